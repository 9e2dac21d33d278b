// Kaldi fbank -> LFR -> CMVN frontend (WavFrontend.forward, funasr/frontends/wav_frontend.py:118-158).
//
// Algorithm = kaldi-native-fbank as vendored by the reference and used by its C++ runtime
// (runtime/onnxruntime/src/paraformer.cpp:21-31,298-312) with the WavFrontend options:
// 16 kHz, 25 ms / 10 ms, snip_edges, dither 0, remove_dc_offset, preemph 0.97, hamming,
// 512-point power spectrum, 80 mel bins 20 Hz..8 kHz (mel = 1127 ln(1 + f/700)),
// log(max(e, FLT_EPSILON)):
//   frame f: x = 32768 * wav[160 f .. 160 f + 399]              (feature-window.cc:121-176)
//            x -= mean(x); x[i] -= 0.97 x[i-1] (x[0] -= 0.97 x[0]); x *= hamming  (:177-247)
//            P[k] = |FFT512(x)[k]|^2, k < 256                  (feature-functions.cc:28-47)
//            e[m] = sum_k W[m][k] P[k];  fbank[m] = log(max(e, eps))  (feature-fbank.cc:73-118)
// LFR (apply_lfr, wav_frontend.py:58-74): row i = frames clamp(6i + j - 3, 0, N-1), j = 0..6.
// CMVN (apply_cmvn, :41-55): (x + shift) * scale.
//
// One wave per frame: samples, DC mean (sequential f32 sum) and the window in f32 (as knf), the FFT in
// f64 in LDS (knf runs Ooura's rdft in double; after the f32 rounding of its outputs the two FFTs
// agree), power / mel sums in f32 in knf's order, the log as f64 rounded to f32. Bit-identical to the
// compiled knf on >= 99.9 % of log-mel entries (the rest differ by one ulp: glibc's logf is not
// correctly rounded everywhere).
#include <math.h>

#include <vector>

#include "pfm_common.h"

namespace {

constexpr int FL = 400, FS = 160, NFFT = 512, NBIN = 256, NMEL = 80, LFR_M = 7, LFR_N = 6;
constexpr int FPB = 4;   // frames (waves) per workgroup; each wave owns its LDS slice

// Orders one wave's LDS writes before its later LDS reads by other lanes (no workgroup barrier:
// waves never share LDS here).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__host__ __device__ inline int frames_of(int n) { return n < FL ? 0 : 1 + (n - FL) / FS; }

__global__ __launch_bounds__(256) void fbank_kernel(const float* __restrict__ wav, const int* __restrict__ nsamp,
                                                    int B, int S_max, int N_cap, const float* __restrict__ window,
                                                    const double2* __restrict__ tw, const float* __restrict__ melw,
                                                    const int* __restrict__ mlo, const int* __restrict__ mhi,
                                                    float* __restrict__ fb) {
    __shared__ double2 buf[FPB][NFFT];
    __shared__ __attribute__((aligned(16))) float xs[FPB][NFFT];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long gf = (long long)blockIdx.x * FPB + w;     // global frame slot = b * N_cap + f
    const int b = (int)(gf / N_cap), f = (int)(gf % N_cap);
    const bool active = b < B && f < frames_of(min(nsamp[min(b, B - 1)], S_max));
    double2* z = buf[w];
    float* x = xs[w];
    if (active) {
        const float* src = wav + (long long)b * S_max + (long long)f * FS;
        // 1. load + scale; the DC mean as knf's sequential f32 sum / 400 (feature-window.cc:179-190):
        //    one lane walks the 400 samples in order (an f64 or tree sum rounds differently)
        for (int i = lane; i < FL; i += 64) x[i] = src[i] * 32768.0f;
        wave_sync();
        float s = 0.f;
        if (lane == 0) {
#pragma unroll 4
            for (int i = 0; i < FL; i += 4) {
                const float4 v = *reinterpret_cast<const float4*>(x + i);
                s += v.x; s += v.y; s += v.z; s += v.w;
            }
        }
        const float mean = __shfl(s, 0) / (float)FL;
        // 2. DC removal, pre-emphasis (uses the un-emphasised neighbour), window
        float y[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const int i = lane + 64 * j;
            if (i < FL) {
                const float cur = x[i] - mean;
                const float prev = (i > 0 ? x[i - 1] : x[0]) - mean;
                y[j] = (cur - 0.97f * prev) * window[i];
            }
        }
        // 3. bit-reversed load into the complex FFT buffer (zero-padded to 512)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = lane + 64 * j;
            const int r = __brev((unsigned)i) >> (32 - 9);
            const double v = (j < 7 && i < FL) ? (double)y[j] : 0.0;
            z[r] = make_double2(v, 0.0);
        }
        wave_sync();
        // 4. radix-2 DIT FFT, 9 stages, 256 butterflies per stage = 4 per lane
        for (int s = 1; s <= 9; ++s) {
            const int half = 1 << (s - 1);
            const int tstep = NFFT >> s;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int bf = lane + 64 * j;
                const int grp = bf / half, pos = bf % half;
                const int i0 = grp * 2 * half + pos, i1 = i0 + half;
                const double2 wv = tw[pos * tstep];
                const double2 a = z[i0], c = z[i1];
                const double tr = c.x * wv.x - c.y * wv.y, ti = c.x * wv.y + c.y * wv.x;
                z[i0] = make_double2(a.x + tr, a.y + ti);
                z[i1] = make_double2(a.x - tr, a.y - ti);
            }
            wave_sync();
        }
        // 5. power spectrum in f32 (values rounded to f32 first, as knf copies the FFT back to float)
        for (int k = lane; k < NBIN; k += 64) {
            const float re = (float)z[k].x, im = (float)z[k].y;
            x[k] = re * re + im * im;
        }
        wave_sync();
        // 6. mel energies (sequential f32 sum over the bin's support) + log floor
        float* out = fb + ((long long)b * N_cap + f) * NMEL;
        for (int m = lane; m < NMEL; m += 64) {
            float e = 0.f;
            for (int k = mlo[m]; k <= mhi[m]; ++k) e += melw[m * NBIN + k] * x[k];
            // log(max(e, FLT_EPSILON)) (feature-fbank.cc:102-108) as the f64 log rounded once: the
            // correctly rounded logf (ocml's f32 logf is within an ulp, not rounded the same way)
            out[m] = (float)log((double)fmaxf(e, 1.1920928955078125e-07f));
        }
    }
}

__global__ __launch_bounds__(256) void lfr_cmvn_kernel(const float* __restrict__ fb, const int* __restrict__ nsamp,
                                                       int B, int S_max, int N_cap, const float* __restrict__ cmvn,
                                                       float* __restrict__ feats, int T_cap, int* __restrict__ T_out) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // one float4 of output
    const int q = LFR_M * NMEL / 4;                                           // 140 float4 per row
    if (gid >= (long long)B * T_cap * q) return;
    const int c4 = (int)(gid % q);
    const long long row = gid / q;
    const int b = (int)(row / T_cap), i = (int)(row % T_cap);
    const int N = frames_of(min(nsamp[b], S_max));
    const int T = (N + LFR_N - 1) / LFR_N;
    if (c4 == 0 && i == 0) T_out[b] = T;
    float4 v = make_float4(0, 0, 0, 0);
    if (i < T) {
        const int col = c4 * 4, j = col / NMEL, m = col % NMEL;
        int fi = i * LFR_N + j - (LFR_M - 1) / 2;
        fi = fi < 0 ? 0 : (fi > N - 1 ? N - 1 : fi);
        v = *(const float4*)(fb + ((long long)b * N_cap + fi) * NMEL + m);
        if (cmvn) {
            const float4 sh = *(const float4*)(cmvn + col), sc = *(const float4*)(cmvn + LFR_M * NMEL + col);
            v.x = (v.x + sh.x) * sc.x; v.y = (v.y + sh.y) * sc.y;
            v.z = (v.z + sh.z) * sc.z; v.w = (v.w + sh.w) * sc.w;
        }
    }
    *(float4*)(feats + row * (LFR_M * NMEL) + c4 * 4) = v;
}

// Online LFR (WavFrontendOnline.apply_lfr, wav_frontend.py:275-310, + apply_cmvn): row r stacks the
// m frames frames[idx[r * m + j]], j = 0..m-1 (indices computed on the host from the splice-cache and
// frame counts, the only state the reference's as_strided depends on). One float4 of output per thread.
__global__ __launch_bounds__(256) void lfr_gather_kernel(const float* __restrict__ frames, const int* __restrict__ idx,
                                                         int rows, int m, const float* __restrict__ cmvn,
                                                         float* __restrict__ out) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int q = m * NMEL / 4;
    if (gid >= (long long)rows * q) return;
    const int c4 = (int)(gid % q);
    const int r = (int)(gid / q);
    const int col = c4 * 4, j = col / NMEL, mm = col % NMEL;
    float4 v = *(const float4*)(frames + (long long)idx[r * m + j] * NMEL + mm);
    if (cmvn) {
        const float4 sh = *(const float4*)(cmvn + col), sc = *(const float4*)(cmvn + m * NMEL + col);
        v.x = (v.x + sh.x) * sc.x; v.y = (v.y + sh.y) * sc.y;
        v.z = (v.z + sh.z) * sc.z; v.w = (v.w + sh.w) * sc.w;
    }
    *(float4*)(out + (long long)r * (m * NMEL) + col) = v;
}

}  // namespace

hipError_t pfm_fbank_raw_launch(const float* wav, const int* nsamp, int B, int S_max, const unsigned char* tables,
                                float* fb, int N_cap, hipStream_t st) {
    const float* melw = (const float*)tables;
    const int* lo = (const int*)(tables + NMEL * NBIN * 4);
    const int* hi = lo + NMEL;
    const float* window = (const float*)(hi + NMEL);
    const size_t twoff = ((size_t)(NMEL * NBIN * 4 + NMEL * 8 + FL * 4) + 15) & ~size_t(15);
    const double2* tw = (const double2*)(tables + twoff);
    const long long nfr = (long long)B * N_cap;
    {
        hipError_t e = hipMemsetAsync(fb, 0, (size_t)nfr * NMEL * 4, st);
        if (e != hipSuccess) return e;
    }
    if (nfr == 0) return hipSuccess;
    hipLaunchKernelGGL(fbank_kernel, dim3((unsigned)((nfr + FPB - 1) / FPB)), dim3(256), 0, st, wav, nsamp, B, S_max,
                       N_cap, window, tw, melw, lo, hi, fb);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_lfr_gather_launch(const float* frames, const int* idx, int rows, int m, const float* cmvn, float* out,
                                 hipStream_t st) {
    const long long n4 = (long long)rows * (m * NMEL / 4);
    if (n4 == 0) return hipSuccess;
    hipLaunchKernelGGL(lfr_gather_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, frames, idx, rows, m,
                       cmvn, out);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

int pfm_fbank_frames(int nsamp) {
    const int n = frames_of(nsamp);
    return (n + LFR_N - 1) / LFR_N;
}

// Host tables mirroring knf: hamming window (double -> float, feature-window.cc:25-55), mel
// triangles in f32 (mel-computations.cc:107-221), twiddles exp(-2 pi i k / 512) in f64.
void pfm_fbank_tables(float* melw, int* lo, int* hi, float* window, double* tw /*[2*256]*/) {
    const double a = 2.0 * M_PI / (FL - 1);
    for (int i = 0; i < FL; ++i) window[i] = (float)(0.54 - 0.46 * cos(a * (double)i));
    // knf evaluates MelScale at run time with the C library's logf; a constant-folded logf(20 Hz) /
    // logf(8 kHz) is correctly rounded instead and moves the triangle edges by an ulp (bins 0, 9-12)
    auto mel = [](float f) { return 1127.0f * logf(1.0f + f / 700.0f); };
    const float fft_bin_width = 16000.0f / NFFT;
    volatile float f_low = 20.0f, f_high = 8000.0f;
    const float mlow = mel(f_low), mhigh = mel(f_high);
    const float delta = (mhigh - mlow) / (NMEL + 1);
    for (int m = 0; m < NMEL; ++m) {
        const float left = mlow + m * delta, center = mlow + (m + 1) * delta, right = mlow + (m + 2) * delta;
        lo[m] = -1; hi[m] = -2;
        for (int k = 0; k < NBIN; ++k) {
            const float mf = mel(fft_bin_width * k);
            float wv = 0.f;
            if (mf > left && mf < right) {
                wv = mf <= center ? (mf - left) / (center - left) : (right - mf) / (right - center);
                if (lo[m] < 0) lo[m] = k;
                hi[m] = k;
            }
            melw[m * NBIN + k] = wv;
        }
    }
    for (int k = 0; k < NBIN; ++k) {
        tw[2 * k] = cos(-2.0 * M_PI * k / NFFT);
        tw[2 * k + 1] = sin(-2.0 * M_PI * k / NFFT);
    }
}

size_t pfm_fbank_table_bytes() { return NMEL * NBIN * 4 + NMEL * 4 * 2 + FL * 4 + NBIN * 16 + 64; }

// tables: device block laid out [melw | lo | hi | window | pad | tw]
hipError_t pfm_fbank_launch(const float* wav, const int* nsamp, int B, int S_max, const float* cmvn,
                            const unsigned char* tables, float* fb_ws, int N_cap, float* feats, int T_cap, int* T_out,
                            hipStream_t st) {
    const float* melw = (const float*)tables;
    const int* lo = (const int*)(tables + NMEL * NBIN * 4);
    const int* hi = lo + NMEL;
    const float* window = (const float*)(hi + NMEL);
    const size_t twoff = ((size_t)(NMEL * NBIN * 4 + NMEL * 8 + FL * 4) + 15) & ~size_t(15);
    const double2* tw = (const double2*)(tables + twoff);
    const long long nfr = (long long)B * N_cap;
    if (nfr > 0) {
        hipLaunchKernelGGL(fbank_kernel, dim3((unsigned)((nfr + FPB - 1) / FPB)), dim3(256), 0, st, wav, nsamp, B, S_max,
                           N_cap, window, tw, melw, lo, hi, fb_ws);
        PFM_LAUNCH_CHECK();
    }
    const long long n4 = (long long)B * T_cap * (LFR_M * NMEL / 4);
    hipLaunchKernelGGL(lfr_cmvn_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, fb_ws, nsamp, B, S_max,
                       N_cap, cmvn, feats, T_cap, T_out);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

size_t pfm_fbank_twoff() { return ((size_t)(NMEL * NBIN * 4 + NMEL * 8 + FL * 4) + 15) & ~size_t(15); }
int pfm_fbank_nframes(int nsamp) { return frames_of(nsamp); }
