// Fused masked multi-head attention for SAN-M self-attention and decoder cross-attention.
//
// Replaces MultiHeadedAttentionSANM.forward/forward_attention (funasr/models/sanm/attention.py:
// 254-311) and MultiHeadedAttentionCrossAtt.forward (attention.py:631-717):
//     out = softmax((q * d_k^-0.5) k^T, -inf on keys t >= len) v,   d_k = 128
// without materialising the [T, T] score matrix (flash-style online softmax).
//
// One workgroup = 4 waves = 128 query rows of one (utterance, head); each wave owns 32 rows.
// The products are computed SWAPPED: S^T = K.Q^T and O^T = V^T.P^T, so in every MFMA
// accumulator the query row is the lane (q = lane & 31) and keys / head dims run over the
// registers. The running max / sum of a query row is therefore lane-local (one xor-32
// shuffle joins the two half-waves) and the O rescale is a per-lane scalar multiply.
//
// f32 ("exact"): v_mfma_f32_32x32x2_f32 — S^T 64 MFMA + O^T 64 MFMA per 32-key tile.
// bf16 ("fast"): v_mfma_f32_32x32x16_bf16 — 8 + 8 MFMA per tile; P^T feeds the second
//   product straight from the S^T accumulator registers (k-order permuted accordingly) and
//   V is staged transposed in LDS.
#include <stdlib.h>

#include <stdint.h>

#include "pfm_common.h"
#include "pfm_stream.h"

namespace {

constexpr int DK = 128;
constexpr int KT = 32;            // keys per tile
constexpr int QW = 32;            // query rows per wave

struct AttnArgs {
    const void* q; RowMap qmap;   // query rows: row m = b*Tq + t; head h at +h*DK
    const void* k; RowMap kmap;   // key rows:   row m = b*Tk + t
    const void* v; RowMap vmap;
    float* o; long long ldo;      // output rows b*Tq + t, head h at column h*DK (f32)
    void* o2; int o2_dtype;       // optional bf16 copy (fast mode)
    const int* klen;              // [B] valid keys
    int Tq, Tk;
    float scale;
    // optional fused FSMN memory block (encoder self-attention, fast mode): fout[b*Tq + t][h*DK + c] =
    // mask * (sum_k fw[k][h*DK + c] * vm[t - 5 + k] + vm[t]), vm = V rows masked by klen (K = 11, left 5)
    const float* fw; bf16* fout; long long fld; int fD;
    float* fout32 = nullptr;      // EXACT mode (x6 kernel): the same FSMN block in f32 (fout's row stride fld)
    // optional streaming cache retain, fused (bf16 kernels; kv_retain_kernel of k_stream.hip): after the key loop the
    // blocks of query tile 0 copy head h's K and V columns of stream b's new cache rows — the last min(C, cl + tw -
    // drop) key rows — into the slot's cache rows (rt_W elements, V at rt_voff). The key rows are the gathered
    // [cache ; window] buffer, the cache a different array, so no block reads what another writes.
    const SPrm* rt_prm = nullptr;
    bf16* rt_cache = nullptr;
    int rt_C = 0, rt_drop = 0, rt_dec = 0, rt_W = 0, rt_voff = 0;
    const int* rt_ntok = nullptr;   // decoder caches move only for streams whose decoder ran
};

// ---- f32 tile geometry (bytes)
constexpr int KP32 = DK * 4 + 16;   // K tile row pitch 528 B: ds_read_b128 rows conflict-free
constexpr int VP32 = DK * 4;        // V tile row pitch 512 B (ds_read_b32 per lane, no conflict)
constexpr int LDS32 = 2 * (KT * KP32 + KT * VP32);
// ---- bf16 tile geometry
constexpr int KP16 = DK * 2 + 16;   // 272 B
constexpr int VTP16 = KT * 2 + 8;   // V^T row (one head dim, 32 keys) pitch 72 B: b64 reads conflict-free
constexpr int LDS16 = 2 * (KT * KP16 + DK * VTP16);

__device__ __forceinline__ int kappa(int e) { return (e & 3) + 8 * (e >> 2); }

// x combined with lane ^ 32's x by one v_permlane32_swap (the swap of x with itself leaves {own, partner} in every lane,
// in an order that depends on the half; max and + are commutative, so the result equals op(x, __shfl_xor(x, 32)) bit
// for bit — without the ds_bpermute round trip through the LDS pipe)
__device__ __forceinline__ float xor32_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_add(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <typename T> struct AttnLds;

// XCD-aware block order: consecutive linear block ids go to the 8 XCDs round-robin, so with the plain order the
// query blocks of one (utterance, head) land on different XCDs and each fetches the K / V rows from HBM into its own
// L2. Here the nq query blocks of one (utterance, head) take linear ids 8 apart (i, i + 8, ...): the same XCD, dispatched
// together, so the later ones read the key tiles from that L2. A bijection of the grid; results are unchanged.
__device__ __forceinline__ void attn_block(int& qt, int& h, int& b) {
    qt = blockIdx.x; h = blockIdx.y; b = blockIdx.z;
    const int nq = gridDim.x, nbh = gridDim.y * gridDim.z;
    if (nq > 1 && (nbh & 7) == 0) {
        const int id = blockIdx.x + nq * (blockIdx.y + gridDim.y * blockIdx.z);
        const int g = id / (8 * nq), r = id - g * 8 * nq;
        const int bh = 8 * g + (r & 7);
        qt = r >> 3;
        h = bh % gridDim.y;
        b = bh / gridDim.y;
    }
}

__global__ __launch_bounds__(256) void attn_f32_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int qt, h, b;
    attn_block(qt, h, b);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 31, fh = lane >> 5;
    const int klen = min(a.klen[b], a.Tk);
    const float* Q = (const float*)a.q;
    const float* K = (const float*)a.k;
    const float* V = (const float*)a.v;

    // Q fragment in registers: lane (q = fr) holds dims 8kq + 4fh + c, pre-scaled like q_h * d_k^-0.5
    const int qrow = qt * 128 + wid * QW + fr;
    float4 qf[16];
    {
        const bool ok = qrow < a.Tq;
        const float* qp = Q + a.qmap.off((long long)b * a.Tq + (ok ? qrow : 0)) + h * DK;
#pragma unroll
        for (int kq = 0; kq < 16; ++kq) {
            float4 x = ok ? *(const float4*)(qp + kq * 8 + fh * 4) : make_float4(0, 0, 0, 0);
            qf[kq] = make_float4(x.x * a.scale, x.y * a.scale, x.z * a.scale, x.w * a.scale);
        }
    }
    f32x16 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[d][e] = 0.f;
    float mrun = -INFINITY, lrun = 0.f;

    const int ntiles = (klen + KT - 1) / KT;
    // staging: K and V tiles, 32 rows x 512 B each = 1024 x 16 B chunks each; 4+4 per thread
    auto stage = [&](int t, int s) {
        unsigned char* Ks = smem + s * (KT * KP32 + KT * VP32);
        unsigned char* Vs = Ks + KT * KP32;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i, row = c >> 5, ch = c & 31;
            const int key = t * KT + row;
            float4 kx = make_float4(0, 0, 0, 0), vx = make_float4(0, 0, 0, 0);
            if (key < klen) {
                const long long m = (long long)b * a.Tk + key;
                kx = *(const float4*)(K + a.kmap.off(m) + h * DK + ch * 4);
                vx = *(const float4*)(V + a.vmap.off(m) + h * DK + ch * 4);
            }
            *(float4*)(Ks + row * KP32 + ch * 16) = kx;
            *(float4*)(Vs + row * VP32 + ch * 16) = vx;
        }
    };
    if (ntiles > 0) stage(0, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (t + 1 < ntiles) stage(t + 1, cur ^ 1);
        const unsigned char* Ks = smem + cur * (KT * KP32 + KT * VP32);
        const float* Vs = (const float*)(Ks + KT * KP32);
        // S^T[key][q] = sum_d K[key][d] Q[q][d]
        f32x16 s;
#pragma unroll
        for (int e = 0; e < 16; ++e) s[e] = 0.f;
#pragma unroll
        for (int kq = 0; kq < 16; ++kq) {
            const float4 kx = *(const float4*)(Ks + fr * KP32 + kq * 32 + fh * 16);
            s = __builtin_amdgcn_mfma_f32_32x32x2f32(kx.x, qf[kq].x, s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_32x32x2f32(kx.y, qf[kq].y, s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_32x32x2f32(kx.z, qf[kq].z, s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_32x32x2f32(kx.w, qf[kq].w, s, 0, 0, 0);
        }
        // lane holds S^T[key = kappa(e) + 4fh][q = fr]; mask keys >= klen
        float mt = -INFINITY;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int key = t * KT + kappa(e) + 4 * fh;
            if (key >= klen) s[e] = -INFINITY;
            mt = fmaxf(mt, s[e]);
        }
        mt = xor32_max(mt);
        const float mnew = fmaxf(mrun, mt);
        const float corr = expf(mrun - mnew);
        float ls = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            s[e] = expf(s[e] - mnew);
            ls += s[e];
        }
        ls = xor32_add(ls);
        lrun = lrun * corr + ls;
        mrun = mnew;
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[d][e] *= corr;
        // O^T[d][q] += sum_key V[key][d] P[q][key]; MFMA step e sums keys kappa(e) (+4 on half 1)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const float* vr = Vs + (kappa(e) + 4 * fh) * (VP32 / 4);
#pragma unroll
            for (int d = 0; d < 4; ++d)
                o[d] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr[d * 32 + fr], s[e], o[d], 0, 0, 0);
        }
        __syncthreads();
    }
    if (qrow >= a.Tq) return;
    const float inv = (klen > 0) ? 1.f / lrun : 0.f;
    float* op = a.o ? a.o + ((long long)b * a.Tq + qrow) * a.ldo + h * DK : nullptr;
    bf16* op2 = a.o2 ? (bf16*)a.o2 + ((long long)b * a.Tq + qrow) * a.ldo + h * DK : nullptr;
    const bool x3 = a.o2_dtype == DT_X3;   // split output (planes a.fD apart): the out-projection's operand
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {   // registers 4g..4g+3 are 4 consecutive head dims
            const int col = d * 32 + 8 * g + 4 * fh;
            const float v[4] = {o[d][4 * g] * inv, o[d][4 * g + 1] * inv, o[d][4 * g + 2] * inv, o[d][4 * g + 3] * inv};
            if (op) *(float4*)(op + col) = make_float4(v[0], v[1], v[2], v[3]);
            if (op2) {
                if (x3) {
                    bf16x4 p0, p1, p2;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        bf16 u, w, z;
                        split3_bf16(v[i], u, w, z);
                        p0[i] = u; p1[i] = w; p2[i] = z;
                    }
                    *(bf16x4*)(op2 + col) = p0;
                    *(bf16x4*)(op2 + col + a.fD) = p1;
                    *(bf16x4*)(op2 + col + 2 * a.fD) = p2;
                } else {
                    bf16x4 t = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
                    *(bf16x4*)(op2 + col) = t;
                }
            }
        }
}

// ---- EXACT mode on bf16 MFMA: split-bf16 emulation of the f32 kernel above (same swapped products,
// same online softmax in f32). Every f32 operand x is split as x0 + x1 + x2 (bf16, exact), and each f32
// product a.b becomes a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0 on v_mfma_f32_32x32x16_bf16 (dropped
// terms <= 2^-25 |ab|, f32 accumulation): S^T = K.Q^T and O^T = V^T.P^T at f32 accuracy for 6x the
// bf16 MFMA work, i.e. 2.7x the f32-MFMA ceiling. 8 waves = 256 query rows per workgroup; 32-key tiles
// staged from f32 rows into LDS as three bf16 planes (K row-major, V transposed in the permuted key
// order that P^T takes straight from the S^T accumulator registers), double-buffered.
constexpr int X6_KT = 32;
constexpr int X6_KP = DK * 2 + 16;            // K plane row pitch 272 B (32 key rows)
constexpr int X6_VP = X6_KT * 2 + 16;         // V^T plane row pitch 80 B (128 dim rows): b128 reads conflict-free
constexpr int X6_KPL = X6_KT * X6_KP, X6_VPL = DK * X6_VP;
constexpr int X6_STG = 3 * (X6_KPL + X6_VPL);
constexpr int X6_LDS = 2 * X6_STG;

__device__ __forceinline__ void x6_split(float x, bf16& a, bf16& b, bf16& c) {
    a = f2bf(x);
    const float r = x - bf2f(a);
    b = f2bf(r);
    c = f2bf(r - bf2f(b));
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// c += a.b with a = a0+a1+a2, b = b0+b1+b2 (small products first)
__device__ __forceinline__ f32x16 mfma_x6(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                          const bf16x8& b1, const bf16x8& b2, f32x16 c) {
    c = mfma32(a2, b0, c);
    c = mfma32(a1, b1, c);
    c = mfma32(a0, b2, c);
    c = mfma32(a1, b0, c);
    c = mfma32(a0, b1, c);
    return mfma32(a0, b0, c);
}

// Fused FSMN memory block, EXACT mode (f32 V in, f32 out): the arithmetic of fsmn_win_kernel<11, float, 5>
// (fma chain over the 11 taps ascending from 0, then + x[t]; rows t >= klen are 0). Thread = 4 channels x
// 8 rows of the block's QB rows x this head's 128 channels; the window comes from global memory (V was just
// streamed by the key loop). No barriers: threads past Tq simply stop.
template <int QB, int NTH>
__device__ __forceinline__ void fsmn_epilogue_f32(const AttnArgs& a, int qt, int h, int b, int klen) {
    constexpr int FK = 11, FL = 5, CQ = DK / 4, RPT = 8, RG = NTH / CQ;
    static_assert(QB % (RG * RPT) == 0, "whole passes of RG x RPT rows");
    const int cq = threadIdx.x % CQ, rg = threadIdx.x / CQ;
    const int c = h * DK + cq * 4;
    const float* V = (const float*)a.v;
    float4 w[FK];
#pragma unroll
    for (int k = 0; k < FK; ++k) w[k] = *(const float4*)(a.fw + (long long)k * a.fD + c);
#pragma unroll 1
    for (int pass = 0; pass < QB / (RG * RPT); ++pass) {
        const int t0 = qt * QB + (pass * RG + rg) * RPT;
        if (t0 >= a.Tq) break;
        float4 x[RPT + FK - 1];
#pragma unroll
        for (int i = 0; i < RPT + FK - 1; ++i) {
            const int tc = min(max(t0 - FL + i, 0), a.Tk - 1);
            x[i] = *(const float4*)(V + a.vmap.off((long long)b * a.Tk + tc) + c);
        }
#pragma unroll
        for (int i = 0; i < RPT + FK - 1; ++i) {
            const int tt = t0 - FL + i;
            if (!(tt >= 0 && tt < klen)) x[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int t = t0 + i;
            if (t >= a.Tq) break;
            float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t < klen) {
                float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int k = 0; k < FK; ++k) {
                    acc.x = fmaf(w[k].x, x[i + k].x, acc.x);
                    acc.y = fmaf(w[k].y, x[i + k].y, acc.y);
                    acc.z = fmaf(w[k].z, x[i + k].z, acc.z);
                    acc.w = fmaf(w[k].w, x[i + k].w, acc.w);
                }
                const float4 self = x[i + FL];
                y = make_float4(acc.x + self.x, acc.y + self.y, acc.z + self.z, acc.w + self.w);
            }
            *(float4*)(a.fout32 + ((long long)b * a.Tq + t) * a.fld + c) = y;
        }
    }
}

// VAR (diagnostic instantiations for standalone timing; the library instantiates VAR 0): 1 no staging after tile
// 0, 2 no softmax, 3 no PV products, 4 no QK products
template <int VAR = 0>
__global__ __launch_bounds__(512) void attn_x6_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int qt, h, b;
    attn_block(qt, h, b);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 31, fh = lane >> 5;
    const int klen = min(a.klen[b], a.Tk);
    const float* Q = (const float*)a.q;
    const float* K = (const float*)a.k;
    const float* V = (const float*)a.v;

    // Q^T fragments (B operand): lane (q = fr) holds dims 16ks + 8fh + j, pre-scaled, split in three
    const int qrow = qt * 256 + wid * QW + fr;
    bf16x8 q0[8], q1[8], q2[8];
    {
        const bool ok = qrow < a.Tq;
        const float* qp = Q + a.qmap.off((long long)b * a.Tq + (ok ? qrow : 0)) + h * DK;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const float4 x0 = ok ? *(const float4*)(qp + ks * 16 + fh * 8) : make_float4(0, 0, 0, 0);
            const float4 x1 = ok ? *(const float4*)(qp + ks * 16 + fh * 8 + 4) : make_float4(0, 0, 0, 0);
            const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                bf16 u, v, w;
                x6_split(xv[j] * a.scale, u, v, w);
                q0[ks][j] = u; q1[ks][j] = v; q2[ks][j] = w;
            }
        }
    }
    f32x16 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[d][e] = 0.f;
    float mrun = -INFINITY, lrun = 0.f;
    const int ntiles = (klen + X6_KT - 1) / X6_KT;

    // staging of one 32-key tile: threads 0..255 take a 4-key x 4-dim block of V (written transposed,
    // key quad at its permuted slot: P^T k-step s lane half fh holds keys 16s + 8(j>>2) + 4fh + (j&3)),
    // threads 256..511 four 4-dim chunks of K rows; keys >= klen are zeros
    auto stage = [&](int t, int sbuf) {
        unsigned char* Ks = smem + sbuf * X6_STG;
        unsigned char* Vs = Ks + 3 * X6_KPL;
        if (tid < 256) {
            const int kq4 = tid >> 5, dq = tid & 31;   // keys 4kq4.., dims 4dq..
            float xv[4][4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = t * X6_KT + 4 * kq4 + r;
                float4 x = make_float4(0, 0, 0, 0);
                if (key < klen) x = *(const float4*)(V + a.vmap.off((long long)b * a.Tk + key) + h * DK + 4 * dq);
                xv[r][0] = x.x; xv[r][1] = x.y; xv[r][2] = x.z; xv[r][3] = x.w;
            }
            const int s16 = kq4 >> 2, w4 = kq4 & 3, pos = ((w4 & 1) << 1) | (w4 >> 1);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                bf16x4 p0, p1, p2;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    bf16 u, v, w;
                    x6_split(xv[r][c], u, v, w);
                    p0[r] = u; p1[r] = v; p2[r] = w;
                }
                const int off = (4 * dq + c) * X6_VP + s16 * 32 + pos * 8;
                *(bf16x4*)(Vs + off) = p0;
                *(bf16x4*)(Vs + X6_VPL + off) = p1;
                *(bf16x4*)(Vs + 2 * X6_VPL + off) = p2;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = (tid - 256) + 256 * i, row = c >> 5, ch = c & 31;
                const int key = t * X6_KT + row;
                float4 x = make_float4(0, 0, 0, 0);
                if (key < klen) x = *(const float4*)(K + a.kmap.off((long long)b * a.Tk + key) + h * DK + ch * 4);
                const float xv[4] = {x.x, x.y, x.z, x.w};
                bf16x4 p0, p1, p2;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    bf16 u, v, w;
                    x6_split(xv[e], u, v, w);
                    p0[e] = u; p1[e] = v; p2[e] = w;
                }
                const int off = row * X6_KP + ch * 8;
                *(bf16x4*)(Ks + off) = p0;
                *(bf16x4*)(Ks + X6_KPL + off) = p1;
                *(bf16x4*)(Ks + 2 * X6_KPL + off) = p2;
            }
        }
    };
    if (ntiles > 0) stage(0, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (VAR != 1 && t + 1 < ntiles) stage(t + 1, cur ^ 1);
        const unsigned char* Ks = smem + (VAR == 1 ? 0 : cur) * X6_STG;
        const unsigned char* Vs = Ks + 3 * X6_KPL;
        // S^T[key][q]: A = K rows (key = fr, dims 16ks + 8fh ..), B = Q^T
        f32x16 s;
#pragma unroll
        for (int e = 0; e < 16; ++e) s[e] = 0.f;
#pragma unroll
        for (int ks = 0; ks < (VAR == 4 ? 0 : 8); ++ks) {
            const unsigned char* kp = Ks + fr * X6_KP + ks * 32 + fh * 16;
            const bf16x8 k0 = *(const bf16x8*)kp, k1 = *(const bf16x8*)(kp + X6_KPL),
                         k2 = *(const bf16x8*)(kp + 2 * X6_KPL);
            s = mfma_x6(k0, k1, k2, q0[ks], q1[ks], q2[ks], s);
        }
        // identical masking / online softmax to attn_f32_kernel
        if constexpr (VAR == 2) {
            lrun = 1.f;
        } else {
        float mt = -INFINITY;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int key = t * X6_KT + kappa(e) + 4 * fh;
            if (key >= klen) s[e] = -INFINITY;
            mt = fmaxf(mt, s[e]);
        }
        mt = xor32_max(mt);
        const float mnew = fmaxf(mrun, mt);
        const float corr = expf(mrun - mnew);
        float ls = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            s[e] = expf(s[e] - mnew);
            ls += s[e];
        }
        ls = xor32_add(ls);
        lrun = lrun * corr + ls;
        mrun = mnew;
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[d][e] *= corr;
        }
        // O^T[d][q] += V^T.P^T: k step s16 takes accumulator registers 8 s16 .. 8 s16 + 7 as P^T
#pragma unroll
        for (int s16 = 0; s16 < (VAR == 3 ? 0 : 2); ++s16) {
            bf16x8 p0, p1, p2;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                bf16 u, v, w;
                x6_split(s[8 * s16 + j], u, v, w);
                p0[j] = u; p1[j] = v; p2[j] = w;
            }
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const unsigned char* vp = Vs + (32 * d + fr) * X6_VP + s16 * 32 + fh * 16;
                const bf16x8 v0 = *(const bf16x8*)vp, v1 = *(const bf16x8*)(vp + X6_VPL),
                             v2 = *(const bf16x8*)(vp + 2 * X6_VPL);
                o[d] = mfma_x6(v0, v1, v2, p0, p1, p2, o[d]);
            }
        }
        __syncthreads();
    }
    if (qrow < a.Tq) {
    const float inv = (klen > 0) ? 1.f / lrun : 0.f;
    float* op = a.o ? a.o + ((long long)b * a.Tq + qrow) * a.ldo + h * DK : nullptr;
    bf16* op2 = a.o2 ? (bf16*)a.o2 + ((long long)b * a.Tq + qrow) * a.ldo + h * DK : nullptr;
    const bool x3 = a.o2_dtype == DT_X3;   // split output (planes a.fD apart): the out-projection's operand
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {   // registers 4g..4g+3 are 4 consecutive head dims
            const int col = d * 32 + 8 * g + 4 * fh;
            const float v[4] = {o[d][4 * g] * inv, o[d][4 * g + 1] * inv, o[d][4 * g + 2] * inv, o[d][4 * g + 3] * inv};
            if (op) *(float4*)(op + col) = make_float4(v[0], v[1], v[2], v[3]);
            if (op2) {
                if (x3) {
                    bf16x4 p0, p1, p2;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        bf16 u, w, z;
                        split3_bf16(v[i], u, w, z);
                        p0[i] = u; p1[i] = w; p2[i] = z;
                    }
                    *(bf16x4*)(op2 + col) = p0;
                    *(bf16x4*)(op2 + col + a.fD) = p1;
                    *(bf16x4*)(op2 + col + 2 * a.fD) = p2;
                } else {
                    bf16x4 t = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
                    *(bf16x4*)(op2 + col) = t;
                }
            }
        }
    }
    if (a.fout32) fsmn_epilogue_f32<256, 512>(a, qt, h, b, klen);
}

// ---- bf16 kernel geometry: 64-key tiles; K row-major with a 16-B chunk XOR swizzle (conflict-free
// ds_read_b128 of 16 distinct rows); V row-major with a 320-B pitch so the transposing
// ds_read_b64_tr_b16 reads (4 key rows x 32 B per half-wave) hit 64 distinct banks.
constexpr int KT2 = 64;
constexpr int KROW = DK * 2;                    // 256 B
constexpr int VROW = DK * 2 + 64;               // 320 B
constexpr int KTILE = KT2 * KROW, VTILE = KT2 * VROW;
constexpr int STG2 = KTILE + VTILE;             // 36 KiB per stage
constexpr int FSMN_LDS = (256 + 10) * DK * 2 + 11 * DK * 4;   // fused FSMN window + taps (8-wave kernel)
constexpr int LDS8_FS = 2 * STG2 + FSMN_LDS;            // K/V stages + the FSMN window captured beside them
constexpr float RESCALE_THR = 8.0f;             // lazy O rescale: only when a row max grows by > 8
#ifndef ATTN_CSUB
#define ATTN_CSUB 0
#endif
#ifndef ATTN_LMFMA
#define ATTN_LMFMA 0
#endif

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// Fused FSMN memory block for the block's QB query rows x this head's DK channels (encoder
// self-attention: query row == key row). `win` holds V rows [t0-5, t0+QB+5) of head h (rows outside [0, klen)
// as zeros; captured by the key loop) followed by the 11 taps of the head's channels; thread = 8 rows x 8
// channels. Same f32 operation order as fsmn_win_kernel<11, bf16, 5> (taps ascending, then + x[t]).
template <int QB, int NTH>
__device__ __forceinline__ void fsmn_epilogue(const AttnArgs& a, const unsigned char* win, int qt, int h, int b,
                                              int klen) {
    constexpr int FK = 11, FL = 5, FR = QB + FK - 1, RB = DK * 2;   // 256-B rows
    static_assert(NTH == (QB / 8) * (DK / 8), "one thread per 8 rows x 8 channels");
    __syncthreads();                                   // every window row and tap is in LDS
    const int t0 = qt * QB;
    const unsigned char* xs = win;
    const float* ws = (const float*)(win + FR * RB);
    const int rb = threadIdx.x / (DK / 8), c8 = (threadIdx.x % (DK / 8)) * 8;
    float y[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) y[i][j] = 0.f;
    // every window row is read once (18 rows for 8 outputs x 11 taps) and feeds each output it touches; an output's
    // taps still accumulate in ascending k (row r = i + k ascending), the order of fsmn_win_kernel
    float w8[FK][8];
#pragma unroll
    for (int k = 0; k < FK; ++k) {
        const float4 wa = *(const float4*)(ws + k * DK + c8), wb = *(const float4*)(ws + k * DK + c8 + 4);
        w8[k][0] = wa.x; w8[k][1] = wa.y; w8[k][2] = wa.z; w8[k][3] = wa.w;
        w8[k][4] = wb.x; w8[k][5] = wb.y; w8[k][6] = wb.z; w8[k][7] = wb.w;
    }
#pragma unroll
    for (int r = 0; r < 8 + FK - 1; ++r) {
        const bf16x8 x = *(const bf16x8*)(xs + (rb * 8 + r) * RB + c8 * 2);
        float xf[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xf[j] = bf2f(x[j]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int k = r - i;
            if (k < 0 || k >= FK) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) y[i][j] = fmaf(w8[k][j], xf[j], y[i][j]);
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int t = t0 + rb * 8 + i;
        if (t >= a.Tq) break;
        const bf16x8 xself = *(const bf16x8*)(xs + (rb * 8 + i + FL) * RB + c8 * 2);
        bf16x8 ob;
#pragma unroll
        for (int j = 0; j < 8; ++j) ob[j] = f2bf(t < klen ? y[i][j] + bf2f(xself[j]) : 0.f);
        *(bf16x8*)(a.fout + ((long long)b * a.Tq + t) * a.fld + h * DK + c8) = ob;
    }
}

// VAR (diagnostic instantiations for standalone timing — results are wrong; the library instantiates
// VAR 0 only): 1 no K/V loads after tile 0, 2 no softmax (P = S), 3 no PV products, 4 no QK products,
// 5 no key loop (prologue + epilogue only)
// Fused FSMN epilogue (8 waves): the block's V window [t0 - 5, t0 + 261) is captured into its own LDS region from
// the staging registers as the key tiles stream through (rows < klen; the others zeroed up front), so the epilogue
// starts from LDS (re-loading the window from global memory after the key loop: 37.8 -> 35.5 us per encoder group
// launch, tools/attn_bench.hip). bf16-only outputs are stored 16 B per lane: permlane32 swaps pair the two
// half-waves' 8-B pieces of a row (35.5 -> 33.5 us). Both bit-identical to the earlier forms. Measured and not
// kept: two K/V tiles in flight (register staging two tiles ahead: +1.5 %), static priority 1 for the younger half
// of the waves (within noise).
template <int NWV, int VAR = 0>
__global__ __launch_bounds__(NWV * 64, 8 / NWV) void attn_bf16_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NT = NWV * 64, QBLK = NWV * QW;
    int qt, h, b;
    attn_block(qt, h, b);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 31, fh = lane >> 5;
    const int klen = min(a.klen[b], a.Tk);
    const bf16* Q = (const bf16*)a.q;
    const bf16* K = (const bf16*)a.k;
    const bf16* V = (const bf16*)a.v;

    // Q fragment (B operand of S^T = K.Q^T): lane (q = fr) holds dims 16kq + 8fh + j, pre-scaled by
    // d_k^-0.5 * log2(e): scores arrive in log2 units, so each probability is one subtract + v_exp_f32
    const int qrow = qt * QBLK + wid * QW + fr;
    const float qs = a.scale * 1.4426950408889634f;
    bf16x8 qf[8];
    {
        const bool ok = qrow < a.Tq;
        const bf16* qp = Q + a.qmap.off((long long)b * a.Tq + (ok ? qrow : 0)) + h * DK;
#pragma unroll
        for (int kq = 0; kq < 8; ++kq) {
            bf16x8 x;
            if (ok) x = *(const bf16x8*)(qp + kq * 16 + fh * 8);
            else
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = (bf16)0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = f2bf(bf2f(x[j]) * qs);
            qf[kq] = x;
        }
    }
    f32x16 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[d][e] = 0.f;
    float mused = -INFINITY, lrun = 0.f;
    // ATTN_LMFMA: the row sums come from the matrix core, P^T against an all-ones A fragment (every accumulator register
    // of lane q then holds sum_key bf16(P[q][key]): the normaliser of exactly the P the PV products used)
    f32x16 ol;
#pragma unroll
    for (int e = 0; e < 16; ++e) ol[e] = 0.f;
    const int ntiles = (klen + KT2 - 1) / KT2;

    // register staging: each thread moves (64 rows x 16 chunks) / NT chunks of K and of V per tile.
    // An utterance's key rows are `ld` apart (plain map, or one segment per utterance: launcher check),
    // so a chunk's source is utterance base + row * row_bytes + chunk * 16 with 32-bit offsets; rows
    // past klen load the clamped last valid row (masked to -inf in the last tile's scores).
    constexpr int CPT = KT2 * 16 / NT;
    static_assert(CPT == 2 || CPT == 4, "staging struct holds 2 or 4 16-B chunks of K and of V per thread");
    const char* kbase = (const char*)(K + a.kmap.off((long long)b * a.Tk) + h * DK);
    const char* vbase = (const char*)(V + a.vmap.off((long long)b * a.Tk) + h * DK);
    const unsigned krb = (unsigned)a.kmap.ld * 2u, vrb = (unsigned)a.vmap.ld * 2u;
    const int lastrow = max(klen - 1, 0);
    // Named members returned by value (register arrays indexed before unrolling went to scratch).
    struct Stg { uint4 k0, k1, k2, k3, v0, v1, v2, v3; };
    auto ld1 = [&](int t, int c, uint4& kk, uint4& vv) {
        const unsigned row = (unsigned)min(t * KT2 + (c >> 4), lastrow);
        const unsigned cb = (unsigned)(c & 15) * 16u;
        kk = *(const uint4*)(kbase + (row * krb + cb));
        vv = *(const uint4*)(vbase + (row * vrb + cb));
    };
    auto gload = [&](int t) -> Stg {
        Stg r;
        ld1(t, tid, r.k0, r.v0);
        ld1(t, tid + NT, r.k1, r.v1);
        if constexpr (CPT == 4) {
            ld1(t, tid + 2 * NT, r.k2, r.v2);
            ld1(t, tid + 3 * NT, r.k3, r.v3);
        }
        return r;
    };
    auto st1 = [&](unsigned char* base, int c, const uint4& kk, const uint4& vv) {
        const int row = c >> 4, ch = c & 15;
        *(uint4*)(base + row * KROW + ((ch ^ (row & 15)) << 4)) = kk;
        *(uint4*)(base + KTILE + row * VROW + ch * 16) = vv;
    };
    // the block's FSMN window (V rows [fw0, fw0 + QBLK + 10) of this head) lives at smem + 2 STG2
    constexpr bool CAP = NWV == 8;
    const bool cap = CAP && a.fout != nullptr;
    const int fw0 = qt * QBLK - 5;
    unsigned char* fxs = smem + 2 * STG2;
    auto fcap = [&](int t, int c, const uint4& vv) {
        const int row = t * KT2 + (c >> 4), r = row - fw0;
        if (r >= 0 && r < QBLK + 10 && row < klen) *(uint4*)(fxs + r * (DK * 2) + (c & 15) * 16) = vv;
    };
    auto sstore = [&](int s, const Stg& r, int t) {
        unsigned char* base = smem + s * STG2;
        st1(base, tid, r.k0, r.v0);
        st1(base, tid + NT, r.k1, r.v1);
        if constexpr (CPT == 4) {
            st1(base, tid + 2 * NT, r.k2, r.v2);
            st1(base, tid + 3 * NT, r.k3, r.v3);
        }
        if constexpr (CAP) {
            if (cap) {
                fcap(t, tid, r.v0);
                fcap(t, tid + NT, r.v1);
                if constexpr (CPT == 4) {
                    fcap(t, tid + 2 * NT, r.v2);
                    fcap(t, tid + 3 * NT, r.v3);
                }
            }
        }
    };
    // per-lane constants of the transposed V read: lane 4q+p of its 16-lane group addresses key
    // row q, head dims 4p..4p+3 of the group's 16-column block
    const int tg = lane >> 4, ti = lane & 15;
    const int tr_key = 4 * (tg >> 1) + (ti >> 2);
    const int tr_col = 16 * (tg & 1) + 4 * (ti & 3);

    auto compute = [&](int t) {
        const unsigned char* Ks = smem + (t & 1) * STG2;
        const unsigned char* Vs = Ks + KTILE;
        f32x16 s[2];
        // all 16 K fragments of the tile are read before the first product (graduated lgkmcnt waits): left to
        // the scheduler, each ds_read was followed by lgkmcnt(0) and its MFMA, one LDS latency per product
        bf16x8 kx[2][8];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const int row = kb * 32 + fr;
#pragma unroll
            for (int kq = 0; kq < 8; ++kq) kx[kb][kq] = *(const bf16x8*)(Ks + row * KROW + (((2 * kq + fh) ^ (row & 15)) << 4));
        }
        __builtin_amdgcn_sched_barrier(0);
        // ATTN_CSUB: the QK^T chain starts from C = -mused (the running max; 0 before the first tile), so the common
        // path's probabilities are exp2(s) with no per-score subtract (only a tile that moves the max subtracts)
        const float mb = ATTN_CSUB ? (mused == -INFINITY ? 0.f : mused) : 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int e = 0; e < 16; ++e) s[kb][e] = ATTN_CSUB ? -mb : 0.f;
            if constexpr (VAR == 4) continue;
#pragma unroll
            for (int kq = 0; kq < 8; ++kq) s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kx[kb][kq], qf[kq], s[kb], 0, 0, 0);
        }
        // lane holds S^T[key = t*64 + kb*32 + kappa(e) + 4fh][q = fr]
        if constexpr (VAR != 2) {
        if ((t + 1) * KT2 > klen) {   // only the last tile can hold keys past klen
            // a real branch: as a plain `if` the compiler if-converted the masking onto every tile (32 compares +
            // 32 selects per tile); the empty volatile asm keeps it out of the common path
            asm volatile("" ::: "memory");
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int key = t * KT2 + kb * 32 + kappa(e) + 4 * fh;
                    if (key >= klen) s[kb][e] = -INFINITY;
                }
        }
        float mt = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int e = 0; e < 16; ++e) mt = fmaxf(mt, s[kb][e]);
        mt = xor32_max(mt);
        if constexpr (ATTN_CSUB) {   // s holds QK^T - mb: the max test and the rare subtract in those units
            if (mt + mb > mused + RESCALE_THR * 1.4426950408889634f) {   // lazy rescale (log2 units)
                const float corr = __builtin_amdgcn_exp2f(mused - (mt + mb));
                lrun *= corr;
#pragma unroll
                for (int d = 0; d < 4; ++d)
#pragma unroll
                    for (int e = 0; e < 16; ++e) o[d][e] *= corr;
                if constexpr (ATTN_LMFMA) ol *= corr;
                mused = mt + mb;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int e = 0; e < 16; ++e) s[kb][e] -= mt;
            }
        } else if (mt > mused + RESCALE_THR * 1.4426950408889634f) {   // lazy rescale (log2 units; rare after tile 0)
            const float corr = __builtin_amdgcn_exp2f(mused - mt);
            lrun *= corr;
#pragma unroll
            for (int d = 0; d < 4; ++d)
#pragma unroll
                for (int e = 0; e < 16; ++e) o[d][e] *= corr;
            if constexpr (ATTN_LMFMA) ol *= corr;
            mused = mt;
        }
        float ls = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                s[kb][e] = __builtin_amdgcn_exp2f(ATTN_CSUB ? s[kb][e] : s[kb][e] - mused);
                if constexpr (!ATTN_LMFMA) ls += s[kb][e];
            }
        if constexpr (!ATTN_LMFMA) {
            ls = xor32_add(ls);
            lrun += ls;
        }
        } else {
            lrun = 1.f;
        }
        if constexpr (VAR == 3) return;
        // O^T[d][q] += sum_key V[key][d] P[q][key]; P^T from the accumulator registers (k-step st of
        // key block kb = registers 8st..8st+7: key 16st + 8(j>>2) + 4fh + (j&3)), V^T by tr reads
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                bf16x8 pb;
#pragma unroll
                for (int j = 0; j < 8; ++j) pb[j] = f2bf(s[kb][8 * st + j]);
                const int key0 = kb * 32 + 16 * st + tr_key;
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const unsigned char* vp = Vs + key0 * VROW + (d * 32 + tr_col) * 2;
                    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)vp);
                    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(vp + 8 * VROW));
                    bf16x8 va;
                    __builtin_memcpy(&va, &lo, 8);
                    __builtin_memcpy(((char*)&va) + 8, &hi, 8);
                    o[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb, o[d], 0, 0, 0);
                }
                if constexpr (ATTN_LMFMA) {
                    bf16x8 ones;
#pragma unroll
                    for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.f;
                    ol = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pb, ol, 0, 0, 0);
                }
            }
        }
    };

    // One staging set: tile t+1 is fetched into registers before tile t's products and written to
    // the other LDS buffer after them (that buffer's last reader, tile t-1, finished before the
    // previous barrier), so the fetch has one tile of compute to land. The fetch index is clamped so
    // every iteration issues the same loads (the last one is unused).
    const Stg first = gload(0);
    if constexpr (CAP) {
        if (cap) {   // rows of the window outside [0, klen) are zeros; the taps of this head after the window
            float4 tw = make_float4(0.f, 0.f, 0.f, 0.f);
            constexpr int NW4 = 11 * (DK / 4);
            if (tid < NW4) tw = *(const float4*)(a.fw + (long long)(tid / (DK / 4)) * a.fD + h * DK + (tid % (DK / 4)) * 4);
            for (int i = tid; i < (QBLK + 10) * 16; i += NT) {
                const int row = fw0 + (i >> 4);
                if (row < 0 || row >= klen) *(uint4*)(fxs + (i >> 4) * (DK * 2) + (i & 15) * 16) = make_uint4(0, 0, 0, 0);
            }
            if (tid < NW4) *(float4*)(fxs + (QBLK + 10) * (DK * 2) + tid * 16) = tw;
        }
    }
    if (ntiles > 0) sstore(0, first, 0);
    __syncthreads();
    for (int t = 0; t < (VAR == 5 ? 0 : ntiles); ++t) {
        const Stg nx = VAR == 1 ? first : gload(min(t + 1, ntiles - 1));
        compute(t);
        if (t + 1 < ntiles) sstore((t + 1) & 1, nx, t + 1);
        __syncthreads();
    }
    if constexpr (ATTN_LMFMA) {
        if constexpr (VAR != 2) lrun = ol[0];
    }
    {
        if (!a.o && a.o2) {   // bf16 rows only: 8 x 16-B stores per lane (the two half-waves hold 8-B pieces of a row)
            const float inv = (klen > 0) ? 1.f / lrun : 0.f;
            bf16* op2 = (bf16*)a.o2 + ((long long)b * a.Tq + (qrow < a.Tq ? qrow : 0)) * a.ldo + h * DK;
#pragma unroll
            for (int d = 0; d < 4; ++d)
#pragma unroll
                for (int g = 0; g < 4; g += 2) {
                    uint2 pa, pb;
                    {
                        bf16x4 t4 = {f2bf(o[d][4 * g] * inv), f2bf(o[d][4 * g + 1] * inv), f2bf(o[d][4 * g + 2] * inv),
                                     f2bf(o[d][4 * g + 3] * inv)};
                        __builtin_memcpy(&pa, &t4, 8);
                        bf16x4 u4 = {f2bf(o[d][4 * g + 4] * inv), f2bf(o[d][4 * g + 5] * inv),
                                     f2bf(o[d][4 * g + 6] * inv), f2bf(o[d][4 * g + 7] * inv)};
                        __builtin_memcpy(&pb, &u4, 8);
                    }
                    auto rx = __builtin_amdgcn_permlane32_swap(pa.x, pb.x, false, false);
                    auto ry = __builtin_amdgcn_permlane32_swap(pa.y, pb.y, false, false);
                    if (qrow < a.Tq)
                        *(uint4*)(op2 + d * 32 + 8 * g + 8 * fh) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
                }
        }
    }
    if (qrow < a.Tq && (a.o || !a.o2)) {
        const float inv = (klen > 0) ? 1.f / lrun : 0.f;
        float* op = a.o ? a.o + ((long long)b * a.Tq + qrow) * a.ldo + h * DK : nullptr;
        bf16* op2 = a.o2 ? (bf16*)a.o2 + ((long long)b * a.Tq + qrow) * a.ldo + h * DK : nullptr;
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int g = 0; g < 4; ++g) {   // registers 4g..4g+3 are 4 consecutive head dims
                const int col = d * 32 + 8 * g + 4 * fh;
                const float v0 = o[d][4 * g] * inv, v1 = o[d][4 * g + 1] * inv;
                const float v2 = o[d][4 * g + 2] * inv, v3 = o[d][4 * g + 3] * inv;
                if (op) *(float4*)(op + col) = make_float4(v0, v1, v2, v3);
                if (op2) {
                    bf16x4 t4 = {f2bf(v0), f2bf(v1), f2bf(v2), f2bf(v3)};
                    *(bf16x4*)(op2 + col) = t4;
                }
            }
    }
    if constexpr (NWV == 8) {
        if (a.fout) fsmn_epilogue<QBLK, NT>(a, fxs, qt, h, b, klen);
    }
    if (a.rt_cache && qt == 0 && !(a.rt_dec && a.rt_ntok[b] < 1)) {
        const SPrm p = a.rt_prm[b];
        const int len0 = (a.rt_dec ? p.cld : p.cle) + p.tw - a.rt_drop;
        const int ncl = min(a.rt_C, len0);
        for (int e = tid; e < ncl * 32; e += NT) {   // 16 16-B chunks of K and 16 of V per row (128 head dims)
            const int j = e >> 5, c = e & 31;
            const unsigned row = (unsigned)(len0 - ncl + j), cb = (unsigned)(c & 15) * 16u;
            const uint4 val = c < 16 ? *(const uint4*)(kbase + (row * krb + cb)) : *(const uint4*)(vbase + (row * vrb + cb));
            *(uint4*)((char*)a.rt_cache +
                      (((long long)p.slot * a.rt_C + j) * a.rt_W + (c < 16 ? 0 : a.rt_voff) + h * DK) * 2 + cb) = val;
        }
    }
}

}  // namespace

// q/k/v: head-concatenated rows (head h at column h*128). o: f32 [B*Tq, ldo] (may be null in
// bf16 mode when only o2 is wanted). heads*128 columns per row.
hipError_t pfm_attention_small(int dtype, const void* q, RowMap qmap, const void* k, RowMap kmap, const void* v,
                               RowMap vmap, float* o, void* o2, long long ldo, const int* klen, int B, int Tq, int Tk,
                               int heads, int dk, float scale, hipStream_t st);

hipError_t pfm_attention_fsmn(int dtype, const void* q, RowMap qmap, const void* k, RowMap kmap, const void* v,
                              RowMap vmap, float* o, long long ldo, void* o2, const int* klen, int B, int Tq,
                              int Tk, int heads, int dk, float scale, const float* fsmn_wT, bf16* fsmn_out,
                              long long fsmn_ld, hipStream_t st) {
    if (dk != DK) {   // 32 / 64-wide heads (CT-Transformer): k_punc.hip; no fused FSMN there
        if (fsmn_out) return hipErrorInvalidValue;
        return pfm_attention_small(dtype, q, qmap, k, kmap, v, vmap, o, o2, ldo, klen, B, Tq, Tk, heads, dk, scale, st);
    }
    if (B <= 0 || Tq <= 0) return hipSuccess;
    AttnArgs a;
    a.q = q; a.qmap = qmap; a.k = k; a.kmap = kmap; a.v = v; a.vmap = vmap;
    a.o = o; a.ldo = ldo; a.o2 = o2; a.o2_dtype = DT_BF16; a.klen = klen; a.Tq = Tq; a.Tk = Tk; a.scale = scale;
    a.fw = fsmn_wT; a.fout = fsmn_out; a.fld = fsmn_ld; a.fD = heads * DK;
    if (fsmn_out) {   // fused FSMN: bf16 8-wave kernel only, self-attention, 16-B aligned rows
        const PfmKnobs& kn = pfm_knobs();
        if (dtype != DT_BF16 || Tq != Tk || kn.attn_waves != 8 || fsmn_ld % 8 ||
            vmap.ld % 8 || ((uintptr_t)fsmn_out % 16) || !fsmn_wT)
            return hipErrorInvalidValue;
    }
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)attn_f32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS32);
        (void)hipFuncSetAttribute((const void*)attn_x6_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, X6_LDS);
        (void)hipFuncSetAttribute((const void*)attn_bf16_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * STG2);
        (void)hipFuncSetAttribute((const void*)attn_bf16_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS8_FS);
    }
    // bf16 kernels address an utterance's key rows as base + t * ld (32-bit offsets)
    auto contiguous = [&](const RowMap& m) {
        return (m.rows_per_seg <= 0 || m.rows_per_seg == Tk) && (long long)Tk * m.ld * 2 < (1ll << 31);
    };
    if (dtype == DT_BF16 && (!contiguous(kmap) || !contiguous(vmap))) return hipErrorInvalidValue;
    if (dtype == DT_F32 && pfm_knobs().exact_x6 && ldo % 4 == 0 && ((uintptr_t)o % 16) == 0 &&
        ((uintptr_t)o2 % 8) == 0) {   // EXACT mode on split-bf16 MFMA (f32 accuracy; 4-column output stores)
        dim3 grid((Tq + 255) / 256, heads, B), block(512);
        hipLaunchKernelGGL(attn_x6_kernel<0>, grid, block, X6_LDS, st, a);
    } else if (dtype == DT_F32) {
        dim3 grid((Tq + 127) / 128, heads, B), block(256);
        hipLaunchKernelGGL(attn_f32_kernel, grid, block, LDS32, st, a);
    } else {
        const int nw = pfm_knobs().attn_waves;
        if (nw == 8) {
            dim3 grid((Tq + 255) / 256, heads, B), block(512);
            hipLaunchKernelGGL((attn_bf16_kernel<8>), grid, block, a.fout ? LDS8_FS : 2 * STG2, st, a);
        } else {
            dim3 grid((Tq + 127) / 128, heads, B), block(256);
            hipLaunchKernelGGL(attn_bf16_kernel<4>, grid, block, 2 * STG2, st, a);
        }
    }
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// EXACT mode (split-bf16 x6 attention) with the output written as the split operand of the out-projection:
// out3 rows of 3 x heads x 128 bf16 (x0 | x1 | x2 planes, heads x 128 apart). q/k/v f32.
// fsmn_wT / fsmn_out (optional, both or neither): the encoder's FSMN memory block (K 11, left 5) on v in
// the epilogue, f32 rows of fsmn_ld floats (self-attention only: Tq == Tk).
hipError_t pfm_attention_x3(const float* q, RowMap qmap, const float* k, RowMap kmap, const float* v, RowMap vmap,
                            bf16* out3, const int* klen, int B, int Tq, int Tk, int heads, int dk, float scale,
                            const float* fsmn_wT, float* fsmn_out, long long fsmn_ld, hipStream_t st) {
    if (B <= 0 || Tq <= 0) return hipSuccess;
    if (dk != DK || !pfm_knobs().exact_x6) return hipErrorInvalidValue;
    if ((fsmn_out != nullptr) != (fsmn_wT != nullptr)) return hipErrorInvalidValue;
    if (fsmn_out && (Tq != Tk || fsmn_ld % 4 || vmap.ld % 4 || vmap.rows_per_seg > 0 || ((uintptr_t)fsmn_out % 16) ||
                     ((uintptr_t)v % 16) || ((uintptr_t)fsmn_wT % 16)))
        return hipErrorInvalidValue;
    AttnArgs a;
    a.q = q; a.qmap = qmap; a.k = k; a.kmap = kmap; a.v = v; a.vmap = vmap;
    a.o = nullptr; a.ldo = 3LL * heads * DK; a.o2 = out3; a.o2_dtype = DT_X3; a.klen = klen; a.Tq = Tq; a.Tk = Tk;
    a.scale = scale; a.fw = fsmn_wT; a.fout = nullptr; a.fld = fsmn_ld; a.fD = heads * DK;
    a.fout32 = fsmn_out;
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)attn_x6_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, X6_LDS);
    }
    dim3 grid((Tq + 255) / 256, heads, B), block(512);
    hipLaunchKernelGGL(attn_x6_kernel<0>, grid, block, X6_LDS, st, a);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// bf16 attention over a streaming step's gathered keys with the cache retain fused (AttnArgs rt_*): the key buffer is
// [n][Tk][2 heads 128] (K | V), the cache [slots][C][2 heads 128]. hipErrorNotSupported (nothing launched) for shapes
// the bf16 kernels do not take: the caller then runs the attention and kv_retain_kernel separately.
hipError_t pfm_attention_retain(const void* q, RowMap qmap, const void* kv, int B, int Tq, int Tk, void* o2, long long ldo,
                                const int* klen, int heads, int dk, float scale, const SPrm* prm, void* cache, int C,
                                int drop, int dec, const int* ntok, hipStream_t st) {
    if (B <= 0 || Tq <= 0) return hipSuccess;
    const int D = heads * DK;
    if (dk != DK || !o2 || (dec && !ntok) || ((uintptr_t)kv % 16) || ((uintptr_t)cache % 16) ||
        (long long)Tk * 2 * D * 2 >= (1ll << 31))
        return hipErrorNotSupported;
    AttnArgs a;
    const RowMap km = rowmap_seg(Tk, (long long)Tk * 2 * D, 2 * D);
    a.q = q; a.qmap = qmap; a.k = kv; a.kmap = km; a.v = (const bf16*)kv + D; a.vmap = km;
    a.o = nullptr; a.ldo = ldo; a.o2 = o2; a.o2_dtype = DT_BF16; a.klen = klen; a.Tq = Tq; a.Tk = Tk; a.scale = scale;
    a.fw = nullptr; a.fout = nullptr; a.fld = 0; a.fD = D;
    a.rt_prm = prm; a.rt_cache = (bf16*)cache; a.rt_C = C; a.rt_drop = drop; a.rt_dec = dec; a.rt_W = 2 * D;
    a.rt_voff = D; a.rt_ntok = ntok;
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)attn_bf16_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STG2);
        (void)hipFuncSetAttribute((const void*)attn_bf16_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS8_FS);
    }
    // chunk-sized steps (<= 128 query rows: every streaming step) take the 4-wave kernel: the same per-wave arithmetic
    // (bit-identical output), half the waves and a smaller kernel on a launch chain where only latency counts
    // (2.20 -> 2.135 ms per chunk at one stream, profiles/r04y_stream_attn_waves.txt)
    if (pfm_knobs().attn_waves == 8 && Tq > 128) {
        dim3 grid((Tq + 255) / 256, heads, B), block(512);
        hipLaunchKernelGGL((attn_bf16_kernel<8>), grid, block, 2 * STG2, st, a);
    } else {
        dim3 grid((Tq + 127) / 128, heads, B), block(256);
        hipLaunchKernelGGL(attn_bf16_kernel<4>, grid, block, 2 * STG2, st, a);
    }
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_attention(int dtype, const void* q, RowMap qmap, const void* k, RowMap kmap, const void* v,
                         RowMap vmap, float* o, long long ldo, void* o2, const int* klen, int B, int Tq,
                         int Tk, int heads, int dk, float scale, hipStream_t st) {
    return pfm_attention_fsmn(dtype, q, qmap, k, kmap, v, vmap, o, ldo, o2, klen, B, Tq, Tk, heads, dk, scale, nullptr,
                              nullptr, 0, st);
}

int pfm_attention_lds_bytes(int dtype) { return dtype == DT_F32 ? LDS32 : 2 * STG2; }
