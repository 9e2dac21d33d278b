// Fused SAN-M feed-forward sub-layer of the FAST-mode encoder (gfx950), one launch per layer:
//
//   x  <- x + W2 . relu(W1 . LN2(x) + b1) + b2          (sanm/encoder.py:138-145,
//                                                        transformer/positionwise_feed_forward.py:14-34)
//   xn <- LN1_next(x)  (optional: the next layer's norm1, its QKV projection's bf16 A operand)
//
// d_model 512, hidden 2048. One workgroup (8 waves) owns 64 rows end to end:
//   prologue  LN2 of its rows (f32 two-pass statistics) -> bf16 A image in LDS (64 x 512, 64 KiB)
//   loop over 8 hidden chunks of 256:
//     phase 1  H^T[256 x 64] = W1_c . A^T  (16 k32 steps; wave w owns hidden rows 32w..32w+31)
//              -> relu(+ b1) -> bf16 H image in LDS (64 x 256, 32 KiB)
//     phase 2  Y^T[512 x 64] += W2_c . H^T (8 k32 steps x two 256-row halves; wave w owns output
//              columns 32w..32w+31 of each half; accumulators stay in registers for the whole loop)
//   epilogue  Y^T -> LDS (f32 rows) -> x + Y + b2 (f32 out) and LN1_next -> bf16
// The 2048-wide hidden activation never leaves the CU: per layer this deletes the H round trip
// (M x 2048 bf16 written + read) and both standalone LayerNorm passes of the unfused path.
//
// Weights stream through a 4-slot LDS ring of 16 KiB tiles by global_load_lds (3 tiles in flight).
// The tiles are pre-packed once per weight upload (ffn_pack_kernel) into the exact LDS image the
// fragment reads expect, bank swizzle included, so every DMA is a linear 1 KiB copy per wave.
// Per chunk: 16 W1 tiles [256 hidden x 32 k] then 16 W2 tiles [256 out x 32 hidden] (k step s,
// half eta = tile 2s + eta). Tile rows are 64 B (4 x 16-B slots, slot XOR f2(row)).
// Fragment reads are software-pipelined one tile ahead of the MFMAs (tile t+1's ds_reads are issued
// right after the barrier that publishes it, while tile t's MFMAs drain).
#include <stdint.h>

#include "pfm_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int FD = 512, FF = 2048, BM = 64;
constexpr int HC = 256, NCH = FF / HC;          // hidden chunk, chunks
constexpr int TILE = 16384, TPC = 32, NTILE = NCH * TPC;
constexpr int OP_TILES = 32;                    // out-projection Wo [512][512]: 16 k steps x 2 halves (W2 format)
constexpr int QK_TILES = 3 * OP_TILES;          // next layer's Wqkv [1536][512]: three Wo-format passes
constexpr int OFF_AN = 0, OFF_H = 65536, OFF_RING = 98304, LDS_BYTES = 163840;
constexpr int OFF_RED = LDS_BYTES - 4096, OFF_STATS = OFF_RED - 512;   // DEC epilogue (above the Y image)
#ifndef FFN_XB
#define FFN_XB 2
#endif
constexpr int YP = 516;                         // epilogue f32 row pitch (floats)

static_assert(OFF_RING + 4 * TILE == LDS_BYTES, "LDS plan");
static_assert(BM * YP * 4 <= OFF_STATS, "epilogue image below the DEC statistics");

// 64-B tile rows: physical 16-B slot = logical slot ^ f2(row). Conflict-free for 16x16x32 fragment
// reads (16 consecutive rows, slot = lane >> 4): every ds_read_b128 lane group covers 16 distinct
// bank positions.
__device__ __forceinline__ int f2(int row) { return (row >> 2) & 2; }

__device__ __forceinline__ bf16x8 ld128(const unsigned char* p) { return *(const bf16x8*)p; }

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float pick4(float v0, float v1, float v2, float v3, int g) {
    return g == 0 ? v0 : (g == 1 ? v1 : (g == 2 ? v2 : v3));
}

template <int N> __device__ __forceinline__ void vm_wait() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else static_assert(N < 0, "vm_wait: unsupported count");
}

template <int HB> struct Frag { bf16x8 w[HB]; bf16x8 a[4]; };

// VAR (diagnostic instantiations for standalone timing; the library instantiates VAR 0 only): 0 = the kernel; 1 = no weight DMA (stale ring); 2 = no MFMAs;
// 3 = every tile streams ring tiles 0..3 of the layer (L2-hot 64 KiB); 4 = prologue + epilogue only (no
// tile loop); 5 = VAR 1 without the per-tile barriers (MFMA + fragment reads alone); OP only: 6 = prologue, phase 0 and
// LN2, then exit; 7 = VAR 6 without phase 0 (the I/O of the OP transition alone)
//
// OP (the attention sub-layer's out-projection folded in front): the block starts from the attention output
// O and the FSMN output F (bf16 rows) instead of x:
//   phase 0   Y0^T[512 x 64] = Wo . O^T   (O image in the A slot; 32 Wo tiles in W2 format lead the ring)
//   x1 = ((Y0 + bo) + F) + x  (x optional: layer 0 has no residual)  kept in the phase-2 accumulators,
//   LN2(x1) -> bf16 A image (row statistics reduced across the 8 waves through LDS), accumulators += b2,
//   then the FFN loop above accumulates W2 . H on top: the epilogue stores x2 = accumulators directly.
// x1 never leaves the CU (one kernel and one HBM round trip of the residual stream less per layer).
//
// QK (MODE 4; diagnostic: instantiated by tools/ffn_bench.hip only, measured slower than the separate GEMM): after the
// FFN, x2 goes out from the accumulators, LN1_next(x2) becomes the bf16 A image and phase 3 streams the next layer's Wqkv
// as 96 more Wo-format tiles (Xn receives q|k|v rows of 1536, c1 the biases).
//
// DEC (Paraformer decoder feed-forward, sanm/positionwise_feed_forward.py:12-33): y = W2 . LN_F(relu(W1 x' + b1)),
// x' = LN1(x) (the prologue), w2 without bias. LN_F over the 2048-wide hidden is folded through W2:
//   y = rstd . (W2g . h - mu . c1) + c2,   W2g = W2 diag(gamma_F) (packed bf16), c1 = rowsum(W2g), c2 = W2 beta_F,
// with mu / rstd of the bf16 hidden h accumulated chunk by chunk (sum, sum of squares) and reduced across the
// 8 waves in the epilogue. Outputs: xn = LN_next(y) (bf16; the decoder's LN2 or after_norm), xo = y (optional).
// In DEC mode the arguments bo / b2 carry c1 / c2.
//
// NW (waves per workgroup): 8 = wave w owns 32 weight rows of every 256-row tile (2 fragments), the kernel;
// 4 = one wave per SIMD owning 64 weight rows (4 fragments, 192 accumulator registers; each tile's A / H
// fragments read by half as many waves: 32 instead of 48 KiB of LDS reads per tile) measured 16 % slower
// (207 vs 178 us at M = 32,000; bench 24.6 vs 21.6 ms/step) and is not instantiated.
// HR: phase 2 (and phase 0) reads a k step's activation fragments once for both 256-row halves (odd tiles
// copy them from the even tile's registers) instead of re-reading them from LDS.
// PD: ring tiles in flight behind the one being published (2: tile t+3 issued at the top of iteration t, 3:
// tile t+4 — the slot of tile t is free as soon as the barrier retires everyone's fragment reads of it, so
// all 4 ring slots can be streaming; A/B: bench 21.6 (PD 2) -> 20.1 ms/step (PD 3)). The library
// instantiates HR = true, PD = 3 only (the measured-slower combinations were A/B knobs until round 3).
template <int VAR, int MODE = 0, int NW = 8, bool HR = true, int PD = 3>
__global__ __launch_bounds__(64 * NW) void ffn_fused_kernel(const float* __restrict__ X, int M, const float* __restrict__ g2,
                                                        const float* __restrict__ be2, float eps,
                                                        const bf16* __restrict__ Wp, const float* __restrict__ b1,
                                                        const float* __restrict__ b2, float* Xo,
                                                        const float* __restrict__ gn, const float* __restrict__ bn,
                                                        bf16* __restrict__ Xn, const bf16* __restrict__ O,
                                                        const bf16* __restrict__ Fr, const float* __restrict__ bo,
                                                        const float* __restrict__ c1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, r16 = lane & 15;
    const long long m0 = (long long)blockIdx.x * BM;
    constexpr int WR = 256 / NW, HB = WR / 16, RPW = BM / NW, LPW = TILE / (1024 * NW);
    using FragT = Frag<HB>;
    constexpr bool OP = MODE == 1 || MODE == 3 || MODE == 4, DEC = MODE == 2 || MODE == 3;
    constexpr bool EOP = MODE == 1 || MODE == 4, QK = MODE == 4;
    constexpr int T0 = OP ? OP_TILES : 0;      // FFN tiles start after the Wo tiles
    float rs[4] = {0.f, 0.f, 0.f, 0.f}, rq[4] = {0.f, 0.f, 0.f, 0.f};   // DEC: hidden row sums / sums of squares
    constexpr int NT_ALL = NTILE + T0 + (QK ? QK_TILES : 0);

    auto issue = [&](int t) {
        if (t >= NT_ALL || VAR == 1 || VAR == 5) return;
        const bf16* src = Wp + (long long)(VAR == 3 ? (t & 3) : t) * (TILE / 2) + (LPW * w * 64 + lane) * 8;
        unsigned char* dst = smem + OFF_RING + (t & 3) * TILE + LPW * w * 1024;
#pragma unroll
        for (int i = 0; i < LPW; ++i)
            __builtin_amdgcn_global_load_lds((gbl_void*)(src + 512 * i), (lds_void*)(dst + 1024 * i), 16, 0, 0);
    };
    auto bar = [&]() {
        if (VAR == 5) return;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // OP row statistics: lane partials -> the 4 g lanes -> the 8 waves through LDS ([2][8 waves][64 rows] in the
    // H image, which is free between chunks' uses: before chunk 0 and after the last chunk)
    float* red = (float*)(smem + OFF_H);
    auto row_reduce = [&](float (&v)[4], int slot) {
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            v[mb] += __shfl_xor(v[mb], 16, 64);
            v[mb] += __shfl_xor(v[mb], 32, 64);
            if (g == 0) red[slot * 512 + w * 64 + 16 * mb + r16] = v[mb];
        }
        bar();
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            float t = 0.f;
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) t += red[slot * 512 + ww * 64 + 16 * mb + r16];
            v[mb] = t;
        }
    };
    // the lane's 4 consecutive columns 4g .. 4g+3 of the 16 at a wave-uniform address, by scalar loads (a vector load
    // would share vmcnt with the in-flight ring DMAs and drain the ring before its first use)
    auto cols4 = [&](const float* p) {
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = p[k];
        return make_float4(pick4(v[0], v[4], v[8], v[12], g), pick4(v[1], v[5], v[9], v[13], g),
                           pick4(v[2], v[6], v[10], v[14], g), pick4(v[3], v[7], v[11], v[15], g));
    };
    // ---- prologue: LN2 of rows m0 + 8w .. + 7 -> bf16 A image (row pitch 1 KiB, slot ^ (row & 15))
    //      (OP: the attention output rows go to the A image instead; LN2 follows phase 0)
    if constexpr (OP) {
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int m = RPW * w + i;
            const long long row = min(m0 + m, (long long)M - 1);
            const bf16x8 v = *(const bf16x8*)(O + row * FD + 8 * lane);
            *(bf16x8*)(smem + OFF_AN + m * 1024 + ((lane ^ (m & 15)) << 4)) = v;
        }
        issue(0);
        issue(1);
        issue(2);
        if constexpr (PD == 3) issue(3);
    } else {
        float4 xa[RPW], xb[RPW];
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const long long row = min(m0 + RPW * w + i, (long long)M - 1);
            const float* xr = X + row * FD + 8 * lane;
            xa[i] = *(const float4*)xr;
            xb[i] = *(const float4*)(xr + 4);
        }
        issue(0);
        issue(1);
        issue(2);
        if constexpr (PD == 3) issue(3);
        const float4 ga = *(const float4*)(g2 + 8 * lane), gb = *(const float4*)(g2 + 8 * lane + 4);
        const float4 ba = *(const float4*)(be2 + 8 * lane), bb = *(const float4*)(be2 + 8 * lane + 4);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            float v[8] = {xa[i].x, xa[i].y, xa[i].z, xa[i].w, xb[i].x, xb[i].y, xb[i].z, xb[i].w};
            float s = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) s += v[e];
            const float mean = wave_sum(s) * (1.f / FD);
            float q = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) { v[e] -= mean; q += v[e] * v[e]; }
            const float rstd = 1.f / sqrtf(wave_sum(q) * (1.f / FD) + eps);
            const float gg[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
            const float bbv[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e] * rstd * gg[e] + bbv[e]);
            const int m = RPW * w + i;
            *(bf16x8*)(smem + OFF_AN + m * 1024 + ((lane ^ (m & 15)) << 4)) = o;
        }
    }

    f32x4 acc1[HB][4], acc2a[HB][4], acc2b[HB][4];
#pragma unroll
    for (int i = 0; i < HB; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) { acc1[i][j][e] = 0.f; acc2a[i][j][e] = 0.f; acc2b[i][j][e] = 0.f; }

    // fragment reads of tile t: weight rows of this wave (ring slot t & 3) + the activation operand
    // (A image for W1 tiles, H image for W2 tiles)
    auto rd_w = [&](int t, FragT& f) {
        const unsigned char* ring = smem + OFF_RING + (t & 3) * TILE;
#pragma unroll
        for (int hb = 0; hb < HB; ++hb) {
            const int row = WR * w + 16 * hb + r16;
            f.w[hb] = ld128(ring + row * 64 + ((g ^ f2(row)) << 4));
        }
    };
    auto rd_a = [&](int t, FragT& f) {   // W1 tile t: k step j = t & 15 of the A image
        const int j = t & 15;
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
            f.a[mb] = ld128(smem + OFF_AN + (16 * mb + r16) * 1024 + (((4 * j + g) ^ r16) << 4));
    };
    auto rd_h = [&](int t, FragT& f) {   // W2 tile t: k step s = (t & 15) >> 1 of the H image
        const int s2 = (t & 15) >> 1;
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
            f.a[mb] = ld128(smem + OFF_H + (16 * mb + r16) * 512 + (((4 * s2 + g) ^ r16) << 4));
    };
    auto rd1 = [&](int t, FragT& f) { rd_w(t, f); rd_a(t, f); };
    auto rd2 = [&](int t, FragT& f) { rd_w(t, f); rd_h(t, f); };
    // the second half of a k step (odd tile) reuses the first half's activation fragments
    auto rd_w2 = [&](int t, FragT& f, const FragT& prev) {
        rd_w(t, f);
        if constexpr (HR) {
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) f.a[mb] = prev.a[mb];
        } else if constexpr (OP) {
            if (t < OP_TILES) {
                const int j = t >> 1;
#pragma unroll
                for (int mb = 0; mb < 4; ++mb)
                    f.a[mb] = ld128(smem + OFF_AN + (16 * mb + r16) * 1024 + (((4 * j + g) ^ r16) << 4));
            } else {
                rd_h(t, f);
            }
        } else {
            rd_h(t, f);
        }
    };
    // relu(H^T + b1) of chunk c -> bf16 H image [64 rows][256 hidden] (row pitch 512 B, slot ^ (row & 15)).
    // acc1[hb][mb][i] = H^T[hidden 32w + 16hb + 4g + i][row 16mb + r16]. The wave's 32 biases come in by
    // scalar loads (no vector-memory op beside the in-flight LDS-DMA ring).
    auto write_h = [&](int c) {
        const float* bp = b1 + HC * c + WR * w;
#pragma unroll
        for (int hb = 0; hb < HB; ++hb) {
            float bv[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) bv[k] = bp[16 * hb + k];
            float bi[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) bi[i] = pick4(bv[i], bv[4 + i], bv[8 + i], bv[12 + i], g);
            const int hl = WR * w + 16 * hb + 4 * g;
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) {
                const int m = 16 * mb + r16;
                bf16x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = f2bf(fmaxf(acc1[hb][mb][i] + bi[i], 0.f));
                if constexpr (DEC) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float f = bf2f(o[i]);
                        rs[mb] += f;
                        rq[mb] += f * f;
                    }
                }
                *(bf16x4*)(smem + OFF_H + m * 512 + (((hl >> 3) ^ r16) << 4) + ((hl & 7) << 1)) = o;
#pragma unroll
                for (int i = 0; i < 4; ++i) acc1[hb][mb][i] = 0.f;
            }
        }
    };
    auto mm1 = [&](const FragT& f) {
        if (VAR == 2) { asm volatile("" :: "v"(f.w[0]), "v"(f.w[HB - 1]), "v"(f.a[0]), "v"(f.a[1]), "v"(f.a[2]), "v"(f.a[3])); return; }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int hb = 0; hb < HB; ++hb)
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) acc1[hb][mb] = mfma16(f.w[hb], f.a[mb], acc1[hb][mb]);
        __builtin_amdgcn_s_setprio(0);
    };
    auto mm2a = [&](const FragT& f) {
        if (VAR == 2) { asm volatile("" :: "v"(f.w[0]), "v"(f.w[HB - 1]), "v"(f.a[0]), "v"(f.a[1]), "v"(f.a[2]), "v"(f.a[3])); return; }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int nb = 0; nb < HB; ++nb)
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) acc2a[nb][mb] = mfma16(f.w[nb], f.a[mb], acc2a[nb][mb]);
        __builtin_amdgcn_s_setprio(0);
    };
    auto mm2b = [&](const FragT& f) {
        if (VAR == 2) { asm volatile("" :: "v"(f.w[0]), "v"(f.w[HB - 1]), "v"(f.a[0]), "v"(f.a[1]), "v"(f.a[2]), "v"(f.a[3])); return; }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int nb = 0; nb < HB; ++nb)
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) acc2b[nb][mb] = mfma16(f.w[nb], f.a[mb], acc2b[nb][mb]);
        __builtin_amdgcn_s_setprio(0);
    };
    // top of iteration t: tile t+1 landed (tiles t+2 .. t+PD may stay in flight) and visible to every wave,
    // then the DMA of tile t+1+PD into the slot of tile t+PD-3 (PD = 3: tile t, PD = 2: tile t-1), whose
    // fragments every wave read before this barrier
    auto top = [&](int t) {
        if (VAR != 1 && VAR != 5) {
            // tile t+1 landed; tiles t+2 .. t+PD (those that exist) may stay in flight
            if constexpr (PD == 3) {
                if (t + 3 < NT_ALL) vm_wait<2 * LPW>();
                else if (t + 2 < NT_ALL) vm_wait<LPW>();
                else vm_wait<0>();
            } else {
                if (t + 2 < NT_ALL) vm_wait<LPW>();
                else vm_wait<0>();
            }
        }
        bar();
        issue(t + 1 + PD);
    };

    // Software pipeline, iteration t: top(t) -> fragment reads of tile t+1 -> MFMAs of tile t (fragments
    // read in iteration t-1), so the ds_read latency of the next tile hides under this tile's MFMAs.
    if (VAR != 1 && VAR != 5) {   // tile 0 (tiles 1, 2 in flight)
        vm_wait<PD * LPW>();
    }
    bar();
    FragT F0, F1;
    // phase 0 (phase 3): Wo (Wqkv) tile t = k step (t >> 1) & 15 of the O (xn) image in the A slot, half t & 1
    auto rd0 = [&](int t, FragT& f) {
        rd_w(t, f);
        const int j = (t >> 1) & 15;
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
            f.a[mb] = ld128(smem + OFF_AN + (16 * mb + r16) * 1024 + (((4 * j + g) ^ r16) << 4));
    };
    if constexpr (OP) {
        if constexpr (VAR != 7) {
            rd0(0, F0);
            for (int s2 = 0; s2 < OP_TILES / 2 - 1; ++s2) {
                top(2 * s2); rd_w2(2 * s2 + 1, F1, F0); mm2a(F0);
                top(2 * s2 + 1); rd0(2 * s2 + 2, F0); mm2b(F1);
            }
            top(OP_TILES - 2); rd_w2(OP_TILES - 1, F1, F0); mm2a(F0);
            top(OP_TILES - 1); mm2b(F1);
        }
        // x1 = ((Y0 + bo) + F) + x in the accumulator layout: acc2{a,b}[nb][mb][e] = x1[row 16mb + r16]
        // [col 32w + 16nb + 4g + e (+256 for b)]; LN2 row statistics: lane partials -> 4 g lanes -> 8 waves
        float part[4] = {0.f, 0.f, 0.f, 0.f};
        // Addend loads are branch-free (a null X / Fr reads a valid stand-in and is selected away) and issued
        // in two batches of 8 row fragments, so a batch costs one memory latency: with the loads behind
        // per-fragment `if`s the compiler drained vmcnt(0) before every one (16 serial round trips).
        const bool hx = X != nullptr, hf_ = Fr != nullptr;
        const float* xs = hx ? X : bo;
        const long long xst = hx ? FD : 0;
        const bf16* fs = hf_ ? Fr : O;
        float4 bv[2][HB];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
            for (int nb = 0; nb < HB; ++nb) bv[hf][nb] = *(const float4*)(bo + 256 * hf + WR * w + 16 * nb + 4 * g);
        constexpr int XB = FFN_XB;   // row blocks per load batch
#pragma unroll
        for (int mh = 0; mh < 4 / XB; ++mh) {
            float4 xv[XB][2][HB];
            bf16x4 fv[XB][2][HB];
#pragma unroll
            for (int mi = 0; mi < XB; ++mi) {
                const long long row = min(m0 + 16 * (XB * mh + mi) + r16, (long long)M - 1);
#pragma unroll
                for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                    for (int nb = 0; nb < HB; ++nb) {
                        const int n = 256 * hf + WR * w + 16 * nb + 4 * g;
                        xv[mi][hf][nb] = *(const float4*)(xs + row * xst + n);
                        fv[mi][hf][nb] = *(const bf16x4*)(fs + row * FD + n);
                    }
            }
#pragma unroll
            for (int mi = 0; mi < XB; ++mi) {
                const int mb = XB * mh + mi;
                const long long row = min(m0 + 16 * mb + r16, (long long)M - 1);
#pragma unroll
                for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                    for (int nb = 0; nb < HB; ++nb) {
                        const int n = 256 * hf + WR * w + 16 * nb + 4 * g;
                        f32x4& a = hf ? acc2b[nb][mb] : acc2a[nb][mb];
                        const float4 bb4 = bv[hf][nb];
                        const float4 x4 = hx ? xv[mi][hf][nb] : make_float4(0.f, 0.f, 0.f, 0.f);
                        const bf16x4 f4 = fv[mi][hf][nb];
                        a[0] += bb4.x; a[1] += bb4.y; a[2] += bb4.z; a[3] += bb4.w;
                        if (hf_) {
                            a[0] += bf2f(f4[0]); a[1] += bf2f(f4[1]); a[2] += bf2f(f4[2]); a[3] += bf2f(f4[3]);
                        }
                        a[0] += x4.x; a[1] += x4.y; a[2] += x4.z; a[3] += x4.w;
                        if constexpr (MODE == 3) {   // the decoder keeps x1 (the FSMN step adds it back)
                            if (m0 + 16 * mb + r16 < M) *(float4*)(Xo + row * FD + n) = make_float4(a[0], a[1], a[2], a[3]);
                        }
                        part[mb] += (a[0] + a[1]) + (a[2] + a[3]);
                    }
            }
        }
        row_reduce(part, 0);   // its barrier also retires every wave's phase-0 reads of the O image
        float mean[4], q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) mean[mb] = part[mb] * (1.f / FD);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int nb = 0; nb < HB; ++nb) {
                    const f32x4& a = hf ? acc2b[nb][mb] : acc2a[nb][mb];
#pragma unroll
                    for (int e = 0; e < 4; ++e) { const float d = a[e] - mean[mb]; q[mb] += d * d; }
                }
        row_reduce(q, 1);
        float4 gv[2][HB], bev[2][HB], c2v[2][HB];   // per-column constants, loaded once (not per row block)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
            for (int nb = 0; nb < HB; ++nb) {
                const int n = 256 * hf + WR * w + 16 * nb + 4 * g;
                gv[hf][nb] = *(const float4*)(g2 + n);
                bev[hf][nb] = *(const float4*)(be2 + n);
                c2v[hf][nb] = EOP ? *(const float4*)(b2 + n) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            const int m = 16 * mb + r16;
            const float rstd = 1.f / sqrtf(q[mb] * (1.f / FD) + eps);
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int nb = 0; nb < HB; ++nb) {
                    const int n = 256 * hf + WR * w + 16 * nb + 4 * g;
                    f32x4& a = hf ? acc2b[nb][mb] : acc2a[nb][mb];
                    const float4 gg = gv[hf][nb], be = bev[hf][nb];
                    bf16x4 o = {f2bf((a[0] - mean[mb]) * rstd * gg.x + be.x), f2bf((a[1] - mean[mb]) * rstd * gg.y + be.y),
                                f2bf((a[2] - mean[mb]) * rstd * gg.z + be.z), f2bf((a[3] - mean[mb]) * rstd * gg.w + be.w)};
                    *(bf16x4*)(smem + OFF_AN + m * 1024 + (((n >> 3) ^ (m & 15)) << 4) + ((n & 7) << 1)) = o;
                    if constexpr (EOP) {   // encoder: x2 = (x1 + b2) + W2 . H
                        const float4 c2 = c2v[hf][nb];
                        a[0] += c2.x; a[1] += c2.y; a[2] += c2.z; a[3] += c2.w;
                    } else {                      // decoder: the FFN output has no residual
                        a[0] = 0.f; a[1] = 0.f; a[2] = 0.f; a[3] = 0.f;
                    }
                }
        }
        bar();   // the LN2 image is complete before chunk 0's first fragment reads
        if constexpr (VAR == 6 || VAR == 7) {
            vm_wait<0>();
            return;
        }
    }
    rd1(T0, F0);
    for (int c = 0; c < (VAR == 4 ? 0 : NCH); ++c) {
        const int tb = T0 + TPC * c;
        // phase 1: 16 W1 tiles (H^T of this chunk), fragments alternate F0 / F1
        for (int j = 0; j < 14; j += 2) {
            top(tb + j); rd1(tb + j + 1, F1); mm1(F0);
            top(tb + j + 1); rd1(tb + j + 2, F0); mm1(F1);
        }
        top(tb + 14); rd1(tb + 15, F1); mm1(F0);
        // last W1 tile: H must be complete in LDS before tile tb+16's H fragments are read
        top(tb + 15); rd_w(tb + 16, F0); mm1(F1); write_h(c); bar(); rd_h(tb + 16, F0);
        // phase 2: 16 W2 tiles (k step s: half 0 -> acc2a, half 1 -> acc2b)
        for (int s2 = 0; s2 < 7; ++s2) {
            const int t = tb + 16 + 2 * s2;
            top(t); rd_w2(t + 1, F1, F0); mm2a(F0);
            top(t + 1); rd2(t + 2, F0); mm2b(F1);
        }
        top(tb + 30); rd_w2(tb + 31, F1, F0); mm2a(F0);
        if (c + 1 < NCH) { top(tb + 31); rd1(tb + 32, F0); }
        mm2b(F1);
    }

    if constexpr (QK) {
        // ---- QK epilogue: x2 (the accumulators) -> Xo straight from the accumulator layout; LN1_next(x2) -> bf16
        //      xn image in the A slot (row statistics across the 8 waves, as LN2 after phase 0). Every wave is past
        //      top(tb + 30) of the last chunk, hence past its last H read: the H image holds the reduction.
        float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            const long long row = m0 + 16 * mb + r16;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int nb = 0; nb < HB; ++nb) {
                    const int n = 256 * hf + WR * w + 16 * nb + 4 * g;
                    const f32x4& a = hf ? acc2b[nb][mb] : acc2a[nb][mb];
                    if (row < M) *(float4*)(Xo + row * FD + n) = make_float4(a[0], a[1], a[2], a[3]);
                    part[mb] += (a[0] + a[1]) + (a[2] + a[3]);
                }
        }
        row_reduce(part, 0);   // its barrier retires every wave's fragment reads of the last ring tile
        constexpr int T3 = T0 + NTILE;   // tiles T3 .. T3 + 2 were issued during the last chunk
        issue(T3 + 3);
        float mean[4], q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) mean[mb] = part[mb] * (1.f / FD);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int nb = 0; nb < HB; ++nb) {
                    const f32x4& a = hf ? acc2b[nb][mb] : acc2a[nb][mb];
#pragma unroll
                    for (int e = 0; e < 4; ++e) { const float d = a[e] - mean[mb]; q[mb] += d * d; }
                }
        row_reduce(q, 1);
        float4 gv[2][HB], bev[2][HB];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
            for (int nb = 0; nb < HB; ++nb) {
                gv[hf][nb] = cols4(gn + 256 * hf + WR * w + 16 * nb);
                bev[hf][nb] = cols4(bn + 256 * hf + WR * w + 16 * nb);
            }
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            const int m = 16 * mb + r16;
            const float rstd = 1.f / sqrtf(q[mb] * (1.f / FD) + eps);
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int nb = 0; nb < HB; ++nb) {
                    const int n = 256 * hf + WR * w + 16 * nb + 4 * g;
                    f32x4& a = hf ? acc2b[nb][mb] : acc2a[nb][mb];
                    const float4 gg = gv[hf][nb], be = bev[hf][nb];
                    bf16x4 o = {f2bf((a[0] - mean[mb]) * rstd * gg.x + be.x), f2bf((a[1] - mean[mb]) * rstd * gg.y + be.y),
                                f2bf((a[2] - mean[mb]) * rstd * gg.z + be.z), f2bf((a[3] - mean[mb]) * rstd * gg.w + be.w)};
                    *(bf16x4*)(smem + OFF_AN + m * 1024 + (((n >> 3) ^ (m & 15)) << 4) + ((n & 7) << 1)) = o;
                    a[0] = 0.f; a[1] = 0.f; a[2] = 0.f; a[3] = 0.f;
                }
        }
        vm_wait<PD * LPW>();   // tile T3 landed (the x2 stores ahead of tile T3 + 3 retire with it)
        bar();                 // ... and the xn image is complete
        // ---- phase 3: QKV_next[64 x 1536] = xn . Wqkv^T + bqkv in three passes of 512 columns (32 Wo-format
        //      tiles each); outputs bf16 rows of 1536 in Xn, biases in c1
        rd0(T3, F0);
        for (int p = 0; p < 3; ++p) {
            const int tp = T3 + OP_TILES * p;
            for (int s2 = 0; s2 < OP_TILES / 2 - 1; ++s2) {
                top(tp + 2 * s2); rd_w2(tp + 2 * s2 + 1, F1, F0); mm2a(F0);
                top(tp + 2 * s2 + 1); rd0(tp + 2 * s2 + 2, F0); mm2b(F1);
            }
            top(tp + OP_TILES - 2); rd_w2(tp + OP_TILES - 1, F1, F0); mm2a(F0);
            if (p < 2) { top(tp + OP_TILES - 1); rd0(tp + OP_TILES, F0); }
            mm2b(F1);
            const float* bq = c1 + 512 * p;
            float4 bv[2][HB];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int nb = 0; nb < HB; ++nb) bv[hf][nb] = cols4(bq + 256 * hf + WR * w + 16 * nb);
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) {
                const long long row = m0 + 16 * mb + r16;
#pragma unroll
                for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                    for (int nb = 0; nb < HB; ++nb) {
                        f32x4& a = hf ? acc2b[nb][mb] : acc2a[nb][mb];
                        const float4 b4 = bv[hf][nb];
                        const bf16x4 o = {f2bf(a[0] + b4.x), f2bf(a[1] + b4.y), f2bf(a[2] + b4.z), f2bf(a[3] + b4.w)};
                        if (row < M) *(bf16x4*)(Xn + row * (3 * FD) + 512 * p + 256 * hf + WR * w + 16 * nb + 4 * g) = o;
                        a[0] = 0.f; a[1] = 0.f; a[2] = 0.f; a[3] = 0.f;
                    }
            }
        }
        return;
    }

    if (VAR == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ---- epilogue: Y^T accumulators -> f32 row image; x + Y + b2 -> Xo; LN1_next -> Xn
    //      (OP: the accumulators already hold x1 + b2 + W2 . H)
    float4 xa[RPW], xb[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        if constexpr (OP || DEC) {
            xa[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            xb[i] = xa[i];
        } else {
            const long long row = min(m0 + RPW * w + i, (long long)M - 1);
            const float* xr = X + row * FD + 8 * lane;
            xa[i] = *(const float4*)xr;
            xb[i] = *(const float4*)(xr + 4);
        }
    }
    __syncthreads();   // every wave is past its last ring / A / H read (no DMA in flight here)
    float2* stats = (float2*)(smem + OFF_STATS);   // DEC: per row (mu, rstd) of the hidden
    if constexpr (DEC) {
        float* red = (float*)(smem + OFF_RED);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            rs[mb] += __shfl_xor(rs[mb], 16, 64);
            rs[mb] += __shfl_xor(rs[mb], 32, 64);
            rq[mb] += __shfl_xor(rq[mb], 16, 64);
            rq[mb] += __shfl_xor(rq[mb], 32, 64);
            if (g == 0) {
                red[w * 64 + 16 * mb + r16] = rs[mb];
                red[512 + w * 64 + 16 * mb + r16] = rq[mb];
            }
        }
        __syncthreads();
        if (tid < BM) {
            float sm = 0.f, sq = 0.f;
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) { sm += red[ww * 64 + tid]; sq += red[512 + ww * 64 + tid]; }
            const float mu = sm * (1.f / FF);
            const float var = fmaxf(sq * (1.f / FF) - mu * mu, 0.f);
            stats[tid] = make_float2(mu, 1.f / sqrtf(var + eps));
        }
    }
    float* Y = (float*)smem;
#pragma unroll
    for (int nb = 0; nb < HB; ++nb)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            const int m = 16 * mb + r16;
            const int n = WR * w + 16 * nb + 4 * g;
            *(f32x4*)(Y + m * YP + n) = acc2a[nb][mb];
            *(f32x4*)(Y + m * YP + 256 + n) = acc2b[nb][mb];
        }
    bar();
    float4 c2a = *(const float4*)(b2 + 8 * lane), c2b = *(const float4*)(b2 + 8 * lane + 4);
    if constexpr (MODE == 1) {
        c2a = make_float4(0.f, 0.f, 0.f, 0.f);
        c2b = c2a;
    }
    float4 c1a = make_float4(0.f, 0.f, 0.f, 0.f), c1b = c1a;
    if constexpr (DEC) {
        c1a = *(const float4*)(c1 + 8 * lane);
        c1b = *(const float4*)(c1 + 8 * lane + 4);
    }
    float4 na = {0, 0, 0, 0}, nbv = {0, 0, 0, 0}, qa = {0, 0, 0, 0}, qb = {0, 0, 0, 0};
    if (Xn) {
        na = *(const float4*)(gn + 8 * lane); nbv = *(const float4*)(gn + 8 * lane + 4);
        qa = *(const float4*)(bn + 8 * lane); qb = *(const float4*)(bn + 8 * lane + 4);
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int m = RPW * w + i;
        const long long row = m0 + m;
        const f32x4 ya = *(const f32x4*)(Y + m * YP + 8 * lane), yb = *(const f32x4*)(Y + m * YP + 8 * lane + 4);
        float v[8] = {ya[0] + c2a.x + xa[i].x, ya[1] + c2a.y + xa[i].y, ya[2] + c2a.z + xa[i].z,
                      ya[3] + c2a.w + xa[i].w, yb[0] + c2b.x + xb[i].x, yb[1] + c2b.y + xb[i].y,
                      yb[2] + c2b.z + xb[i].z, yb[3] + c2b.w + xb[i].w};
        if constexpr (DEC) {
            const float2 st = stats[m];
            const float c1v[8] = {c1a.x, c1a.y, c1a.z, c1a.w, c1b.x, c1b.y, c1b.z, c1b.w};
            const float c2v[8] = {c2a.x, c2a.y, c2a.z, c2a.w, c2b.x, c2b.y, c2b.z, c2b.w};
            const float yv[8] = {ya[0], ya[1], ya[2], ya[3], yb[0], yb[1], yb[2], yb[3]};
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = st.y * (yv[e] - st.x * c1v[e]) + c2v[e];
        }
        if (row < M && Xo && MODE != 3) {
            float* orow = Xo + row * FD + 8 * lane;
            *(float4*)orow = make_float4(v[0], v[1], v[2], v[3]);
            *(float4*)(orow + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
        if (Xn) {
            float s = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) s += v[e];
            const float mean = wave_sum(s) * (1.f / FD);
            float q = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) { v[e] -= mean; q += v[e] * v[e]; }
            const float rstd = 1.f / sqrtf(wave_sum(q) * (1.f / FD) + eps);
            const float gg[8] = {na.x, na.y, na.z, na.w, nbv.x, nbv.y, nbv.z, nbv.w};
            const float bb[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e] * rstd * gg[e] + bb[e]);
            if (row < M) *(bf16x8*)(Xn + row * FD + 8 * lane) = o;
        }
    }
}

// Pack one layer's bf16 W1 [2048][512] / W2 [512][2048] into the 256 ring tiles (16 KiB each) in
// LDS-image order. Tile t: chunk c = t >> 5; t & 16 ? W2 tile (k step s = (t & 15) >> 1, half eta = t & 1)
// : W1 tile (k step t & 15). Unit u (16 B) of a tile: row u >> 2, physical slot u & 3 holding logical
// slot (u & 3) ^ f2(row), i.e. 8 consecutive k.
__global__ __launch_bounds__(256) void ffn_pack_kernel(const bf16* __restrict__ W1, const bf16* __restrict__ W2,
                                                       bf16* __restrict__ Wp) {
    const int gid = blockIdx.x * 256 + threadIdx.x;   // < NTILE * 1024
    const int t = gid >> 10, u = gid & 1023;
    const int c = t >> 5, j = t & 15, row = u >> 2, ls = (u & 3) ^ f2(row);
    const bf16* src;
    if (t & 16) {
        const int s = j >> 1, eta = j & 1;
        src = W2 + (long long)(256 * eta + row) * FF + HC * c + 32 * s + 8 * ls;
    } else {
        src = W1 + (long long)(HC * c + row) * FD + 32 * j + 8 * ls;
    }
    *(bf16x8*)(Wp + (long long)gid * 8) = *(const bf16x8*)src;
}

// Wo [512 out][512 in] -> 32 tiles in the W2 tile format: tile t = k step t >> 1, half t & 1 (rows
// 256 (t & 1) + row), so phase 0 reads them exactly like phase 2 reads a chunk's W2 tiles.
__global__ __launch_bounds__(256) void ffn_pack_o_kernel(const bf16* __restrict__ Wo, bf16* __restrict__ Wp) {
    const int gid = blockIdx.x * 256 + threadIdx.x;   // < OP_TILES * 1024
    const int t = gid >> 10, u = gid & 1023;
    const int row = u >> 2, ls = (u & 3) ^ f2(row);
    const bf16* src = Wo + (long long)(256 * (t & 1) + row) * FD + 32 * (t >> 1) + 8 * ls;
    *(bf16x8*)(Wp + (long long)gid * 8) = *(const bf16x8*)src;
}

// DEC packing: W1 tiles as ffn_pack_kernel; W2 tiles from f32 W2 scaled by gamma_F along k (W2g = bf16(W2 g)).
__global__ __launch_bounds__(256) void ffn_pack_dec_kernel(const bf16* __restrict__ W1, const float* __restrict__ W2,
                                                           const float* __restrict__ gF, bf16* __restrict__ Wp) {
    const int gid = blockIdx.x * 256 + threadIdx.x;   // < NTILE * 1024
    const int t = gid >> 10, u = gid & 1023;
    const int c = t >> 5, j = t & 15, row = u >> 2, ls = (u & 3) ^ f2(row);
    bf16x8 o;
    if (t & 16) {
        const int s = j >> 1, eta = j & 1, k0 = HC * c + 32 * s + 8 * ls;
        const float* src = W2 + (long long)(256 * eta + row) * FF + k0;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(src[e] * gF[k0 + e]);
    } else {
        o = *(const bf16x8*)(W1 + (long long)(HC * c + row) * FD + 32 * j + 8 * ls);
    }
    *(bf16x8*)(Wp + (long long)gid * 8) = o;
}

// c1[o] = sum_k bf16(W2[o][k] g[k]) (the packed values), c2[o] = sum_k W2[o][k] b[k]; one block per output row
__global__ __launch_bounds__(256) void ffn_dec_consts_kernel(const float* __restrict__ W2, const float* __restrict__ gF,
                                                             const float* __restrict__ bF, float* __restrict__ c1,
                                                             float* __restrict__ c2) {
    __shared__ float r1[256], r2[256];
    const int o = blockIdx.x, t = threadIdx.x;
    float s1 = 0.f, s2 = 0.f;
    for (int k = t; k < FF; k += 256) {
        const float wv = W2[(long long)o * FF + k];
        s1 += bf2f(f2bf(wv * gF[k]));
        s2 += wv * bF[k];
    }
    r1[t] = s1; r2[t] = s2;
    __syncthreads();
    for (int n = 128; n > 0; n >>= 1) {
        if (t < n) { r1[t] += r1[t + n]; r2[t] += r2[t + n]; }
        __syncthreads();
    }
    if (t == 0) { c1[o] = r1[0]; c2[o] = r2[0]; }
}

}  // namespace

size_t pfm_ffn_packed_elems() { return (size_t)NTILE * TILE / 2; }

hipError_t pfm_ffn_pack_dec(const bf16* W1, const float* W2, const float* gF, const float* bF, bf16* Wp, float* c1,
                            float* c2, hipStream_t st) {
    hipLaunchKernelGGL(ffn_pack_dec_kernel, dim3(NTILE * 1024 / 256), dim3(256), 0, st, W1, W2, gF, Wp);
    PFM_LAUNCH_CHECK();
    hipLaunchKernelGGL(ffn_dec_consts_kernel, dim3(FD), dim3(256), 0, st, W2, gF, bF, c1, c2);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// the LN_F fold constants alone (c1 = rowsum(bf16(W2 diag(gamma_F))), c2 = W2 beta_F), for k_ffn2.hip's split decoder pack
hipError_t pfm_ffn_dec_consts(const float* W2, const float* gF, const float* bF, float* c1, float* c2, hipStream_t st) {
    hipLaunchKernelGGL(ffn_dec_consts_kernel, dim3(FD), dim3(256), 0, st, W2, gF, bF, c1, c2);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// Fused decoder feed-forward (ffn_fused_kernel DEC): x f32 [M, 512] -> xn = LN_next(W2 LN_F(relu(W1 LN1(x) + b1)))
// bf16 [M, 512] (+ the f32 FFN output in xo when non-null). Wp / c1 / c2 from pfm_ffn_pack_dec.
// With o (bf16 [M, 512], the previous block's cross-attention output) and bo: that block's out-projection runs
// first (mode 3): x1 = x + o Wo^T + bo is written to xo (f32, may alias x) and the FFN runs on x1; Wp then
// points at the 32 Wo tiles that precede the FFN tiles.
template <int VAR, int MODE, int NW, bool HR, int PD>
static void ffn_launch(hipStream_t st, int M, const float* x, const float* g, const float* be, float eps, const bf16* Wp,
                const float* b1, const float* b2, float* xo, const float* gn, const float* bn, bf16* xn, const bf16* o,
                const bf16* f, const float* bo, const float* c1) {
    static bool attr_done = false;   // one flag per instantiation
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)ffn_fused_kernel<VAR, MODE, NW, HR, PD>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    }
    hipLaunchKernelGGL((ffn_fused_kernel<VAR, MODE, NW, HR, PD>), dim3((M + BM - 1) / BM), dim3(64 * NW), LDS_BYTES, st, x, M,
                       g, be, eps, Wp, b1, b2, xo, gn, bn, xn, o, f, bo, c1);
}

template <int VAR, int MODE>
static void ffn_launch_nw(hipStream_t st, int M, const float* x, const float* g, const float* be, float eps, const bf16* Wp,
                   const float* b1, const float* b2, float* xo, const float* gn, const float* bn, bf16* xn, const bf16* o,
                   const bf16* f, const float* bo, const float* c1) {
    ffn_launch<VAR, MODE, 8, true, 3>(st, M, x, g, be, eps, Wp, b1, b2, xo, gn, bn, xn, o, f, bo, c1);
}

// Fused decoder feed-forward (ffn_fused_kernel DEC): x f32 [M, 512] -> xn = LN_next(W2 LN_F(relu(W1 LN1(x) + b1)))
// bf16 [M, 512] (+ the f32 FFN output in xo when non-null). Wp / c1 / c2 from pfm_ffn_pack_dec.
// With o (bf16 [M, 512], the previous block's cross-attention output) and bo: that block's out-projection runs
// first (mode 3): x1 = x + o Wo^T + bo is written to xo (f32, may alias x) and the FFN runs on x1; Wp then
// points at the 32 Wo tiles that precede the FFN tiles.
hipError_t pfm_ffn_fused_dec(const float* x, int M, const float* g1, const float* be1, float eps, const bf16* Wp,
                             const float* b1, const float* c1, const float* c2, float* xo, const float* gn,
                             const float* bn, bf16* xn, const bf16* o, const float* bo, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (!xn || !gn || !bn || !c1 || !c2 || (o && (!bo || !xo || !x))) return hipErrorInvalidValue;
    if (((uintptr_t)x | (uintptr_t)xo | (uintptr_t)Wp | (uintptr_t)xn | (uintptr_t)c1 | (uintptr_t)c2 | (uintptr_t)o |
         (uintptr_t)bo) % 16)
        return hipErrorInvalidValue;
    if (o)
        ffn_launch_nw<0, 3>(st, M, x, g1, be1, eps, Wp, b1, c2, xo, gn, bn, xn, o, nullptr, bo, c1);
    else
        ffn_launch_nw<0, 2>(st, M, x, g1, be1, eps, Wp, b1, c2, xo, gn, bn, xn, nullptr, nullptr, nullptr, c1);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
size_t pfm_ffn_packed_o_elems() { return (size_t)OP_TILES * TILE / 2; }

hipError_t pfm_ffn_pack_o(const bf16* Wo, bf16* Wp, hipStream_t st) {
    hipLaunchKernelGGL(ffn_pack_o_kernel, dim3(OP_TILES * 1024 / 256), dim3(256), 0, st, Wo, Wp);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_ffn_pack(const bf16* W1, const bf16* W2, bf16* Wp, hipStream_t st) {
    hipLaunchKernelGGL(ffn_pack_kernel, dim3(NTILE * 1024 / 256), dim3(256), 0, st, W1, W2, Wp);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// x [M, 512] f32 (read), xo [M, 512] f32 (may alias x: every workgroup reads its rows before writing
// them), Wp = pfm_ffn_pack output; gn / bn / xn optional (all three or none).
hipError_t pfm_ffn_fused(const float* x, int M, const float* g2, const float* be2, float eps, const bf16* Wp,
                         const float* b1, const float* b2, float* xo, const float* gn, const float* bn, bf16* xn,
                         hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if ((xn != nullptr) != (gn != nullptr && bn != nullptr)) return hipErrorInvalidValue;
    if (((uintptr_t)x | (uintptr_t)xo | (uintptr_t)Wp | (uintptr_t)xn) % 16) return hipErrorInvalidValue;
    const bf16* z = nullptr;
    const float* zf = nullptr;
    ffn_launch_nw<0, 0>(st, M, x, g2, be2, eps, Wp, b1, b2, xo, gn, bn, xn, z, z, zf, zf);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// The attention sub-layer's out-projection folded in front of the FFN (see ffn_fused_kernel, OP):
//   x1 = O Wo^T + bo + f (+ x)   (x optional)
//   xo = x1 + W2 relu(W1 LN2(x1) + b1) + b2 ;  xn = LN_next(xo) (optional, as pfm_ffn_fused)
// o, f: bf16 [M, 512]; Wop: pfm_ffn_pack_o output immediately followed by the layer's pfm_ffn_pack tiles.
hipError_t pfm_ffn_fused_op(const bf16* o, const bf16* f, const float* bo, const float* x, int M, const float* g2,
                            const float* be2, float eps, const bf16* Wop, const float* b1, const float* b2, float* xo,
                            const float* gn, const float* bn, bf16* xn, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if ((xn != nullptr) != (gn != nullptr && bn != nullptr) || !o || !f || !bo) return hipErrorInvalidValue;
    if (((uintptr_t)x | (uintptr_t)xo | (uintptr_t)Wop | (uintptr_t)xn | (uintptr_t)o | (uintptr_t)f | (uintptr_t)bo) % 16)
        return hipErrorInvalidValue;
    ffn_launch_nw<0, 1>(st, M, x, g2, be2, eps, Wop, b1, b2, xo, gn, bn, xn, o, f, bo, nullptr);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
