// bf16 MFMA GEMM family for the FAST-mode projections (gfx950).
//
//   C[M,N] = epi( A[M,K] . W[N,K]^T ),  A/W bf16 K-contiguous rows, f32 accumulate.
//
// Cfg<BM, BN, WGM, WGN, BK, NS>: block tile BM x BN on WGM x WGN waves; each wave owns a
// (BM/WGM) x (BN/WGN) tile = MI x NI blocks of v_mfma_f32_32x32x16_bf16; K-step BK; NS-stage
// LDS ring. Staging is global_load_lds_dwordx4 straight into LDS; an LDS-DMA writes lane-linear
// 1 KiB pieces, so the bank swizzle is applied on the SOURCE address: LDS slot s of row r holds
// logical 16-B chunk s ^ swz(r), which makes every ds_read_b128 fragment read (16 distinct rows
// per lane group, same chunk) conflict-free. Counted vmcnt waits + raw s_barrier per K-step.
// Epilogue: each wave re-lays its 32-row sub-tiles row-major in its own LDS slice; lanes then
// handle float4 column groups of whole rows (16-B bias/residual loads, 16-B f32 / 8-B bf16
// stores), or scan rows for the fused row-argmax of the output layer.
// Launcher contract: K % BK == 0, row strides % 8 == 0 (16-B aligned rows). Rows beyond M / N
// are clamped to valid memory and dropped in the epilogue.
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "pfm_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

template <int BM_, int BN_, int WGM_, int WGN_, int BK_, int NS_, int PP_ = 0, int MF_ = 0> struct Cfg {
    static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_, BK = BK_, NS = NS_;
    // MFMA shape: 0 = v_mfma_f32_32x32x16_bf16, 1 = v_mfma_f32_16x16x32_bf16 (one-barrier schedule only)
    static constexpr int MF = MF_;
    // schedule: 0 = one barrier per K-step; 1 = ping-pong (wave-row groups staggered by one barrier,
    // one K-step per phase); 2 = 8-phase (quadrant phases, one half-tile of DMA per phase, staggered)
    static constexpr int PP = PP_;
    static constexpr int NW = WGM * WGN, NT = NW * 64;
    static constexpr int WTM = BM / WGM, WTN = BN / WGN;
    static constexpr int MI = WTM / 32, NI = WTN / 32;
    static constexpr int ROWB = BK * 2, CPR = ROWB / 16, RPP = 1024 / ROWB;
    static constexpr int TA = BM * ROWB, TW = BN * ROWB, STAGE = TA + TW;
    static constexpr int PA = TA / 1024 / NW, PW = TW / 1024 / NW;
    static constexpr int EP = WTN + 4;                 // staged epilogue row pitch (floats)
    static constexpr int EPW = 32 * EP * 4;            // epilogue LDS bytes per wave
    static constexpr int LDS = (NS * STAGE > NW * EPW) ? NS * STAGE : NW * EPW;
    static_assert(TA % (1024 * NW) == 0 && TW % (1024 * NW) == 0, "tile not divisible into DMA pieces");
    static_assert(WTN == 64, "epilogue / argmax partials assume 64-column wave tiles");
    static_assert(MF == 0 || ((PP == 0 || PP == 2) && BK % 32 == 0), "16x16x32 MFMA: one-barrier or 8-phase schedule");
    static_assert(PP != 1 || (WGM == 2 && NS >= 3), "ping-pong needs two wave-row groups and >= 3 stages");
    static_assert(PP != 2 || (BM == 256 && BN == 256 && WGM == 2 && WGN == 4 && BK == 64 && NS == 2),
                  "8-phase schedule: 256x256 tile, 2x4 waves, BK 64, two K-tile buffers");
    static_assert(PP != 3 || (BM == 256 && BN == 256 && WGM == 2 && WGN == 4 && BK == 32 && NS == 4),
                  "k-step phase schedule: 256x256 tile, 2x4 waves, BK 32, four K-tile buffers");
    __device__ static inline int swz(int row) { return CPR == 8 ? ((row >> 1) & 7) : ((row >> 2) & 3); }
};

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

template <int P> __device__ __forceinline__ void wait_vm(int rem) {
    if (rem >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
    else if (rem == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <class C>
__global__ __launch_bounds__(C::NT) void gemm_bf16_kernel(const bf16* __restrict__ A, RowMap amap,
                                                          const bf16* __restrict__ W, long long ldw, int M, int N,
                                                          int K, int tiles_m, int tiles_n, int gm, GemmEpi epi) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BK = C::BK, NS = C::NS, ROWB = C::ROWB, MI = C::MI, NI = C::NI, PA = C::PA, PW = C::PW;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    // grouped order: consecutive tiles walk down gm tile-rows before moving one tile-column right, so
    // the ~32 tiles an XCD runs at once share gm A-row bands and a few W-column bands in its 4 MiB L2
    // (row-major order streamed all of W once per tile-row on the wide-N projections)
    int tm, tn;
    if (gm > 0) {
        const int gsz = gm * tiles_n, g = wg / gsz, idx = wg - g * gsz;
        const int rows = min(gm, tiles_m - g * gm);
        tm = g * gm + idx % rows;
        tn = idx / rows;
    } else {
        tm = wg / tiles_n;
        tn = wg % tiles_n;
    }
    const int m0 = tm * C::BM, n0 = tn * C::BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / C::WGN, wn = wid % C::WGN;
    const int fr = lane & 31, fh = lane >> 5;

    const bf16* ga[PA];
    const bf16* gw[PW];
    {
        const int sub = lane / C::CPR, slot = lane % C::CPR;
#pragma unroll
        for (int j = 0; j < PA; ++j) {
            const int row = C::RPP * (PA * wid + j) + sub;
            ga[j] = A + amap.off(min(m0 + row, M - 1)) + (slot ^ C::swz(row)) * 8;
        }
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const int row = C::RPP * (PW * wid + j) + sub;
            gw[j] = W + (long long)min(n0 + row, N - 1) * ldw + (slot ^ C::swz(row)) * 8;
        }
    }
    // split-bf16 emulation of an f32 GEMM (epi.x6_k > 0): K step k0 of the K' = 6 x6_k loop reads A
    // segment pa = {2,1,0,1,0,0}[s] and W plane pw = {0,1,2,0,1,0}[s] of segment s = k0 / x6_k (a K step
    // never straddles segments: x6_k % BK == 0). Small products first.
    // bf16x3 (x6_terms 3): segments 3..5 only.
    // split WEIGHTS only (x6_terms 2, fast mode's precise-weight projections): A is one plain bf16 operand [M, x6_k],
    // W two planes w = w0 + w1 (x6_ws apart); K' = 2 x6_k runs (A, W1) then (A, W0).
    const int xk = epi.x6_k, xt = epi.x6_terms, sg0 = xt == 3 ? 3 : 0;
    auto koff_a = [&](int k0) -> int {
        if (!xk) return k0;
        const int s0 = k0 / xk, kk = k0 - s0 * xk, sg = s0 + sg0;
        if (xt == 2) return kk;
        return (sg == 0 ? 2 : (sg == 1 || sg == 3) ? 1 : 0) * xk + kk;
    };
    auto koff_w = [&](int k0) -> long long {
        if (!xk) return k0;
        const int s0 = k0 / xk, kk = k0 - s0 * xk, sg = s0 + sg0;
        if (xt == 2) return (long long)(s0 == 0 ? 1 : 0) * epi.x6_ws + kk;
        return (long long)(sg == 1 || sg == 4 ? 1 : sg == 2 ? 2 : 0) * epi.x6_ws + kk;
    };
    auto stage = [&](int k0, int s) {
        unsigned char* base = smem + s * C::STAGE;
        const int ka = koff_a(k0);
        const long long kw = koff_w(k0);
#pragma unroll
        for (int j = 0; j < PA; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void*)(ga[j] + ka), (lds_void*)(base + (PA * wid + j) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int j = 0; j < PW; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void*)(gw[j] + kw),
                                             (lds_void*)(base + C::TA + (PW * wid + j) * 1024), 16, 0, 0);
    };

    f32x16 acc[MI][NI];
    // MF 1: 16x16 blocks, block (i4, j4) = rows 16 i4.., cols 16 j4.. of the wave tile;
    // C/D map col = lane & 15, row = 4 (lane >> 4) + reg
    f32x4 acc4[C::MF ? 2 * MI : 1][C::MF ? 2 * NI : 1];
    if constexpr (C::MF == 0) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    } else {
#pragma unroll
        for (int i = 0; i < 2 * MI; ++i)
#pragma unroll
            for (int j = 0; j < 2 * NI; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc4[i][j][e] = 0.f;
    }
    int aoff[MI], asw[MI], woff[NI], wsw[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int row = wm * C::WTM + i * 32 + fr;
        aoff[i] = row * ROWB;
        asw[i] = C::swz(row);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const int row = wn * C::WTN + j * 32 + fr;
        woff[j] = C::TA + row * ROWB;
        wsw[j] = C::swz(row);
    }

    const int nk = K / BK;
    if constexpr (C::PP != 2 && C::PP != 3) {
#pragma unroll
        for (int s = 0; s < NS - 1; ++s)
            if (s < nk) stage(s * BK, s);
    }
    if constexpr (C::PP == 3) {
        // k-step phases (BK 32 = 2 phases per K-tile, 4 K-tile buffers): phase (j, kk) runs the 8 MFMAs
        // of k-step kk of K-tile j over the whole 128x64 wave tile (6 fragment reads: A m-blocks 0..3,
        // B n-blocks 0..1) and issues ONE 16-KiB operand tile of K-tile j+3 (phase kk=0: its A tile,
        // kk=1: its W tile; 2 DMA pieces per wave). R = reads + DMA -> barrier -> M = MFMAs -> barrier;
        // wave-row group 1 runs one barrier behind.
        //  WAR: K-tile j+3 goes to buffer (j-1)&3, whose last reads were in the phase before (j, 0).
        //  RAW: K-tile j+3 is first read in phase (j+3, 0); it is retired at the end of phase (j+2, 1)
        //       with vmcnt(8) (the 4 operand tiles issued in the 4 phases after it stay in flight); G0
        //       waits after M, G1 after R, both before the common barrier ahead of the first read.
        const bf16* osrc[2][2];
        {
            const int sub = lane >> 2, slot = lane & 3;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = 16 * (2 * wid + j) + sub;
                osrc[0][j] = A + amap.off(min(m0 + row, M - 1)) + (slot ^ C::swz(row)) * 8;
                osrc[1][j] = W + (long long)min(n0 + row, N - 1) * ldw + (slot ^ C::swz(row)) * 8;
            }
        }
        auto issue = [&](int tile, int op) -> bool {
            if (tile >= nk) return false;
            unsigned char* base = smem + (tile & 3) * C::STAGE + op * C::TA;
            const long long ko = op ? koff_w(tile * BK) : (long long)koff_a(tile * BK);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(osrc[op][j] + ko),
                                                 (lds_void*)(base + (2 * wid + j) * 1024), 16, 0, 0);
            return true;
        };
        auto bar = [&]() {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        };
        const int grp = wm;
        // retire K-tile `need` (all its DMA) with `after` K-tiles' worth of later issues allowed in flight
        auto wait_tile = [&](int need, int tj) {
            if (need >= nk) return;
            const int later = min(nk, tj + 4) - (need + 1);   // K-tiles issued after `need` (2 ops each)
            if (later >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        };
        auto phase = [&](int j, int kk) {
            const unsigned char* sb = smem + (j & 3) * C::STAGE;
            const int c = 2 * kk + fh;
            bf16x8 af[MI], bfr[NI];
#pragma unroll
            for (int jn = 0; jn < NI; ++jn) bfr[jn] = *(const bf16x8*)(sb + woff[jn] + ((c ^ wsw[jn]) << 4));
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = *(const bf16x8*)(sb + aoff[i] + ((c ^ asw[i]) << 4));
            issue(j + 3, kk);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (grp == 1 && kk == 1) wait_tile(j + 1, j);
            bar();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int jn = 0; jn < NI; ++jn)
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[jn], acc[i][jn], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            if (grp == 0 && kk == 1) wait_tile(j + 1, j);
            bar();
        };
        // prologue: K-tiles 0, 1, 2 in flight; K-tile 0 retired
#pragma unroll
        for (int t = 0; t < 3; ++t) { issue(t, 0); issue(t, 1); }
        {
            const int later = min(nk, 3) - 1;
            if (later >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (grp == 1) bar();
        for (int j = 0; j < nk; ++j) {
            phase(j, 0);
            phase(j, 1);
        }
        if (grp == 0) bar();   // match group 1's stagger barrier
    } else if constexpr (C::PP == 2) {
        // 8-phase schedule (2 K-tiles per iteration, even tile -> buffer 0, odd -> buffer 1). Each phase
        // computes one quadrant of the wave's 128x64 tile for one K-tile (8 MFMAs): q0 = m-blocks 0,1 x
        // n-block 0 (reads A(m0,1) + B(n0)), q1 = m0,1 x n1 (reads B(n1)), q2 = m2,3 x n1 (reads A(m2,3)),
        // q3 = m2,3 x n0 (reads B(n0)). Per phase: R = fragment reads + ONE half-tile (16 KiB: A rows
        // 0-127 / 128-255, W rows 0-127 / 128-255; 2 DMA pieces per wave) -> barrier -> M = MFMAs ->
        // barrier; wave-row group 1 runs one barrier behind (ping-pong on every SIMD).
        //  WAR: a buffer's A halves are restaged from the phase after their last read (q2), its W
        //       halves from the phase after q3; reads are retired (lgkmcnt 0) before the barrier ending R.
        //  RAW: a K-tile's last half is issued >= 1 phase before the wait that retires it (end of phases
        //       3 and 7: vmcnt(2) = only the phase's own half-tile in flight; G0 waits after M, G1
        //       after R, both before the common barrier that precedes the first read).
        const bf16* hsrc[4][2];
        {
            const int sub = lane >> 3, slot = lane & 7;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int prow = 8 * (2 * wid + j) + sub;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int row = hh * 128 + prow;
                    hsrc[hh][j] = A + amap.off(min(m0 + row, M - 1)) + (slot ^ C::swz(row)) * 8;
                    hsrc[2 + hh][j] = W + (long long)min(n0 + row, N - 1) * ldw + (slot ^ C::swz(row)) * 8;
                }
            }
        }
        auto issue = [&](int tile, int hh) -> bool {
            if (tile >= nk) return false;
            unsigned char* base = smem + (tile & 1) * C::STAGE + (hh >> 1) * C::TA + (hh & 1) * 16384;
            const long long ko = (hh >> 1) ? koff_w(tile * BK) : (long long)koff_a(tile * BK);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(hsrc[hh][j] + ko),
                                                 (lds_void*)(base + (2 * wid + j) * 1024), 16, 0, 0);
            return true;
        };
        auto bar = [&]() {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        };
        const int grp = wm;
        bf16x8 aF[2][4], bF[4];
        // MF 1: quadrant = 4 m16 x 2 n16 blocks over two 32-deep k-substeps (16 MFMAs, 8 A + 4 B reads)
        bf16x8 aF16[4][2], bF16[2][2];
        const int r16 = lane & 15, g16 = lane >> 4, sw16 = C::swz(r16);
        auto phase16 = [&](int tile, int q, int itile, int ih, bool wait_after) {
            const unsigned char* sb = smem + (tile & 1) * C::STAGE;
            const int i0 = (q >= 2) ? 4 : 0, j0 = (q == 1 || q == 2) ? 2 : 0;
            // B first (4 reads), then A (8): an lgkmcnt count would retire B before A
            if (q != 2) {
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                    for (int kq = 0; kq < 2; ++kq)
                        bF16[jj][kq] = *(const bf16x8*)(sb + C::TA + (wn * C::WTN + (j0 + jj) * 16 + r16) * ROWB +
                                                        (((4 * kq + g16) ^ sw16) << 4));
            }
            if (q == 0 || q == 2) {
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
#pragma unroll
                    for (int kq = 0; kq < 2; ++kq)
                        aF16[ii][kq] = *(const bf16x8*)(sb + (wm * C::WTM + (i0 + ii) * 16 + r16) * ROWB +
                                                        (((4 * kq + g16) ^ sw16) << 4));
            }
            const bool did = issue(itile, ih);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (grp == 1 && wait_after) {
                if (did) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            bar();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int kq = 0; kq < 2; ++kq)
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
                        acc4[i0 + ii][j0 + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aF16[ii][kq], bF16[jj][kq],
                                                                                        acc4[i0 + ii][j0 + jj], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            if (grp == 0 && wait_after) {
                if (did) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            bar();
        };
        auto phase = [&](int tile, int q, int itile, int ih, bool wait_after) {
            if constexpr (C::MF == 1) { phase16(tile, q, itile, ih, wait_after); return; }
            const unsigned char* sb = smem + (tile & 1) * C::STAGE;
            const int i0 = (q >= 2) ? 2 : 0, jn = (q == 1 || q == 2) ? 1 : 0;
            if (q == 0 || q == 2) {
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
                        aF[ii][kk] = *(const bf16x8*)(sb + aoff[i0 + ii] + (((2 * kk + fh) ^ asw[i0 + ii]) << 4));
            }
            if (q != 2) {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    bF[kk] = *(const bf16x8*)(sb + woff[jn] + (((2 * kk + fh) ^ wsw[jn]) << 4));
            }
            const bool did = issue(itile, ih);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (grp == 1 && wait_after) {
                if (did) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            bar();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
                    acc[i0 + ii][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aF[ii][kk], bF[kk], acc[i0 + ii][jn], 0,
                                                                              0, 0);
            __builtin_amdgcn_s_setprio(0);
            if (grp == 0 && wait_after) {
                if (did) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            bar();
        };
        // prologue: K-tile 0 whole, K-tile 1's first half (its A0) in flight
#pragma unroll
        for (int hh = 0; hh < 4; ++hh) issue(0, hh);
        if (issue(1, 0)) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (grp == 1) bar();
        for (int e = 0; e < nk; e += 2) {
            const int o = e + 1;
            phase(e, 0, o, 1, false);
            phase(e, 1, o, 2, false);
            phase(e, 2, o, 3, false);
            phase(e, 3, e + 2, 0, true);
            phase(o, 0, e + 2, 1, false);
            phase(o, 1, e + 2, 2, false);
            phase(o, 2, e + 2, 3, false);
            phase(o, 3, o + 2, 0, true);
        }
        if (grp == 0) bar();   // match group 1's stagger barrier
    } else if constexpr (C::PP == 1) {
        // Ping-pong schedule. Wave-row group g = wm (0/1; the two groups share every SIMD). Per K-tile t
        // each wave runs an R phase (issue the DMA for stage t+NS-1, read all fragments of stage t,
        // lgkmcnt(0)) and an M phase (the MFMAs), each closed by an s_barrier. Group 1 starts one
        // barrier late, so one group's LDS reads + DMA issue overlap the other group's MFMAs.
        // Common barrier numbering: G0 runs R(t) before #2t+1 and M(t) before #2t+2; G1 runs R(t)
        // before #2t+2 and M(t) before #2t+3.
        //  RAW: every wave retires its own stage-(t+1) DMA before common barrier #2t+2 (G0: end of
        //       M(t), G1: end of R(t)); readers of stage t+1 start after #2t+2 (G0) / #2t+3 (G1).
        //  WAR: stage t+NS-1 overwrites buffer (t-1)%NS in R(t), i.e. after #2t (G0) / #2t+1 (G1);
        //       the last reads of that buffer (R(t-1)) were retired before #2t-1 (G0) / #2t (G1).
        constexpr int P = PA + PW;
        const int grp = wm;
        auto retire_next = [&](int kt) {   // stage kt+1 landed (own pieces)
            const int rem = nk - 2 - kt;    // stages issued beyond kt+1
            if (rem >= NS - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P * (NS - 2)) : "memory");
            else if (NS - 2 >= 2 && rem == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        };
        // stage 0 complete and visible to everyone before either group reads it
        if (nk - 1 >= NS - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P * (NS - 2)) : "memory");
        else if (NS - 2 >= 2 && nk - 1 == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (grp == 1) __builtin_amdgcn_s_barrier();
        for (int kt = 0; kt < nk; ++kt) {
            __builtin_amdgcn_sched_barrier(0);
            if (kt + NS - 1 < nk) stage((kt + NS - 1) * BK, (kt + NS - 1) % NS);
            const unsigned char* sb = smem + (kt % NS) * C::STAGE;
            bf16x8 af[BK / 16][MI], bfr[BK / 16][NI];
#pragma unroll
            for (int kq = 0; kq < BK / 16; ++kq) {
                const int c = 2 * kq + fh;
#pragma unroll
                for (int j = 0; j < NI; ++j) bfr[kq][j] = *(const bf16x8*)(sb + woff[j] + ((c ^ wsw[j]) << 4));
#pragma unroll
                for (int i = 0; i < MI; ++i) af[kq][i] = *(const bf16x8*)(sb + aoff[i] + ((c ^ asw[i]) << 4));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (grp == 1 && kt + 1 < nk) retire_next(kt);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int kq = 0; kq < BK / 16; ++kq)
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NI; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kq][i], bfr[kq][j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            if (grp == 0 && kt + 1 < nk) retire_next(kt);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
        if (grp == 0) __builtin_amdgcn_s_barrier();   // match group 1's stagger barrier
    } else if constexpr (C::MF == 1) {
        // 16x16x32 fragments: lane (r = lane & 15, g = lane >> 4) reads row r of a 16-row block, K chunk
        // 4 kq + g of the 32-wide k-substep kq (the same source-side swizzle keeps the 16 rows x 4 chunks
        // of every ds_read_b128 lane group on distinct banks)
        const int r16 = lane & 15, g16 = lane >> 4;
        // 16-row blocks start at multiples of 16 rows, so the row swizzle depends on r16 only and every
        // block's fragment address is one base + a compile-time offset (ds_read immediate)
        const int sw = C::swz(r16);
        const int abase = (wm * C::WTM + r16) * ROWB, wbase = C::TA + (wn * C::WTN + r16) * ROWB;
        for (int kt = 0; kt < nk; ++kt) {
            wait_vm<PA + PW>(min(NS - 2, nk - 1 - kt));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (kt + NS - 1 < nk) stage((kt + NS - 1) * BK, (kt + NS - 1) % NS);
            const unsigned char* sb = smem + (kt % NS) * C::STAGE;
#pragma unroll
            for (int kq = 0; kq < BK / 32; ++kq) {
                const int co = ((4 * kq + g16) ^ sw) << 4;
                const unsigned char* pa = sb + abase + co;
                const unsigned char* pw = sb + wbase + co;
                bf16x8 af[2 * MI], bfr[2 * NI];
#pragma unroll
                for (int i = 0; i < 2 * MI; ++i) af[i] = *(const bf16x8*)(pa + i * 16 * ROWB);
#pragma unroll
                for (int j = 0; j < 2 * NI; ++j) bfr[j] = *(const bf16x8*)(pw + j * 16 * ROWB);
#pragma unroll
                for (int i = 0; i < 2 * MI; ++i)
#pragma unroll
                    for (int j = 0; j < 2 * NI; ++j)
                        acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc4[i][j], 0, 0, 0);
            }
        }
    } else
    for (int kt = 0; kt < nk; ++kt) {
        wait_vm<PA + PW>(min(NS - 2, nk - 1 - kt));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + NS - 1 < nk) stage((kt + NS - 1) * BK, (kt + NS - 1) % NS);
        const unsigned char* sb = smem + (kt % NS) * C::STAGE;
#pragma unroll
        for (int kq = 0; kq < BK / 16; ++kq) {
            const int c = 2 * kq + fh;
            bf16x8 af[MI], bfr[NI];
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = *(const bf16x8*)(sb + aoff[i] + ((c ^ asw[i]) << 4));
#pragma unroll
            for (int j = 0; j < NI; ++j) bfr[j] = *(const bf16x8*)(sb + woff[j] + ((c ^ wsw[j]) << 4));
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NI; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- epilogue (C/D map: col = lane&31, row = (e&3) + 8(e>>2) + 4(lane>>5))
    if (epi.vec_ok || epi.amax_val) {
        constexpr int EP = C::EP;
        float* ep = (float*)(smem + wid * C::EPW);
        const bool f32o = epi.out_dtype == DT_F32;
        // a lane's output columns are the same for every row it writes: one bias load, before any store
        const bool st16 = epi.st16_ok && !(epi.res0 || epi.res1);
        const int colv = n0 + wn * 64 + (st16 ? (lane & 7) * 8 : (lane & 15) * 4);
        float4 bb = make_float4(0.f, 0.f, 0.f, 0.f), bb2 = bb;
        if (epi.out && epi.bias && colv < N) {
            bb = *(const float4*)(epi.bias + colv);
            if (st16) bb2 = *(const float4*)(epi.bias + colv + 4);
        }
        // consume it here, before any store: otherwise paths that skip rows leave it "pending" and the
        // compiler re-waits vmcnt(0) (draining the stores issued since) at every use below
        asm volatile("" ::"v"(bb.x), "v"(bb.y), "v"(bb.z), "v"(bb.w), "v"(bb2.x), "v"(bb2.y), "v"(bb2.z),
                     "v"(bb2.w));
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            if constexpr (C::MF == 0) {
#pragma unroll
                for (int j = 0; j < NI; ++j)
#pragma unroll
                    for (int e = 0; e < 16; ++e) ep[((e & 3) + 8 * (e >> 2) + 4 * fh) * EP + j * 32 + fr] = acc[i][j][e];
            } else {
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                    for (int j = 0; j < 2 * NI; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            ep[(ii * 16 + 4 * (lane >> 4) + e) * EP + j * 16 + (lane & 15)] = acc4[2 * i + ii][j][e];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (epi.amax_val) {
                // fused row-argmax of the output layer over this wave's 64 columns: 2 lanes per staged
                // row scan 32 columns each in order (first index wins ties, like torch.argmax)
                const int rr = lane >> 1, half = lane & 1;
                const int cb = n0 + wn * 64 + half * 32;
                float bv = -INFINITY;
                int bi = 0x7fffffff;
                for (int cc = 0; cc < 32; ++cc) {
                    const int col = cb + cc;
                    if (col < N) {
                        const float v = ep[rr * EP + half * 32 + cc] * epi.alpha + (epi.bias ? epi.bias[col] : 0.f);
                        if (v > bv) { bv = v; bi = col; }
                    }
                }
                const float ov = __shfl_xor(bv, 1, 64);
                const int oi = __shfl_xor(bi, 1, 64);
                if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
                const int row = m0 + wm * C::WTM + i * 32 + rr;
                if (half == 0 && row < M) {
                    const long long p = (long long)row * epi.n_tiles + (n0 + wn * 64) / 64;
                    epi.amax_val[p] = bv;
                    epi.amax_idx[p] = bi;
                }
            }
            if (st16) {
#pragma unroll
                for (int sidx = 0; sidx < 4; ++sidx) {
                    const int f = lane + 64 * sidx, rr = f >> 3, c8 = f & 7;
                    const int row = m0 + wm * C::WTM + i * 32 + rr;
                    const int col = n0 + wn * 64 + c8 * 8;
                    if (row >= M || col >= N) continue;
                    float4 v = *(const float4*)(ep + rr * EP + c8 * 8);
                    float4 u = *(const float4*)(ep + rr * EP + c8 * 8 + 4);
                    v.x = v.x * epi.alpha + bb.x; v.y = v.y * epi.alpha + bb.y;
                    v.z = v.z * epi.alpha + bb.z; v.w = v.w * epi.alpha + bb.w;
                    u.x = u.x * epi.alpha + bb2.x; u.y = u.y * epi.alpha + bb2.y;
                    u.z = u.z * epi.alpha + bb2.z; u.w = u.w * epi.alpha + bb2.w;
                    if (epi.relu) {
                        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
                        u.x = fmaxf(u.x, 0.f); u.y = fmaxf(u.y, 0.f); u.z = fmaxf(u.z, 0.f); u.w = fmaxf(u.w, 0.f);
                    }
                    bf16x8 t = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w), f2bf(u.x), f2bf(u.y), f2bf(u.z), f2bf(u.w)};
                    *(bf16x8*)((bf16*)epi.out + epi.out_map.off(row) + col) = t;
                }
            } else if (C::MI <= 2 && epi.res_batch && (epi.res0 || epi.res1) && epi.out) {
                // (64-row wave tiles only: with 128-row tiles the extra registers spill)
                // residual loads of 4 row groups first, then their stores (vmcnt retires in order: a load
                // queued behind a store waits for it)
#pragma unroll
                for (int sb = 0; sb < 8; sb += 4) {
                    float4 r0[4], r1[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int f = lane + 64 * (sb + q), rr = f >> 4, c4 = f & 15;
                        const long long row = min(m0 + wm * C::WTM + i * 32 + rr, M - 1);
                        const int col = min(n0 + wn * 64 + c4 * 4, N - 4);
                        r0[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                        r1[q] = r0[q];
                        if (epi.res0) {
                            if (epi.res0_bf16) {
                                const bf16x4 t = *(const bf16x4*)((const bf16*)epi.res0 + row * epi.ld_res0 + col);
                                r0[q] = make_float4(bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3]));
                            } else {
                                r0[q] = *(const float4*)(epi.res0 + row * epi.ld_res0 + col);
                            }
                        }
                        if (epi.res1) r1[q] = *(const float4*)(epi.res1 + row * epi.ld_res1 + col);
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int f = lane + 64 * (sb + q), rr = f >> 4, c4 = f & 15;
                        const int row = m0 + wm * C::WTM + i * 32 + rr;
                        const int col = n0 + wn * 64 + c4 * 4;
                        if (row >= M || col >= N) continue;
                        float4 v = *(const float4*)(ep + rr * EP + c4 * 4);
                        v.x = v.x * epi.alpha + bb.x; v.y = v.y * epi.alpha + bb.y;
                        v.z = v.z * epi.alpha + bb.z; v.w = v.w * epi.alpha + bb.w;
                        if (epi.relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
                        v.x += r0[q].x + r1[q].x; v.y += r0[q].y + r1[q].y;
                        v.z += r0[q].z + r1[q].z; v.w += r0[q].w + r1[q].w;
                        const long long ob = epi.out_map.off(row) + col;
                        if (f32o) *(float4*)((float*)epi.out + ob) = v;
                        else {
                            bf16x4 t = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                            *(bf16x4*)((bf16*)epi.out + ob) = t;
                        }
                        if (epi.out2) {
                            bf16x4 t = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                            *(bf16x4*)((bf16*)epi.out2 + epi.out2_map.off(row) + col) = t;
                        }
                    }
                }
            } else
#pragma unroll
            for (int sidx = 0; sidx < 8; ++sidx) {
                if (!epi.out) break;
                const int f = lane + 64 * sidx, rr = f >> 4, c4 = f & 15;
                const int row = m0 + wm * C::WTM + i * 32 + rr;
                const int col = n0 + wn * 64 + c4 * 4;
                if (row >= M || col >= N) continue;
                float4 v = *(const float4*)(ep + rr * EP + c4 * 4);
                v.x = v.x * epi.alpha + bb.x; v.y = v.y * epi.alpha + bb.y;
                v.z = v.z * epi.alpha + bb.z; v.w = v.w * epi.alpha + bb.w;
                if (epi.relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
                if (epi.res0) {
                    float4 r0;
                    if (epi.res0_bf16) {
                        const bf16x4 rb = *(const bf16x4*)((const bf16*)epi.res0 + (long long)row * epi.ld_res0 + col);
                        r0 = make_float4(bf2f(rb[0]), bf2f(rb[1]), bf2f(rb[2]), bf2f(rb[3]));
                    } else {
                        r0 = *(const float4*)(epi.res0 + (long long)row * epi.ld_res0 + col);
                    }
                    v.x += r0.x; v.y += r0.y; v.z += r0.z; v.w += r0.w;
                }
                if (epi.res1) {
                    const float4 r1 = *(const float4*)(epi.res1 + (long long)row * epi.ld_res1 + col);
                    v.x += r1.x; v.y += r1.y; v.z += r1.z; v.w += r1.w;
                }
                const long long ob = epi.out_map.off(row) + col;
                if (f32o) *(float4*)((float*)epi.out + ob) = v;
                else if (epi.out_dtype == DT_X3) {   // EXACT-mode split operand of the next GEMM: planes N apart
                    const float vv[4] = {v.x, v.y, v.z, v.w};
                    bf16x4 p0, p1, p2;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        bf16 u, w, z;
                        split3_bf16(vv[e], u, w, z);
                        p0[e] = u; p1[e] = w; p2[e] = z;
                    }
                    *(bf16x4*)((bf16*)epi.out + ob) = p0;
                    *(bf16x4*)((bf16*)epi.out + ob + N) = p1;
                    *(bf16x4*)((bf16*)epi.out + ob + 2 * N) = p2;
                } else {
                    bf16x4 t = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                    *(bf16x4*)((bf16*)epi.out + ob) = t;
                }
                if (epi.out2) {
                    bf16x4 t = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                    *(bf16x4*)((bf16*)epi.out2 + epi.out2_map.off(row) + col) = t;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        return;
    }
    // scalar fallback epilogue (odd N / strides): straight from the accumulators
    if constexpr (C::MF == 1) {   // re-pack the 16x16 blocks into the 32x32 register map
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        float* ep = (float*)(smem + wid * C::EPW);
        constexpr int EP = C::EP;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int j = 0; j < 2 * NI; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        ep[(ii * 16 + 4 * (lane >> 4) + e) * EP + j * 16 + (lane & 15)] = acc4[2 * i + ii][j][e];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int j = 0; j < NI; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = ep[((e & 3) + 8 * (e >> 2) + 4 * fh) * EP + j * 32 + fr];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = m0 + wm * C::WTM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
            if (row >= M) continue;
            const long long ob = epi.out_map.off(row);
#pragma unroll
            for (int j = 0; j < NI; ++j) {
                const int col = n0 + wn * C::WTN + j * 32 + fr;
                if (col >= N) continue;
                float v = acc[i][j][e] * epi.alpha;
                if (epi.bias) v += epi.bias[col];
                if (epi.relu) v = fmaxf(v, 0.f);
                if (epi.res0)
                    v += epi.res0_bf16 ? bf2f(((const bf16*)epi.res0)[(long long)row * epi.ld_res0 + col])
                                       : epi.res0[(long long)row * epi.ld_res0 + col];
                if (epi.res1) v += epi.res1[(long long)row * epi.ld_res1 + col];
                if (epi.out_dtype == DT_F32) ((float*)epi.out)[ob + col] = v;
                else ((bf16*)epi.out)[ob + col] = f2bf(v);
                if (epi.out2) ((bf16*)epi.out2)[epi.out2_map.off(row) + col] = f2bf(v);
            }
        }
    }
}

// Persistent variant: gridDim.x = min(tiles, CUs) blocks; block b walks tiles slot(b), slot(b)+grid, ...
// The LDS-DMA ring runs over the flattened (tile, k-step) sequence, so the next tile's first NS-1
// stages are in flight while the current tile finishes and runs its epilogue; the epilogue stages
// 16-row halves of each wave's 32-row sub-tiles in a wave-private LDS slice next to the ring, and its
// stores drain behind the next tile's MFMAs. Blocks that share an XCD (bid % 8) take consecutive
// tile slots, so each XCD's L2 holds a compact band of A rows / W columns.
template <class C, int EPR>
__global__ __launch_bounds__(C::NT) void gemm_bf16_persist_kernel(const bf16* __restrict__ A, RowMap amap,
                                                                  const bf16* __restrict__ W, long long ldw, int M,
                                                                  int N, int K, int tiles_m, int tiles_n, GemmEpi epi) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BK = C::BK, NS = C::NS, ROWB = C::ROWB, MI = C::MI, NI = C::NI, PA = C::PA, PW = C::PW;
    constexpr int EP = C::EP, EPH = EPR * EP * 4;   // EPR-row epilogue chunks (8 or 16)
    static_assert(EPR == 8 || EPR == 16, "epilogue chunk rows");
    const int ntiles = tiles_m * tiles_n;
    const int nb = gridDim.x, bid = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = bid % 8;
    const int slot = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int my_tiles = slot < ntiles ? (ntiles - 1 - slot) / nb + 1 : 0;
    const int nk = K / BK;
    const int total = my_tiles * nk;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / C::WGN, wn = wid % C::WGN;
    const int fr = lane & 31, fh = lane >> 5;
    const int sub = lane / C::CPR, sl = lane % C::CPR;
    int arow[PA], wrow[PW], acol[PA], wcol[PW];
#pragma unroll
    for (int j = 0; j < PA; ++j) {
        arow[j] = C::RPP * (PA * wid + j) + sub;
        acol[j] = (sl ^ C::swz(arow[j])) * 8;
    }
#pragma unroll
    for (int j = 0; j < PW; ++j) {
        wrow[j] = C::RPP * (PW * wid + j) + sub;
        wcol[j] = (sl ^ C::swz(wrow[j])) * 8;
    }
    auto stage = [&](int g, int s) {
        const int ti = g / nk, kt = g - ti * nk;
        const int t = slot + ti * nb;
        const int tm = t / tiles_n, tn = t - tm * tiles_n;
        const int k0 = kt * BK;
        unsigned char* base = smem + s * C::STAGE;
#pragma unroll
        for (int j = 0; j < PA; ++j)
            __builtin_amdgcn_global_load_lds(
                (gbl_void*)(A + amap.off(min(tm * C::BM + arow[j], M - 1)) + acol[j] + k0),
                (lds_void*)(base + (PA * wid + j) * 1024), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < PW; ++j)
            __builtin_amdgcn_global_load_lds(
                (gbl_void*)(W + (long long)min(tn * C::BN + wrow[j], N - 1) * ldw + wcol[j] + k0),
                (lds_void*)(base + C::TA + (PW * wid + j) * 1024), 16, 0, 0);
    };
    int aoff[MI], asw[MI], woff[NI], wsw[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int row = wm * C::WTM + i * 32 + fr;
        aoff[i] = row * ROWB;
        asw[i] = C::swz(row);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const int row = wn * C::WTN + j * 32 + fr;
        woff[j] = C::TA + row * ROWB;
        wsw[j] = C::swz(row);
    }
    f32x16 acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    float* ep = (float*)(smem + NS * C::STAGE + wid * EPH);
    const bool f32o = epi.out_dtype == DT_F32;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < total) stage(s, s);
    for (int g = 0; g < total; ++g) {
        wait_vm<PA + PW>(min(NS - 2, total - 1 - g));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (g + NS - 1 < total) stage(g + NS - 1, (g + NS - 1) % NS);
        const unsigned char* sb = smem + (g % NS) * C::STAGE;
#pragma unroll
        for (int kq = 0; kq < BK / 16; ++kq) {
            const int c = 2 * kq + fh;
            bf16x8 af[MI], bfr[NI];
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = *(const bf16x8*)(sb + aoff[i] + ((c ^ asw[i]) << 4));
#pragma unroll
            for (int j = 0; j < NI; ++j) bfr[j] = *(const bf16x8*)(sb + woff[j] + ((c ^ wsw[j]) << 4));
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NI; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        const int ti = g / nk;
        if (g - ti * nk != nk - 1) continue;
        // ---- epilogue of tile t (wave-private LDS slice; no block barrier)
        const int t = slot + ti * nb;
        const int tm = t / tiles_n, tn = t - tm * tiles_n;
        const int m0 = tm * C::BM, n0 = tn * C::BN;
        const int c4 = lane & 15, col = n0 + wn * 64 + c4 * 4;
        float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
        if (epi.bias && col < N) bb = *(const float4*)(epi.bias + col);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
#pragma unroll
            for (int h = 0; h < 32 / EPR; ++h) {
                constexpr int EC = EPR / 2;   // accumulator elements per chunk: rows 8(e>>2)+(e&3)+4fh
#pragma unroll
                for (int j = 0; j < NI; ++j)
#pragma unroll
                    for (int e = EC * h; e < EC * h + EC; ++e)
                        ep[((e & 3) + 8 * ((e >> 2) - 2 * EC * h / 8) + 4 * fh) * EP + j * 32 + fr] = acc[i][j][e];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int sidx = 0; sidx < EPR / 4; ++sidx) {
                    const int rr = (lane >> 4) + 4 * sidx;
                    const int row = m0 + wm * C::WTM + i * 32 + EPR * h + rr;
                    if (row >= M || col >= N) continue;
                    float4 v = *(const float4*)(ep + rr * EP + c4 * 4);
                    v.x = v.x * epi.alpha + bb.x; v.y = v.y * epi.alpha + bb.y;
                    v.z = v.z * epi.alpha + bb.z; v.w = v.w * epi.alpha + bb.w;
                    if (epi.relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
                    if (epi.res0) {
                        float4 r0;
                        if (epi.res0_bf16) {
                            const bf16x4 rb = *(const bf16x4*)((const bf16*)epi.res0 + (long long)row * epi.ld_res0 + col);
                            r0 = make_float4(bf2f(rb[0]), bf2f(rb[1]), bf2f(rb[2]), bf2f(rb[3]));
                        } else {
                            r0 = *(const float4*)(epi.res0 + (long long)row * epi.ld_res0 + col);
                        }
                        v.x += r0.x; v.y += r0.y; v.z += r0.z; v.w += r0.w;
                    }
                    if (epi.res1) {
                        const float4 r1 = *(const float4*)(epi.res1 + (long long)row * epi.ld_res1 + col);
                        v.x += r1.x; v.y += r1.y; v.z += r1.z; v.w += r1.w;
                    }
                    const long long ob = epi.out_map.off(row) + col;
                    if (f32o) *(float4*)((float*)epi.out + ob) = v;
                    else {
                        bf16x4 tt = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                        *(bf16x4*)((bf16*)epi.out + ob) = tt;
                    }
                    if (epi.out2) {
                        bf16x4 tt = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                        *(bf16x4*)((bf16*)epi.out2 + epi.out2_map.off(row) + col) = tt;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        // retire the bias load on every path (all rows of a tail tile may be skipped): a load left
        // pending across the back-edge makes the compiler drain the whole DMA ring (vmcnt(0)) before
        // those registers are reused in the next k-step
        asm volatile("" ::"v"(bb.x), "v"(bb.y), "v"(bb.z), "v"(bb.w));
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    }
}

// tile configurations (PFM_GEMM_CFG selects one per launch for A/B runs; 0 = automatic)
using C1 = Cfg<256, 256, 2, 4, 64, 2>;   // 128 KiB LDS, 8 waves, wave 128x64, 1 block/CU
using C2 = Cfg<256, 128, 4, 2, 32, 3>;   // 72 KiB, 8 waves, wave 64x64, 2 blocks/CU
using C3 = Cfg<128, 128, 2, 2, 64, 2>;   // 64 KiB, 4 waves, wave 64x64, 2 blocks/CU
using C4 = Cfg<128, 256, 2, 4, 32, 3>;   // 72 KiB, 8 waves, wave 64x64, 2 blocks/CU
using C5 = Cfg<256, 256, 2, 4, 32, 4>;   // 128 KiB, BK 32 x 4 stages
using C6 = Cfg<256, 256, 2, 4, 32, 4, 1>;   // 128 KiB, BK 32 x 4 stages, ping-pong wave groups
using C7 = Cfg<256, 256, 2, 4, 32, 3>;   // persistent: 96 KiB ring + 34 KiB epilogue slices (16-row chunks)
using C8 = Cfg<256, 256, 2, 4, 32, 4>;   // persistent: 128 KiB ring + 17 KiB slices (8-row chunks)
using C9 = Cfg<256, 256, 2, 4, 64, 2>;   // persistent: 2 x 64 KiB ring + 17 KiB slices
using C10 = Cfg<256, 128, 2, 2, 32, 3>;  // 4 waves (wave 128x64), 72 KiB: 2 blocks/CU -> epilogue/main-loop overlap
using C11 = Cfg<256, 128, 2, 2, 32, 2>;  // 4 waves, 48 KiB
using C12 = Cfg<256, 128, 2, 2, 64, 2>;  // 4 waves, 96 KiB (1 block/CU; control)
using C13 = Cfg<256, 256, 2, 4, 64, 2, 2>;  // 8-phase schedule (K % 128 == 0)
using C14 = Cfg<256, 256, 2, 4, 32, 4, 3>;  // k-step phases, BK 32 x 4 buffers
using C15 = Cfg<256, 256, 2, 4, 64, 2, 0, 1>;  // C1 on v_mfma_f32_16x16x32_bf16
using C16 = Cfg<128, 256, 2, 4, 32, 3, 0, 1>;  // C4 on v_mfma_f32_16x16x32_bf16
using C17 = Cfg<256, 256, 2, 4, 64, 2, 2, 1>;  // 8-phase schedule on v_mfma_f32_16x16x32_bf16 (K % 128 == 0)

template <class C>
hipError_t launch(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K, const GemmEpi& e2,
                  hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<C>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  C::LDS);
    }
    const int tiles_m = (M + C::BM - 1) / C::BM, tiles_n = (N + C::BN - 1) / C::BN;
    // grouped tile order (4 tile-rows per group) for the wide-N projections (memory K|V, vocabulary:
    // +6 % measured), row-major otherwise; PFM_GEMM_GM overrides per launch (A/B)
    const int gm = pfm_knobs().gemm_gm >= 0 ? pfm_knobs().gemm_gm : (tiles_n >= 16 ? 4 : 0);
    hipLaunchKernelGGL((gemm_bf16_kernel<C>), dim3(tiles_m * tiles_n), dim3(C::NT), C::LDS, st, (const bf16*)A, amap,
                       (const bf16*)W, ldw, M, N, K, tiles_m, tiles_n, gm, e2);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

template <class C, int EPR>
hipError_t launch_persist(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                          const GemmEpi& e2, hipStream_t st) {
    constexpr int LDS = C::NS * C::STAGE + C::NW * EPR * C::EP * 4;
    static_assert(LDS <= 160 * 1024, "persistent GEMM LDS budget");
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)(gemm_bf16_persist_kernel<C, EPR>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS);
    }
    const int tiles_m = (M + C::BM - 1) / C::BM, tiles_n = (N + C::BN - 1) / C::BN;
    const int grid = std::min(tiles_m * tiles_n, num_cus());
    hipLaunchKernelGGL((gemm_bf16_persist_kernel<C, EPR>), dim3(grid), dim3(C::NT), LDS, st, (const bf16*)A, amap,
                       (const bf16*)W, ldw, M, N, K, tiles_m, tiles_n, e2);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

int f_gemm_cfg_forced() { const int f = pfm_knobs().gemm_cfg; return f >= 1 && f <= 17 ? f : 0; }

int pick_cfg(int M, int N, int K, bool amax) {
    const int f = pfm_knobs().gemm_cfg;   // PFM_GEMM_CFG (per call): lets one process A/B configurations
    if (f >= 1 && f <= 17) return f;
    // Default (measured on the path, tools/bench_ab.py with the two concurrent encoder groups: 24.2 vs
    // 25.0-25.3 ms/step for the policies below). Grids are counted in 256x256 tiles; each encoder group
    // sees half the batch's rows:
    //  - N <= 512 with K >= 1024 (FFN w2, CIF conv) on the 8-phase 16x16x32 schedule (C17);
    //  - >= one 256x256 tile per CU (QKV, FFN w1, memory K|V) on the one-barrier 16x16x32 kernel (C15);
    //  - everything else (out-projections, decoder-sized M, the fused-argmax vocabulary GEMM) on
    //    128x256 tiles, two blocks per CU (C4).
    // (alternative policies measured slower on the path and removed in round 3: the earlier grid-size
    // policy C15 / C4, C13 for decoder-sized M, C4 for the 512-wide decoder GEMMs, the 8-phase schedules
    // for the >= 256-tile grids; 256x128 tiles for the one-group QKV 22.08 vs 21.68 ms. C3 for the
    // decoder projections: 10.9 vs 13.3 us at M = 7392, K = 512; 26.0 vs 35.5 us at K = 2048)
    const long long big = (long long)((M + 255) / 256) * ((N + 255) / 256);
    if (amax) return big >= 512 ? 15 : 4;
    if (N <= 512 && K % 128 == 0 && K >= 1024 && big >= 120) return 17;
    if (big >= 256) return 15;
    if (N <= 512 && big < 120) return 3;   // decoder-sized M: 128x128 tiles fill more CUs
    return 4;
}

}  // namespace

bool pfm_gemm_bf16_256_ok(RowMap amap, long long ldw, int K) {
    return K % 64 == 0 && ldw % 8 == 0 && amap.ld % 8 == 0 && (amap.rows_per_seg <= 0 || amap.seg_stride % 8 == 0);
}

// argmax partials: one per (row, 64-column block), row stride rounded up to 256 columns
int pfm_gemm_bf16_256_amax_tiles(int N) { return (N + 255) / 256 * 4; }

hipError_t pfm_gemm_bf16_256(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                             const GemmEpi& epi, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (!pfm_gemm_bf16_256_ok(amap, ldw, K)) return hipErrorInvalidValue;
    GemmEpi e2 = epi;
    e2.vec_ok = epi_vec_ok(epi, N);
    {
        const RowMap& om = epi.out_map;
        e2.st16_ok = e2.vec_ok && epi.out && epi.out_dtype == DT_BF16 && !epi.out2 && !epi.amax_val && N % 8 == 0 &&
                     om.ld % 8 == 0 && (om.rows_per_seg <= 0 || om.seg_stride % 8 == 0) &&
                     ((uintptr_t)epi.out % 16) == 0 && pfm_knobs().gemm_st16;
    }
    e2.res_batch = pfm_knobs().gemm_resbatch;   // residual loads batched ahead of the stores
    if (epi.out && epi.out_dtype == DT_X3) {   // split output: the general vector epilogue path only
        if (!e2.vec_ok || epi.amax_val || epi.out2 || epi.out_map.ld % 4) return hipErrorInvalidValue;
        e2.res_batch = 0;
    }
    int cfg = pick_cfg(M, N, K, epi.amax_val != nullptr);
    // EXACT mode's x6 GEMMs (x6_terms 6) stay on ONE MFMA shape whatever the grid: every output element is then
    // the same chain of v_mfma_f32_16x16x32_bf16 over k = 0, 32, 64, ... (C15 / C16 / C17 differ in tile size and
    // schedule, not in any element's accumulation order), so a row's result does not depend on how many rows
    // share the launch — a batch of 1 and a batch of 64 (or one data-parallel shard) decode an utterance
    // identically. The grid only picks the tile: >= 256 256-tiles C15, the 8-phase C17 for N <= 512 / K >= 1024,
    // else the 128 x 256 C16 (the 32x32x16 C3 / C4 it replaces rounded differently).
    if (epi.x6_k && epi.x6_terms != 2 && epi.x6_terms != 3 && f_gemm_cfg_forced() == 0) {
        const long long big = (long long)((M + 255) / 256) * ((N + 255) / 256);
        cfg = (N <= 512 && K % 128 == 0 && K >= 1024 && big >= 120) ? 17 : big >= 256 ? 15 : 16;
    } else if (epi.x6_k && cfg != 1 && cfg != 3 && cfg != 4 && cfg != 13 && cfg != 15 && cfg != 16 && cfg != 17) {
        cfg = 15;
    }
    if (epi.x6_k && (K != (epi.x6_terms == 3 ? 3 : epi.x6_terms == 2 ? 2 : 6) * epi.x6_k || epi.x6_k % 64))
        return hipErrorInvalidValue;
    switch (cfg) {
        case 2: return launch<C2>(A, amap, W, ldw, M, N, K, e2, st);
        case 3: return launch<C3>(A, amap, W, ldw, M, N, K, e2, st);
        case 4: return launch<C4>(A, amap, W, ldw, M, N, K, e2, st);
        case 5: return launch<C5>(A, amap, W, ldw, M, N, K, e2, st);
        case 6: return launch<C6>(A, amap, W, ldw, M, N, K, e2, st);
        case 7: if (!e2.amax_val && e2.vec_ok) return launch_persist<C7, 16>(A, amap, W, ldw, M, N, K, e2, st);
                return launch<C1>(A, amap, W, ldw, M, N, K, e2, st);
        case 8: if (!e2.amax_val && e2.vec_ok) return launch_persist<C8, 8>(A, amap, W, ldw, M, N, K, e2, st);
                return launch<C1>(A, amap, W, ldw, M, N, K, e2, st);
        case 9: if (!e2.amax_val && e2.vec_ok) return launch_persist<C9, 8>(A, amap, W, ldw, M, N, K, e2, st);
                return launch<C1>(A, amap, W, ldw, M, N, K, e2, st);
        case 10: return launch<C10>(A, amap, W, ldw, M, N, K, e2, st);
        case 11: return launch<C11>(A, amap, W, ldw, M, N, K, e2, st);
        case 12: return launch<C12>(A, amap, W, ldw, M, N, K, e2, st);
        case 13: if (K % 128 == 0) return launch<C13>(A, amap, W, ldw, M, N, K, e2, st);
                 return launch<C1>(A, amap, W, ldw, M, N, K, e2, st);
        case 14: return launch<C14>(A, amap, W, ldw, M, N, K, e2, st);
        case 16: return launch<C16>(A, amap, W, ldw, M, N, K, e2, st);
        case 17: if (K % 128 == 0) return launch<C17>(A, amap, W, ldw, M, N, K, e2, st);
                 return launch<C15>(A, amap, W, ldw, M, N, K, e2, st);
        case 1: return launch<C1>(A, amap, W, ldw, M, N, K, e2, st);
        default: return launch<C15>(A, amap, W, ldw, M, N, K, e2, st);
    }
}

