// Fused SAN-M encoder feed-forward sub-layer, 128 rows per workgroup (gfx950, fast mode). The encoder modes of
// k_ffn.hip with the same arithmetic (see there for the reference citations), plus the next layer's QKV:
//   MODE 0  encoder:       x2 = x + W2 relu(W1 LN2(x) + b1) + b2                 (sanm/encoder.py:138-145)
//   MODE 1  encoder + OP:  x1 = O Wo^T + bo + F (+ x), then MODE 0 on x1          (sanm/encoder.py:120-145)
//   MODE 4  MODE 1, then the next layer's q|k|v = LN1_next(x2) Wqkv^T + bq        (sanm/attention.py:275-288)
//   MODE 5  MODE 4 with the v rows of Wqkv as two bf16 planes (w = w0 + w1, fast mode's precise-weight option:
//           PFM_FAST_XW bit 4): the v pass streams 32 more tiles, accumulated into the same registers
//   MODE 6  MODE 5 with Wo as two bf16 planes too (PFM_FAST_XW bit 8): phase 0 streams 32 more tiles
//   MODE 3  MODE 1 with Wo as two bf16 planes (the last layer under PFM_FAST_XW bit 8)
//   MODE 7  decoder FFN (PositionwiseFeedForwardDecoderSANM, sanm/positionwise_feed_forward.py:12-33, in a
//           DecoderLayerSANM, paraformer/decoder.py:95-101): y = W2 LN_F(relu(W1 LN1(x) + b1)), xn = LN_next(y),
//           the 2048-wide hidden SPLIT over two workgroups per 128-row tile (below)
//   MODE 8  MODE 7 with the previous block's cross-attention out-projection in front (decoder.py:113-119):
//           x1 = x + O Wo^T + bo -> Xo (the residual the FSMN step adds back), the FFN on LN1(x1)
// with the next LayerNorm of the result as a bf16 output (the consumer GEMM's operand; MODE 4: the QKV rows).
//
// Decoder split (MODE 7 / 8). A decoder group has ~7.4k rows (B x L): 58 row tiles of 128, too few workgroups for
// the chip when each streams all 4.5 MB of a block's weights. Each tile is owned by TWO workgroups, one per half of
// the hidden (1024 units: 32 chunks of W1 rows / W2 columns, 2048 stream fragments each): both compute the tile's
// LN1 (and phase 0), then each its half of y = W2g h (W2g = W2 diag(gamma_F), LN_F folded through W2 as in
// k_ffn.hip DEC: y = rstd (W2g h - mu c1) + c2) and its half of the LN_F statistics (sum, sum of squares of the bf16
// hidden, by v_dot2c_f32_bf16 on the packed relu output). Both publish their f32 partial (256 KiB, accumulator
// order) and statistics, then one agent-scope acq_rel add on the tile's counter: the workgroup that arrives second
// adds the other's partial (float addition commutes: the result does not depend on the arrival order), applies the
// fold and LN_next, stores xn and resets the counter; the first one exits. No workgroup waits for another, so the
// protocol needs no co-residency. The two halves of a tile take block ids b and b + 8 (one XCD: the partner's
// partial and the shared input rows come from the same L2).
//
// Why a second kernel: k_ffn.hip owns 64 rows per workgroup, so every workgroup streams all 4.5 MB of the
// layer's weights through L2 -> LDS for 64 rows (64 FLOP per weight byte), and its A / H images fill the LDS
// beside the weight ring. Here a workgroup owns 128 rows with 4 waves (one per SIMD, up to 512 VGPRs each) on
// v_mfma_f32_32x32x16_bf16; each wave owns 32 rows and keeps EVERYTHING of them in registers:
//   act[32]  the B operand fragments of its rows (O in phase 0, then LN(x1)): 128 VGPRs
//   acc[16]  the 512-wide f32 output rows Y^T[512 x 32] (x1 + b2 + W2 H): 256 AGPRs
//   acc1     one hidden chunk H^T[32 x 32] of phase 1, converted in registers into phase 2's B operand
// The 32x32 accumulator has the row (lane) as its column and the features in registers, so the next
// product that sums over features takes it with no lane movement (cdna_hip_programming.md §3 "an
// accumulator tile as the next MFMA's operand"); the k order inside each 16-deep step is permuted
// (element j of lane half h <-> feature 16s + 8(j>>2) + 4h + (j&3) of its 32-block) and the weights are
// packed in that order. The LDS holds only the weight ring (8 x 16 KiB tiles, one 1 KiB MFMA fragment per
// 32x16 weight block, read lane-linearly: conflict-free) and the per-column vectors. Weight bytes per row
// halve against k_ffn.hip and no activation ever goes through LDS.
//
// Weight stream (pfm_ffn2_pack*), one 1 KiB fragment per MFMA, in MFMA issue order:
//   [OP: Wo fragments, four output blocks interleaved per k step: (ob 4g, ks) .. (ob 4g+3, ks), then ks+1]
//   head  P1(0): the 32 W1 fragments of hidden chunk 0 (k steps 0..31, one accumulator chain seeded with b1)
//   body c (c = 0..62), 64 fragments: slots 3m, 3m+1 = P1(c+1) k steps 2m, 2m+1, slot 3m+2 = P2(c)
//         output block m, hidden k step 0 (m < 16); slots 48..63 = P2(c) output blocks 0..15, hidden k step 1
//   tail  P2(63): output blocks 0..15 of k step 0, then of k step 1
// so phase 1 of chunk c+1 runs under phase 2 of chunk c (a software pipeline), and relu(H + b1) of chunk c+1 -> bf16
// (phase 2's B operand, double-buffered) is issued between the last 16 MFMAs of the body instead of in a drain
// between the phases. (Phase 1 first in the body — slots 0..31 — with the relu spread over the other 30 gaps: its
// compute was faster without DMA / barriers, 192.5 vs 197.4 us, but the launch 0.7 % slower; not kept.)
// Tile t is published (landed + every wave done with tile t-2) by one barrier placed PD fragments before its
// first read; the DMA of tile t-2+RS into the freed slot is spread over the following 16 MFMAs (one 1 KiB piece
// per wave every 4 fragments), so no wave issues a burst of LDS-DMA beside an idle matrix pipe.
#include <stdint.h>

#include "pfm_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int FD = 512, FF = 2048, BM = 128, NW = 4, HC = 32, NCH = FF / HC;   // 64 hidden chunks
constexpr int FE = 512;                  // bf16 elements per fragment (32 rows x 16 k)
constexpr int TF = 16;                   // fragments per ring tile (16 KiB)
constexpr int RS = 8;                    // ring slots
constexpr int GW = TF / NW;              // LDS-DMA pieces (1 KiB) per wave per tile
constexpr int RING = RS * TF * 1024;     // 128 KiB
constexpr int OPF = 16 * 32;             // phase-0 fragments: Wo = 16 output blocks x 32 k steps
constexpr int CHF = 64;                  // fragments per hidden chunk: 32 W1 k steps + 16 x 2 W2
#ifndef FFN2_PD
#define FFN2_PD 7
#endif
constexpr int PD = FFN2_PD;              // fragment reads in flight ahead of their MFMA
#ifndef FFN2_OPI
#define FFN2_OPI 4
#endif
constexpr int OPI = FFN2_OPI;           // phase-0 output blocks interleaved per k step (1 = back-to-back chains)
constexpr int NB = 8;                    // fragment register slots (divides TF, CHF and OPF; the drains name all 8)
// per-column vectors staged in LDS behind the ring (float offsets)
constexpr int V_G = 0, V_B = 512, V_C2 = 1024, V_GN = 1536, V_BN = 2048, V_BO = 2560, V_B1 = 3072;
constexpr int QKF = 3 * OPF;             // MODE 4 phase 3: the next layer's Wqkv, three passes of 512 output features
constexpr int V_BQ = V_B1 + FF;          // MODE 4: the next layer's q|k|v biases
constexpr int NVEC = V_BQ + 3 * FD;
constexpr int LDS_BYTES = RING + NVEC * 4;   // 157,696 B
static_assert(LDS_BYTES <= 163840, "LDS plan");
static_assert(PD < TF && TF % NB == 0 && CHF % NB == 0 && OPF % NB == 0 && PD < NB, "stream plan");

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Every MFMA of the kernel is an asm statement with an explicit register file, so the allocator cannot trade
// the 16 output blocks (acc[16] = all 256 AGPRs, "a") against phase 1's accumulator (acc1, 16 VGPRs, "v"):
// with the builtin, acc1 claimed an AGPR block and one output block bounced through scratch every chunk.
// hipcc pads no hazards around inline asm (cdna_hip_programming.md §5.7 item 2), so the kernel keeps them:
//   * the first MFMA of a chain takes the inline constant 0 as C; later ones accumulate into the same registers,
//     back to back (XDL D -> the next XDL's whole C: 0 wait states) or with other MFMAs in between (phase 0
//     interleaves four output blocks, phase 1 is one chain of 32 from its C = b1; 1, 2 and 4 interleaved blocks measured
//     bit-identical);
//   * D -> any other reader: 24 wait states (covers the 16-pass XDL distance of 19; xdl_drain(), fenced by
//     sched_barrier, before the transition / epilogue VALU reads the accumulators; mfma_v_drain() before the relu
//     of acc1 — 13 states measured too few: the next-LayerNorm output read stale accumulators);
//   * a VALU-written operand -> MFMA: s_nop 1 (valu_to_mfma(), after the relu writes phase 2's B operand and
//     after the transition writes act).
// A comes from ds_read (ordered by lgkmcnt), B from act / hf.
__device__ __forceinline__ void mfma_a0(f32x16& d, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&a"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_a(f32x16& d, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma32_v0(f32x16& d, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma32_vc(f32x16& d, const bf16x8& a, const bf16x8& b, const f32x16& c) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(d) : "v"(a), "v"(b), "v"(c));
}
__device__ __forceinline__ void mfma32_v(f32x16& d, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_v_drain(f32x16& d) { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(d)); }
// The drain names every output block ("+a"): the compiler's copies of an accumulator into VGPRs (it keeps some
// blocks there for the epilogue) can then only come after the wait states — a nop without operands let the
// allocator place the copy of the last-written block right behind its MFMA, before the nops (stale values).
__device__ __forceinline__ void xdl_drain(f32x16 (&a)[16]) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+a"(a[0]), "+a"(a[1]), "+a"(a[2]), "+a"(a[3]), "+a"(a[4]), "+a"(a[5]), "+a"(a[6]), "+a"(a[7]),
                   "+a"(a[8]), "+a"(a[9]), "+a"(a[10]), "+a"(a[11]), "+a"(a[12]), "+a"(a[13]), "+a"(a[14]),
                   "+a"(a[15])::"memory");
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void valu_to_mfma() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

template <int N> __device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N <= 63, "vm_wait: vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
static_assert((RS - 3) * GW == 20, "vm_wait counts");

// the hidden chunk's biases (4 x 16 B of this lane) by asm ds_reads: hipcc would precede a plain LDS read of
// the staging area with vmcnt(0) (draining the in-flight ring DMA), and a scalar load would turn every counted
// LDS wait of the chunk into lgkmcnt(0). hipcc does not count these reads: b1_wait() orders them (LDS returns
// in order, and at the point of use only the PD younger fragment reads may still be outstanding).
__device__ __forceinline__ void b1_read(f32x4& d, const void* lds) {
    asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"((unsigned)(uintptr_t)lds) : "memory");
}
// the per-column vectors of the VALU phases, by the same asm reads: a plain LDS read makes hipcc wait vmcnt(0)
// first (it cannot tell the vector area from the LDS-DMA ring), which in the epilogue serialised every group of
// output stores behind the next vector read. vec_wait() retires all LDS reads issued so far.
__device__ __forceinline__ f32x4 vec_read(const float* lds) {
    f32x4 d;
    asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"((unsigned)(uintptr_t)lds) : "memory");
    return d;
}

// feature index (within its 32-block) of register reg of a 32x32 accumulator in lane half h
__device__ __forceinline__ int acc_col(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// bf16 outputs of one 32-feature block as two 16-B stores per lane: lane half h holds features 8q + 4h .. +3 of the
// four register groups q; permlane32 swaps hand each half-wave the other half's piece of groups q (h = 0: q even,
// h = 1: q odd), so every lane stores 8 consecutive features of its row (8-B stores were store-issue bound)
__device__ __forceinline__ void store_bf16_block(bf16* row, const bf16x4 (&o)[4], int h) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        uint2 pa, pb;
        __builtin_memcpy(&pa, &o[2 * j], 8);
        __builtin_memcpy(&pb, &o[2 * j + 1], 8);
        const auto rx = __builtin_amdgcn_permlane32_swap(pa.x, pb.x, false, false);
        const auto ry = __builtin_amdgcn_permlane32_swap(pa.y, pb.y, false, false);
        *(uint4*)(row + 16 * j + 8 * h) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
    }
}

// VAR (diagnostic builds of tools/ffn2_bench.hip only; the library instantiates VAR 0): 1 = no weight DMA and no
// DMA waits (stale ring), 2 = no MFMAs, 3 = neither DMA nor barriers (MFMA + fragment reads alone), 5 = the
// prologue / transition / epilogue alone (no stream: zero chunks, no phase-0 MFMAs), 4 = every tile streamed from
// the same L2-hot 64 KiB (wrong math; prices L2 misses of the weight stream), 6 = the DMA of a tile issued as one
// burst at its publishing barrier (the pre-round-4 schedule), 7 = no phase-3 (q|k|v) stores, 8 = no x2 store,
// 9 = the full kernel with phase timestamps (s_memrealtime, 100 MHz) of wave 0 written past row M of Xo
// (16 x u64 per workgroup: the caller provides the room), 10 = no relu VALU (the hidden operand stale: prices the
// activation's VALU inside the stream), 11 = no wait states between phase 1's last MFMAs and the relu (wrong math), 12 = 10 with the stamps of 9
template <int MODE, int VAR = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void ffn2_kernel(
    const float* __restrict__ X, int M, const float* __restrict__ g, const float* __restrict__ be, float eps,
    const bf16* __restrict__ Wp, const float* __restrict__ b1, const float* __restrict__ b2, float* Xo,
    const float* __restrict__ gn, const float* __restrict__ bn, bf16* __restrict__ Xn, const bf16* __restrict__ O,
    const bf16* __restrict__ Fr, const float* __restrict__ bo, const float* __restrict__ c1, float* part,
    unsigned* cnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* vec = (float*)(smem + RING);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    static_assert(MODE == 0 || MODE == 1 || MODE == 3 || (MODE >= 4 && MODE <= 10), "encoder / decoder modes");
    constexpr bool DEC = MODE >= 7;                // decoder FFN (LN_F folded through W2)
    constexpr bool SPLIT = MODE == 7 || MODE == 8; // ... its hidden split over two workgroups per tile
    constexpr bool OP = MODE == 1 || MODE == 3 || (MODE >= 4 && MODE <= 6) || MODE == 8 || MODE == 10;   // Wo in front
    constexpr bool QK = MODE >= 4 && MODE <= 6;    // + the next layer's QKV
    constexpr bool XV = MODE == 5 || MODE == 6;    // + the v rows' second weight plane
    constexpr bool XO = MODE == 3 || MODE == 6;    // + Wo's second weight plane
    constexpr int NCHK = SPLIT ? NCH / 2 : NCH;    // hidden chunks this workgroup streams
    constexpr int F0 = OP ? (XO ? 2 : 1) * OPF : 0, F3 = F0 + NCHK * CHF, NF = F3 + (QK ? QKF + (XV ? OPF : 0) : 0),
                  NT = NF / TF;
    // DEC: tile t's halves are blocks 16 (t >> 3) + (t & 7) and that + 8 (the same XCD)
    const int bid = blockIdx.x;
    const int tile = SPLIT ? ((bid >> 4) << 3) | (bid & 7) : bid, half = SPLIT ? (bid >> 3) & 1 : 0;
    if (SPLIT && (long long)tile * BM >= M) return;   // grid padding (both halves of such a tile leave)
    const long long rg = (long long)tile * BM + 32 * w + r;   // this lane's row
    const bool live = rg < M;
    const long long rc = live ? rg : (long long)M - 1;               // clamped for loads
    unsigned long long tsv[16];                                       // VAR 9: phase timestamps (uniform)
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (VAR == 9 || VAR == 12) {
            __builtin_amdgcn_sched_barrier(0);
            tsv[i] = __builtin_amdgcn_s_memrealtime();
            if (i == 3) tsv[14] = __builtin_amdgcn_s_memtime();   // shader clock across the FFN stream
            if (i == 4) tsv[15] = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_s_waitcnt(0xC07F);                    // lgkmcnt(0): no stamp left in flight
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    stamp(0);

    // ---- per-column vectors -> LDS (before any LDS-DMA is in flight: their waits drain nothing)
    for (int i = tid; i < FD; i += 256) {
        vec[V_G + i] = g[i];
        vec[V_B + i] = be[i];
        vec[V_C2 + i] = b2[i];
        if (Xn) { vec[V_GN + i] = gn[i]; vec[V_BN + i] = bn[i]; }
        if constexpr (OP) vec[V_BO + i] = bo[i];
    }
    for (int i = tid; i < NCHK * HC; i += 256) vec[V_B1 + i] = b1[NCHK * HC * half + i];   // DEC: this half's biases
    if constexpr (QK)
        for (int i = tid; i < 3 * FD; i += 256) vec[V_BQ + i] = c1[i];
    if constexpr (DEC)   // LN_F folded through W2: c1 = rowsum(W2g) (c2 = W2 beta_F arrives as b2)
        for (int i = tid; i < FD; i += 256) vec[V_BQ + i] = c1[i];
    __syncthreads();

    // ---- weight ring: tile t -> slot t % RS; this wave moves fragments GW w .. GW w + GW - 1 of each tile
    // DEC: the layer block holds [Wo | half-0 stream][Wo | half-1 stream] (split) or [Wo | stream]; no out-projection
    // in front (MODE 7 / 9): the Wo slot is skipped
    const bf16* wbase = DEC ? Wp + (long long)half * (OPF + NCHK * CHF) * FE + (OP ? 0 : (long long)OPF * FE) : Wp;
    const bf16* wsrc = wbase + (long long)GW * w * FE + lane * 8;
    // piece p (0..3) of tile t: one 1 KiB LDS-DMA per wave. The four pieces of a wave are 1 KiB apart in both
    // spaces, so they share one address and one M0 and differ only in the instruction's immediate offset.
    static_assert(GW == 4, "LDS-DMA pieces per tile");
    auto piece = [&](int t, int p) {
        if (t >= NT || VAR == 1 || VAR == 3 || VAR == 5) return;
        const bf16* src = wsrc + (long long)(VAR == 4 ? (t & 3) : t) * TF * FE;   // VAR 4: an L2-hot 64 KiB stream
        unsigned char* dst = smem + (t % RS) * (TF * 1024) + GW * w * 1024;
        if (p == 0) __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 0, 0);
        else if (p == 1) __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 1024, 0);
        else if (p == 2) __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 2048, 0);
        else __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 3072, 0);
    };
    auto issue = [&](int t) {
#pragma unroll
        for (int p = 0; p < GW; ++p) piece(t, p);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // publish tile t: it landed (RS-3 newer tiles may stay in flight: every piece of tiles up to t-3+RS was issued
    // before this point). The same barrier retires tile t-2: every wave consumed its last fragment (the MFMA waited
    // for the read) before reaching this barrier, so its slot takes tile t-2+RS at once — no LDS wait at the
    // barrier, the PD fragment reads of tile t stay in flight. Piece 0 goes out here, pieces 1..3 four, eight and
    // twelve fragments later (step_pre), all before the next publishing barrier.
    auto top = [&](int t) {
        if (t >= NT || VAR == 3 || VAR == 5) return;
        if (VAR == 1) {}
        else if (t + RS - 3 < NT) vm_wait<(RS - 3) * GW>();
        else vm_wait<0>();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (VAR == 6) issue(t - 2 + RS);
        else piece(t - 2 + RS, 0);
    };
    // Fragment reads are asm ds_reads with hand-counted waits (the compiler's wait analysis lost count across the
    // asm MFMAs and the loop back edge and drained every read in flight ~10 times per chunk). LDS reads return in
    // order: before MFMA f, the reads of fragments f+1 .. f+PD are the only younger ones, so lgkmcnt(PD) covers
    // fragment f. The wait statement names the destination ("+v"),
    // so no consumer of it is scheduled above the wait.
    bf16x8 wf[NB];
    const unsigned ring_lane = (unsigned)(uintptr_t)smem + lane * 16;
    auto rd = [&](int f, int fs, bf16x8& dst) {   // fs = f mod TF at compile time (the immediate offset)
        const unsigned a = ring_lane + ((f / TF) % RS) * (TF * 1024);
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(a), "i"((fs % TF) * 1024));
    };
    auto frag_wait = [&](bf16x8& d) { asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(d) : "i"(PD)); };
#pragma unroll
    for (int t = 0; t < RS - 2; ++t) issue(t);
    if constexpr (VAR == 6) {
        issue(RS - 2);
    } else {   // pieces 2, 3 of tile RS-2 go out at positions 2 and 6 of tile 0 (step_pre's spread schedule)
        piece(RS - 2, 0);
        piece(RS - 2, 1);
    }

    // ---- prologue: B-operand fragments of this lane's row (phase 0: O rows; else LN(x)) and the accumulator
    bf16x8 act[32];
    f32x16 acc[16];
    // LayerNorm statistics of a 512-wide row split over lanes r, r+32 (256 features each)
    // (two-pass: mean, then the centred sum of squares, like the unfused LayerNorm kernels)
    auto half_mean = [&](float s) { return (s + __shfl_xor(s, 32, 64)) * (1.f / FD); };
    auto half_rstd = [&](float q) { return 1.f / sqrtf((q + __shfl_xor(q, 32, 64)) * (1.f / FD) + eps); };
    // The VALU phases (prologue, transition, epilogue) touch the accumulators one output block at a time: the
    // block is copied to VGPRs, used / updated and written back between scheduling fences, so at most one block
    // (plus a batch of loads) is in VGPRs at once — left to itself the allocator pulled the whole array into
    // VGPRs and spilled it to scratch.
    auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };
    auto acc_get = [&](int ob) {
        f32x16 t = acc[ob];
        asm volatile("" : "+v"(t));
        return t;
    };
    auto acc_put = [&](int ob, f32x16 t) {
        acc[ob] = t;
        asm volatile("" : "+a"(acc[ob]));
    };
    auto acc_stats = [&](float& mean, float& rstd) {
        float s = 0.f;
#pragma unroll
        for (int ob = 0; ob < 16; ++ob) {
            fence();
            const f32x16 t = acc_get(ob);
#pragma unroll
            for (int e = 0; e < 16; ++e) s += t[e];
        }
        fence();
        mean = half_mean(s);
        float q = 0.f;
#pragma unroll
        for (int ob = 0; ob < 16; ++ob) {
            fence();
            const f32x16 t = acc_get(ob);
#pragma unroll
            for (int e = 0; e < 16; ++e) { const float d = t[e] - mean; q += d * d; }
        }
        fence();
        rstd = half_rstd(q);
    };
    // LN of block ob (values t, register e = feature 8(e>>2) + 4h + (e&3) of the block) with the vectors at
    // vg / vb -> the B fragments of k steps 2 ob, 2 ob + 1 (the permuted order the W1 fragments are packed in)
    // four column vectors (vector areas va, vb of block ob: register groups q = 0..3) by asm reads, one wait
    auto vec_block = [&](int va, int vb, int ob, f32x4 (&A)[4], f32x4 (&B)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            A[q] = vec_read(vec + va + 32 * ob + 8 * q + 4 * h);
            B[q] = vec_read(vec + vb + 32 * ob + 8 * q + 4 * h);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(B[0]), "+v"(B[1]),
                     "+v"(B[2]), "+v"(B[3]));
    };
    auto ln_block = [&](int ob, const f32x16& t, float mean, float rstd, int vg = V_G, int vbb = V_B) {
        f32x4 G[4], Bt[4];
        vec_block(vg, vbb, ob, G, Bt);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                act[2 * ob + (q >> 1)][4 * (q & 1) + i] = f2bf((t[4 * q + i] - mean) * rstd * G[q][i] + Bt[q][i]);
    };
    // acc[ob] = (keep ? acc[ob] + vector at V_C2 : 0) for every block (the accumulator start of the FFN)
    auto acc_c2 = [&](int ob, f32x16 t, bool keep) {
        if (keep) {
            f32x4 C[4], Cd[4];
            vec_block(V_C2, V_C2, ob, C, Cd);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i) t[4 * q + i] += C[q][i];
        } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) t[e] = 0.f;
        }
        acc_put(ob, t);
    };
    // acc = ((acc or 0) + bias) + f) + hx * x over the row, in four batches of 4 output blocks whose loads
    // (16 float4 of x, 16 x 8 B of f) are all issued before the first use: one memory round trip per batch (loads
    // interleaved with their uses were serialised, each wait also draining the in-flight weight DMA)
    auto add_rows = [&](bool from_zero, const float* xp, long long xst, float hx, const bf16* fp, int vb) {
        constexpr int NBT = 4, KB = 64 / NBT;
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt) {
            fence();
            float4 xv[KB];
            bf16x4 fv[KB];
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                const int kk = KB * bt + k, col = 32 * (kk / 4) + 8 * (kk % 4) + 4 * h;
                xv[k] = *(const float4*)(xp + rc * xst + col);
                if (fp) fv[k] = *(const bf16x4*)(fp + rc * FD + col);
            }
            fence();
#pragma unroll
            for (int j = 0; j < KB / 4; ++j) {
                const int ob = (KB / 4) * bt + j;
                f32x16 t;
                if (from_zero) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) t[e] = 0.f;
                } else {
                    t = acc_get(ob);
                }
                f32x4 Bv[4], Bd[4];
                if (vb >= 0) {
                    vec_block(vb, vb, ob, Bv, Bd);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) Bv[q] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = 4 * j + q;
                    const float xs[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float fvi = fp ? bf2f(fv[k][i]) : 0.f;
                        t[4 * q + i] = ((t[4 * q + i] + Bv[q][i]) + fvi) + hx * xs[i];
                    }
                }
                acc_put(ob, t);
                fence();
            }
        }
    };
    if constexpr (OP) {
#pragma unroll
        for (int ks = 0; ks < 32; ++ks) act[ks] = *(const bf16x8*)(O + rc * FD + 16 * ks + 8 * h);
    } else {
        // the row into the accumulators (batched loads), its LayerNorm -> act, then the accumulator start
        // (x + b2, the residual the FFN output lands on)
        add_rows(true, X, FD, 1.f, nullptr, -1);
        float mean, rstd;
        acc_stats(mean, rstd);
#pragma unroll
        for (int ob = 0; ob < 16; ++ob) {
            fence();
            const f32x16 t = acc_get(ob);
            ln_block(ob, t, mean, rstd);
            // the decoder FFN output has no residual (and w_2 no bias): its first phase-2 MFMAs start from C = 0
            // instead (zeroed accumulators here made the allocator spill the stream's operands)
            if constexpr (!DEC) acc_c2(ob, t, true);
        }
        fence();
    }

    // ---- tile 0 landed everywhere (the compiler's wait for the activation loads drained the ring DMA too)
    vm_wait<0>();
    bar();
    stamp(1);
#pragma unroll
    for (int f = 0; f < PD; ++f) rd(f, f, wf[f]);

    // one stream step: fragment f (compile-time position fs within the stream's unrolled section, fs = f mod 16):
    // publish the next tile when its first read is due, issue this wave's spread DMA pieces of the tile whose slot
    // that barrier freed, read fragment f+PD, wait for fragment f (then its MFMA)
    // (past the stream's end the read-ahead keeps going: in-bounds reads of stale ring slots nobody consumes,
    // so every step has the same wait)
    // (the publishing position TF - PD must differ from the piece positions 14, 2 and 6)
    static_assert(TF == 16 && PD >= 5 && PD <= 7, "publish / DMA spread positions");
    auto step_pre = [&](int f, int fs) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        const int ps = fs % TF;
        if (ps == TF - PD) top(f / TF + 1);        // position 9: publish tile f/16 + 1 (DMA piece 0 of tile f/16 + 7)
        else if constexpr (VAR != 6) {
            if (ps == 14) piece(f / TF - 1 + RS, 1);
            else if (ps == 2) piece(f / TF - 2 + RS, 2);
            else if (ps == 6) piece(f / TF - 2 + RS, 3);
        }
        rd(f + PD, fs + PD, wf[(fs + PD) % NB]);
        frag_wait(wf[fs % NB]);
        __builtin_amdgcn_sched_barrier(0);
    };

    if constexpr (OP) {   // phase 0: Y0^T += Wo . O^T; fragment f -> output block 4 (f >> 7) + (f & 3), k step (f >> 2) & 31
#pragma unroll
        for (int pp = 0; pp < 16 / OPI; ++pp)
#pragma unroll
            for (int ks = 0; ks < 32; ++ks)
#pragma unroll
                for (int e = 0; e < OPI; ++e) {
                    const int f = 32 * OPI * pp + OPI * ks + e, ob = OPI * pp + e;
                    step_pre(f, f);
                    if (VAR == 2 || VAR == 5) asm volatile("" :: "v"(wf[f % NB]));
                    else if (ks == 0) mfma_a0(acc[ob], wf[f % NB], act[0]);
                    else mfma_a(acc[ob], wf[f % NB], act[ks]);
                }
        if constexpr (XO) {   // Wo's second plane: the same fragment order, into the same accumulators
#pragma unroll
            for (int pp = 0; pp < 16 / OPI; ++pp)
#pragma unroll
                for (int ks = 0; ks < 32; ++ks)
#pragma unroll
                    for (int e = 0; e < OPI; ++e) {
                        const int f = OPF + 32 * OPI * pp + OPI * ks + e, ob = OPI * pp + e;
                        step_pre(f, f);
                        if (VAR == 2 || VAR == 5) asm volatile("" :: "v"(wf[f % NB]));
                        else mfma_a(acc[ob], wf[f % NB], act[ks]);
                    }
        }
        // The read-ahead of the stream's first PD fragments is in flight. An asm ds_read's destination counts as
        // written at the statement, so across the VALU-heavy transition the compiler spilled those registers to
        // scratch before the data landed (garbage operands for the first phase-1 MFMAs on some waves): retire the
        // reads here and issue them again after the transition.
        stamp(2);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wf[0]), "+v"(wf[1]), "+v"(wf[2]), "+v"(wf[3]), "+v"(wf[4]),
                     "+v"(wf[5]), "+v"(wf[6]), "+v"(wf[7]));
        xdl_drain(acc);
        // x1 = ((Y0 + bo) + F) + x (the separate GEMM epilogue's order; layer 0: no x; the decoder: no F)
        add_rows(false, X ? X : bo, X ? FD : 0, X ? 1.f : 0.f, DEC ? nullptr : Fr, V_BO);
        if constexpr (DEC) {   // the decoder keeps x1 (its FSMN step adds the FFN's LN_next output back onto it)
            if (half == 0 && live) {
#pragma unroll
                for (int ob = 0; ob < 16; ++ob) {
                    fence();
                    const f32x16 t = acc_get(ob);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        *(float4*)(Xo + rg * FD + 32 * ob + 8 * q + 4 * h) =
                            make_float4(t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]);
                }
                fence();
            }
        }
        float mean, rstd;
        acc_stats(mean, rstd);
#pragma unroll
        for (int ob = 0; ob < 16; ++ob) {   // LN2(x1) -> act; accumulators: x1 + b2 (decoder: LN1(x1), from zero)
            fence();
            const f32x16 t = acc_get(ob);
            ln_block(ob, t, mean, rstd);
            if constexpr (!DEC) acc_c2(ob, t, true);   // decoder: phase 2 starts from C = 0 (see the prologue)
        }
        fence();
    }
    // the LayerNorm's bf16 operand materialised before the MFMAs (see relu_q: the conversions must not sink into the
    // MFMA stream past valu_to_mfma's wait states)
#pragma unroll
    for (int ks = 0; ks < 32; ++ks) asm volatile("" : "+v"(act[ks]));
    if constexpr (OP) {   // the stream's first PD fragments again (see the end of phase 0)
#pragma unroll
        for (int f = 0; f < PD; ++f) rd(F0 + f, f, wf[f % NB]);
    }
    valu_to_mfma();
    stamp(3);

    // ---- the FFN stream (see the header): head P1(0), bodies c = 0..62 (P1(c+1) under P2(c)), tail P2(63)
    // Phase 1 is one accumulator chain seeded with b1 (the first MFMA takes the chunk's biases as C: back-to-back
    // MFMAs on one accumulator issue at the same rate as on several), so the activation is relu(H) alone: two
    // v_cvt_pk_bf16_f32 and two v_pk_max_i16 per group of 4 features (a bf16 is negative iff its 16-bit pattern is,
    // so the integer max with 0 is the relu, and it commutes with the round-to-nearest). The f32 add + max + convert
    // per feature it replaces cost 12 us of a 215 us launch (VAR 10): the stream's MFMA gaps are full (a ds_read, its
    // counted wait and the MFMA's issue), so every VALU instruction added there costs its issue time.
    f32x16 acc1;                // phase 1 of one chunk (H^T = W1 . act + b1)
    float hs = 0.f, hq = 0.f;   // DEC: sum / sum of squares of this lane's bf16 hidden (LN_F statistics)
    bf16x8 hfa[2], hfb[2];      // phase 2's B operand (hidden k steps 0, 1) of even / odd chunks
    f32x4 bqa[4], bqb[4];       // b1 of even / odd chunks: features 8q + 4h .. +3 (accumulator register groups)
    auto b1_issue = [&](int c, f32x4 (&bq)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < 4; ++q) b1_read(bq[q], vec + V_B1 + HC * c + 8 * q + 4 * h);
    };
    // phase 1, k step j of a chunk (stream fragment f, position fs); k step 0 starts the chain from the biases
    // (read a body earlier: the named wait only tells the compiler they landed — the step's own fragment wait,
    // lgkmcnt(PD), already covered them)
    auto p1 = [&](int f, int fs, int j, f32x4 (&bq)[4]) __attribute__((always_inline)) {
        step_pre(f, fs);
        if (VAR == 2) {
            asm volatile("" :: "v"(wf[fs % NB]));
        } else if (j == 0) {
            asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]) : "i"(PD));
            const f32x8 c01 = __builtin_shufflevector(bq[0], bq[1], 0, 1, 2, 3, 4, 5, 6, 7);
            const f32x8 c23 = __builtin_shufflevector(bq[2], bq[3], 0, 1, 2, 3, 4, 5, 6, 7);
            const f32x16 cb = __builtin_shufflevector(c01, c23, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
            mfma32_vc(acc1, wf[fs % NB], act[0], cb);
        } else {
            mfma32_v(acc1, wf[fs % NB], act[j]);
        }
    };
    // phase 2: output block k & 15, hidden k step k >> 4; first: chunk 0's k step 0 of a decoder launch (C = 0)
    auto p2 = [&](int f, int fs, int k, const bf16x8 (&hb)[2], bool first = false) __attribute__((always_inline)) {
        step_pre(f, fs);
        if (VAR == 2) asm volatile("" :: "v"(wf[fs % NB]), "v"(hb[k >> 4]));
        else if (DEC && first && k < 16) mfma_a0(acc[k & 15], wf[fs % NB], hb[k >> 4]);
        else mfma_a(acc[k & 15], wf[fs % NB], hb[k >> 4]);
    };
    // phase 1's last MFMAs drained (24 wait states before a VALU reads their results)
    auto acc1_ready = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (VAR != 11) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc1));
        __builtin_amdgcn_sched_barrier(0);
    };
    // relu(H) -> bf16 for register group q (4 features) into hb
    auto relu_q = [&](int q, bf16x8 (&hb)[2]) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (VAR != 10 && VAR != 12) {
            const bf16x4 t = {f2bf(acc1[4 * q]), f2bf(acc1[4 * q + 1]), f2bf(acc1[4 * q + 2]), f2bf(acc1[4 * q + 3])};
            uint2 u;
            __builtin_memcpy(&u, &t, 8);
            asm volatile("v_pk_max_i16 %0, %0, 0\n\tv_pk_max_i16 %1, %1, 0" : "+v"(u.x), "+v"(u.y));
            __builtin_memcpy(((char*)&hb[q >> 1]) + 8 * (q & 1), &u, 8);
            if constexpr (DEC) {   // LN_F statistics of the values phase 2 consumes: two packed pairs per group
                bf16x2 p0, p1, one;
                const unsigned uo = 0x3f803f80u;   // (1.0, 1.0)
                __builtin_memcpy(&p0, &u.x, 4);
                __builtin_memcpy(&p1, &u.y, 4);
                __builtin_memcpy(&one, &uo, 4);
                hs = __builtin_amdgcn_fdot2_f32_bf16(p0, one, hs, false);
                hs = __builtin_amdgcn_fdot2_f32_bf16(p1, one, hs, false);
                hq = __builtin_amdgcn_fdot2_f32_bf16(p0, p0, hq, false);
                hq = __builtin_amdgcn_fdot2_f32_bf16(p1, p1, hq, false);
            }
        } else {
            asm volatile("" :: "v"(acc1));
        }
        // pin the packed bf16 here: left alone, instruction selection sinks the v_cvt_pk_bf16_f32 next to the operand's
        // first MFMA, past every scheduling fence, with no wait state between the VALU write and the MFMA read
        asm volatile("" : "+v"(hb[q >> 1]));
        __builtin_amdgcn_sched_barrier(0);
    };
    // body c: slots 3m, 3m+1 = P1(c+1) k steps 2m, 2m+1; slot 3m+2 = P2(c) block m, hidden k step 0; slots 48..63 =
    // P2(c) blocks 0..15, hidden k step 1, with relu(c+1) in four groups behind slots 50, 52, 54, 56; b1 of chunk
    // c+2 is read at the body's start (bqn: the buffer chunk c's biases left)
    auto body = [&](int c, const bf16x8 (&hcur)[2], bf16x8 (&hnext)[2], f32x4 (&bqc)[4], f32x4 (&bqn)[4],
                    bool first = false) __attribute__((always_inline)) {
        const int fb = F0 + 32 + CHF * c;
        if (c + 2 < NCHK) b1_issue(c + 2, bqn);
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            p1(fb + 3 * m, 3 * m, 2 * m, bqc);
            p1(fb + 3 * m + 1, 3 * m + 1, 2 * m + 1, bqc);
            p2(fb + 3 * m + 2, 3 * m + 2, m, hcur, first);
        }
#pragma unroll
        for (int i = 48; i < 64; ++i) {
            p2(fb + i, i, 16 + (i - 48), hcur);
            if (i == 49) acc1_ready();
            if (i >= 50 && i <= 56 && (i & 1) == 0) relu_q((i - 50) >> 1, hnext);
        }
        valu_to_mfma();
    };
    if constexpr (VAR != 5) {
        b1_issue(0, bqa);
        b1_issue(1, bqb);
#pragma unroll
        for (int j = 0; j < 32; ++j) p1(F0 + j, j, j, bqa);   // head: P1(0)
        acc1_ready();
#pragma unroll
        for (int q = 0; q < 4; ++q) relu_q(q, hfa);
        valu_to_mfma();
        int c0 = 0;
        if constexpr (DEC) {   // chunk 0's phase 2 starts the accumulators (C = 0): its body peeled
            body(0, hfa, hfb, bqb, bqa, true);
            body(1, hfb, hfa, bqa, bqb);
            c0 = 2;
        }
        for (int c = c0; c < NCHK - 2; c += 2) {
            body(c, hfa, hfb, bqb, bqa);
            body(c + 1, hfb, hfa, bqa, bqb);
        }
        body(NCHK - 2, hfa, hfb, bqb, bqa);
        const int ft = F0 + 32 + CHF * (NCHK - 1);
#pragma unroll
        for (int k = 0; k < 32; ++k) p2(ft + k, k, k, hfb);   // tail: P2(63)
    }
    stamp(4);
    if constexpr (QK || DEC)   // the stream's read-ahead (phase 3's first fragments): retired before the epilogue
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wf[0]), "+v"(wf[1]), "+v"(wf[2]), "+v"(wf[3]), "+v"(wf[4]),
                     "+v"(wf[5]), "+v"(wf[6]), "+v"(wf[7]));
    xdl_drain(acc);

    // ---- DEC: publish this half's partial y and LN_F statistics; the second workgroup of the tile to arrive
    //      combines both halves (see the header), the first one is done
    if constexpr (DEC) {
        hs += __shfl_xor(hs, 32, 64);   // lanes r and r + 32 hold the two halves of each 32-feature group
        hq += __shfl_xor(hq, 32, 64);
    }
    if constexpr (SPLIT) {
        constexpr long long WPART = 16 * 1024;   // floats of one wave's partial: 16 blocks x 16 registers x 64 lanes
        float* mine = part + ((long long)(2 * tile + half) * NW + w) * WPART;
#pragma unroll
        for (int ob = 0; ob < 16; ++ob) {
            fence();
            const f32x16 t = acc_get(ob);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *(float4*)(mine + ob * 1024 + q * 256 + lane * 4) = make_float4(t[4 * q], t[4 * q + 1], t[4 * q + 2],
                                                                                  t[4 * q + 3]);
        }
        fence();
        float2* stats = (float2*)(part + (long long)2 * gridDim.x / 2 * NW * WPART);   // behind every tile's partials
        if (h == 0) stats[(long long)(2 * tile + half) * BM + 32 * w + r] = make_float2(hs, hq);
        vm_wait<0>();      // every store of this wave completed (visible at the device's coherence point)
        __syncthreads();   // ... of every wave
        unsigned* arrived = (unsigned*)smem;   // the ring is idle: no DMA in flight after the stream
        if (tid == 0)   // release this workgroup's partial; acquire the partner's when it came first
            arrived[0] = __hip_atomic_fetch_add(cnt + tile, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (*(volatile unsigned*)arrived == 0) return;   // first: the partner combines the tile
        if (tid == 0) __hip_atomic_store(cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
        const float* other = part + ((long long)(2 * tile + (half ^ 1)) * NW + w) * WPART;
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {   // the partner's partial in four batches of 4 blocks (16 float4 in flight)
            fence();
            float4 ov[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                ov[k] = *(const float4*)(other + (4 * bt + k / 4) * 1024 + (k % 4) * 256 + lane * 4);
            fence();
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ob = 4 * bt + j;
                f32x16 t = acc_get(ob);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 o4 = ov[4 * j + q];
                    t[4 * q] += o4.x; t[4 * q + 1] += o4.y; t[4 * q + 2] += o4.z; t[4 * q + 3] += o4.w;
                }
                acc_put(ob, t);
                fence();
            }
        }
        const float2 so = stats[(long long)(2 * tile + (half ^ 1)) * BM + 32 * w + r];
        hs += so.x;
        hq += so.y;
    }
    if constexpr (DEC) {
        // y = rstd (W2g h - mu c1) + c2 over the whole hidden (k_ffn.hip DEC's fold; one-pass variance of the bf16 h)
        const float mu = hs * (1.f / FF);
        const float rsf = 1.f / sqrtf(fmaxf(hq * (1.f / FF) - mu * mu, 0.f) + eps);
#pragma unroll
        for (int ob = 0; ob < 16; ++ob) {
            fence();
            f32x16 t = acc_get(ob);
            f32x4 C1[4], C2[4];
            vec_block(V_BQ, V_C2, ob, C1, C2);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i) t[4 * q + i] = rsf * (t[4 * q + i] - mu * C1[q][i]) + C2[q][i];
            if (!OP && Xo && live) {   // MODE 7 / 9 with xo: the FFN output y itself (the op tests; the path passes none)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *(float4*)(Xo + rg * FD + 32 * ob + 8 * q + 4 * h) =
                        make_float4(t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]);
            }
            acc_put(ob, t);
        }
        fence();
    }
    // ---- epilogue (no DMA in flight: the last tiles were waited for by their tops)
    if (!DEC && live && Xo && VAR != 8) {
#pragma unroll
        for (int ob = 0; ob < 16; ++ob) {
            fence();
            const f32x16 t = acc_get(ob);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *(float4*)(Xo + rg * FD + 32 * ob + 8 * q + 4 * h) = make_float4(t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]);
        }
        fence();
    }
    stamp(5);
    if constexpr (QK) {
        // ---- phase 3: the next layer's q|k|v = LN1_next(x2) Wqkv^T + b in three passes of 512 output features,
        //      the LayerNorm output as the B operand in registers (the W1 k order: Wqkv packed by ffn2_pack_qkv);
        //      Xn receives bf16 rows of 1536, c1 holds the biases
        float mean, rstd;
        acc_stats(mean, rstd);
#pragma unroll
        for (int ob = 0; ob < 16; ++ob) {
            fence();
            const f32x16 t = acc_get(ob);
            ln_block(ob, t, mean, rstd, V_GN, V_BN);
        }
        fence();
#pragma unroll
        for (int ks = 0; ks < 32; ++ks) asm volatile("" : "+v"(act[ks]));
#pragma unroll
        for (int f = 0; f < PD; ++f) rd(F3 + f, f, wf[f % NB]);
        valu_to_mfma();
        stamp(6);
        // three passes of 512 output features (the whole accumulator); a pass's epilogue (bias, bf16, 16-B stores)
        // runs between the passes. (Six passes of 256 with the previous pass's stores issued in the MFMA shadow from
        // the other accumulator half spilled the LayerNorm operand to scratch inside the loop: not kept.)
        for (int p = 0; p < 3; ++p) {
            const int fp = F3 + OPF * p;
#pragma unroll
            for (int pp = 0; pp < 4; ++pp)
#pragma unroll
                for (int ks = 0; ks < 32; ++ks)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int fs = 128 * pp + 4 * ks + e, ob = 4 * pp + e;
                        step_pre(fp + fs, fs);
                        if (VAR == 2 || VAR == 5) asm volatile("" :: "v"(wf[fs % NB]));
                        else if (ks == 0) mfma_a0(acc[ob], wf[fs % NB], act[0]);
                        else mfma_a(acc[ob], wf[fs % NB], act[ks]);
                    }
            if constexpr (XV) {   // the v pass: the second plane's fragments, same order, into the same accumulators
                if (p == 2) {
#pragma unroll
                    for (int pp = 0; pp < 4; ++pp)
#pragma unroll
                        for (int ks = 0; ks < 32; ++ks)
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const int fs = OPF + 128 * pp + 4 * ks + e, ob = 4 * pp + e;
                                step_pre(fp + fs, fs);
                                if (VAR == 2 || VAR == 5) asm volatile("" :: "v"(wf[fs % NB]));
                                else mfma_a(acc[ob], wf[fs % NB], act[ks]);
                            }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wf[0]), "+v"(wf[1]), "+v"(wf[2]), "+v"(wf[3]), "+v"(wf[4]),
                         "+v"(wf[5]), "+v"(wf[6]), "+v"(wf[7]));
            xdl_drain(acc);
            if (p == 0) stamp(7);
            else if (p == 1) stamp(9);
            else stamp(11);
            if (live && VAR != 7) {
#pragma unroll
                for (int ob = 0; ob < 16; ++ob) {
                    fence();
                    const f32x16 t = acc_get(ob);
                    f32x4 Bq[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) Bq[q] = vec_read(vec + V_BQ + FD * p + 32 * ob + 8 * q + 4 * h);
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(Bq[0]), "+v"(Bq[1]), "+v"(Bq[2]), "+v"(Bq[3]));
                    bf16x4 o[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q)
#pragma unroll
                        for (int i = 0; i < 4; ++i) o[q][i] = f2bf(t[4 * q + i] + Bq[q][i]);
                    store_bf16_block(Xn + rg * (3 * FD) + FD * p + 32 * ob, o, h);
                }
                fence();
            }
            if (p < 2) {
#pragma unroll
                for (int f = 0; f < PD; ++f) rd(fp + OPF + f, f, wf[f % NB]);
            }
            valu_to_mfma();
            if (p == 0) stamp(8);
            else if (p == 1) stamp(10);
            else stamp(12);
        }
        if constexpr (VAR == 9 || VAR == 12) {   // the stores retired, then the record
            vm_wait<0>();
            stamp(13);
            if (tid < 16) {
                unsigned long long v = tsv[0];
#pragma unroll
                for (int i = 1; i < 16; ++i) v = tid == i ? tsv[i] : v;
                ((unsigned long long*)(Xo + (long long)M * FD))[16 * blockIdx.x + tid] = v;
            }
        }
        return;
    }
    if (Xn) {
        float mean, rstd;
        acc_stats(mean, rstd);
        if (live) {
#pragma unroll
            for (int ob = 0; ob < 16; ++ob) {
                fence();
                const f32x16 t = acc_get(ob);
                f32x4 G[4], Bt[4];
                vec_block(V_GN, V_BN, ob, G, Bt);
                bf16x4 o[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[q][i] = f2bf((t[4 * q + i] - mean) * rstd * G[q][i] + Bt[q][i]);
                store_bf16_block(Xn + rg * FD + 32 * ob, o, h);
            }
            fence();
        }
    }
}

// ---- packing: one thread per 16-B piece (fragment f, lane l = 32 hh + m) in stream order
// within-block feature of element j of lane half hh in k step s (the accumulator's register order)
__device__ __forceinline__ int perm_k(int s, int hh, int j) { return 16 * s + 8 * (j >> 2) + 4 * hh + (j & 3); }

// FFN stream position q (0..4095, see the header) -> hidden chunk c, W1 (P1) or W2 (P2) fragment, index j:
// P1 j = W1 rows [32c, 32c+32) x k step j of the 512 inputs (permuted k); P2 j = W2 rows [32 (j & 15), +32) x hidden
// k step j >> 4 of the chunk's 32 hidden (permuted).
__device__ __forceinline__ void ffn2_stream_frag(int q, int& c, bool& w1, int& j) {
    constexpr int TAIL = 32 + (NCH - 1) * CHF;
    if (q < 32) { c = 0; w1 = true; j = q; return; }
    if (q >= TAIL) { c = NCH - 1; w1 = false; j = q - TAIL; return; }
    const int b = (q - 32) / CHF, i = (q - 32) % CHF;
    if (i < 48) {
        const int m = i / 3, rr = i % 3;
        if (rr < 2) { c = b + 1; w1 = true; j = 2 * m + rr; }
        else { c = b; w1 = false; j = m; }
    } else {
        c = b; w1 = false; j = 16 + (i - 48);
    }
}

__global__ __launch_bounds__(256) void ffn2_pack_kernel(const bf16* __restrict__ W1, const bf16* __restrict__ W2,
                                                        bf16* __restrict__ Wp) {
    const int gid = blockIdx.x * 256 + threadIdx.x;   // < NCH * CHF * 64
    const int f = gid >> 6, l = gid & 63, m = l & 31, hh = l >> 5;
    int c, j;
    bool w1;
    ffn2_stream_frag(f, c, w1, j);
    bf16x8 o;
    if (w1) {
        const int kb = j >> 1, s = j & 1;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = W1[(long long)(HC * c + m) * FD + 32 * kb + perm_k(s, hh, e)];
    } else {
        const int ob = j & 15, s = j >> 4;
        const long long rowb = (long long)(32 * ob + m) * FF + HC * c;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = W2[rowb + perm_k(s, hh, e)];
    }
    *(bf16x8*)(Wp + (long long)gid * 8) = o;
}

// Wo [512 out][512 in] -> phase-0 fragments f = 128 p + 4 ks + e: output block 4p + e, k step ks (natural k: the O rows
// are loaded in natural order)
__global__ __launch_bounds__(256) void ffn2_pack_o_kernel(const bf16* __restrict__ Wo, bf16* __restrict__ Wp) {
    const int gid = blockIdx.x * 256 + threadIdx.x;   // < OPF * 64
    const int f = gid >> 6, l = gid & 63, m = l & 31, hh = l >> 5;
    const int ob = OPI * (f / (32 * OPI)) + f % OPI, ks = (f / OPI) % 32;
    *(bf16x8*)(Wp + (long long)gid * 8) = *(const bf16x8*)(Wo + (long long)(32 * ob + m) * FD + 16 * ks + 8 * hh);
}

// the next layer's Wqkv [1536 out][512 in] -> phase-3 fragments: three passes of 512 output features (rows 512 p ..),
// fragment f of a pass = output block 4 (f >> 7) + (f & 3), k step (f >> 2) & 31, with W1's permuted k (the B operand
// is the LayerNorm output in act)
__global__ __launch_bounds__(256) void ffn2_pack_qkv_kernel(const bf16* __restrict__ Wq, bf16* __restrict__ Wp, int p0) {
    const int gid = blockIdx.x * 256 + threadIdx.x;   // < (3 - p0) * OPF * 64
    const int fq = gid >> 6, l = gid & 63, m = l & 31, hh = l >> 5;
    const int p = p0 + fq / OPF, f = fq % OPF;
    const int ob = 4 * (f >> 7) + (f & 3), ks = (f >> 2) & 31;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e)
        o[e] = Wq[(long long)(FD * p + 32 * ob + m) * FD + 32 * (ks >> 1) + perm_k(ks & 1, hh, e)];
    *(bf16x8*)(Wp + (long long)gid * 8) = o;
}

// decoder half stream h (MODE 7 / 8): fragment q of the 32-chunk stream of hidden chunks 32 h .. 32 h + 31, W1 rows of
// the chunk (permuted k, as ffn2_pack_kernel) and W2g = bf16(W2 diag(gamma_F)) columns of the chunk (the value
// k_ffn.hip's DEC pack and ffn_dec_consts_kernel use, so c1 = rowsum of exactly these bf16 values)
__global__ __launch_bounds__(256) void ffn2_pack_dec_kernel(const bf16* __restrict__ W1, const float* __restrict__ W2,
                                                            const float* __restrict__ gF, bf16* __restrict__ Wp, int hh0,
                                                            int NCHH) {
    const int TAIL = 32 + (NCHH - 1) * CHF;
    const int gid = blockIdx.x * 256 + threadIdx.x;   // < NCHH * CHF * 64
    const int q = gid >> 6, l = gid & 63, m = l & 31, hh = l >> 5;
    int c, j;
    bool w1;
    if (q < 32) { c = 0; w1 = true; j = q; }
    else if (q >= TAIL) { c = NCHH - 1; w1 = false; j = q - TAIL; }
    else {
        const int b = (q - 32) / CHF, i = (q - 32) % CHF;
        if (i < 48) {
            const int mm = i / 3, rr = i % 3;
            if (rr < 2) { c = b + 1; w1 = true; j = 2 * mm + rr; }
            else { c = b; w1 = false; j = mm; }
        } else {
            c = b; w1 = false; j = 16 + (i - 48);
        }
    }
    const int cg = NCHH * hh0 + c;   // global hidden chunk
    bf16x8 o;
    if (w1) {
        const int kb = j >> 1, s = j & 1;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = W1[(long long)(HC * cg + m) * FD + 32 * kb + perm_k(s, hh, e)];
    } else {
        const int ob = j & 15, s = j >> 4;
        const long long rowb = (long long)(32 * ob + m) * FF;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = HC * cg + perm_k(s, hh, e);
            o[e] = f2bf(W2[rowb + k] * gF[k]);
        }
    }
    *(bf16x8*)(Wp + (long long)gid * 8) = o;
}

template <int MODE>
hipError_t ffn2_launch(hipStream_t st, int M, const float* x, const float* g, const float* be, float eps, const bf16* Wp,
                       const float* b1, const float* b2, float* xo, const float* gn, const float* bn, bf16* xn,
                       const bf16* o, const bf16* f, const float* bo, const float* c1, float* part = nullptr,
                       unsigned* cnt = nullptr) {
    static bool attr_done = false;   // one flag per instantiation
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)ffn2_kernel<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    }
    const int tiles = (M + BM - 1) / BM;
    const int grid = (MODE == 7 || MODE == 8) ? 16 * ((tiles + 7) / 8) : tiles;   // split: two halves per tile, 8 apart
    hipLaunchKernelGGL(ffn2_kernel<MODE>, dim3(grid), dim3(64 * NW), LDS_BYTES, st, x, M, g, be, eps, Wp, b1, b2, xo, gn,
                       bn, xn, o, f, bo, c1, part, cnt);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

// packed sizes equal k_ffn.hip's (pfm_ffn_packed_elems / pfm_ffn_packed_o_elems): the buffers are shared
static_assert((size_t)NCH * CHF * FE == (size_t)2048 * 1024, "FFN pack size");
static_assert((size_t)OPF * FE == (size_t)512 * 512, "Wo pack size");

hipError_t pfm_ffn2_pack(const bf16* W1, const bf16* W2, bf16* Wp, hipStream_t st) {
    hipLaunchKernelGGL(ffn2_pack_kernel, dim3(NCH * CHF * 64 / 256), dim3(256), 0, st, W1, W2, Wp);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// the next layer's Wqkv [1536][512] -> QKF fragments behind the layer's FFN tiles (ffn2_kernel MODE 4)
hipError_t pfm_ffn2_pack_qkv(const bf16* Wqkv, bf16* Wp, hipStream_t st) {
    hipLaunchKernelGGL(ffn2_pack_qkv_kernel, dim3(QKF * 64 / 256), dim3(256), 0, st, Wqkv, Wp, 0);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// MODE 5: the v rows' second plane (rows 1024..1535 of a [1536][512] plane) -> OPF more fragments behind the QKV ones
hipError_t pfm_ffn2_pack_qkv_v(const bf16* Wqkv_lo, bf16* Wp, hipStream_t st) {
    hipLaunchKernelGGL(ffn2_pack_qkv_kernel, dim3(OPF * 64 / 256), dim3(256), 0, st, Wqkv_lo, Wp, 2);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_ffn2_pack_o(const bf16* Wo, bf16* Wp, hipStream_t st) {
    hipLaunchKernelGGL(ffn2_pack_o_kernel, dim3(OPF * 64 / 256), dim3(256), 0, st, Wo, Wp);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// Same contracts as pfm_ffn_fused / pfm_ffn_fused_op (k_ffn.hip), pfm_ffn2_pack* weights.
hipError_t pfm_ffn2_fused(const float* x, int M, const float* g2, const float* be2, float eps, const bf16* Wp,
                          const float* b1, const float* b2, float* xo, const float* gn, const float* bn, bf16* xn,
                          hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if ((xn != nullptr) != (gn != nullptr && bn != nullptr) || !x || !b1 || !b2 || !g2 || !be2) return hipErrorInvalidValue;
    if (!al16(x) || !al16(xo) || !al16(Wp) || !al16(xn) || !al16(b1) || !al16(b2)) return hipErrorInvalidValue;
    return ffn2_launch<0>(st, M, x, g2, be2, eps, Wp, b1, b2, xo, gn, bn, xn, nullptr, nullptr, nullptr, nullptr);
}

hipError_t pfm_ffn2_fused_op(const bf16* o, const bf16* f, const float* bo, const float* x, int M, const float* g2,
                             const float* be2, float eps, const bf16* Wop, const float* b1, const float* b2, float* xo,
                             const float* gn, const float* bn, bf16* xn, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if ((xn != nullptr) != (gn != nullptr && bn != nullptr) || !o || !f || !bo || !xo || !b1 || !b2)
        return hipErrorInvalidValue;
    if (!al16(x) || !al16(xo) || !al16(Wop) || !al16(xn) || !al16(o) || !al16(f) || !al16(bo)) return hipErrorInvalidValue;
    return ffn2_launch<1>(st, M, x, g2, be2, eps, Wop, b1, b2, xo, gn, bn, xn, o, f, bo, nullptr);
}

// MODE 4: pfm_ffn2_fused_op plus the next layer's q|k|v projection: x2 -> xo (f32), qkv = LN1_next(x2) Wqkv^T + bq
// (bf16 [M, 1536]); Wop: the Wo fragments, the FFN stream and pfm_ffn2_pack_qkv's fragments, contiguous.
hipError_t pfm_ffn2_fused_op_qkv(const bf16* o, const bf16* f, const float* bo, const float* x, int M, const float* g2,
                                 const float* be2, float eps, const bf16* Wop, const float* b1, const float* b2, float* xo,
                                 const float* gn, const float* bn, const float* bq, bf16* qkv, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (!o || !f || !bo || !xo || !b1 || !b2 || !gn || !bn || !bq || !qkv) return hipErrorInvalidValue;
    if (!al16(x) || !al16(xo) || !al16(Wop) || !al16(qkv) || !al16(o) || !al16(f) || !al16(bo) || !al16(bq))
        return hipErrorInvalidValue;
    return ffn2_launch<4>(st, M, x, g2, be2, eps, Wop, b1, b2, xo, gn, bn, qkv, o, f, bo, bq);
}

// MODE 5: MODE 4 with Wop's QKV fragments followed by pfm_ffn2_pack_qkv_v's (the v rows' second weight plane);
// xo_planes: MODE 6, Wop starts with Wo's two planes (pfm_ffn2_pack_o of each, back to back)
hipError_t pfm_ffn2_fused_op_qkv_xv(const bf16* o, const bf16* f, const float* bo, const float* x, int M,
                                    const float* g2, const float* be2, float eps, const bf16* Wop, const float* b1,
                                    const float* b2, float* xo, const float* gn, const float* bn, const float* bq,
                                    bf16* qkv, bool xo_planes, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (!o || !f || !bo || !xo || !b1 || !b2 || !gn || !bn || !bq || !qkv) return hipErrorInvalidValue;
    if (!al16(x) || !al16(xo) || !al16(Wop) || !al16(qkv) || !al16(o) || !al16(f) || !al16(bo) || !al16(bq))
        return hipErrorInvalidValue;
    if (xo_planes) return ffn2_launch<6>(st, M, x, g2, be2, eps, Wop, b1, b2, xo, gn, bn, qkv, o, f, bo, bq);
    return ffn2_launch<5>(st, M, x, g2, be2, eps, Wop, b1, b2, xo, gn, bn, qkv, o, f, bo, bq);
}

// ---- decoder FFN, hidden split over two workgroups per 128-row tile (ffn2_kernel MODE 7 / 8)
// Packed block of one decoder FFN: [Wo fragments | half-0 stream][Wo fragments | half-1 stream] (the Wo slots hold the
// previous block's out-projection, packed twice; MODE 7 leaves them unused).
// (split = false: one [Wo | full stream] block of the same size, for the unsplit 128-row MODE 9 / 10)
size_t pfm_ffn2_dec_packed_elems() { return (size_t)2 * (OPF + NCH / 2 * CHF) * FE; }

hipError_t pfm_ffn2_pack_dec(const bf16* W1, const float* W2, const float* gF, const bf16* Wo, bf16* Wp, hipStream_t st,
                             bool split) {
    const int nh = split ? 2 : 1, nchh = NCH / nh;
    const size_t hs = (size_t)(OPF + nchh * CHF) * FE;
    for (int hh = 0; hh < nh; ++hh) {
        if (Wo) {
            hipLaunchKernelGGL(ffn2_pack_o_kernel, dim3(OPF * 64 / 256), dim3(256), 0, st, Wo, Wp + hh * hs);
            PFM_LAUNCH_CHECK();
        }
        hipLaunchKernelGGL(ffn2_pack_dec_kernel, dim3(nchh * CHF * 64 / 256), dim3(256), 0, st, W1, W2, gF,
                           Wp + hh * hs + (size_t)OPF * FE, hh, nchh);
        PFM_LAUNCH_CHECK();
    }
    return hipSuccess;
}

// scratch of one launch over M rows: the partials (two halves x 128 rows x 512 f32 per tile slot of the grid) and the
// LN_F statistics behind them; counters: one per tile slot, zero before the first launch (every launch leaves them 0)
size_t pfm_ffn2_dec_scratch_floats(int M) {
    const size_t slots = (size_t)8 * (((M + BM - 1) / BM + 7) / 8);
    return slots * 2 * NW * 16 * 1024 + slots * 2 * BM * 2;
}
size_t pfm_ffn2_dec_counters(int M) { return (size_t)8 * (((M + BM - 1) / BM + 7) / 8); }

// x f32 [M, 512] -> xn = LN_next(W2 LN_F(relu(W1 LN1(x1) + b1))) bf16 [M, 512]; with o (bf16 [M, 512]) and bo: x1 = x +
// o Wo^T + bo, written to xo (f32, may alias x); else x1 = x and xo (optional) receives y. Wp: pfm_ffn2_pack_dec; c1 / c2: the LN_F fold constants
// (pfm_ffn_pack_dec); part / cnt: pfm_ffn2_dec_scratch_floats(M) floats / pfm_ffn2_dec_counters(M) zeroed counters,
// private to this launch's stream (the split MODE 7 / 8; both null: the unsplit MODE 9 / 10 on a split = false pack).
hipError_t pfm_ffn2_fused_dec(const float* x, int M, const float* g1, const float* be1, float eps, const bf16* Wp,
                              const float* b1, const float* c1, const float* c2, float* xo, const float* gn,
                              const float* bn, bf16* xn, const bf16* o, const float* bo, float* part, unsigned* cnt,
                              hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (!x || !xn || !gn || !bn || !c1 || !c2 || !b1 || (o && (!bo || !xo))) return hipErrorInvalidValue;
    if (!part || !cnt) {   // unsplit: one workgroup per 128-row tile streams the whole hidden (MODE 9 / 10)
        if (!al16(x) || !al16(xo) || !al16(Wp) || !al16(xn) || !al16(o) || !al16(bo)) return hipErrorInvalidValue;
        if (o) return ffn2_launch<10>(st, M, x, g1, be1, eps, Wp, b1, c2, xo, gn, bn, xn, o, nullptr, bo, c1);
        return ffn2_launch<9>(st, M, x, g1, be1, eps, Wp, b1, c2, xo, gn, bn, xn, nullptr, nullptr, nullptr, c1);
    }
    if (!al16(x) || !al16(xo) || !al16(Wp) || !al16(xn) || !al16(o) || !al16(bo) || !al16(part)) return hipErrorInvalidValue;
    if (o) return ffn2_launch<8>(st, M, x, g1, be1, eps, Wp, b1, c2, xo, gn, bn, xn, o, nullptr, bo, c1, part, cnt);
    return ffn2_launch<7>(st, M, x, g1, be1, eps, Wp, b1, c2, xo, gn, bn, xn, nullptr, nullptr, nullptr, c1, part, cnt);
}

// MODE 3: pfm_ffn2_fused_op with Wop = Wo's two planes, then the FFN fragments (the last layer under bit 8)
hipError_t pfm_ffn2_fused_op_xo(const bf16* o, const bf16* f, const float* bo, const float* x, int M, const float* g2,
                                const float* be2, float eps, const bf16* Wop, const float* b1, const float* b2,
                                float* xo, const float* gn, const float* bn, bf16* xn, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if ((xn != nullptr) != (gn != nullptr && bn != nullptr) || !o || !f || !bo || !xo || !b1 || !b2)
        return hipErrorInvalidValue;
    if (!al16(x) || !al16(xo) || !al16(Wop) || !al16(xn) || !al16(o) || !al16(f) || !al16(bo)) return hipErrorInvalidValue;
    return ffn2_launch<3>(st, M, x, g2, be2, eps, Wop, b1, b2, xo, gn, bn, xn, o, f, bo, nullptr);
}
