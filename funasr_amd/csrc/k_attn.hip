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
#include "pfm_common.h"

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

template <typename T> struct AttnLds;

__global__ __launch_bounds__(256) void attn_f32_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
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
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float mnew = fmaxf(mrun, mt);
        const float corr = expf(mrun - mnew);
        float ls = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            s[e] = expf(s[e] - mnew);
            ls += s[e];
        }
        ls += __shfl_xor(ls, 32, 64);
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
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int col = d * 32 + kappa(e) + 4 * fh;
            const float v = o[d][e] * inv;
            if (op) op[col] = v;
            if (op2) op2[col] = f2bf(v);
        }
}

__global__ __launch_bounds__(256) void attn_bf16_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 31, fh = lane >> 5;
    const int klen = min(a.klen[b], a.Tk);
    const bf16* Q = (const bf16*)a.q;
    const bf16* K = (const bf16*)a.k;
    const bf16* V = (const bf16*)a.v;

    const int qrow = qt * 128 + wid * QW + fr;
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
            for (int j = 0; j < 8; ++j) x[j] = f2bf(bf2f(x[j]) * a.scale);
            qf[kq] = x;
        }
    }
    f32x16 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[d][e] = 0.f;
    float mrun = -INFINITY, lrun = 0.f;
    const int ntiles = (klen + KT - 1) / KT;
    // K tile: 32 rows x 256 B = 512 chunks; V tile 32 keys x 256 B = 512 chunks -> 2+2 per thread
    auto stage = [&](int t, int s) {
        unsigned char* Ks = smem + s * (KT * KP16 + DK * VTP16);
        unsigned char* Vt = Ks + KT * KP16;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = tid + 256 * i, row = c >> 4, ch = c & 15;
            const int key = t * KT + row;
            uint4 kx = make_uint4(0, 0, 0, 0), vx = make_uint4(0, 0, 0, 0);
            if (key < klen) {
                const long long m = (long long)b * a.Tk + key;
                kx = *(const uint4*)(K + a.kmap.off(m) + h * DK + ch * 8);
                vx = *(const uint4*)(V + a.vmap.off(m) + h * DK + ch * 8);
            }
            *(uint4*)(Ks + row * KP16 + ch * 16) = kx;
            const unsigned short* vs = (const unsigned short*)&vx;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                *(unsigned short*)(Vt + (ch * 8 + j) * VTP16 + row * 2) = vs[j];
        }
    };
    if (ntiles > 0) stage(0, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (t + 1 < ntiles) stage(t + 1, cur ^ 1);
        const unsigned char* Ks = smem + cur * (KT * KP16 + DK * VTP16);
        const unsigned char* Vt = Ks + KT * KP16;
        f32x16 s;
#pragma unroll
        for (int e = 0; e < 16; ++e) s[e] = 0.f;
#pragma unroll
        for (int kq = 0; kq < 8; ++kq) {
            const bf16x8 kx = *(const bf16x8*)(Ks + fr * KP16 + kq * 32 + fh * 16);
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kx, qf[kq], s, 0, 0, 0);
        }
        float mt = -INFINITY;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int key = t * KT + kappa(e) + 4 * fh;
            if (key >= klen) s[e] = -INFINITY;
            mt = fmaxf(mt, s[e]);
        }
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float mnew = fmaxf(mrun, mt);
        const float corr = __expf(mrun - mnew);
        float ls = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            s[e] = __expf(s[e] - mnew);
            ls += s[e];
        }
        ls += __shfl_xor(ls, 32, 64);
        lrun = lrun * corr + ls;
        mrun = mnew;
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[d][e] *= corr;
        // P^T as B operand: k-step st uses registers 8st..8st+7; element j of half fh is key
        // 16st + 8(j>>2) + 4fh + (j&3). V^T operand element j must be that same key.
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            bf16x8 pb;
#pragma unroll
            for (int j = 0; j < 8; ++j) pb[j] = f2bf(s[8 * st + j]);
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const unsigned char* vr = Vt + (d * 32 + fr) * VTP16;
                const uint2 lo = *(const uint2*)(vr + (16 * st + 4 * fh) * 2);
                const uint2 hi = *(const uint2*)(vr + (16 * st + 8 + 4 * fh) * 2);
                uint4 vv = make_uint4(lo.x, lo.y, hi.x, hi.y);
                bf16x8 va;
                __builtin_memcpy(&va, &vv, 16);
                o[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb, o[d], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    if (qrow >= a.Tq) return;
    const float inv = (klen > 0) ? 1.f / lrun : 0.f;
    float* op = a.o ? a.o + ((long long)b * a.Tq + qrow) * a.ldo + h * DK : nullptr;
    bf16* op2 = a.o2 ? (bf16*)a.o2 + ((long long)b * a.Tq + qrow) * a.ldo + h * DK : nullptr;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int col = d * 32 + kappa(e) + 4 * fh;
            const float v = o[d][e] * inv;
            if (op) op[col] = v;
            if (op2) op2[col] = f2bf(v);
        }
}

}  // namespace

// q/k/v: head-concatenated rows (head h at column h*128). o: f32 [B*Tq, ldo] (may be null in
// bf16 mode when only o2 is wanted). heads*128 columns per row.
hipError_t pfm_attention(int dtype, const void* q, RowMap qmap, const void* k, RowMap kmap, const void* v,
                         RowMap vmap, float* o, long long ldo, void* o2, const int* klen, int B, int Tq,
                         int Tk, int heads, int dk, float scale, hipStream_t st) {
    if (dk != DK) return hipErrorInvalidValue;
    if (B <= 0 || Tq <= 0) return hipSuccess;
    AttnArgs a;
    a.q = q; a.qmap = qmap; a.k = k; a.kmap = kmap; a.v = v; a.vmap = vmap;
    a.o = o; a.ldo = ldo; a.o2 = o2; a.o2_dtype = DT_BF16; a.klen = klen; a.Tq = Tq; a.Tk = Tk; a.scale = scale;
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)attn_f32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS32);
        (void)hipFuncSetAttribute((const void*)attn_bf16_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS16);
    }
    dim3 grid((Tq + 127) / 128, heads, B), block(256);
    if (dtype == DT_F32) hipLaunchKernelGGL(attn_f32_kernel, grid, block, LDS32, st, a);
    else hipLaunchKernelGGL(attn_bf16_kernel, grid, block, LDS16, st, a);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

int pfm_attention_lds_bytes(int dtype) { return dtype == DT_F32 ? LDS32 : LDS16; }
