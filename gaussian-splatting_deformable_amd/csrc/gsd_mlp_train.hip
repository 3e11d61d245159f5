// gsd_mlp_train.hip -- the deformation network's TRAINING path (DirectTemporalNeRF, scene/gaussian_model.py:242-316,
// positional encoding :33-82) at float32 accuracy on the bf16 matrix cores.
//
// The reference trains the network in float32 with autograd (torch GEMMs).  gfx950 has no TF32/xf32 and its f32
// MFMA runs at the f32 vector rate (157 TF), 1/16 of bf16.  Every f32 operand here is split into three bf16 terms,
// a = hi + mid + lo (hi = bf16(a), mid = bf16(a - hi), lo = bf16(a - hi - mid): 24 bits of mantissa, the f32 value
// to 2^-25), and a product a.b is formed from the six leading partial products hi.hi + hi.mid + mid.hi + hi.lo +
// mid.mid + lo.hi (the three dropped ones are below 2^-24 of |a b|, under f32's own rounding), each exact in the f32
// accumulator of v_mfma_f32_32x32x16_bf16: "BF16x6".  Six bf16 MFMAs cost 6/16 of the f32 MFMA time for the same
// product, so the f32-accurate GEMMs run on a 2.67x higher roof (419 TF).
//
// Layout.  Activations live FEATURE-MAJOR in HBM, [feature][ldp] (ldp = P rounded up to 256): the forward writes
// every layer's post-ReLU output h_l (the backward's ReLU masks and weight-gradient operands), the backward writes
// the pre-activation gradients g_l.  The MFMA operand maps then need no transposes:
//   k_mlp_gemm_dma   Y^T = A . X^T for a tile of 256 Gaussians (8 waves x 32): A = the layer's weights W (forward)
//                or W^T (backward), pre-split and packed fragment-major by k_mlp_pack; both A and the activation rows
//                copied global -> LDS by LDS-DMA three k-steps ahead; lane (h, c) reads features 16 ks + 8 h + j of
//                Gaussian c and splits them in registers.  Epilogues: bias + ReLU -> h_l (forward), bias -> the
//                heads' (P, 58) outputs, or the ReLU mask of h_l -> g_l and the encoding's gradient rows (backward).
//   k_mlp_wgrad  dW = g . X^T over the Gaussians: both operands feature-major, so lane (h, c) reads 8 consecutive
//                Gaussians of one feature row (32 B); split-K over Gaussian chunks into per-wave partials, plus the
//                bias gradient's row sums of g; k_mlp_wgrad_reduce sums the partials in a fixed order.
//   k_mlp_encode / k_mlp_encode_bwd   enc(x), enc(t) feature-major; dL/dx from dL/d enc(x) through the stored
//                sin / cos (d sin(2^i x) = 2^i cos(2^i x) dx: no trig in the backward).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "gsd_kernels.h"

// GSD_ABLATE (timing experiments only, never a product build): bit 1 drops the GEMM epilogue's global stores, 2 its
// MFMAs, 4 the fused forward's activation stores, 8 its MFMAs, 16 the weight-gradient MFMAs, 64 the fused forward's
// weight copies, 128 the GEMM's copies, 256 the fused forward's per-k-step wait + barrier, 512 five of its six
// copies per k-step, 2048 the fused forward's weight copies through registers
// (a load one k-step ahead, then a ds_write; results exact).  The results are then garbage; the durations say what each part costs.
#ifndef GSD_ABLATE
#define GSD_ABLATE 0
#endif

namespace gsd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---- the three-term split ----
struct Split8 {
    bf16x8 hi, mid, lo;
};
__device__ __forceinline__ Split8 split8(const float (&v)[8]) {
    Split8 s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 h = (__bf16)v[j];
        const float r1 = v[j] - (float)h;   // exact: v and h share their leading bits
        const __bf16 m = (__bf16)r1;
        const float r2 = r1 - (float)m;     // exact
        s.hi[j] = h;
        s.mid[j] = m;
        s.lo[j] = (__bf16)r2;
    }
    return s;
}

// acc += A . B to f32 accuracy from the splits (the six leading products, smallest first)
__device__ __forceinline__ f32x16 mfma_x6(const Split8& a, const Split8& b, f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.lo, b.hi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.mid, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.lo, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.hi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.mid, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.hi, acc, 0, 0, 0);
    return acc;
}
template <int ABL>
__device__ __forceinline__ f32x16 mfma_x6_abl(const Split8& a, const Split8& b, f32x16 acc) {
    if constexpr (ABL != 0) {
        acc[0] += (float)a.hi[0] * (float)b.hi[0] + (float)a.lo[1] * (float)b.lo[1];
        return acc;
    } else {
        return mfma_x6(a, b, acc);
    }
}

// ---- weights: the reference's pieces, the padded input layout ----
__device__ __forceinline__ int mlp_col(int map, int k) {
    if (map == 1) return k < 63 ? k : (k == 63 ? -1 : (k < 85 ? k - 1 : -1));
    if (map == 2) return k < 63 ? k : (k == 63 ? -1 : k - 1);
    return k;
}
// pointer to element (row, col) of the piece holding `row`, or null past the rows
__device__ __forceinline__ float* mlp_elem(const MlpWeightRef& w, int row, int col) {
    if (row < 0 || col < 0 || row >= w.row_off[w.n_pieces]) return nullptr;
    int i = 0;
#pragma unroll
    for (int q = 1; q < 4; ++q) i += (q < w.n_pieces && row >= w.row_off[q]) ? 1 : 0;
    return w.W[i] + (size_t)(row - w.row_off[i]) * w.ldw + col;
}

// ---- weight packing: A[m][k] of a layer (W or W^T, zero-padded, input columns mapped) into split fragments ----
// out[((ks * RB + rb) * 3 + s) * 64 + lane] = split s of A[32 rb + (lane & 31)][16 ks + 8 (lane >> 5) + 0..7]
__device__ __forceinline__ void mlp_pack_one(const MlpPackParams& p, int t);
__global__ __launch_bounds__(256) void k_mlp_pack(MlpPackParams p) { mlp_pack_one(p, blockIdx.x * 256 + threadIdx.x); }
// several packs in one launch (grid.y = the job): one launch per direction instead of nine or ten ~6-us ones
__global__ __launch_bounds__(256) void k_mlp_pack_multi(MlpPackBatch b) {
    if ((int)blockIdx.y < b.n) mlp_pack_one(b.job[blockIdx.y], blockIdx.x * 256 + threadIdx.x);
}
__device__ __forceinline__ void mlp_pack_one(const MlpPackParams& p, int t) {
    const int RW = p.m16 ? 16 : 32, KW = p.m16 ? 32 : 16;   // fragment rows and k-step depth
    const int RB = p.M / RW, KS = p.K / KW;
    if (t >= KS * RB * 64) return;
    const int lane = t & 63, rb = (t >> 6) % RB, ks = (t >> 6) / RB;
    const int m = RW * rb + (lane & (RW - 1));
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        int k;
        if (p.m16) {
            const int q = lane >> 4;
            k = 32 * ks + (ks >= p.perm_from ? 16 * (j >> 2) + 4 * q + (j & 3) : 8 * q + j);
        } else {
            const int h = lane >> 5;
            k = 16 * ks + (ks >= p.perm_from ? 8 * (j >> 2) + 4 * h + (j & 3) : 8 * h + j);
        }
        // forward: A = W, rows m = output features, columns k = (padded) input features; backward: A = W^T
        const float* e = p.transpose ? mlp_elem(p.w, k, mlp_col(p.w.map, m + p.m_off))
                                     : mlp_elem(p.w, m, mlp_col(p.w.map, k));
        v[j] = e ? *e : 0.f;
    }
    const Split8 s = split8(v);
    bf16x8* o = reinterpret_cast<bf16x8*>(p.out) + (size_t)((ks * RB + rb) * 3) * 64 + lane;
    o[0] = s.hi;
    o[64] = s.mid;
    o[128] = s.lo;
}

// the heads' four biases (or any pieces) gathered into one padded vector
__global__ void k_mlp_gather_bias(MlpWeightRef b, float* __restrict__ dst, int n_pad) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= n_pad) return;
    const float* e = mlp_elem(b, n, 0);
    dst[n] = e ? *e : 0.f;
}

// The heads' incoming gradients -> [dst_rows][ldp] feature-major (rows past 58 zero).  A workgroup takes 64
// Gaussians: each head's 64 rows are one contiguous run, read coalesced into LDS, then written per feature.
__global__ __launch_bounds__(256) void k_mlp_rows_to_features(int P, int ldp, MlpHeadsIn src, float* __restrict__ dst,
                                                              int dst_rows) {
    __shared__ float tile[64][65];
    const int g0 = blockIdx.x * 64;
    const int ng = min(64, P - g0);   // Gaussians of this block (<= 0 past P)
    for (int i = threadIdx.x; i < 64 * 64; i += 256) tile[i / 64][i % 64] = 0.f;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float* sp = src.src[k];
        const int w = kMlpHeadCol[k + 1] - kMlpHeadCol[k], ld = src.ld[k];
        if (!sp || ng <= 0) continue;
        for (int i = threadIdx.x; i < ng * w; i += 256) {
            const int gg = i / w, col = i - gg * w;
            tile[gg][kMlpHeadCol[k] + col] = sp[(size_t)(g0 + gg) * ld + col];
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * dst_rows; i += 256) {
        const int r = i / 64, gg = i % 64;
        dst[(size_t)r * ldp + g0 + gg] = r < 64 ? tile[gg][r] : 0.f;
    }
}

// ---- the positional encoding (gaussian_model.py:33-82), feature-major ----
// E rows: 0-2 x, then per frequency i the sin of the 3 coordinates and their cos (3 + 6 i + 3 s + d), 63 = 0;
// ET rows: 0 t, 1 + 2 i sin(2^i t), 2 + 2 i cos(2^i t), 21-31 = 0.
__global__ __launch_bounds__(256) void k_mlp_encode(int P, int ldp, const float* __restrict__ x,
                                                    const float* __restrict__ t, float* __restrict__ E,
                                                    float* __restrict__ ET) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= ldp) return;
    const bool in = g < P;
    const float v[3] = {in ? x[3 * g] : 0.f, in ? x[3 * g + 1] : 0.f, in ? x[3 * g + 2] : 0.f};
    const float tv = in ? t[g] : 0.f;
#pragma unroll
    for (int d = 0; d < 3; ++d) E[(size_t)d * ldp + g] = v[d];
#pragma unroll 1
    for (int i = 0; i < 10; ++i) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float a = ldexpf(v[d], i);   // x * 2^i, exact as torch's x * freqs
            E[(size_t)(3 + 6 * i + d) * ldp + g] = sinf(a);
            E[(size_t)(6 + 6 * i + d) * ldp + g] = cosf(a);
        }
        const float a = ldexpf(tv, i);
        ET[(size_t)(1 + 2 * i) * ldp + g] = sinf(a);
        ET[(size_t)(2 + 2 * i) * ldp + g] = cosf(a);
    }
    E[(size_t)63 * ldp + g] = 0.f;
    ET[g] = tv;
#pragma unroll 1
    for (int r = 21; r < 32; ++r) ET[(size_t)r * ldp + g] = 0.f;
}

// dL/dx = dL/dE[identity rows] + sum_i 2^i (dL/dsin_i cos_i - dL/dcos_i sin_i), the sin / cos read back from E
__global__ __launch_bounds__(256) void k_mlp_encode_bwd(int P, int ldp, const float* __restrict__ E,
                                                        const float* __restrict__ dE, float* __restrict__ dx,
                                                        int accumulate) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= P) return;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        float s = dE[(size_t)d * ldp + g];
#pragma unroll 1
        for (int i = 0; i < 10; ++i) {
            const size_t rs = (size_t)(3 + 6 * i + d) * ldp + g, rc = (size_t)(6 + 6 * i + d) * ldp + g;
            s += ldexpf(dE[rs] * E[rc] - dE[rc] * E[rs], i);
        }
        dx[3 * g + d] = accumulate ? dx[3 * g + d] + s : s;
    }
}

// The GEMM epilogue: accumulator register q of row block r holds row
// n = 32 (rb0 + r) + 8 (q >> 2) + 4 h + (q & 3) of Gaussian g = g0 + c.  The hidden-row epilogues (forward ReLU,
// backward mask) go out through LDS: the wave writes its 32 x 32 block transposed into st and stores each row's 32
// Gaussians as 16-B pieces -- four 1-KB store instructions per block instead of sixteen 256-B ones (the one-dword
// stores were store-issue bound: 30 % of the forward GEMM's time, 44 % of the backward's).
template <int MODE, int RB>
__device__ __forceinline__ void gemm_epilogue(const MlpGemmParams& p, const f32x16 (&acc)[RB],
                                              const unsigned (&bits_in)[RB], float (*st)[36], int rb0, int g0,
                                              int lane) {
    const int h = lane >> 5, c = lane & 31, g = g0 + c;
    const int srow = lane >> 3, scol = 4 * (lane & 7);   // the transposed read: rows srow + 8 i, columns scol..+3
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int nb = 32 * (rb0 + r);   // the block's first row
        if (MODE == kMlpFwdHeads) {      // the four heads' outputs per Gaussian: 58 floats, written as is
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 b4 = *reinterpret_cast<const float4*>(p.bias + nb + 8 * j + 4 * h);
                const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int n = nb + 8 * j + 4 * h + i;
                    if (n < 58 && g < p.P) mlp_store_head(p.heads, g, n, acc[r][4 * j + i] + bq[i]);
                }
            }
            continue;
        }
        float v[16];
        if (MODE == kMlpFwdRelu) {
            unsigned bits_out = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 b4 = *reinterpret_cast<const float4*>(p.bias + nb + 8 * j + 4 * h);
                const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float y = relu_nan(acc[r][4 * j + i] + bq[i]);
                    v[4 * j + i] = y;
                    bits_out |= (!(y <= 0.f) ? 1u : 0u) << (4 * j + i);
                }
            }
            if (p.mask_out) p.mask_out[(size_t)((rb0 + r) * 2 + h) * p.ldp + g] = (unsigned short)bits_out;
        } else {   // backward: rows < n_a -> the encoding's gradient (no ReLU), the rest masked by h
            const bool enc_rows = nb < p.n_a;   // n_a is a multiple of 32: per block
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const float a = acc[r][q];
                if (enc_rows) {
                    v[q] = a;
                } else if (p.mask_in) {
                    v[q] = (bits_in[r] >> q) & 1u ? a : 0.f;   // threshold_backward
                } else if (p.mask) {
                    const int n = nb + 8 * (q >> 2) + 4 * h + (q & 3);
                    v[q] = p.mask[(size_t)(n - p.n_a) * p.ldp + g] > 0.f ? a : 0.f;   // threshold_backward(g, h, 0)
                } else {
                    v[q] = 0.f;
                }
            }
            if (!enc_rows && !p.mask_in && !p.mask) continue;   // no mask: those rows are dropped
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) st[8 * (q >> 2) + 4 * h + (q & 3)][c] = v[q];
        wave_lds_handoff();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = srow + 8 * i, n = nb + row;
            const float4 y = *reinterpret_cast<const float4*>(&st[row][scol]);
            float* d;
            bool acc_old = false;
            if (MODE == kMlpBwdMask && nb < p.n_a) {
                d = p.dst_a + (size_t)n * p.ldp + g0 + scol;
                acc_old = p.accumulate_a != 0;
            } else {
                d = p.dst + (size_t)(MODE == kMlpBwdMask ? n - p.n_a : n) * p.ldp + g0 + scol;
            }
            float4 o = y;
            if (acc_old) {
                const float4 old = *reinterpret_cast<const float4*>(d);
                o = make_float4(old.x + y.x, old.y + y.y, old.z + y.z, old.w + y.w);
            }
            if constexpr (!(GSD_ABLATE & 1)) *reinterpret_cast<float4*>(d) = o;
            else if (o.x == 1234.5f) *reinterpret_cast<float4*>(d) = o;
        }
        wave_lds_handoff();   // the next block's writes stay behind these reads
    }
}

// ---- Y^T = A X^T for a tile of 256 Gaussians and all of the launch's output rows ----
// A = the layer's W (forward) or W^T (backward), pre-split into three bf16 planes by k_mlp_pack (fragment-major);
// X^T = the feature-major activations, split in registers; 6 MFMAs (32x32x16 bf16) per row block and k-step.
// Eight waves (two per SIMD) own 256 Gaussians and all of the launch's row blocks.  Every k-step, the workgroup
// copies the operands of k-step ks + 3 global -> LDS with global_load_lds_dwordx4 (no VGPR round trip): the
// A fragments (RB x 3 chunks of 1 KB, fragment-major as k_mlp_pack wrote them) and the 16 activation rows of its
// 256 Gaussians (1 KB each).  Each wave issues the same number of copies per stage (chunks past RB x 3 re-copy chunk
// 0 into padding), so one counted `s_waitcnt vmcnt(per-stage copies)` before the k-step's raw s_barrier retires the
// stage the next k-step reads while the two newest stay in flight: the copies cross the barrier instead of draining at
// every k-step.  All LDS is one array (a
// second __shared__ object made hipcc wait for every copy before each LDS read, cdna_hip_programming.md §5).
template <int RB>
struct GemmDmaLds {
    static constexpr int kChunks = RB * 3;             // 1-KB fragment chunks of A per k-step
    static constexpr int kAPer = (kChunks + 7) / 8;    // copies per wave per k-step for A
    static constexpr int kASlot = kAPer * 8 * 1024;
    static constexpr int kXSlot = 16 * 1024;           // 16 feature rows x 256 Gaussians x 4 B
    static constexpr int kSlots = 4;                   // k-step ks reads slot ks % 4 while ks + 1 .. ks + 3 are staged
    static constexpr int kX0 = kSlots * kASlot;
    static constexpr int kBytes = kX0 + kSlots * kXSlot;   // <= 160 KB (>= 36 KB: the epilogue's scratch aliases it)
    static constexpr int kPerStage = kAPer + 2;        // copies per wave per k-step (A, then two activation rows)
};

template <int N>
__device__ __forceinline__ void wait_vm() {   // s_waitcnt vmcnt(N): two stages of copies stay in flight
    static_assert(N == 6 || N == 8 || N == 10, "copies per two stages");
    if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
}

__device__ __forceinline__ void raw_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// one 16-B-per-lane global -> LDS copy (1 KB per wave-instruction at lds + 16 lane).  A non-template function: with
// the builtin written inside the kernel template, the host pass silently dropped the kernel's launch stubs.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ void dma16(const void* src, unsigned char* lds) {
    __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)lds, 16, 0, 0);
}

// Stage k-step KS_IN (clamped: past the end a harmless re-copy, so every stage issues the same count) into ring
// slot SLOT.  (A macro: as a lambda or a helper template inside the kernel template, the host pass silently failed to
// instantiate the kernel's launch stub.)
#define GSD_GEMM_DMA_ISSUE(KS_IN, SLOT)                                                                         \
    do {                                                                                                        \
        const int ks_ = min((KS_IN), KS - 1), slot_ = (SLOT);                                                   \
        _Pragma("unroll") for (int i_ = 0; i_ < L::kAPer; ++i_) {                                               \
            const int ch_ = wave + 8 * i_;                                                                      \
            dma16(F + (size_t)ks_ * kstride + (size_t)(ch_ < L::kChunks ? ch_ : 0) * 64 + lane,                 \
                  s_mem + slot_ * L::kASlot + ch_ * 1024);                                                       \
        }                                                                                                       \
        const float* xs_ = ks_ < p.ks0 ? p.src0 + (size_t)(16 * ks_) * p.ldp                                    \
                                       : p.src1 + (size_t)(16 * (ks_ - p.ks0)) * p.ldp;                         \
        _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                                      \
            const int r_ = 2 * wave + i_;                                                                       \
            dma16(xs_ + (size_t)r_ * p.ldp + blockIdx.x * 256 + 4 * lane,                                      \
                  s_mem + L::kX0 + slot_ * L::kXSlot + r_ * 1024);                                               \
        }                                                                                                       \
    } while (0)

template <int MODE, int RB>
__global__ __launch_bounds__(512) void k_mlp_gemm_dma(MlpGemmParams p) {
    using L = GemmDmaLds<RB>;
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[L::kBytes];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31, wave = tid >> 6;
    const int gw = blockIdx.x * 256 + wave * 32;      // the wave's first Gaussian (< ldp)
    const int KS = p.ks0 + p.ks1;
    const int rb0 = blockIdx.y * RB;
    const size_t kstride = (size_t)p.rb * 3 * 64;     // 16-B fragments per k-step of the packed A
    const bf16x8* F = reinterpret_cast<const bf16x8*>(p.frags) + (size_t)rb0 * 3 * 64;
    f32x16 acc[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r] = f32x16{};
    unsigned bits_in[RB];   // backward: the forward's ReLU words, loaded ahead (used after the loop)
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        bits_in[r] = 0xffffu;
        if (MODE == kMlpBwdMask && p.mask_in) {
            const int rm = rb0 + r - p.n_a / 32;
            if (rm >= 0) bits_in[r] = p.mask_in[(size_t)(rm * 2 + h) * p.ldp + gw + c];
        }
    }
    GSD_GEMM_DMA_ISSUE(0, 0);
    GSD_GEMM_DMA_ISSUE(1, 1);
    GSD_GEMM_DMA_ISSUE(2, 2);
    wait_vm<2 * L::kPerStage>();   // k-step 0 landed (this wave's copies) ...
    raw_barrier();                 // ... and every wave's
    for (int ks = 0; ks < KS; ++ks) {
        const int slot = ks & 3;
        // k-step ks + 3 into the slot k-step ks - 1 read (every wave is past it)
        if constexpr (!(GSD_ABLATE & 128)) GSD_GEMM_DMA_ISSUE(ks + 3, (ks + 3) & 3);
        const float* xrow = reinterpret_cast<const float*>(s_mem + L::kX0 + slot * L::kXSlot) + wave * 32 + c;
        float xv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] = xrow[(8 * h + j) * 256];
        const Split8 b = split8(xv);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + slot * L::kASlot);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            Split8 a;
            a.hi = sa[(r * 3) * 64 + lane];
            a.mid = sa[(r * 3 + 1) * 64 + lane];
            a.lo = sa[(r * 3 + 2) * 64 + lane];
            acc[r] = mfma_x6_abl<GSD_ABLATE & 2>(a, b, acc[r]);
        }
        wait_vm<2 * L::kPerStage>();   // k-step ks + 1 landed; ks + 2 and ks + 3 stay in flight across the barrier
        raw_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's re-copies, before the scratch reuses the rings
    raw_barrier();
    float(*st)[36] = reinterpret_cast<float(*)[36]>(s_mem) + wave * 32;
    gemm_epilogue<MODE, RB>(p, acc, bits_in, st, rb0, gw, lane);
}

#undef GSD_GEMM_DMA_ISSUE

// ---- the training forward fused across the layers ----
// One workgroup of four waves (one per SIMD, ~400 registers each) takes 128 Gaussians through all nine layers.  A
// wave keeps its 32 Gaussians' activations in registers: layer l's accumulators (32 rows x 32 Gaussians per row
// block, column on the lane) become, after bias and ReLU, layer l + 1's B operand with no lane movement -- k-step
// 2 rb + s is accumulator registers 8 s .. 8 s + 7 of row block rb, which is why the weights of the layers fed this
// way are packed with the accumulator-order k permutation (MlpPackParams::perm_from).  Only the weights move: the
// split fragments of one k-step (24 KB) are copied global -> LDS by LDS-DMA into a four-slot ring three k-steps
// ahead and shared by the four waves (a wave reading them from L2 itself, as the bf16 k_mlp_fwd does, would need
// ~4x the L2 bandwidth); the ring runs straight through the eight hidden layers (122 k-steps), the heads get their
// own.  Every hidden output still goes to HBM (the backward's operands and ReLU words), but no layer re-reads its
// input: 1 GB per layer at P = 1M instead of 2.
constexpr int kFusedStep = 8 * 3 * 64;   // bf16x8 per hidden k-step: 8 row blocks x 3 splits x 64 lanes (24 KB)

// s_waitcnt vmcnt(N) with a compile-time N: the copies and stores younger than the stage being retired
template <int N>
__device__ __forceinline__ void wait_vm_c() {
    static_assert(N >= 0 && N < 64, "vmcnt is six bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// dma16 as inline asm (M0 written and restored in the same statement): the compiler does not see this copy, so it
// neither drains it before unrelated LDS reads nor counts it -- every wait on it is the caller's s_waitcnt vmcnt.
// lds: the wave-uniform LDS byte address.
__device__ __forceinline__ void dma16_asm(const void* src, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(lds_ptr_t)(const_cast<void*>(p));
}

// the same with N known only after unrolling (a loop counter): constant-folds to one case
__device__ __forceinline__ void wait_vm_u(int n) {
    switch (n) {
#define GSD_VM_CASE(N) \
    case N: wait_vm_c<N>(); break;
#define GSD_VM_CASE8(N) GSD_VM_CASE(N) GSD_VM_CASE(N + 1) GSD_VM_CASE(N + 2) GSD_VM_CASE(N + 3) GSD_VM_CASE(N + 4) \
    GSD_VM_CASE(N + 5) GSD_VM_CASE(N + 6) GSD_VM_CASE(N + 7)
        GSD_VM_CASE8(0) GSD_VM_CASE8(8) GSD_VM_CASE8(16) GSD_VM_CASE8(24) GSD_VM_CASE8(32) GSD_VM_CASE8(40)
#undef GSD_VM_CASE8
#undef GSD_VM_CASE
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (unreachable: every count used is < 48)
    }
}

// global stores a k-step of a fused layer issues (the layer before's output rows and ReLU words, see below): all of
// them, and those issued after the k-step's last weight copy (row blocks 5-7 and the ReLU word)
constexpr int kActStores = 8;   // 4-B row stores per activation k-step (a 16-B form via a quad transpose was 1.5 % slower)
__device__ __forceinline__ constexpr int fused_stores(int kse, int ks, int prev) {
    return ks < 0 ? prev : (ks < kse ? 0 : kActStores + (ks - kse < 8 ? 1 : 0));
}
__device__ __forceinline__ constexpr int fused_stores_late(int kse, int ks, int prev) {
    return ks < 0 ? (prev ? 3 : 0) : (ks < kse ? 0 : 3 + (ks - kse < 8 ? 1 : 0));
}

// elements 2 jp, 2 jp + 1 of split8 (one dword of each plane)
__device__ __forceinline__ void split_pair(const float (&v)[8], int jp, Split8& s) {
#pragma unroll
    for (int j = 2 * jp; j < 2 * jp + 2; ++j) {
        const __bf16 h = (__bf16)v[j];
        const float r1 = v[j] - (float)h;
        const __bf16 m = (__bf16)r1;
        s.hi[j] = h;
        s.mid[j] = m;
        s.lo[j] = (__bf16)(r1 - (float)m);
    }
}

// MFMA m (0-5, smallest product first) of mfma_x6
template <int M>
__device__ __forceinline__ f32x16 mfma_x6_part(const Split8& a, const Split8& b, f32x16 acc) {
    if constexpr (GSD_ABLATE & 8) {
        acc[M] += (float)a.hi[M] * (float)b.hi[M];
        return acc;
    }
    if constexpr (M == 0) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.lo, b.hi, acc, 0, 0, 0);
    if constexpr (M == 1) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.mid, acc, 0, 0, 0);
    if constexpr (M == 2) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.lo, acc, 0, 0, 0);
    if constexpr (M == 3) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.hi, acc, 0, 0, 0);
    if constexpr (M == 4) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.mid, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.hi, acc, 0, 0, 0);
}

// One hidden layer's k-steps -- KSE from the encoding registers (xe: enc(x) k-steps 0-3, then xt: enc(t) k-steps
// 4-5), then KSA from the activation registers -- fully unrolled so that every register-array index is a constant.
// s: the global k-step of the layer's first (its ring slot is s & 3).  A k-step is 48 MFMAs (8 row blocks x 6), and
// everything else it does is placed one piece per MFMA gap (sched_barriers fix the order), where its issue hides
// under the MFMA's 32 cycles instead of adding to them:
//  - the next row block's three fragments, read from LDS at the row block's start;
//  - the copy of k-step s + ks + 3 (of this layer, or of the next one's first three) into the slot k-step
//    s + ks - 1 read: 24 chunks of 1 KB, six per wave (shared by the four waves), one per row block 0-5 (gap 1);
//  - one of the eight rows of the PREVIOUS layer's output this k-step consumes (act[ks - KSE]) to HBM per row block
//    (gap 3), and on the first eight k-steps that row block's ReLU word (row block 7, gap 5): the output stores ride
//    under the MFMAs instead of stalling an epilogue, and act is live anyway;
//  - the three-term split of the NEXT k-step's B operand, a pair of elements per gap (row blocks 1-4, gap 5);
// then s_waitcnt vmcnt(the stores and copies issued after k-step s + ks + 1's last copy) and a raw barrier.
// PREV: the stores of each of the layer before's last two k-steps (0 after layer 0).
// ST = false (the evaluation without autograd, k_mlp_fwd_fused<false>): no output stores at all, and the waits count
// the copies only.
template <int KSE, int KSA, int PREV, bool ST = true>
__device__ __forceinline__ void fused_hidden_layer(const MlpFusedParams& p, unsigned char* s_mem, int s, int l,
                                                   int wave, int lane, unsigned voff_h, unsigned voff_b,
                                                   const float (&xe)[4][8], const float (&xt)[2][8],
                                                   const float (&act)[16][8], const unsigned (&bits)[8],
                                                   f32x16 (&acc)[8], bf16x8 (&R)[6]) {
    constexpr int KS = KSE + KSA;
    const bf16x8* fc = reinterpret_cast<const bf16x8*>(p.frags[l]) + lane;
    // past the last hidden layer: its own last k-step again (a harmless re-copy keeps the per-step count uniform)
    const bf16x8* fn = l < 7 ? reinterpret_cast<const bf16x8*>(p.frags[l + 1]) + lane : fc + (KS - 1) * kFusedStep;
    const int ldp = p.ldp;
    float* Hp = KSA ? p.H[l - 1] : nullptr;
    unsigned short* Bp = KSA ? p.bits[l - 1] : nullptr;
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = f32x16{};
    // the B operand of k-step ks (a constant index after unrolling)
    auto operand = [&](int ks) -> const float(&)[8] {
        if (ks < KSE) return ks < 4 ? xe[ks < 4 ? ks : 0] : xt[ks >= 4 && ks < 6 ? ks - 4 : 0];
        return act[ks >= KSE ? ks - KSE : 0];
    };
    Split8 b = split8(operand(0));
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int kk = ks + 3;
        const bf16x8* f = kk < KS ? fc + kk * kFusedStep : (l < 7 ? fn + (kk - KS) * kFusedStep : fn);
        const unsigned dst = lds_addr(s_mem) + ((s + kk) & 3) * (24 * 1024);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + ((s + ks) & 3) * (24 * 1024));
        const int k2 = ks >= KSE ? ks - KSE : 0;   // act[k2][r]: row 16 k2 + 8 (r >> 2) + 4 h + (r & 3)
        const bool stores = ST && ks >= KSE && !(GSD_ABLATE & 4);
        Split8 bn = b;
        Split8 a;
        a.hi = sa[lane];
        a.mid = sa[64 + lane];
        a.lo = sa[128 + lane];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            Split8 an = a;
            if (r + 1 < 8) {
                an.hi = sa[((r + 1) * 3) * 64 + lane];
                an.mid = sa[((r + 1) * 3 + 1) * 64 + lane];
                an.lo = sa[((r + 1) * 3 + 2) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<0>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<1>(a, b, acc[r]);
            if (r < ((GSD_ABLATE & 512) ? 1 : 6) && !(GSD_ABLATE & 64)) {
                const int ch = wave + 4 * r;
                if constexpr (GSD_ABLATE & 2048) {
                    // k-step ks + 2's chunk (loaded one k-step ago) to LDS, then k-step ks + 3's into the register
                    *reinterpret_cast<bf16x8*>(s_mem + ((s + ks + 2) & 3) * (24 * 1024) + ch * 1024 + 16 * lane) = R[r];
                    R[r] = f[ch * 64];
                } else {
                    dma16_asm(f + ch * 64, __builtin_amdgcn_readfirstlane(dst + ch * 1024));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<2>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<3>(a, b, acc[r]);
            // nontemporal: the 8 GB of hidden outputs stream past L2 instead of evicting the weights every
            // workgroup re-reads from it (2 % faster than plain stores)
            if (stores)
                __builtin_nontemporal_store(act[k2][r], Hp + (size_t)(16 * k2 + 8 * (r >> 2) + (r & 3)) * ldp + voff_h);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<4>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<5>(a, b, acc[r]);
            if (r >= 1 && r <= 4 && ks + 1 < KS) split_pair(operand(ks + 1 < KS ? ks + 1 : 0), r - 1, bn);
            if (r == 7 && stores && k2 < 8)
                __builtin_nontemporal_store((unsigned short)bits[k2 < 8 ? k2 : 0], Bp + (size_t)(2 * k2) * ldp + voff_b);
            __builtin_amdgcn_sched_barrier(0);
            a = an;
        }
        b = bn;
        if constexpr (GSD_ABLATE & 2048) {
            raw_barrier();   // the ds_writes (lgkmcnt) before it; the loads and stores stay in flight
        } else if constexpr (!(GSD_ABLATE & 256)) {
            wait_vm_u((ST ? fused_stores_late(KSE, ks - 2, PREV) + fused_stores(KSE, ks - 1, PREV) +
                                fused_stores(KSE, ks, PREV) : 0) + 12);
            raw_barrier();
        }
    }
}

// bias (from LDS) + ReLU into the next layer's B operand (k-step 2 rb + s8 = registers 8 s8 .. 8 s8 + 7) and the
// ReLU words; no global access (their stores ride in the next layer's k-steps)
__device__ __forceinline__ void fused_hidden_epilogue(const float* s_bias, int h, const f32x16 (&acc)[8],
                                                      float (&act)[16][8], unsigned (&bits)[8]) {
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
        unsigned w = 0;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
            const float4 b4 = *reinterpret_cast<const float4*>(s_bias + 32 * rb + 8 * q4 + 4 * h);
            const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = 4 * q4 + i;
                const float y = relu_nan(acc[rb][q] + bq[i]);
                act[2 * rb + (q >> 3)][q & 7] = y;
                w |= (!(y <= 0.f) ? 1u : 0u) << q;
            }
        }
        bits[rb] = w;
    }
}

// kStore = false: the evaluation without autograd (the reference's f32 network under torch.no_grad(), render.py:46 ->
// gaussian_model.py:290-316): the same kernel without the hidden outputs' and ReLU words' stores (8 KB per Gaussian
// of HBM writes), p.H / p.bits unused -- only the heads are written.
template <bool kStore>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1))) void k_mlp_fwd_fused(MlpFusedParams p) {
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[4 * 24 * 1024];
    // the biases in an LDS object of their own: the compiler then knows the ring's copies cannot write them and
    // reads them without draining the copies in flight (one LDS array: an s_waitcnt vmcnt(0) per epilogue)
    __shared__ __attribute__((aligned(16))) float s_bias[8 * 256 + 64];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31, wave = tid >> 6;
    const int g = blockIdx.x * 128 + wave * 32 + c;   // < ldp (the grid covers ldp / 128 workgroups)
    const unsigned voff_h = (unsigned)(4 * h) * (unsigned)p.ldp + (unsigned)g;   // row 4 h of a layer's output
    const unsigned voff_b = (unsigned)h * (unsigned)p.ldp + (unsigned)g;         // ReLU word of half h
#pragma unroll
    for (int l = 0; l < 8; ++l) s_bias[256 * l + tid] = p.bias[l][tid];
    if (tid < 64) s_bias[2048 + tid] = p.bias_heads[tid];
    // the encoding in the B operand's natural order: lane half h holds rows 16 ks + 8 h + j
    float xe[4][8], xt[2][8];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) xe[ks][j] = p.E[(size_t)(16 * ks + 8 * h + j) * p.ldp + g];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) xt[ks][j] = p.ET[(size_t)(16 * ks + 8 * h + j) * p.ldp + g];
    // before the first copy: plain loads never wait behind one.  The builtin (0xf70: vmcnt 0, the other counters
    // free), not asm, so that the compiler knows these loads are done and sets no waits of its own on them later
    __builtin_amdgcn_s_waitcnt(0xf70);
    __syncthreads();   // the biases in LDS
    float act[16][8];
    unsigned bits[8];
    f32x16 acc[8];
    bf16x8 R[6];
    if constexpr (GSD_ABLATE & 2048) {
        const bf16x8* f0 = reinterpret_cast<const bf16x8*>(p.frags[0]) + lane;
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int ch = wave + 4 * i;
                R[i] = f0[k * kFusedStep + ch * 64];
                if (k < 2) *reinterpret_cast<bf16x8*>(s_mem + k * (24 * 1024) + ch * 1024 + 16 * lane) = R[i];
            }
        __syncthreads();
    } else {
        const bf16x8* f0 = reinterpret_cast<const bf16x8*>(p.frags[0]) + lane;
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int ch = wave + 4 * i;
                dma16_asm(f0 + k * kFusedStep + ch * 64,
                          __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + k * (24 * 1024) + ch * 1024));
            }
        wait_vm_c<12>();
        raw_barrier();
    }
    constexpr int PV = kStore ? 8 : 0;
    fused_hidden_layer<6, 0, 0, kStore>(p, s_mem, 0, 0, wave, lane, voff_h, voff_b, xe, xt, act, bits, acc, R);
    fused_hidden_epilogue(s_bias, h, acc, act, bits);
    fused_hidden_layer<0, 16, 0, kStore>(p, s_mem, 6, 1, wave, lane, voff_h, voff_b, xe, xt, act, bits, acc, R);
    fused_hidden_epilogue(s_bias + 256, h, acc, act, bits);
#pragma unroll 1
    for (int l = 2; l <= 4; ++l) {
        fused_hidden_layer<0, 16, PV, kStore>(p, s_mem, 6 + 16 * (l - 1), l, wave, lane, voff_h, voff_b, xe, xt, act,
                                              bits, acc, R);
        fused_hidden_epilogue(s_bias + 256 * l, h, acc, act, bits);
    }
    fused_hidden_layer<4, 16, PV, kStore>(p, s_mem, 70, 5, wave, lane, voff_h, voff_b, xe, xt, act, bits, acc, R);
    fused_hidden_epilogue(s_bias + 256 * 5, h, acc, act, bits);
#pragma unroll 1
    for (int l = 6; l <= 7; ++l) {
        fused_hidden_layer<0, 16, PV, kStore>(p, s_mem, 90 + 16 * (l - 6), l, wave, lane, voff_h, voff_b, xe, xt, act,
                                              bits, acc, R);
        fused_hidden_epilogue(s_bias + 256 * l, h, acc, act, bits);
    }
    // the heads (58 outputs, two row blocks): their own ring over the same LDS, 6 chunks per k-step (two copies per
    // wave, the last two re-copy chunk 0); the last hidden layer's output rides under their MFMAs as above
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    const bf16x8* fh = reinterpret_cast<const bf16x8*>(p.frags[8]) + lane;
#define GSD_HEADS_ISSUE(KS)                                                                                    \
    do {                                                                                                       \
        const int k_ = min((KS), 15);                                                                          \
        _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                                     \
            const int ch_ = wave + 4 * i_;                                                                     \
            dma16_asm(fh + k_ * (2 * 3 * 64) + (ch_ < 6 ? ch_ : 0) * 64,                                       \
                      __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + ((KS) & 3) * (8 * 1024) + ch_ * 1024));   \
        }                                                                                                      \
    } while (0)
    f32x16 ho[2] = {f32x16{}, f32x16{}};
    GSD_HEADS_ISSUE(0);
    GSD_HEADS_ISSUE(1);
    GSD_HEADS_ISSUE(2);
    wait_vm_c<4>();
    raw_barrier();
    float* H7 = p.H[7];
    unsigned short* B7 = p.bits[7];
    const int ldp = p.ldp;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
        GSD_HEADS_ISSUE(ks + 3);
        const Split8 b = split8(act[ks]);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + (ks & 3) * (8 * 1024));
        if constexpr (kStore) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                __builtin_nontemporal_store(act[ks][j], H7 + (size_t)(16 * ks + 8 * (j >> 2) + (j & 3)) * ldp + voff_h);
            if (ks < 8)
                __builtin_nontemporal_store((unsigned short)bits[ks < 8 ? ks : 0], B7 + (size_t)(2 * ks) * ldp + voff_b);
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            Split8 a;
            a.hi = sa[(r * 3) * 64 + lane];
            a.mid = sa[(r * 3 + 1) * 64 + lane];
            a.lo = sa[(r * 3 + 2) * 64 + lane];
            ho[r] = mfma_x6(a, b, ho[r]);
        }
        wait_vm_u(4 + (kStore ? (ks >= 2 ? fused_stores(0, ks - 2, 0) : 0) + (ks >= 1 ? fused_stores(0, ks - 1, 0) : 0) +
                                    fused_stores(0, ks, 0)
                              : 0));
        raw_barrier();
    }
#undef GSD_HEADS_ISSUE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's re-copies: nothing left in flight at exit
    if (g < p.P) {
        const float* bh = s_bias + 2048;
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const float4 b4 = *reinterpret_cast<const float4*>(bh + 32 * r + 8 * q4 + 4 * h);
                const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int n = 32 * r + 8 * q4 + 4 * h + i;
                    if (n < 58) mlp_store_head(p.heads, g, n, ho[r][4 * q4 + i] + bq[i]);
                }
            }
    }
}

// ---- the layer-fused forward at two waves per SIMD (k_mlp_fwd_fused16) ----
// k_mlp_fwd_fused holds 32 Gaussians per wave in ~450 registers: one wave per SIMD, so the issue of every weight copy
// and activation store stalls that wave's MFMA stream (the ablations of DESIGN.md §7: the MFMA work and the copy /
// store issue add up).  Here a wave holds 16 Gaussians on v_mfma_f32_16x16x32_bf16 -- 16 row blocks of 16 output
// rows, k-steps of 32 -- in 64 accumulator and 64 activation registers, so the workgroup's eight waves run two per
// SIMD and one wave's copies, stores and splits issue while the other's MFMAs run.  The weight fragments are read
// from LDS twice as often per MAC (a 16 x 32 fragment per 16 x 16 output block): 128 B/clk of the array's 256 for
// ds_read_b128.  The ring: three 48-KB slots (k-step t + 2 copied while t is multiplied), the biases beside it.
// Operand maps (lane l: q = l >> 4, c = l & 15, the Gaussian):
//   A fragment: row 16 rb + c, columns 32 ks + kcol(q, j), j = 0..7 (k_mlp_pack m16: natural kcol 8 q + j, or the
//               accumulator order 16 (j >> 2) + 4 q + (j & 3))
//   B operand:  element j of k-step ks = input feature 32 ks + kcol(q, j) of Gaussian c
//   C:          acc[rb][i] = output row 16 rb + 4 q + i
// so row blocks 2 s and 2 s + 1 of a layer's output are the next layer's k-step s with no lane movement.  The hidden
// outputs and ReLU words go to HBM in the layouts k_mlp_fwd_fused writes (the backward reads them unchanged).
typedef float f32x4 __attribute__((ext_vector_type(4)));
// the layer loops of the 16-wide kernels: one copy of a layer's code in the product; GSD_MLP_UNROLL_LAYERS (a check
// build only, tests/test_codegen.py) unrolls them so that the text order of the code is its issue order
#ifdef GSD_MLP_UNROLL_LAYERS
#define GSD_LAYER_LOOP _Pragma("unroll")
#else
#define GSD_LAYER_LOOP _Pragma("unroll 1")
#endif
constexpr int kF16Step = 16 * 3 * 64;   // bf16x8 per hidden k-step (48 KB)
constexpr int kF16Slot = 48 * 1024;

template <int M>
__device__ __forceinline__ f32x4 mfma16_part(const Split8& a, const Split8& b, f32x4 acc) {
    if constexpr (M == 0) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, acc, 0, 0, 0);
    if constexpr (M == 1) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.mid, acc, 0, 0, 0);
    if constexpr (M == 2) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, acc, 0, 0, 0);
    if constexpr (M == 3) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.hi, acc, 0, 0, 0);
    if constexpr (M == 4) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.mid, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, acc, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16_x6(const Split8& a, const Split8& b, f32x4 acc) {
    acc = mfma16_part<0>(a, b, acc);
    acc = mfma16_part<1>(a, b, acc);
    acc = mfma16_part<2>(a, b, acc);
    acc = mfma16_part<3>(a, b, acc);
    acc = mfma16_part<4>(a, b, acc);
    return mfma16_part<5>(a, b, acc);
}

// nontemporal row stores through a buffer descriptor built from wave-uniform values (the base: a k-step's first
// row), the lane's part a 32-bit offset: no 64-bit address per store held in registers.  v: element (row, g) with
// `row` rows (uniform) past base and `voff` = (its row within the group) * ldp + g (per lane), in elements.
__device__ __forceinline__ void store_row_nt(float v, const float* base, unsigned voff, int row_elems) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)(4 * voff), 4 * row_elems, 2);
}
__device__ __forceinline__ void store_row(float v, const float* base, unsigned voff, int row_elems) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)(4 * voff), 4 * row_elems, 0);
}
__device__ __forceinline__ float load_row(const float* base, unsigned voff, int row_elems) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, -1, 0x00020000);
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(4 * voff), 4 * row_elems, 0));
}
__device__ __forceinline__ void store_word_nt(unsigned w, const unsigned short* base, unsigned voff) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(base), 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)w, r, (int)(2 * voff), 0, 2);
}

// dma16_asm with a wave-uniform base (SGPRs) and the lane's 32-bit byte offset: no 64-bit address per copy in
// registers (the chunk's offset folds into the base)
__device__ __forceinline__ void dma16_sa(const void* sbase, unsigned voff, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds)
                 : "memory");
}

// global stores a k-step issues, all after its weight copies: 8 activation rows and a ReLU word (the k-steps fed by
// the layer before); ks < 0: the layer before's last k-step (prev)
__device__ __forceinline__ constexpr int f16_stores(int kse, int ks, int prev) {
    return ks < 0 ? prev : (ks < kse ? 0 : 9);
}

// One hidden layer (KSE encoding k-steps: enc(x) 0-1, then enc(t); then KSA activation k-steps), fully unrolled.  s:
// the layer's first global k-step (ring slot (s + ks) % 3).  Per k-step: 16 row blocks x 6 MFMAs, and in their gaps
// the next row block's fragments (LDS), k-step s + ks + 2's six copies per wave (row blocks 0-5), the previous layer's
// eight output rows this k-step consumes and its ReLU word (row blocks 6-14), the next B operand's split (1-4); then
// a counted vmcnt (k-step s + ks + 1 landed) and a raw barrier.
template <int KSE, int KSA, int PREV, bool ST>
__device__ __forceinline__ void fused16_layer(const MlpFusedParams& p, unsigned char* s_mem, int s, int l, int wave,
                                              int lane, unsigned voff_dma, unsigned voff_h, unsigned voff_b, bool bit_lane,
                                              const float (&xe)[2][8], const float (&xt)[8], const float (&act)[8][8],
                                              const unsigned (&bits)[8], f32x4 (&acc)[16]) {
    constexpr int KS = KSE + KSA;
    constexpr int kStepB = kF16Step * 16;   // bytes per k-step
    const char* fc = reinterpret_cast<const char*>(p.frags[l]);
    const char* fn = l < 7 ? reinterpret_cast<const char*>(p.frags[l + 1]) : fc + (KS - 1) * kStepB;
    const int ldp = p.ldp;
    float* Hp = KSA ? p.H[l - 1] : nullptr;
    unsigned short* Bp = KSA ? p.bits[l - 1] : nullptr;
    const int s3 = s % 3;
    const unsigned base = lds_addr(s_mem);
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = f32x4{};
    auto operand = [&](int ks) -> const float(&)[8] {
        if (ks < KSE) return ks < 2 ? xe[ks < 2 ? ks : 0] : xt;
        return act[ks >= KSE ? ks - KSE : 0];
    };
    auto slot = [&](int k) -> unsigned {   // k: a compile-time offset from s
        int t = s3 + k % 3;
        t = t >= 3 ? t - 3 : t;
        return (unsigned)t * kF16Slot;
    };
    Split8 b = split8(operand(0));
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int kk = ks + 2;
        const char* f = kk < KS ? fc + kk * kStepB : (l < 7 ? fn + (kk - KS) * kStepB : fn);
        const unsigned dst = base + slot(kk);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + slot(ks));
        const int k2 = ks >= KSE ? ks - KSE : 0;
        const bool stores = ST && ks >= KSE;
        Split8 bn = b;
        Split8 a;
        a.hi = sa[lane];
        a.mid = sa[64 + lane];
        a.lo = sa[128 + lane];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            Split8 an = a;
            if (r + 1 < 16) {
                an.hi = sa[((r + 1) * 3) * 64 + lane];
                an.mid = sa[((r + 1) * 3 + 1) * 64 + lane];
                an.lo = sa[((r + 1) * 3 + 2) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<0>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<1>(a, b, acc[r]);
            if (r < 6)   // chunk wave + 8 r: bytes 8192 r + 16 tid of the k-step
                dma16_sa(f + 8192 * r, voff_dma, __builtin_amdgcn_readfirstlane(dst + (wave + 8 * r) * 1024));
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<2>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<3>(a, b, acc[r]);
            if (stores && r >= 6 && r < 14) {
                const int e = r - 6;   // act[k2][e]: row 32 k2 + 16 (e >> 2) + 4 q + (e & 3)
                store_row_nt(act[k2][e < 8 ? e : 0], Hp + (size_t)(32 * k2) * ldp, voff_h,
                             (16 * (e >> 2) + (e & 3)) * ldp);
            }
            if (stores && r == 14 && bit_lane) store_word_nt(bits[k2], Bp + (size_t)(2 * k2) * ldp, voff_b);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<4>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<5>(a, b, acc[r]);
            if (r >= 1 && r <= 4 && ks + 1 < KS) split_pair(operand(ks + 1 < KS ? ks + 1 : 0), r - 1, bn);
            __builtin_amdgcn_sched_barrier(0);
            a = an;
        }
        b = bn;
        wait_vm_u((ST ? f16_stores(KSE, ks - 1, PREV) + f16_stores(KSE, ks, PREV) : 0) + 6);
        raw_barrier();
    }
}

// bias (LDS) + ReLU into the next layer's B operand (k-step rb32 = row blocks 2 rb32, 2 rb32 + 1) and the ReLU words
// in k_mlp_fwd_fused's layout (word 2 rb32 + h, bit 4 q4 + i = row 32 rb32 + 8 q4 + 4 h + i): lane (q, c) holds
// half of word 2 rb32 + (q & 1), lane (q ^ 2, c) the other half
__device__ __forceinline__ void fused16_epilogue(const float* s_bias, int q, const f32x4 (&acc)[16],
                                                 float (&act)[8][8], unsigned (&bits)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        unsigned w = 0;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const float4 b4 = *reinterpret_cast<const float4*>(s_bias + 16 * (2 * k + a) + 4 * q);
            const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float y = relu_nan(acc[2 * k + a][i] + bq[i]);
                act[k][4 * a + i] = y;
                w |= (!(y <= 0.f) ? 1u : 0u) << (8 * a + i);
            }
        }
        w <<= 4 * (q >> 1);
        bits[k] = w | (unsigned)__shfl_xor((int)w, 32);
    }
}

template <bool kStore>
__global__ __launch_bounds__(512) void k_mlp_fwd_fused16(MlpFusedParams p) {
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[3 * kF16Slot];
    __shared__ __attribute__((aligned(16))) float s_bias[8 * 256 + 64];
    const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, c = lane & 15, wave = tid >> 6;
    const int g = blockIdx.x * 128 + wave * 16 + c;   // < ldp (the grid covers ldp / 128 workgroups)
    const int ldp = p.ldp;
    const unsigned voff_h = (unsigned)(4 * q) * (unsigned)ldp + (unsigned)g;      // row 4 q of a layer's output
    const unsigned voff_b = (unsigned)(q & 1) * (unsigned)ldp + (unsigned)g;      // ReLU word of half q & 1
    const bool bit_lane = q < 2;
    const unsigned voff_dma = 16u * (unsigned)tid;
#pragma unroll
    for (int i = 0; i < 4; ++i) s_bias[512 * i + tid] = p.bias[(512 * i + tid) >> 8][(512 * i + tid) & 255];
    if (tid < 64) s_bias[2048 + tid] = p.bias_heads[tid];
    float xe[2][8], xt[8];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) xe[ks][j] = p.E[(size_t)(32 * ks + 8 * q + j) * ldp + g];
#pragma unroll
    for (int j = 0; j < 8; ++j) xt[j] = p.ET[(size_t)(8 * q + j) * ldp + g];
    __builtin_amdgcn_s_waitcnt(0xf70);   // plain loads done before the first copy (as k_mlp_fwd_fused)
    __syncthreads();
    {
        const char* f0 = reinterpret_cast<const char*>(p.frags[0]);
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int i = 0; i < 6; ++i)
                dma16_sa(f0 + k * (kF16Step * 16) + 8192 * i, voff_dma,
                         __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + k * kF16Slot + (wave + 8 * i) * 1024));
    }
    wait_vm_c<6>();
    raw_barrier();
    float act[8][8];
    unsigned bits[8];
    f32x4 acc[16];
    constexpr int PV = kStore ? 9 : 0;
    fused16_layer<3, 0, 0, kStore>(p, s_mem, 0, 0, wave, lane, voff_dma, voff_h, voff_b, bit_lane, xe, xt, act, bits, acc);
    fused16_epilogue(s_bias, q, acc, act, bits);
    fused16_layer<0, 8, 0, kStore>(p, s_mem, 3, 1, wave, lane, voff_dma, voff_h, voff_b, bit_lane, xe, xt, act, bits, acc);
    fused16_epilogue(s_bias + 256, q, acc, act, bits);
GSD_LAYER_LOOP
    for (int l = 2; l <= 4; ++l) {
        fused16_layer<0, 8, PV, kStore>(p, s_mem, 3 + 8 * (l - 1), l, wave, lane, voff_dma, voff_h, voff_b, bit_lane, xe, xt,
                                        act, bits, acc);
        fused16_epilogue(s_bias + 256 * l, q, acc, act, bits);
    }
    fused16_layer<2, 8, PV, kStore>(p, s_mem, 35, 5, wave, lane, voff_dma, voff_h, voff_b, bit_lane, xe, xt, act, bits, acc);
    fused16_epilogue(s_bias + 256 * 5, q, acc, act, bits);
GSD_LAYER_LOOP
    for (int l = 6; l <= 7; ++l) {
        fused16_layer<0, 8, PV, kStore>(p, s_mem, 45 + 8 * (l - 6), l, wave, lane, voff_dma, voff_h, voff_b, bit_lane, xe, xt,
                                        act, bits, acc);
        fused16_epilogue(s_bias + 256 * l, q, acc, act, bits);
    }
    // the heads (58 outputs, four row blocks of 16, eight k-steps): their own ring of four 16-KB slots over the same
    // LDS, 12 chunks per k-step (two copies per wave; waves 4-7 re-copy chunk 0 into the slot's padding); layer 7's
    // output and ReLU words ride under their MFMAs
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    const char* fh = reinterpret_cast<const char*>(p.frags[8]);
    // chunk wave: bytes 16 tid of the k-step; chunk wave + 8: 8192 + 16 tid for waves 0-3, chunk 0 (16 lane) again
    // for waves 4-7
    const unsigned voff_h2 = wave < 4 ? 8192u + voff_dma : 16u * (unsigned)lane;
#define GSD_H16_ISSUE(KS)                                                                                      \
    do {                                                                                                       \
        const char* f_ = fh + min((KS), 7) * (4 * 3 * 64 * 16);                                                \
        dma16_sa(f_, voff_dma, __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + ((KS) & 3) * (16 * 1024) + wave * 1024)); \
        dma16_sa(f_, voff_h2,                                                                                  \
                 __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + ((KS) & 3) * (16 * 1024) + (wave + 8) * 1024)); \
    } while (0)
    f32x4 ho[4] = {f32x4{}, f32x4{}, f32x4{}, f32x4{}};
    GSD_H16_ISSUE(0);
    GSD_H16_ISSUE(1);
    GSD_H16_ISSUE(2);
    wait_vm_c<4>();
    raw_barrier();
    float* H7 = p.H[7];
    unsigned short* B7 = p.bits[7];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        GSD_H16_ISSUE(ks + 3);
        const Split8 b = split8(act[ks]);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + (ks & 3) * (16 * 1024));
        if constexpr (kStore) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
                store_row_nt(act[ks][e], H7 + (size_t)(32 * ks) * ldp, voff_h, (16 * (e >> 2) + (e & 3)) * ldp);
            if (bit_lane) store_word_nt(bits[ks], B7 + (size_t)(2 * ks) * ldp, voff_b);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            Split8 a;
            a.hi = sa[(r * 3) * 64 + lane];
            a.mid = sa[(r * 3 + 1) * 64 + lane];
            a.lo = sa[(r * 3 + 2) * 64 + lane];
            ho[r] = mfma16_x6(a, b, ho[r]);
        }
        wait_vm_u(4 + f16_stores(0, ks - 2, 0) * kStore + f16_stores(0, ks - 1, 0) * kStore +
                  f16_stores(0, ks, 0) * kStore);
        raw_barrier();
    }
#undef GSD_H16_ISSUE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's re-copies: nothing left in flight at exit
    if (g < p.P) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 b4 = *reinterpret_cast<const float4*>(s_bias + 2048 + 16 * r + 4 * q);
            const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = 16 * r + 4 * q + i;
                if (n < 58) mlp_store_head(p.heads, g, n, ho[r][i] + bq[i]);
            }
        }
    }
}

// ---- the backward's dX chain fused across the layers ----
// g_{l-1} = (W_l^T g_l) masked by the forward's ReLU words of h_l, from the heads' gradient g8 down to g0, in one
// kernel the way k_mlp_fwd_fused runs the forward: a wave keeps its 32 Gaussians' gradient in registers, layer l's
// accumulators becoming (masked) layer l - 1's B operand with no lane movement (W^T packed with the accumulator-order
// k permutation, k_mlp_pack perm_from 0; the first step's g8 comes in natural order from the heads' row-major
// gradients), the packed W^T k-steps (24 KB) shared by the four waves through a four-slot LDS ring fed by LDS-DMA
// three k-steps ahead (as the forward; copies through registers measured 1.3 % slower there).  Every g_l goes to HBM
// once (the weight gradients' operand), its rows stored under the next step's MFMAs; nothing is re-read.  The
// mask words of all eight steps (16 B per lane each) are loaded at the start: a load issued inside the ring would be
// waited for by the next k-step's counted wait (the counter retires in order), at HBM latency.  A final two-row-block
// step multiplies g0 by W0^T's enc(x) rows: the encoding's gradient, to which layer 5's enc(x) rows times g5 add --
// formed inside the kernel by enc_pass (a ring of its own, just before step 3, while the B operand holds g5).

// global stores of a chain k-step: all eight act rows, three of them (row blocks 5-7) after the k-step's last copy
__device__ __forceinline__ constexpr int chain_stores(int ks, int prev) { return ks < 0 ? (prev ? 8 : 0) : 8; }
__device__ __forceinline__ constexpr int chain_stores_late(int ks, int prev) { return ks < 0 ? (prev ? 3 : 0) : 3; }

// one step's k-steps.  B operand k-step ks = act[ks]: natural row order (NAT: lane half h holds rows 16 ks + 8 h + j)
// or the accumulator order (rows 16 ks + 8 (j >> 2) + 4 h + (j & 3)); the rows are stored to Gp (+ voff) under the
// MFMAs.  s: the global k-step of the step's first; the ring is fed with k-steps of this step, then of the next
// (fn), or re-copies of this step's last when LAST.  PREV: the step before stored rows (every step but the first).
template <int KS, bool NAT, bool LAST, int PREV>
__device__ __forceinline__ void chain_step(const bf16x8* fc, const bf16x8* fn, float* __restrict__ Gp, unsigned voff,
                                           int ldp, unsigned char* s_mem, int s, int wave, int lane,
                                           const float (&act)[16][8], f32x16 (&acc)[8]) {
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = f32x16{};
    Split8 b = split8(act[0]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int kk = ks + 3;
        const bf16x8* f = kk < KS ? fc + kk * kFusedStep : (LAST ? fc + (KS - 1) * kFusedStep : fn + (kk - KS) * kFusedStep);
        const unsigned dst = lds_addr(s_mem) + ((s + kk) & 3) * (24 * 1024);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + ((s + ks) & 3) * (24 * 1024));
        Split8 bn = b;
        Split8 a;
        a.hi = sa[lane];
        a.mid = sa[64 + lane];
        a.lo = sa[128 + lane];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            Split8 an = a;
            if (r + 1 < 8) {
                an.hi = sa[((r + 1) * 3) * 64 + lane];
                an.mid = sa[((r + 1) * 3 + 1) * 64 + lane];
                an.lo = sa[((r + 1) * 3 + 2) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<0>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<1>(a, b, acc[r]);
            if (r < 6) {
                const int ch = wave + 4 * r;
                dma16_asm(f + ch * 64, __builtin_amdgcn_readfirstlane(dst + ch * 1024));
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<2>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<3>(a, b, acc[r]);
            {
                const int roff = NAT ? r : 8 * (r >> 2) + (r & 3);
                __builtin_nontemporal_store(act[ks][r], Gp + (size_t)(16 * ks + roff) * ldp + voff);
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<4>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma_x6_part<5>(a, b, acc[r]);
            if (r >= 1 && r <= 4 && ks + 1 < KS) split_pair(act[ks + 1 < KS ? ks + 1 : 0], r - 1, bn);
            __builtin_amdgcn_sched_barrier(0);
            a = an;
        }
        b = bn;
        // k-step ks + 1's copies (issued at k-step ks - 2) landed: wait for all but the younger stores and copies
        wait_vm_u(chain_stores_late(ks - 2, PREV) + chain_stores(ks - 1, PREV) + chain_stores(ks, PREV) + 12);
        raw_barrier();
    }
}

// threshold_backward by the forward's ReLU words (w: the step's eight 16-bit words, two per register): act (the
// next step's B operand, accumulator order) = acc where h > 0
__device__ __forceinline__ void chain_mask(const unsigned (&w)[4], const f32x16 (&acc)[8], float (&act)[16][8]) {
#pragma unroll
    for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int q = 0; q < 16; ++q)
            act[2 * rb + (q >> 3)][q & 7] = (w[rb >> 1] >> (16 * (rb & 1) + q)) & 1u ? acc[rb][q] : 0.f;
}

// W^T's 64 enc(x) rows (2 row blocks, accumulator k order, K = 256) times the B operand in act, on a ring of its
// own (s_e: four 8-KB slots; waves 0 and 1 copy two chunks per k-step, 2 and 3 one and re-copy chunk 0 into the
// padding).  Its copies are younger than everything in flight, so its first wait also retires the main ring's
// prefetched k-steps and the stores before it (once per workgroup); the counted waits after it over-wait by its
// copies, never under-wait.  No stores: act's rows go out with the chain step that uses it.
__device__ __forceinline__ void enc_pass(const void* frags, unsigned char* s_e, int wave, int lane,
                                         const float (&act)[16][8], f32x16 (&ho)[2]) {
    const bf16x8* fe = reinterpret_cast<const bf16x8*>(frags) + lane;
#define GSD_E5_ISSUE(KS)                                                                                       \
    do {                                                                                                       \
        const int k_ = min((KS), 15);                                                                          \
        _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                                     \
            const int ch_ = wave + 4 * i_;                                                                     \
            dma16_asm(fe + k_ * (2 * 3 * 64) + (ch_ < 6 ? ch_ : 0) * 64,                                       \
                      __builtin_amdgcn_readfirstlane(lds_addr(s_e) + ((KS) & 3) * (8 * 1024) + ch_ * 1024));     \
        }                                                                                                      \
    } while (0)
    ho[0] = f32x16{};
    ho[1] = f32x16{};
    GSD_E5_ISSUE(0);
    GSD_E5_ISSUE(1);
    GSD_E5_ISSUE(2);
    wait_vm_c<4>();
    raw_barrier();
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
        GSD_E5_ISSUE(ks + 3);
        const Split8 b = split8(act[ks]);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_e + (ks & 3) * (8 * 1024));
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            Split8 a;
            a.hi = sa[(r * 3) * 64 + lane];
            a.mid = sa[(r * 3 + 1) * 64 + lane];
            a.lo = sa[(r * 3 + 2) * 64 + lane];
            ho[r] = mfma_x6(a, b, ho[r]);
        }
        wait_vm_c<4>();   // stage ks + 1 landed; ks + 2 and ks + 3 (two copies each) stay in flight
        raw_barrier();
    }
#undef GSD_E5_ISSUE
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1))) void k_mlp_bwd_chain(MlpChainParams p) {
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[4 * 24 * 1024];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31, wave = tid >> 6;
    const int g = blockIdx.x * 128 + wave * 32 + c;   // < ldp (the grid covers ldp / 128 workgroups)
    const int ldp = p.ldp;
    const unsigned voff_n = (unsigned)(8 * h) * (unsigned)ldp + (unsigned)g;   // natural order: row 8 h
    const unsigned voff_a = (unsigned)(4 * h) * (unsigned)ldp + (unsigned)g;   // accumulator order: row 4 h
    // the mask words of every step (two 16-bit words per 32-bit word), each lane's own: registers would not fit
    __shared__ uint4 s_w[8][256];
    // the ring of the layer-5 enc(x) pass (W5^T's rows 0-63 times g5): 6 chunks of 1 KB per k-step in 8-KB slots
    __shared__ __attribute__((aligned(16))) unsigned char s_e5[4 * 8 * 1024];
    float act[16][8];
    f32x16 acc[8];
    // g8, natural order: act[ks][j] = row 16 ks + 8 h + j of the heads' gradient (58 rows; zero past them and P)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int n = 16 * ks + 8 * h + j;
            const int k = n < 3 ? 0 : (n < 6 ? 1 : (n < 10 ? 2 : 3));
            const int c0 = k == 0 ? 0 : (k == 1 ? 3 : (k == 2 ? 6 : 10));
            const float* src = p.heads.src[k];
            act[ks][j] = (g < p.P && n < 58 && src) ? src[(size_t)g * p.heads.ld[k] + (n - c0)] : 0.f;
        }
#pragma unroll
    for (int ks = 4; ks < 16; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) act[ks][j] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        unsigned wq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned lo = p.bits[i][(size_t)(2 * (2 * q) + h) * ldp + g];
            const unsigned hi = p.bits[i][(size_t)(2 * (2 * q + 1) + h) * ldp + g];
            wq[q] = lo | (hi << 16);
        }
        s_w[i][tid] = make_uint4(wq[0], wq[1], wq[2], wq[3]);
    }
    // before the first copy: plain loads never wait behind one (vmcnt 0, the other counters free; the builtin, so
    // the compiler knows them done)
    __builtin_amdgcn_s_waitcnt(0xf70);
    {
        const bf16x8* f0 = reinterpret_cast<const bf16x8*>(p.frags[0]) + lane;
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int ch = wave + 4 * i;
                dma16_asm(f0 + k * kFusedStep + ch * 64,
                          __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + k * (24 * 1024) + ch * 1024));
            }
    }
    wait_vm_c<12>();
    raw_barrier();
    const bf16x8* F[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) F[i] = reinterpret_cast<const bf16x8*>(p.frags[i]) + lane;
    auto mask = [&](int i) {
        const uint4 wv = s_w[i][tid];
        const unsigned wi[4] = {wv.x, wv.y, wv.z, wv.w};
        chain_mask(wi, acc, act);
    };
    chain_step<4, true, false, 0>(F[0], F[1], p.G[0], voff_n, ldp, s_mem, 0, wave, lane, act, acc);
    mask(0);
    // steps 1-6 (layers 7 .. 2); before step 3 (layer 5), act = g5: W5^T's enc(x) rows times g5 -> dE (added to at
    // the end; held in registers that long, it spilled)
#pragma unroll 1
    for (int i = 1; i < 3; ++i) {
        chain_step<16, false, false, 1>(F[i], F[i + 1], p.G[i], voff_a, ldp, s_mem, 4 + 16 * (i - 1), wave, lane, act,
                                        acc);
        mask(i);
    }
    {
        f32x16 he[2];
        enc_pass(p.frags_e5, s_e5, wave, lane, act, he);
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int q = 0; q < 16; ++q) p.dE[(size_t)(32 * r + 8 * (q >> 2) + 4 * h + (q & 3)) * ldp + g] = he[r][q];
    }
#pragma unroll 1
    for (int i = 3; i < 7; ++i) {
        chain_step<16, false, false, 1>(F[i], F[i + 1], p.G[i], voff_a, ldp, s_mem, 4 + 16 * (i - 1), wave, lane, act,
                                        acc);
        mask(i);
    }
    chain_step<16, false, true, 1>(F[7], F[7], p.G[7], voff_a, ldp, s_mem, 4 + 16 * 6, wave, lane, act, acc);
    mask(7);   // g0
    // the final step: W0^T's enc(x) rows (two row blocks) times g0, added to the layer-5 part in dE; g0's rows
    // stored under it.  Its own ring over the same LDS (6 chunks of 1 KB per k-step in 8-KB slots; waves 0 and 1 copy
    // two chunks, 2 and 3 one and re-copy chunk 0 into the padding), after everything in flight has retired
    f32x16 ho[2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 16; ++q) ho[r][q] = p.dE[(size_t)(32 * r + 8 * (q >> 2) + 4 * h + (q & 3)) * ldp + g];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    const bf16x8* fe = reinterpret_cast<const bf16x8*>(p.frags_e) + lane;
#define GSD_E_ISSUE(KS)                                                                                        \
    do {                                                                                                       \
        const int k_ = min((KS), 15);                                                                          \
        _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                                     \
            const int ch_ = wave + 4 * i_;                                                                     \
            dma16_asm(fe + k_ * (2 * 3 * 64) + (ch_ < 6 ? ch_ : 0) * 64,                                       \
                      __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + ((KS) & 3) * (8 * 1024) + ch_ * 1024));   \
        }                                                                                                      \
    } while (0)
    GSD_E_ISSUE(0);
    GSD_E_ISSUE(1);
    GSD_E_ISSUE(2);
    wait_vm_c<4>();
    raw_barrier();
    float* G0 = p.G[8];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
        GSD_E_ISSUE(ks + 3);
        const Split8 b = split8(act[ks]);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + (ks & 3) * (8 * 1024));
#pragma unroll
        for (int j = 0; j < 8; ++j)
            __builtin_nontemporal_store(act[ks][j], G0 + (size_t)(16 * ks + 8 * (j >> 2) + (j & 3)) * ldp + voff_a);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            Split8 a;
            a.hi = sa[(r * 3) * 64 + lane];
            a.mid = sa[(r * 3 + 1) * 64 + lane];
            a.lo = sa[(r * 3 + 2) * 64 + lane];
            ho[r] = mfma_x6(a, b, ho[r]);
        }
        // stage ks + 1 (issued at k-step ks - 2, or in the prologue) landed: all but the younger copies and stores
        wait_vm_u(4 + (ks >= 2 ? 8 : 0) + (ks >= 1 ? 8 : 0) + 8);
        raw_barrier();
    }
#undef GSD_E_ISSUE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's re-copies: nothing left in flight at exit
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 16; ++q)
            p.dE[(size_t)(32 * r + 8 * (q >> 2) + 4 * h + (q & 3)) * ldp + g] = ho[r][q];
}

// ---- the dX chain at two waves per SIMD (k_mlp_bwd_chain16) ----
// k_mlp_bwd_chain's structure on k_mlp_fwd_fused16's operand maps: eight waves of 16 Gaussians, v_mfma_f32_16x16x32,
// the packed W^T k-steps (48 KB) through a three-slot ring two k-steps ahead.  Per step the next step's ReLU words
// (the eight 16-bit words of the lane's half, 16 B) are loaded at its first k-step, ahead of the copies, so the
// counted waits retire them a k-step later; the mask (k_mlp_fwd_fused16's word layout read back) is applied from
// registers.  The two 64-row passes on W^T's enc(x) rows (layer 5's, times g5 before step 3, and layer 0's, times g0
// at the end) run on a ring of their own over the drained main ring (four 16-KB slots, three ahead); the main ring
// restarts after the first.  Every step's input goes to G[i] under its MFMAs, as in k_mlp_bwd_chain.

// a 4-B LDS-DMA per lane (one 256-B row segment per wave): the ReLU words of the workgroup's 128 Gaussians
__device__ __forceinline__ void dma4_sa(const void* sbase, unsigned voff, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds)
                 : "memory");
}
// the sixteen ReLU-word rows of a step for the workgroup's Gaussians into s_w ([16][128] u16): wave w copies rows
// 2 w, 2 w + 1 (two DMAs per wave, counted by the caller's waits)
__device__ __forceinline__ void chain16_words(const unsigned short* bits, int ldp, int wave, unsigned voff_w2,
                                              unsigned s_w) {
    const int w = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
    for (int j = 0; j < 2; ++j)
        dma4_sa(bits + (size_t)(2 * w + j) * ldp, voff_w2, __builtin_amdgcn_readfirstlane(s_w + (2 * w + j) * 256));
}

// one step: KS k-steps of B = act (NAT: natural rows 32 ks + 8 q + j; else the accumulator order), the rows stored to
// Gp under the MFMAs; s: the step's first k-step in the ring phase (slot s % 3); LAST: the ring is fed re-copies of
// this step's own last k-step (no next step in this ring phase); MASKLD: the next step's ReLU words are loaded into
// wn at k-step 0; PREV: stores of the k-step before (0 at a ring phase's start).
template <int KS, bool NAT, bool LAST, bool MASKLD, int PREV>
__device__ __forceinline__ void chain16_step(const char* fc, const char* fn, float* __restrict__ Gp, int ldp,
                                             unsigned char* s_mem, int s, int wave, int lane, unsigned voff_dma,
                                             unsigned voff_st, const unsigned short* bits_next, unsigned voff_w2,
                                             unsigned s_wn, const float (&act)[8][8], f32x4 (&acc)[16]) {
    constexpr int kStepB = kF16Step * 16;
    const int s3 = s % 3;
    const unsigned base = lds_addr(s_mem);
    auto slot = [&](int k) -> unsigned {
        int t = s3 + k % 3;
        t = t >= 3 ? t - 3 : t;
        return (unsigned)t * kF16Slot;
    };
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = f32x4{};
    Split8 b = split8(act[0]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int kk = ks + 2;
        const char* f = kk < KS ? fc + kk * kStepB : (LAST ? fc + (KS - 1) * kStepB : fn + (kk - KS) * kStepB);
        const unsigned dst = base + slot(kk);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + slot(ks));
        if (MASKLD && ks == 0) chain16_words(bits_next, ldp, wave, voff_w2, s_wn);
        Split8 bn = b;
        Split8 a;
        a.hi = sa[lane];
        a.mid = sa[64 + lane];
        a.lo = sa[128 + lane];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            Split8 an = a;
            if (r + 1 < 16) {
                an.hi = sa[((r + 1) * 3) * 64 + lane];
                an.mid = sa[((r + 1) * 3 + 1) * 64 + lane];
                an.lo = sa[((r + 1) * 3 + 2) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<0>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<1>(a, b, acc[r]);
            if (r < 6) dma16_sa(f + 8192 * r, voff_dma, __builtin_amdgcn_readfirstlane(dst + (wave + 8 * r) * 1024));
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<2>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<3>(a, b, acc[r]);
            if (r >= 6 && r < 14) {
                const int e = r - 6;
                store_row_nt(act[ks][e < 8 ? e : 0], Gp + (size_t)(32 * ks) * ldp, voff_st,
                             (NAT ? e : 16 * (e >> 2) + (e & 3)) * ldp);
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<4>(a, b, acc[r]);
            __builtin_amdgcn_sched_barrier(0);
            acc[r] = mfma16_part<5>(a, b, acc[r]);
            if (r >= 1 && r <= 4 && ks + 1 < KS) split_pair(act[ks + 1 < KS ? ks + 1 : 0], r - 1, bn);
            __builtin_amdgcn_sched_barrier(0);
            a = an;
        }
        b = bn;
        // k-step ks + 1's copies (issued at k-step ks - 1, or before the phase) landed: all but the younger ops
        wait_vm_u((ks == 0 ? PREV : 8) + (MASKLD && ks == 0 ? 2 : 0) + 6 + 8);
        raw_barrier();
    }
}

// threshold_backward by the forward's ReLU words (fused16_epilogue's layout) from s_w: word 2 k + (q & 1) of the
// lane's Gaussian gl (0-127 in the workgroup)
__device__ __forceinline__ void chain16_mask(const unsigned short* s_w, int gl, int q, const f32x4 (&acc)[16],
                                             float (&act)[8][8]) {
    int idx = (q & 1) * 128 + gl;
    asm volatile("" : "+v"(idx));   // formed here, not hoisted to the kernel's start and held (or spilled) till now
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const unsigned wk = (unsigned)s_w[idx + 256 * k] >> (4 * (q >> 1));
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int i = 0; i < 4; ++i) act[k][4 * a + i] = (wk >> (8 * a + i)) & 1u ? acc[2 * k + a][i] : 0.f;
    }
}

// a 64-row pass (four row blocks of 16, K = 256) of W^T's enc(x) rows times act, on a four-slot ring over the drained
// main ring: ho += A act.  Gp: act's rows stored under it (the final step's g0), or null.
template <bool STORE>
__device__ __forceinline__ void chain16_enc_pass(const char* fe, unsigned char* s_mem, int wave, int lane,
                                                 unsigned voff_dma, float* __restrict__ Gp, int ldp, unsigned voff_st,
                                                 const float (&act)[8][8], f32x4 (&ho)[4]) {
    const unsigned voff_2 = wave < 4 ? 8192u + voff_dma : 16u * (unsigned)lane;   // waves 4-7 re-copy chunk 0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
#define GSD_E16_ISSUE(KS)                                                                                      \
    do {                                                                                                       \
        const char* f_ = fe + min((KS), 7) * (4 * 3 * 64 * 16);                                                \
        dma16_sa(f_, voff_dma, __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + ((KS) & 3) * (16 * 1024) + wave * 1024)); \
        dma16_sa(f_, voff_2,                                                                                   \
                 __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + ((KS) & 3) * (16 * 1024) + (wave + 8) * 1024)); \
    } while (0)
    GSD_E16_ISSUE(0);
    GSD_E16_ISSUE(1);
    GSD_E16_ISSUE(2);
    wait_vm_c<4>();
    raw_barrier();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        GSD_E16_ISSUE(ks + 3);
        const Split8 b = split8(act[ks]);
        const bf16x8* sa = reinterpret_cast<const bf16x8*>(s_mem + (ks & 3) * (16 * 1024));
        if constexpr (STORE) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
                store_row_nt(act[ks][e], Gp + (size_t)(32 * ks) * ldp, voff_st, (16 * (e >> 2) + (e & 3)) * ldp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            Split8 a;
            a.hi = sa[(r * 3) * 64 + lane];
            a.mid = sa[(r * 3 + 1) * 64 + lane];
            a.lo = sa[(r * 3 + 2) * 64 + lane];
            ho[r] = mfma16_x6(a, b, ho[r]);
        }
        // k-step ks + 1 (issued at k-step ks - 2, or before the loop) landed
        wait_vm_u(4 + (STORE ? (ks >= 2 ? 8 : 0) + (ks >= 1 ? 8 : 0) + 8 : 0));
        raw_barrier();
    }
#undef GSD_E16_ISSUE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's re-copies: nothing in flight past the pass
    raw_barrier();
}

__global__ __launch_bounds__(512) void k_mlp_bwd_chain16(MlpChainParams p) {
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[3 * kF16Slot];
    // the ReLU words of three steps ([16][128] u16 each): step i's are read at its end from buffer i % 3 while step
    // i + 1's land in (i + 1) % 3 and step i + 2's are issued into (i + 2) % 3 by waves already past step i
    __shared__ __attribute__((aligned(16))) unsigned short s_w[3][16 * 128];
    const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, c = lane & 15, wave = tid >> 6;
    const int gl = wave * 16 + c, g = blockIdx.x * 128 + gl;   // < ldp (the grid covers ldp / 128 workgroups)
    const int ldp = p.ldp;
    const unsigned voff_dma = 16u * (unsigned)tid;
    const unsigned voff_n = (unsigned)(8 * q) * (unsigned)ldp + (unsigned)g;    // natural order: row 8 q
    const unsigned voff_a = (unsigned)(4 * q) * (unsigned)ldp + (unsigned)g;    // accumulator order: row 4 q
    const unsigned voff_w2 = 2u * (unsigned)(blockIdx.x * 128 + 2 * lane);     // words of Gaussians 2 lane, + 1
    const unsigned sw0 = lds_addr(&s_w[0][0]);
    auto swb = [&](int i) -> unsigned { return sw0 + (unsigned)(i % 3) * (16 * 128 * 2); };
    float act[8][8];
    f32x4 acc[16];
    // g8, natural order: act[ks][j] = row 32 ks + 8 q + j of the heads' gradient (58 rows; zero past them and P)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int n = 32 * ks + 8 * q + j;
            const int k = n < 3 ? 0 : (n < 6 ? 1 : (n < 10 ? 2 : 3));
            const int c0 = k == 0 ? 0 : (k == 1 ? 3 : (k == 2 ? 6 : 10));
            const float* src = p.heads.src[k];
            act[ks][j] = (g < p.P && n < 58 && src) ? src[(size_t)g * p.heads.ld[k] + (n - c0)] : 0.f;
        }
#pragma unroll
    for (int ks = 2; ks < 8; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) act[ks][j] = 0.f;
    __builtin_amdgcn_s_waitcnt(0xf70);   // plain loads done before the first copy
    chain16_words(p.bits[0], ldp, wave, voff_w2, swb(0));   // retired with the prologue's wait
    auto prologue = [&](const char* f0) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int i = 0; i < 6; ++i)
                dma16_sa(f0 + k * (kF16Step * 16) + 8192 * i, voff_dma,
                         __builtin_amdgcn_readfirstlane(lds_addr(s_mem) + k * kF16Slot + (wave + 8 * i) * 1024));
        wait_vm_c<6>();
        raw_barrier();
    };
    auto F = [&](int i) { return reinterpret_cast<const char*>(p.frags[i]); };
    // phase A: steps 0-2 (layers 8, 7, 6)
    prologue(F(0));
    chain16_step<2, true, false, true, 0>(F(0), F(1), p.G[0], ldp, s_mem, 0, wave, lane, voff_dma, voff_n, p.bits[1],
                                          voff_w2, swb(1), act, acc);
    chain16_mask(s_w[0], gl, q, acc, act);
    chain16_step<8, false, false, true, 8>(F(1), F(2), p.G[1], ldp, s_mem, 2, wave, lane, voff_dma, voff_a, p.bits[2],
                                           voff_w2, swb(2), act, acc);
    chain16_mask(s_w[1], gl, q, acc, act);
    chain16_step<8, false, true, true, 8>(F(2), F(2), p.G[2], ldp, s_mem, 10, wave, lane, voff_dma, voff_a, p.bits[3],
                                          voff_w2, swb(3), act, acc);
    chain16_mask(s_w[2], gl, q, acc, act);   // g5
    {   // W5^T's enc(x) rows times g5 -> dE (added to at the end)
        f32x4 he[4] = {f32x4{}, f32x4{}, f32x4{}, f32x4{}};
        chain16_enc_pass<false>(reinterpret_cast<const char*>(p.frags_e5), s_mem, wave, lane, voff_dma, nullptr, ldp,
                                voff_a, act, he);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < 4; ++i) store_row(he[r][i], p.dE, voff_a, (16 * r + i) * ldp);
    }
    // phase B: steps 3-7 (layers 5 .. 1)
    prologue(F(3));
    chain16_step<8, false, false, true, 0>(F(3), F(4), p.G[3], ldp, s_mem, 0, wave, lane, voff_dma, voff_a, p.bits[4],
                                           voff_w2, swb(4), act, acc);
    chain16_mask(s_w[0], gl, q, acc, act);
GSD_LAYER_LOOP
    for (int i = 4; i < 7; ++i) {
        chain16_step<8, false, false, true, 8>(F(i), F(i + 1), p.G[i], ldp, s_mem, 8 * (i - 3), wave, lane, voff_dma,
                                               voff_a, p.bits[i + 1], voff_w2, swb(i + 1), act, acc);
        chain16_mask(reinterpret_cast<const unsigned short*>(s_w) + (i % 3) * (16 * 128), gl, q, acc, act);
    }
    chain16_step<8, false, true, false, 8>(F(7), F(7), p.G[7], ldp, s_mem, 32, wave, lane, voff_dma, voff_a, p.bits[7],
                                           voff_w2, swb(8), act, acc);
    chain16_mask(s_w[1], gl, q, acc, act);   // g0 (step 7: buffer 7 % 3)
    // the final pass: W0^T's enc(x) rows times g0, added to the layer-5 part in dE; g0's rows stored under it
    f32x4 ho[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) ho[r][i] = load_row(p.dE, voff_a, (16 * r + i) * ldp);
    chain16_enc_pass<true>(reinterpret_cast<const char*>(p.frags_e), s_mem, wave, lane, voff_dma, p.G[8], ldp, voff_a,
                           act, ho);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) store_row(ho[r][i], p.dE, voff_a, (16 * r + i) * ldp);
}

// ---- dW = G X^T (split-K over Gaussian chunks) and db = row sums of G ----
// One workgroup per Gaussian chunk computes the whole (32 NRB) x (32 KRB) output, one wave per tile of TNB x TKB
// blocks of 32 x 32 (four waves, one per SIMD with 512 registers; or eight, two per SIMD, on half-size tiles; or
// twelve / sixteen, with two threads per row, kHalf).  Each 16-Gaussian step, every thread loads 64 B of one or two
// feature rows (of G or X) -- 32 B of one row with two threads per row --, splits
// them into the three bf16 planes ONCE and writes them to LDS in the MFMA operand layout; the waves then read their
// A (G) and B (X) fragments from there: [row][plane * 2 + h] slots of 16 B, 7 slots per row (112 B: the 16 lanes
// of a b128 read hit 16 distinct bank quads).  Double-buffered: step s + 1 is staged while step s is multiplied.
constexpr int kWgSlots = 7;

template <int NRB, int KRB, int TNB, int TKB>
struct WgradShape {
    static constexpr int TN = NRB / TNB, TK = KRB / TKB, WAVES = TN * TK;
    static_assert(TN * TNB == NRB && TK * TKB == KRB && WAVES <= 16, "wgrad tiling");
    static constexpr int ROWS = 32 * (NRB + KRB);                       // G rows then X rows
    static constexpr int THREADS = 64 * WAVES;
    static constexpr int RPT = (ROWS + THREADS - 1) / THREADS;          // rows staged per thread
};

__device__ __forceinline__ void stage_row(const float (&raw)[16], int p0, int P, bf16x8* __restrict__ slot,
                                          float* bsum) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = p0 + j < P ? raw[j] : 0.f;   // Gaussians past P contribute nothing
    if (bsum) {
#pragma unroll
        for (int j = 0; j < 16; ++j) *bsum += v[j];
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        float w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = v[8 * hh + j];
        const Split8 sp = split8(w);
        slot[0 + hh] = sp.hi;
        slot[2 + hh] = sp.mid;
        slot[4 + hh] = sp.lo;
    }
}

template <int NRB, int KRB, int TNB, int TKB>
__global__ __launch_bounds__(64 * ((NRB / TNB) * (KRB / TKB)))
__attribute__((amdgpu_waves_per_eu((NRB / TNB) * (KRB / TKB) > 8 ? 4 : ((NRB / TNB) * (KRB / TKB) > 4 ? 2 : 1))))
void k_mlp_wgrad(MlpWgradParams p) {
    typedef WgradShape<NRB, KRB, TNB, TKB> S;
    __shared__ bf16x8 s_op[2][S::ROWS][kWgSlots];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31, wave = tid >> 6;
    const int tn = wave / S::TK, tk = wave % S::TK;
    const int p_lo = blockIdx.x * p.chunk, p_hi = min(p.P, p_lo + p.chunk);
    // the rows this thread stages: r = tid + THREADS i; G row r (< 32 NRB) or X row r - 32 NRB
    const float* src[S::RPT];
    float bsum[S::RPT];
#pragma unroll
    for (int i = 0; i < S::RPT; ++i) {
        // (with two threads per row, kHalf below, thread t stages row t / 2)
        const int r = (S::RPT == 1 && S::THREADS >= 2 * S::ROWS && S::WAVES > 8) ? min(tid >> 1, S::ROWS - 1)
                                                                                  : tid + S::THREADS * i;
        bsum[i] = 0.f;
        if (r < 32 * NRB) src[i] = p.G + (size_t)r * p.ldp;
        else {
            const int k = r - 32 * NRB;
            src[i] = k < 32 * p.k_rb0 ? p.X0 + (size_t)k * p.ldp : p.X1 + (size_t)(k - 32 * p.k_rb0) * p.ldp;
        }
    }
    // Each row's 32 Gaussians of two steps are loaded together (eight 16-B loads: whole 128-B lines; one 64-B
    // segment per row and step ran the staging at ~2.8 TB/s), and split + written to LDS one step ahead: step s + 1
    // is staged while step s multiplies.
    // (One row per thread only: with more, e.g. layer 5's 576 rows on 256 threads, the pair of steps in registers
    // spills, so those shapes keep one 16-Gaussian segment per row and step, loaded two steps ahead.)
    constexpr bool kWide = S::RPT == 1 && S::WAVES <= 8;
#ifndef GSD_WGRAD_WHOLE_ROWS
    constexpr bool kHalf = !kWide && S::RPT == 1 && S::THREADS >= 2 * S::ROWS;
#else
    constexpr bool kHalf = false;
#endif
    constexpr int kWid = kWide ? 32 : 16;
    float raw[S::RPT][kWid];
    auto load_into = [&](float (&dst)[S::RPT][kWid], int p0) {
#pragma unroll
        for (int i = 0; i < S::RPT; ++i)
            if (tid + S::THREADS * i < S::ROWS) {
#pragma unroll
                for (int q = 0; q < kWid / 4; ++q) {
                    const float4 f = *reinterpret_cast<const float4*>(src[i] + p0 + 4 * q);
                    dst[i][4 * q] = f.x; dst[i][4 * q + 1] = f.y; dst[i][4 * q + 2] = f.z; dst[i][4 * q + 3] = f.w;
                }
            }
    };
    auto load = [&](int p0) { load_into(raw, p0); };
    auto write_from = [&](const float (&srcv)[S::RPT][kWid], int p0, int buf, int half) {   // half: compile-time
#pragma unroll
        for (int i = 0; i < S::RPT; ++i) {
            const int r = tid + S::THREADS * i;
            if (r < S::ROWS) {
                float v[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = srcv[i][16 * half + j];
                stage_row(v, p0, p_hi, s_op[buf][r], r < 32 * NRB ? &bsum[i] : nullptr);
            }
        }
    };
    auto write = [&](int p0, int buf, int half) { write_from(raw, p0, buf, half); };
    f32x16 acc[TNB][TKB];
#pragma unroll
    for (int i = 0; i < TNB; ++i)
#pragma unroll
        for (int j = 0; j < TKB; ++j) acc[i][j] = f32x16{};
    // one step's multiply: the fragments from LDS buffer bf, six MFMAs per block pair
#define GSD_WGRAD_MMA(bf)                                                                                       \
    do {                                                                                                        \
        Split8 a_[TNB], b_[TKB];                                                                                \
        _Pragma("unroll") for (int i = 0; i < TNB; ++i) {                                                       \
            const bf16x8* sl = s_op[bf][32 * (TNB * tn + i) + c];                                               \
            a_[i].hi = sl[0 + h]; a_[i].mid = sl[2 + h]; a_[i].lo = sl[4 + h];                                  \
        }                                                                                                       \
        _Pragma("unroll") for (int j = 0; j < TKB; ++j) {                                                       \
            const bf16x8* sl = s_op[bf][32 * NRB + 32 * (TKB * tk + j) + c];                                    \
            b_[j].hi = sl[0 + h]; b_[j].mid = sl[2 + h]; b_[j].lo = sl[4 + h];                                  \
        }                                                                                                       \
        _Pragma("unroll") for (int i = 0; i < TNB; ++i)                                                         \
            _Pragma("unroll") for (int j = 0; j < TKB; ++j) acc[i][j] = mfma_x6_abl<GSD_ABLATE & 16>(a_[i], b_[j], acc[i][j]); \
    } while (0)
    if constexpr (kWide) {
        load(p_lo);   // the chunk starts on a 32-Gaussian boundary; reads up to ldp stay inside the padded rows
        write(p_lo, 0, 0);
        __syncthreads();
        // the two waves of a SIMD (w and w + 4) take the step's two phases in opposite orders, so that one's
        // staging VALU runs beside the other's MFMAs instead of both staging, then both multiplying.  The next
        // pair is loaded right after its predecessor's second half is staged (a second register set loading two
        // steps earlier measured slower: 0.77 -> 0.79 ms per 256 x 256 layer, 0.33 -> 0.41 ms for 64 x 256)
        const bool mma_first = S::WAVES == 8 && (wave & 4);
        int buf = 0;
        for (int pb2 = p_lo; pb2 < p_hi; pb2 += 32) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int pb = pb2 + 16 * hh;
                if (pb < p_hi) {   // workgroup-uniform
                    if (mma_first) GSD_WGRAD_MMA(buf);
                    if (pb + 16 < p_hi) {
                        write(pb + 16, buf ^ 1, hh ^ 1);
                        if (hh == 0 && pb2 + 32 < p_hi) load(pb2 + 32);
                    }
                    if (!mma_first) GSD_WGRAD_MMA(buf);
                    __syncthreads();
                    buf ^= 1;
                }
            }
        }
    } else if constexpr (kHalf) {
        // two threads per row, eight Gaussians each: every wave stages (sixteen waves for 512 rows), instead of half
        // of them staging whole 16-Gaussian segments while the other half only multiplies
        const int r = tid >> 1, hv = tid & 1;
        const bool stager = r < S::ROWS;   // (threads past twice the rows only multiply)
        const float* row = src[0];
        float rh[8];
        auto loadh = [&](int p0) {
            if (!stager) return;
            const float4 a = *reinterpret_cast<const float4*>(row + p0 + 8 * hv);
            const float4 b = *reinterpret_cast<const float4*>(row + p0 + 8 * hv + 4);
            rh[0] = a.x; rh[1] = a.y; rh[2] = a.z; rh[3] = a.w; rh[4] = b.x; rh[5] = b.y; rh[6] = b.z; rh[7] = b.w;
        };
        auto writeh = [&](int p0, int bf) {
            if (!stager) return;
            float w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = p0 + 8 * hv + j < p_hi ? rh[j] : 0.f;
            if (r < 32 * NRB) {
#pragma unroll
                for (int j = 0; j < 8; ++j) bsum[0] += w[j];
            }
            const Split8 sp = split8(w);
            s_op[bf][r][0 + hv] = sp.hi;
            s_op[bf][r][2 + hv] = sp.mid;
            s_op[bf][r][4 + hv] = sp.lo;
        };
        int buf = 0;
        loadh(p_lo);
        writeh(p_lo, 0);
        if (p_lo + 16 < p_hi) loadh(p_lo + 16);
        __syncthreads();
        for (int pb = p_lo; pb < p_hi; pb += 16, buf ^= 1) {
            if (pb + 16 < p_hi) {
                writeh(pb + 16, buf ^ 1);
                if (pb + 32 < p_hi) loadh(pb + 32);
            }
            GSD_WGRAD_MMA(buf);
            __syncthreads();
        }
        bsum[0] += __shfl_xor(bsum[0], 1);   // the row's two halves
    } else {
        int buf = 0;
        load(p_lo);
        write(p_lo, 0, 0);
        if (p_lo + 16 < p_hi) load(p_lo + 16);
        __syncthreads();
        for (int pb = p_lo; pb < p_hi; pb += 16, buf ^= 1) {
            if (pb + 16 < p_hi) {
                write(pb + 16, buf ^ 1, 0);
                if (pb + 32 < p_hi) load(pb + 32);
            }
            GSD_WGRAD_MMA(buf);
            __syncthreads();
        }
    }
#undef GSD_WGRAD_MMA
    // partial[chunk][n][k], n = 32 (TNB tn + i) + 8 (q >> 2) + 4 h + (q & 3), k = 32 (TKB tk + j) + c
    float* out = p.partial + (size_t)blockIdx.x * (32 * NRB) * (32 * KRB);
#pragma unroll
    for (int i = 0; i < TNB; ++i) {
#pragma unroll
        for (int j = 0; j < TKB; ++j) {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int n = 32 * (TNB * tn + i) + 8 * (q >> 2) + 4 * h + (q & 3);
                const int k = 32 * (TKB * tk + j) + c;
                out[(size_t)n * (32 * KRB) + k] = acc[i][j][q];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < S::RPT; ++i) {   // the bias gradient: the G rows' sums over this chunk
        if constexpr (kHalf) {
            const int r = tid >> 1;
            if (r < 32 * NRB && !(tid & 1)) p.bias_partial[(size_t)blockIdx.x * (32 * NRB) + r] = bsum[i];
        } else {
            const int r = tid + S::THREADS * i;
            if (r < 32 * NRB) p.bias_partial[(size_t)blockIdx.x * (32 * NRB) + r] = bsum[i];
        }
    }
}

// dW[n][k] = sum over the chunks of partial[chunk][n][k], in a fixed order (deterministic), scattered into the
// reference-shaped pieces (padded columns and rows dropped); in the same launch the bias gradient likewise (the first
// b_blocks workgroups, dispatched first: eight workgroups, each a 489-deep chain of loads, took ~9.5 us in a launch
// of their own, and as the last blocks of this one they ran after the weights' instead of beside).  A workgroup
// owns 32 consecutive outputs; its 8 thread groups sum the chunks c = g, g + 8, ... (loads four chunks ahead) and the
// 8 group sums are combined in group order through LDS.
struct WgradReduceJob {
    int n_rows, k_cols, k_off;
    const float* partial;
    MlpWeightRef dst;
};
__device__ __forceinline__ void wgrad_reduce_block(int n_chunks, const WgradReduceJob& j, int blk, int accumulate,
                                                   float (*red)[32]) {
    const long long n_el = (long long)j.n_rows * j.k_cols;
    const int grp = threadIdx.x >> 5, l = threadIdx.x & 31;
    const long long e = (long long)blk * 32 + l;
    const float* __restrict__ partial = j.partial;
    float s = 0.f;
    if (e < n_el) {
        int c = grp;
        for (; c + 24 < n_chunks; c += 32) {
            const float a = partial[(size_t)c * n_el + e], bb = partial[(size_t)(c + 8) * n_el + e];
            const float d = partial[(size_t)(c + 16) * n_el + e], f = partial[(size_t)(c + 24) * n_el + e];
            s += a; s += bb; s += d; s += f;
        }
        for (; c < n_chunks; c += 8) s += partial[(size_t)c * n_el + e];
    }
    red[grp][l] = s;
    __syncthreads();
    if (grp == 0 && e < n_el) {
        float t = red[0][l];
#pragma unroll
        for (int g = 1; g < 8; ++g) t += red[g][l];
        const int n = (int)(e / j.k_cols), k = (int)(e - (long long)n * j.k_cols);
        float* d = mlp_elem(j.dst, n, mlp_col(j.dst.map, j.k_off + k));
        if (d) *d = accumulate ? *d + t : t;
    }
}
// (two call sites on the kernel arguments themselves: a selected reference to one of them put the job in scratch)
__global__ __launch_bounds__(256) void k_mlp_wgrad_reduce(int n_chunks, WgradReduceJob w, WgradReduceJob b,
                                                          int b_blocks, int accumulate) {
    __shared__ float red[8][32];
    if ((int)blockIdx.x < b_blocks) wgrad_reduce_block(n_chunks, b, blockIdx.x, accumulate, red);
    else wgrad_reduce_block(n_chunks, w, blockIdx.x - b_blocks, accumulate, red);
}

void launch_mlp_pack(const MlpPackParams& p, hipStream_t s) {
    const int n = (p.K / 16) * (p.M / 32) * 64;
    hipLaunchKernelGGL(k_mlp_pack, dim3((n + 255) / 256), dim3(256), 0, s, p);
}
void launch_mlp_pack_batch(const MlpPackBatch& b, hipStream_t s) {
    int n = 0;
    for (int i = 0; i < b.n; ++i) n = std::max(n, (b.job[i].K / 16) * (b.job[i].M / 32) * 64);
    if (b.n > 0) hipLaunchKernelGGL(k_mlp_pack_multi, dim3((n + 255) / 256, b.n), dim3(256), 0, s, b);
}

void launch_mlp_encode(int P, int ldp, const float* x, const float* t, float* E, float* ET, hipStream_t s) {
    hipLaunchKernelGGL(k_mlp_encode, dim3((ldp + 255) / 256), dim3(256), 0, s, P, ldp, x, t, E, ET);
}

void launch_mlp_encode_bwd(int P, int ldp, const float* E, const float* dE, float* dx, int accumulate, hipStream_t s) {
    if (P > 0) hipLaunchKernelGGL(k_mlp_encode_bwd, dim3((P + 255) / 256), dim3(256), 0, s, P, ldp, E, dE, dx, accumulate);
}

// the 320-row backward of layer 5 as two workgroup rows of 5 row blocks (grid.y): 2 waves per SIMD instead of one
// (1.72 ms with all 10 row blocks per workgroup)
template <int MODE>
static void launch_gemm_rb(const MlpGemmParams& p, hipStream_t s) {
    switch (p.rb) {   // 320 rows (layer 5's W^T): two workgroup rows of 5 blocks
        case 2: hipLaunchKernelGGL((k_mlp_gemm_dma<MODE, 2>), dim3(p.ldp / 256), dim3(512), 0, s, p); break;
        case 3: hipLaunchKernelGGL((k_mlp_gemm_dma<MODE, 3>), dim3(p.ldp / 256), dim3(512), 0, s, p); break;
        case 8: hipLaunchKernelGGL((k_mlp_gemm_dma<MODE, 8>), dim3(p.ldp / 256), dim3(512), 0, s, p); break;
        case 10: hipLaunchKernelGGL((k_mlp_gemm_dma<MODE, 5>), dim3(p.ldp / 256, 2), dim3(512), 0, s, p); break;
        default: break;
    }
}

void launch_mlp_fwd_fused(const MlpFusedParams& p, hipStream_t s, bool store) {
    if (p.P <= 0) return;
    if (store) hipLaunchKernelGGL(k_mlp_fwd_fused<true>, dim3(p.ldp / 128), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_mlp_fwd_fused<false>, dim3(p.ldp / 128), dim3(256), 0, s, p);
}
void launch_mlp_fwd_fused16(const MlpFusedParams& p, hipStream_t s, bool store) {
    if (p.P <= 0) return;
    if (store) hipLaunchKernelGGL(k_mlp_fwd_fused16<true>, dim3(p.ldp / 128), dim3(512), 0, s, p);
    else hipLaunchKernelGGL(k_mlp_fwd_fused16<false>, dim3(p.ldp / 128), dim3(512), 0, s, p);
}

void launch_mlp_bwd_chain(const MlpChainParams& p, hipStream_t s) {
    if (p.P > 0) hipLaunchKernelGGL(k_mlp_bwd_chain, dim3(p.ldp / 128), dim3(256), 0, s, p);
}
void launch_mlp_bwd_chain16(const MlpChainParams& p, hipStream_t s) {
    if (p.P > 0) hipLaunchKernelGGL(k_mlp_bwd_chain16, dim3(p.ldp / 128), dim3(512), 0, s, p);
}

void launch_mlp_gemm(const MlpGemmParams& p, int mode, hipStream_t s) {
    if (mode == kMlpFwdRelu) launch_gemm_rb<kMlpFwdRelu>(p, s);
    else if (mode == kMlpFwdHeads) launch_gemm_rb<kMlpFwdHeads>(p, s);
    else launch_gemm_rb<kMlpBwdMask>(p, s);
}

void launch_mlp_wgrad(const MlpWgradParams& p_in, const MlpWeightRef& dst, const MlpWeightRef& dst_b, hipStream_t s) {
    MlpWgradParams p = p_in;
    // 256 x 256: one workgroup per CU (114 KB of LDS), so the chunk grows to cover P in ONE round of 256 workgroups
    // (never past the caller's chunk count, which sizes the partial buffers): 0.732 -> 0.708 ms per layer at 1M (no
    // second, 91 %-full round) and its reduction over 255 partials instead of 489, ~9 us instead of ~24
    // (profiles/round5/deform_mlp_wgrad/; GSD_WGRAD_ROUND1=0 keeps the 2048-Gaussian chunks)
    static const bool round1 = [] {
        const char* e = getenv("GSD_WGRAD_ROUND1");
        return !(e && strcmp(e, "0") == 0);
    }();
    if (round1 && p.n_rb == 8 && p.k_rb == 8)
        p.chunk = std::max(p.chunk, (int)(((long long)p.P + 256 * 32 - 1) / (256 * 32)) * 32);
    const int n_chunks = (p.P + p.chunk - 1) / p.chunk;
    const dim3 grid(n_chunks);
#define GSD_WGRAD(N, K, TN, TK)                                                                            \
    if (p.n_rb == N && p.k_rb == K)                                                                        \
        hipLaunchKernelGGL((k_mlp_wgrad<N, K, TN, TK>), grid, dim3(64 * WgradShape<N, K, TN, TK>::WAVES), 0, s, p);
    // eight waves of half-size tiles, two per SIMD (8 x 8 at P = 1M: 0.92 ms per layer against 1.18 for four waves of
    // 4 x 4 blocks, one per SIMD: the second wave per SIMD hides the staging waits)
    // (layer 5's 320 columns run as two calls, 64 + 256, both on the wide-load 8-wave shapes: 1.47 ms as one call)
    // 256 x 256: sixteen waves of 2 x 2 blocks (four per SIMD, 128 registers, 16-Gaussian loads) -- 0.73 ms per
    // layer at 1M against 0.76 for eight waves of 4 x 2 (two per SIMD, 216 registers, 32-Gaussian loads), which
    // GSD_WGRAD16=0 keeps
    static const bool w16 = [] {
        const char* e = getenv("GSD_WGRAD16");
        return !(e && strcmp(e, "0") == 0);
    }();
    // (round 4, whole-row staging: the narrow shapes with three or four waves per SIMD were slower -- 64 x 256 as 16
    // waves of one block 0.40 ms against 0.30, 256 x 96 as 12 waves of 2 x 1 blocks 0.45 against 0.43)
    if (w16 && p.n_rb == 8 && p.k_rb == 8)
        hipLaunchKernelGGL((k_mlp_wgrad<8, 8, 2, 2>), grid, dim3(64 * WgradShape<8, 8, 2, 2>::WAVES), 0, s, p);
    // Round 5: with two threads staging each row (kHalf in k_mlp_wgrad: every wave stages eight Gaussians of a row
    // per step, instead of half the waves staging whole 16-Gaussian segments while the rest only multiply), the wide
    // shapes pay too: 256 x 256 0.715 -> 0.633 ms, 256 x 96 as twelve waves of 2 x 1 blocks 0.445 -> 0.36, 64 x 256 and
    // 256 x 64 as sixteen waves of one block 0.31 -> 0.295 (profiles/round5/deform_mlp_wgrad/r5aq/);
    // GSD_WGRAD_NARROW_OLD keeps the round-4 narrow shapes
#ifndef GSD_WGRAD_NARROW_OLD
    else GSD_WGRAD(8, 8, 4, 2) else GSD_WGRAD(8, 2, 1, 1) else GSD_WGRAD(8, 10, 4, 5) else GSD_WGRAD(8, 3, 2, 1)
    else GSD_WGRAD(2, 8, 1, 1)
#else
    else GSD_WGRAD(8, 8, 4, 2) else GSD_WGRAD(8, 2, 2, 1) else GSD_WGRAD(8, 10, 4, 5) else GSD_WGRAD(8, 3, 2, 3)
    else GSD_WGRAD(2, 8, 1, 2)
#endif
#undef GSD_WGRAD
    const long long nw = (long long)(32 * p.n_rb) * (32 * p.k_rb);
    const int w_blocks = (int)((nw + 31) / 32), b_blocks = p.skip_bias ? 0 : (32 * p.n_rb + 31) / 32;
    const WgradReduceJob wj{32 * p.n_rb, 32 * p.k_rb, p.k_off, (const float*)p.partial, dst};
    const WgradReduceJob bj{32 * p.n_rb, 1, 0, (const float*)p.bias_partial, dst_b};
    hipLaunchKernelGGL(k_mlp_wgrad_reduce, dim3((unsigned)(w_blocks + b_blocks)), dim3(256), 0, s, n_chunks, wj, bj,
                       b_blocks, p.accumulate);
}

void launch_mlp_rows_to_features(int P, int ldp, const MlpHeadsIn& src, float* dst, int dst_rows, hipStream_t s) {
    hipLaunchKernelGGL(k_mlp_rows_to_features, dim3(ldp / 64), dim3(256), 0, s, P, ldp, src, dst, dst_rows);
}

void launch_mlp_gather_bias(const MlpWeightRef& b, float* dst, int n_pad, hipStream_t s) {
    hipLaunchKernelGGL(k_mlp_gather_bias, dim3((n_pad + 255) / 256), dim3(256), 0, s, b, dst, n_pad);
}

}  // namespace gsd
