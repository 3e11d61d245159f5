// gsd_mlp.hip -- the deformation network's forward (DirectTemporalNeRF, scene/gaussian_model.py:242-316 with the
// positional encoding of :33-82) fused into one kernel on the bf16 matrix cores: the evaluation the module runs
// under autocast-bf16 (gsd_amd.deform_mlp, dtype=torch.bfloat16), without autograd.
//
// torch runs it layer by layer: each of the nine GEMMs streams a (P, 256) activation through HBM (0.5 GB per
// layer at P = 1M in bf16, ~4.7 ms in all).  Here one wave owns 32 Gaussians from the encoding to the heads and
// keeps every activation in registers: a layer's output is computed transposed, Y^T = W X^T, on
// v_mfma_f32_32x32x16_bf16 with the weights as the A operand (rows = output features) and the activations as
// the B operand (columns = the wave's 32 Gaussians), so the f32 accumulator tile of one layer -- its column
// (Gaussian) on the lane, its rows (features) in the 16 registers -- becomes, after bias, ReLU and the bf16
// conversion, the B operand of the next layer with no lane movement and no LDS.  The k order inside each
// 16-wide k-step is then permuted (element j of lane half h is feature 8(j>>2) + 4h + (j&3) of the step); the
// host packs the weights with the same permutation (gsd_amd.deform_mlp.pack_fused_mlp).  The weights (1008 KB
// in bf16) are read as A fragments straight from L2: 1 KB per wave per k-step and row block, coalesced, one
// k-step ahead.  Two waves per SIMD (256 registers each).
//
// Layers (k-steps KS of 16 inputs x row blocks RB of 32 outputs):
//   0      cat(enc(x) 63, enc(t) 21) = 84 -> 96 (natural order)       KS  6, RB 8
//   1-4    256                                                        KS 16, RB 8
//   5      cat(enc(x) 63 -> 64 (natural, weight column 63 zero), h)   KS 20, RB 8
//   6-7    256                                                        KS 16, RB 8
//   heads  dx 3 | d log-scale 3 | d quaternion 4 | dSH 48 = 58 -> 64  KS 16, RB 2
// Bias + ReLU in f32 on the accumulators, each activation rounded to bf16 (as autocast's bf16 GEMM outputs);
// the heads' outputs rounded to bf16 and returned as f32 (the module's .float()).
#include <cstdlib>

#include "gsd_kernels.h"

namespace gsd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#ifndef GSD_MLP_PREFETCH1
#define GSD_MLP_PREFETCH1 1
#endif
constexpr int kMlpPrefetch1 = GSD_MLP_PREFETCH1;  // NC = 1: k-steps of weight fragments in flight

__host__ __device__ constexpr int mlp_ks(int l) { return l == 0 ? 6 : (l == 5 ? 20 : 16); }
__host__ __device__ constexpr int mlp_rb(int l) { return l == kMlpLayers - 1 ? 2 : 8; }
__host__ __device__ constexpr int mlp_frag_off(int l) {
    int o = 0;
    for (int i = 0; i < l; ++i) o += mlp_ks(i) * mlp_rb(i) * 64;
    return o;
}
__host__ __device__ constexpr int mlp_bias_off(int l) {
    int o = 0;
    for (int i = 0; i < l; ++i) o += mlp_rb(i) * 32;
    return o;
}
static_assert(mlp_frag_off(kMlpLayers) == kMlpFrags, "fragment count");
static_assert(mlp_bias_off(kMlpLayers) == kMlpBias, "bias count");

// Feature k of cat(positional_encoding(x), positional_encoding(t)) (gaussian_model.py:33-82: [v, sin(2^i v),
// cos(2^i v)]_{i<10} with the (sin, cos) pair of frequency i over the coordinates: 3 + 6 i + 3 s + d); 0 past 84.
__device__ __forceinline__ float enc_feature(int k, float x0, float x1, float x2, float t) {
    if (k < 3) return k == 0 ? x0 : (k == 1 ? x1 : x2);
    if (k < 63) {
        const int kk = k - 3, i = kk / 6, r = kk - 6 * i, s = r / 3, d = r - 3 * s;
        const float a = ldexpf(d == 0 ? x0 : (d == 1 ? x1 : x2), i);  // x * 2^i, exact as torch's x * freqs
        return s ? cosf(a) : sinf(a);
    }
    if (k < 84) {
        const int e = k - 63;
        if (e == 0) return t;
        const int i = (e - 1) >> 1, s = (e - 1) & 1;
        const float a = ldexpf(t, i);
        return s ? cosf(a) : sinf(a);
    }
    return 0.f;
}

// acc[c][rb] = sum over the k-steps of W-fragment(ks, rb) x in_c(ks), for the wave's NC column blocks of 32
// Gaussians (each A fragment feeds NC MFMAs); the first KS0 steps from in0, the rest from in1.  The fragments of a
// layer are laid out [ks][rb][lane] (one 1-KB wave load each, a k-step's RB of them contiguous); the next k-step's
// are loaded while this one's MFMAs run, and a scheduling barrier per k-step keeps the compiler from hoisting the
// whole layer's loads (which took every register and spilled).  (Sharing each k-step's fragments among the
// workgroup's four waves through an LDS double buffer, one barrier per step, was slower: 2.32 ms against 1.75 at
// P = 1M, NC = 1.)
template <int NC, int KS0, int KS1, int RB>
__device__ __forceinline__ void mlp_layer(const bf16x8* __restrict__ w, const bf16x8 (&in0)[NC][KS0 > 0 ? KS0 : 1],
                                          const bf16x8 (&in1)[NC][KS1 > 0 ? KS1 : 1], f32x16 (&acc)[NC][RB],
                                          int lane) {
    constexpr int KS = KS0 + KS1;
    constexpr int D = NC == 1 ? kMlpPrefetch1 : 1;  // k-steps of fragments in flight (registers: D x RB x 4)
    const bf16x8* wl = w + lane;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[c][rb] = f32x16{};
    bf16x8 a[D + 1][RB];  // ring: step ks reads slot ks % (D + 1)
#pragma unroll
    for (int d = 0; d < D && d < KS; ++d)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) a[d][rb] = wl[(d * RB + rb) * 64];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        if (ks + D < KS) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) a[(ks + D) % (D + 1)][rb] = wl[((ks + D) * RB + rb) * 64];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const bf16x8 b = ks < KS0 ? in0[c][ks < KS0 ? ks : 0] : in1[c][ks >= KS0 ? ks - KS0 : 0];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
                acc[c][rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks % (D + 1)][rb], b, acc[c][rb], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// bias (packed per lane: [rb][h][reg]), ReLU, bf16: accumulator registers 8 s .. 8 s + 7 of row block rb become
// k-step 2 rb + s of the next layer's B operand
template <int NC>
__device__ __forceinline__ void mlp_hidden_epilogue(const f32x16 (&acc)[NC][8], const float* __restrict__ bias, int h,
                                                    bf16x8 (&act)[NC][16]) {
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
        const float4* bq = reinterpret_cast<const float4*>(bias + (rb * 2 + h) * 16);
        float bv[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v = bq[q];
            bv[4 * q] = v.x;
            bv[4 * q + 1] = v.y;
            bv[4 * q + 2] = v.z;
            bv[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    act[c][2 * rb + s][j] = (__bf16)relu_nan(acc[c][rb][8 * s + j] + bv[8 * s + j]);
    }
}

// NC column blocks of 32 Gaussians per wave (1 or 2).  NC = 1 fits 256 registers (5 spilled), so two waves per
// SIMD hide each other's stalls: 1.33 ms at P = 1M.  NC = 2 halves the weight traffic from L2 per MFMA but needs
// ~500 registers, one wave per SIMD: 1.57 ms.
template <int NC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NC == 1 ? 2 : 1))) void k_mlp_fwd(MlpParams p) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int g0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 * NC + (lane & 31);  // column block c: g0 + 32 c
    // The encoding, 96 bf16 features per Gaussian, through LDS: lane half h computes features [48 h, 48 h + 48)
    // of its Gaussians in a loop (one inlined copy of sinf / cosf: 96 unrolled copies spilled ~700 SGPRs), then
    // the B operand of layer 0 (and the encoding's k-steps of layer 5) is read back in natural k order -- lane
    // half h holds features 16 ks + 8 h + j.
    __shared__ __attribute__((aligned(16))) __bf16 s_enc[4][32 * NC][96];
    __bf16(*my)[96] = s_enc[threadIdx.x >> 6];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int g = g0 + 32 * c;
        float x0 = 0.f, x1 = 0.f, x2 = 0.f, t = 0.f;
        if (g < p.P) {
            x0 = p.x[3 * g];
            x1 = p.x[3 * g + 1];
            x2 = p.x[3 * g + 2];
            t = p.t[g];
        }
#pragma unroll 1
        for (int k = 48 * h; k < 48 * h + 48; ++k) my[32 * c + (lane & 31)][k] = (__bf16)enc_feature(k, x0, x1, x2, t);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bf16x8* W = reinterpret_cast<const bf16x8*>(p.frags);
    f32x16 acc[NC][8];
    bf16x8 act[NC][16];
    const bf16x8 none[NC][1] = {};
    {
        bf16x8 enc[NC][6];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int ks = 0; ks < 6; ++ks)
                enc[c][ks] = *reinterpret_cast<const bf16x8*>(&my[32 * c + (lane & 31)][16 * ks + 8 * h]);
        mlp_layer<NC, 6, 0, 8>(W + mlp_frag_off(0), enc, none, acc, lane);
    }
    mlp_hidden_epilogue<NC>(acc, p.bias + mlp_bias_off(0), h, act);
#pragma unroll
    for (int l = 1; l < 8; ++l) {
        if (l == 5) {  // cat(enc(x), h): the encoding's first four k-steps (feature 63 = t meets a zero weight column)
            bf16x8 ex[NC][4];
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int ks = 0; ks < 4; ++ks)
                    ex[c][ks] = *reinterpret_cast<const bf16x8*>(&my[32 * c + (lane & 31)][16 * ks + 8 * h]);
            mlp_layer<NC, 4, 16, 8>(W + mlp_frag_off(5), ex, act, acc, lane);
        } else {
            mlp_layer<NC, 0, 16, 8>(W + mlp_frag_off(l), none, act, acc, lane);
        }
        mlp_hidden_epilogue<NC>(acc, p.bias + mlp_bias_off(l), h, act);
    }
    f32x16 out[NC][2];
    mlp_layer<NC, 0, 16, 2>(W + mlp_frag_off(8), none, act, out, lane);
    const float* bh = p.bias + mlp_bias_off(8);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int g = g0 + 32 * c;
        if (g >= p.P) continue;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int f = 32 * rb + (reg & 3) + 8 * (reg >> 2) + 4 * h;  // this register's output feature
                const float v = (float)(__bf16)(out[c][rb][reg] + bh[(rb * 2 + h) * 16 + reg]);
                if (f < 3) p.d_xyz[3 * g + f] = v;
                else if (f < 6) p.d_scale[3 * g + f - 3] = v;
                else if (f < 10) p.d_rot[4 * g + f - 6] = v;
                else if (f < 58) p.d_sh[48 * g + f - 10] = v;
            }
    }
}

void launch_mlp_fwd(const MlpParams& p, hipStream_t s) {
    if (p.P <= 0) return;
    static const int nc = [] {  // GSD_MLP_NC: column blocks per wave (experiment)
        const char* e = getenv("GSD_MLP_NC");
        return e && atoi(e) == 2 ? 2 : 1;
    }();
    const int per_block = 4 * 32 * nc;
    const dim3 grid((p.P + per_block - 1) / per_block);
    if (nc == 1) hipLaunchKernelGGL(k_mlp_fwd<1>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_mlp_fwd<2>, grid, dim3(256), 0, s, p);
}

}  // namespace gsd

namespace gsd {

// ---- the deformation network's backward, between its GEMMs (gsd_amd.deform_mlp._Linear.backward) ----
// g = gy where y > 0 (ReLU backward; every element when y is null) and the bias gradient's per-block column sums,
// in one pass: torch ran threshold_backward and then sum(0) over g, reading the (P, N) gradient twice.  A
// workgroup owns `rows` consecutive rows; a thread owns a column pair of every (256 / (N/2))-th row of them and
// keeps its two sums in float32; the row lanes are combined through LDS in a fixed order, so part[block][c] is
// deterministic and the caller's sum over blocks is too.
template <typename T>
struct Pair;
template <>
struct Pair<float> {
    typedef float2 V;
    __device__ static float lo(V v) { return v.x; }
    __device__ static float hi(V v) { return v.y; }
    __device__ static V zero() { return make_float2(0.f, 0.f); }
    __device__ static V select(V v, V y, bool relu) {
        return relu ? make_float2(y.x > 0.f ? v.x : 0.f, y.y > 0.f ? v.y : 0.f) : v;
    }
};
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
template <>
struct Pair<__bf16> {
    typedef bf16x2 V;
    __device__ static float lo(V v) { return (float)v.x; }
    __device__ static float hi(V v) { return (float)v.y; }
    __device__ static V zero() { return V{}; }
    __device__ static V select(V v, V y, bool relu) {
        if (!relu) return v;
        V r = v;
        if (!((float)y.x > 0.f)) r.x = (__bf16)0.f;
        if (!((float)y.y > 0.f)) r.y = (__bf16)0.f;
        return r;
    }
};

template <typename T>
__global__ __launch_bounds__(256) void k_relu_bwd_bias(long long P, int N, const T* __restrict__ gy,
                                                        const T* __restrict__ y, T* __restrict__ g,
                                                        float* __restrict__ part, int rows) {
    typedef typename Pair<T>::V V;
    __shared__ float2 red[256];
    const int half = N >> 1, lanes = 256 / half;  // threads per row, rows per pass
    const int tid = threadIdx.x, cp = tid % half, rl = tid / half;
    const long long r0 = (long long)blockIdx.x * rows, r1 = min(P, r0 + rows);
    float s0 = 0.f, s1 = 0.f;
    const bool relu = y != nullptr;
    if (rl < lanes) {
        const V* gy2 = reinterpret_cast<const V*>(gy);
        const V* y2 = reinterpret_cast<const V*>(y);
        V* g2 = reinterpret_cast<V*>(g);
#pragma unroll 4
        for (long long r = r0 + rl; r < r1; r += lanes) {
            const long long e = r * half + cp;
            const V v = Pair<T>::select(gy2[e], relu ? y2[e] : Pair<T>::zero(), relu);
            g2[e] = v;
            s0 += Pair<T>::lo(v);
            s1 += Pair<T>::hi(v);
        }
    }
    red[tid] = make_float2(s0, s1);
    __syncthreads();
    if (tid < half) {
        float2 a = red[tid];
        for (int l = 1; l < lanes; ++l) {
            const float2 b = red[l * half + tid];
            a.x += b.x;
            a.y += b.y;
        }
        part[(size_t)blockIdx.x * N + 2 * tid] = a.x;
        part[(size_t)blockIdx.x * N + 2 * tid + 1] = a.y;
    }
}

int relu_bwd_bias_blocks(long long P, int rows) { return (int)((P + rows - 1) / rows); }

void launch_relu_bwd_bias(long long P, int N, int bf16, const void* gy, const void* y, void* g, float* part,
                          int rows, hipStream_t s) {
    const int nb = relu_bwd_bias_blocks(P, rows);
    if (nb <= 0) return;
    if (bf16)
        hipLaunchKernelGGL(k_relu_bwd_bias<__bf16>, dim3(nb), dim3(256), 0, s, P, N, (const __bf16*)gy,
                           (const __bf16*)y, (__bf16*)g, part, rows);
    else
        hipLaunchKernelGGL(k_relu_bwd_bias<float>, dim3(nb), dim3(256), 0, s, P, N, (const float*)gy,
                           (const float*)y, (float*)g, part, rows);
}

}  // namespace gsd
