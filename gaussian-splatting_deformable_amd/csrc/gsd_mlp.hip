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
// in bf16) are read as A fragments straight from L2: 1 KB per wave per MFMA, coalesced, one k-step ahead.
//
// Layers (k-steps KS of 16 inputs x row blocks RB of 32 outputs):
//   0      cat(enc(x) 63, enc(t) 21) = 84 -> 96 (natural order)       KS  6, RB 8
//   1-4    256                                                        KS 16, RB 8
//   5      cat(enc(x) 63 -> 64 (natural, weight column 63 zero), h)   KS 20, RB 8
//   6-7    256                                                        KS 16, RB 8
//   heads  dx 3 | d log-scale 3 | d quaternion 4 | dSH 48 = 58 -> 64  KS 16, RB 2
// Bias + ReLU in f32 on the accumulators, each activation rounded to bf16 (as autocast's bf16 GEMM outputs);
// the heads' outputs rounded to bf16 and returned as f32 (the module's .float()).
#include "gsd_kernels.h"

namespace gsd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

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

// acc[rb] = sum over the k-steps of W-fragment(ks, rb) x in(ks); the first KS0 steps from in0, the rest from in1.
// The fragments of a layer are laid out [ks][rb][lane] (one 1-KB wave load each, a k-step's RB of them
// contiguous); the next k-step's are loaded while this one's MFMAs run, and a scheduling barrier per k-step keeps
// the compiler from hoisting the whole layer's loads (which took every register and spilled).
template <int KS0, int KS1, int RB>
__device__ __forceinline__ void mlp_layer(const bf16x8* __restrict__ w, const bf16x8 (&in0)[KS0 > 0 ? KS0 : 1],
                                          const bf16x8 (&in1)[KS1 > 0 ? KS1 : 1], f32x16 (&acc)[RB], int lane) {
    constexpr int KS = KS0 + KS1;
    const bf16x8* wl = w + lane;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x16{};
    bf16x8 a[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) a[rb] = wl[rb * 64];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        bf16x8 an[RB];
        if (ks + 1 < KS) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) an[rb] = wl[((ks + 1) * RB + rb) * 64];
        }
        const bf16x8 b = ks < KS0 ? in0[ks < KS0 ? ks : 0] : in1[ks >= KS0 ? ks - KS0 : 0];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rb], b, acc[rb], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (ks + 1 < KS) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) a[rb] = an[rb];
        }
    }
}

// bias (packed per lane: [rb][h][reg]), ReLU, bf16: accumulator registers 8 s .. 8 s + 7 of row block rb become
// k-step 2 rb + s of the next layer's B operand
__device__ __forceinline__ void mlp_hidden_epilogue(const f32x16 (&acc)[8], const float* __restrict__ bias, int h,
                                                    bf16x8 (&act)[16]) {
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
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) act[2 * rb + s][j] = (__bf16)fmaxf(acc[rb][8 * s + j] + bv[8 * s + j], 0.f);
    }
}

__global__ __launch_bounds__(256) void k_mlp_fwd(MlpParams p) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int g = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + (lane & 31);
    const bool live = g < p.P;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f, t = 0.f;
    if (live) {
        x0 = p.x[3 * g];
        x1 = p.x[3 * g + 1];
        x2 = p.x[3 * g + 2];
        t = p.t[g];
    }
    // The encoding, 96 bf16 features per Gaussian, through LDS: lane half h computes features [48 h, 48 h + 48)
    // of its Gaussian in a loop (one inlined copy of sinf / cosf: 96 unrolled copies spilled ~700 SGPRs), then
    // layer 0's B operand is read back in natural k order -- lane half h holds features 16 ks + 8 h + j.
    __shared__ __attribute__((aligned(16))) __bf16 s_enc[4][32][96];
    __bf16(*my)[96] = s_enc[threadIdx.x >> 6];
#pragma unroll 1
    for (int k = 48 * h; k < 48 * h + 48; ++k) my[lane & 31][k] = (__bf16)enc_feature(k, x0, x1, x2, t);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bf16x8 enc[6];
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) enc[ks] = *reinterpret_cast<const bf16x8*>(&my[lane & 31][16 * ks + 8 * h]);
    const bf16x8* W = reinterpret_cast<const bf16x8*>(p.frags);
    f32x16 acc[8];
    bf16x8 act[16];
    const bf16x8 none[1] = {};
    mlp_layer<6, 0, 8>(W + mlp_frag_off(0), enc, none, acc, lane);
    mlp_hidden_epilogue(acc, p.bias + mlp_bias_off(0), h, act);
#pragma unroll
    for (int l = 1; l < 8; ++l) {
        if (l == 5) {  // cat(enc(x), h): enc's first four k-steps (feature 63 = t meets a zero weight column)
            bf16x8 ex[4] = {enc[0], enc[1], enc[2], enc[3]};
            mlp_layer<4, 16, 8>(W + mlp_frag_off(5), ex, act, acc, lane);
        } else {
            mlp_layer<0, 16, 8>(W + mlp_frag_off(l), none, act, acc, lane);
        }
        mlp_hidden_epilogue(acc, p.bias + mlp_bias_off(l), h, act);
    }
    f32x16 out[2];
    mlp_layer<0, 16, 2>(W + mlp_frag_off(8), none, act, out, lane);
    if (!live) return;
    const float* bh = p.bias + mlp_bias_off(8);
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int f = 32 * rb + (reg & 3) + 8 * (reg >> 2) + 4 * h;  // this register's output feature
            const float v = (float)(__bf16)(out[rb][reg] + bh[(rb * 2 + h) * 16 + reg]);
            if (f < 3) p.d_xyz[3 * g + f] = v;
            else if (f < 6) p.d_scale[3 * g + f - 3] = v;
            else if (f < 10) p.d_rot[4 * g + f - 6] = v;
            else if (f < 58) p.d_sh[48 * g + f - 10] = v;
        }
}

void launch_mlp_fwd(const MlpParams& p, hipStream_t s) {
    if (p.P <= 0) return;
    const int waves = (p.P + 31) / 32;
    hipLaunchKernelGGL(k_mlp_fwd, dim3((waves + 3) / 4), dim3(256), 0, s, p);
}

}  // namespace gsd
