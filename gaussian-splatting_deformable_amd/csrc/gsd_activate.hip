// gsd_activate.hip -- the deform/activation preamble of render(), fused.
//
// Reference: gaussian_renderer/__init__.py:79-140 and
// scene/gaussian_model.py:761-797 build the rasterizer inputs with ~10 torch
// kernels (xyz + dx, exp(s + ds), normalize(q + dq), sigmoid(o),
// cat(f_dc, f_rest) + dSH) and ~12 more in the backward.  Here: two
// HBM-bound kernels each way.  Per Gaussian (SH3, offsets present) the forward
// reads 468 B and writes 236 B; the backward reads 312 B (+ the old grads
// when accumulating) and writes 244 B.
//
// Backward accumulation: the parameter gradients can be added in place into
// existing .grad buffers (the FlatGrads slab), which removes autograd's
// separate AccumulateGrad add kernels.
#include "gsd_kernels.h"

namespace gsd {

__global__ __launch_bounds__(256) void k_activate_fwd(ActivateParams p) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= p.P) return;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float x = p.xyz[3 * i + k] + (p.dxyz ? p.dxyz[3 * i + k] : 0.f);
        p.means_out[3 * i + k] = x;
        const float s = p.scaling[3 * i + k] + (p.dscale ? p.dscale[3 * i + k] : 0.f);
        p.scales_out[3 * i + k] = expf(s);
    }
    float4 q = reinterpret_cast<const float4*>(p.rotation)[i];
    if (p.drot) {
        const float4 d = reinterpret_cast<const float4*>(p.drot)[i];
        q = make_float4(q.x + d.x, q.y + d.y, q.z + d.z, q.w + d.w);
    }
    const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);  // F.normalize
    reinterpret_cast<float4*>(p.rot_out)[i] = make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
    p.opac_out[i] = 1.f / (1.f + expf(-p.opacity[i]));
}

// shs_out (P, 1+R, 3) = cat(f_dc (P,1,3), f_rest (P,R,3)) + dsh; one lane per output float, coalesced.
__global__ __launch_bounds__(256) void k_pack_sh(int P, int R, const float* __restrict__ f_dc,
                                                 const float* __restrict__ f_rest, const float* __restrict__ dsh,
                                                 float* __restrict__ shs) {
    const uint32_t row = 3u * (1u + (uint32_t)R);
    const uint32_t n = (uint32_t)P * row;  // host guarantees P * row < 2^32
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u) {
        const uint32_t g = e / row;
        const uint32_t k = e - g * row;
        float v = k < 3 ? f_dc[(size_t)g * 3 + k] : f_rest[(size_t)g * (3 * R) + (k - 3)];
        if (dsh) v += dsh[e];
        shs[e] = v;
    }
}

__global__ __launch_bounds__(256) void k_activate_bwd(ActivateBwdParams p) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= p.P) return;
    const bool acc = p.accumulate != 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float gm = p.g_means[3 * i + k];
        if (p.g_xyz) p.g_xyz[3 * i + k] = acc ? p.g_xyz[3 * i + k] + gm : gm;
        if (p.g_dxyz) p.g_dxyz[3 * i + k] = gm;
        const float s = expf(p.scaling[3 * i + k] + (p.dscale ? p.dscale[3 * i + k] : 0.f));
        const float gs = p.g_scales[3 * i + k] * s;  // d exp(x)/dx = exp(x)
        if (p.g_scaling) p.g_scaling[3 * i + k] = acc ? p.g_scaling[3 * i + k] + gs : gs;
        if (p.g_dscale) p.g_dscale[3 * i + k] = gs;
    }
    float4 q = reinterpret_cast<const float4*>(p.rotation)[i];
    if (p.drot) {
        const float4 d = reinterpret_cast<const float4*>(p.drot)[i];
        q = make_float4(q.x + d.x, q.y + d.y, q.z + d.z, q.w + d.w);
    }
    const float4 go = reinterpret_cast<const float4*>(p.g_rot)[i];
    const float nraw = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    float4 gq;
    if (nraw > 1e-12f) {  // d(q/|q|)/dq = (I - u u^T)/|q|
        const float inv = 1.f / nraw;
        const float4 u = make_float4(q.x * inv, q.y * inv, q.z * inv, q.w * inv);
        const float ug = u.x * go.x + u.y * go.y + u.z * go.z + u.w * go.w;
        gq = make_float4((go.x - u.x * ug) * inv, (go.y - u.y * ug) * inv, (go.z - u.z * ug) * inv,
                         (go.w - u.w * ug) * inv);
    } else {
        gq = make_float4(go.x * 1e12f, go.y * 1e12f, go.z * 1e12f, go.w * 1e12f);
    }
    if (p.g_rotation) {
        float4* d = reinterpret_cast<float4*>(p.g_rotation) + i;
        if (acc) {
            const float4 o = *d;
            *d = make_float4(o.x + gq.x, o.y + gq.y, o.z + gq.z, o.w + gq.w);
        } else {
            *d = gq;
        }
    }
    if (p.g_drot) reinterpret_cast<float4*>(p.g_drot)[i] = gq;
    const float sg = 1.f / (1.f + expf(-p.opacity[i]));
    const float go_ = p.g_opac[i] * sg * (1.f - sg);
    if (p.g_opacity) p.g_opacity[i] = acc ? p.g_opacity[i] + go_ : go_;
}

__global__ __launch_bounds__(256) void k_unpack_sh_bwd(int P, int R, int accumulate, const float* __restrict__ g_shs,
                                                       float* __restrict__ g_fdc, float* __restrict__ g_frest,
                                                       float* __restrict__ g_dsh) {
    const uint32_t row = 3u * (1u + (uint32_t)R);
    const uint32_t n = (uint32_t)P * row;
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u) {
        const uint32_t g = e / row;
        const uint32_t k = e - g * row;
        const float v = g_shs[e];
        float* dst = k < 3 ? (g_fdc ? g_fdc + (size_t)g * 3 + k : nullptr)
                           : (g_frest ? g_frest + (size_t)g * (3 * R) + (k - 3) : nullptr);
        if (dst) *dst = accumulate ? *dst + v : v;
        if (g_dsh) g_dsh[e] = v;
    }
}

static unsigned grid_for(long long n) {
    const long long b = (n + 255) / 256;
    return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

void launch_activate_fwd(const ActivateParams& p, hipStream_t s) {
    if (p.P <= 0) return;
    hipLaunchKernelGGL(k_activate_fwd, dim3((p.P + 255) / 256), dim3(256), 0, s, p);
    if (!p.shs_out) return;  // split SH: the rasterizer reads f_dc / f_rest / dsh in place
    const long long n = (long long)p.P * 3 * (1 + p.R);
    hipLaunchKernelGGL(k_pack_sh, dim3(grid_for(n)), dim3(256), 0, s, p.P, p.R, p.f_dc, p.f_rest, p.dsh, p.shs_out);
}

void launch_activate_bwd(const ActivateBwdParams& p, hipStream_t s) {
    if (p.P <= 0) return;
    hipLaunchKernelGGL(k_activate_bwd, dim3((p.P + 255) / 256), dim3(256), 0, s, p);
    if (!p.g_shs) return;  // split SH: the rasterizer backward wrote the SH gradients itself
    const long long n = (long long)p.P * 3 * (1 + p.R);
    hipLaunchKernelGGL(k_unpack_sh_bwd, dim3(grid_for(n)), dim3(256), 0, s, p.P, p.R, p.accumulate, p.g_shs, p.g_fdc,
                       p.g_frest, p.g_dsh);
}

}  // namespace gsd
