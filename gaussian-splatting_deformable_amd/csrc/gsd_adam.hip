// gsd_adam.hip -- the reference's Adam step over flat parameter / gradient / moment slabs.
//
// Reference: torch.optim.Adam(param_groups, lr=0.0, eps=1e-15) built in training_setup
// (scene/gaussian_model.py:839-856), one group per Gaussian attribute with its own learning rate (the
// xyz group's rescheduled every step, :875-886).  torch (foreach) runs ~8 multi-tensor kernels per
// group; here every parameter of every group lives in one contiguous slab (gsd_amd.optim.FusedAdam),
// so one launch streams the whole state once: per element 16 B read (param, grad, m, v) and 12 B
// written (+4 B when it also clears the gradient for the next step) -- an HBM-bound pass.
//
// Per element, in torch's foreach order (torch/optim/adam.py _multi_tensor_adam):
//   m = lerp(m, g, 1 - beta1)          (m + w (g - m) for w < 0.5)
//   v = v * beta2 + (1 - beta2) * g * g
//   p = p + (-lr / bc1) * (m / (sqrt(v) / sqrt(bc2) + eps))
#include "gsd_kernels.h"

namespace gsd {

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float w1, float beta2, float omb2,
                                          float step_size, float bc2_sqrt, float eps) {
    m = w1 < 0.5f ? m + w1 * (g - m) : g - (g - m) * (1.f - w1);
    v = v * beta2;
    v = v + omb2 * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p + step_size * (m / denom);
}

__global__ __launch_bounds__(256) void k_adam(AdamArgs a, float* __restrict__ param, float* __restrict__ grad,
                                              float* __restrict__ m, float* __restrict__ v) {
    const long long stride = (long long)gridDim.x * 256;
    for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q * 4 < a.n; q += stride) {
        const long long i0 = q * 4;
        // the group of this quad (groups are contiguous, in slab order; a quad may straddle a boundary)
        int gi = 0;
        while (gi + 1 < a.n_groups && i0 >= a.begin[gi + 1]) ++gi;
        const bool whole = i0 + 4 <= a.n && (gi + 1 >= a.n_groups || i0 + 4 <= a.begin[gi + 1]) &&
                           ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                             reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
        if (whole) {
            float4 p4 = reinterpret_cast<float4*>(param)[q];
            const float4 g4 = reinterpret_cast<const float4*>(grad)[q];
            float4 m4 = reinterpret_cast<float4*>(m)[q];
            float4 v4 = reinterpret_cast<float4*>(v)[q];
            const float ss = a.step_size[gi], b2 = a.bc2_sqrt[gi];
            adam_elem(p4.x, g4.x, m4.x, v4.x, a.w1, a.beta2, a.omb2, ss, b2, a.eps);
            adam_elem(p4.y, g4.y, m4.y, v4.y, a.w1, a.beta2, a.omb2, ss, b2, a.eps);
            adam_elem(p4.z, g4.z, m4.z, v4.z, a.w1, a.beta2, a.omb2, ss, b2, a.eps);
            adam_elem(p4.w, g4.w, m4.w, v4.w, a.w1, a.beta2, a.omb2, ss, b2, a.eps);
            reinterpret_cast<float4*>(param)[q] = p4;
            reinterpret_cast<float4*>(m)[q] = m4;
            reinterpret_cast<float4*>(v)[q] = v4;
            if (a.zero_grad) reinterpret_cast<float4*>(grad)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            for (long long i = i0; i < i0 + 4 && i < a.n; ++i) {
                int g = 0;
                while (g + 1 < a.n_groups && i >= a.begin[g + 1]) ++g;
                float pp = param[i], mm = m[i], vv = v[i];
                adam_elem(pp, grad[i], mm, vv, a.w1, a.beta2, a.omb2, a.step_size[g], a.bc2_sqrt[g], a.eps);
                param[i] = pp;
                m[i] = mm;
                v[i] = vv;
                if (a.zero_grad) grad[i] = 0.f;
            }
        }
    }
}

void launch_adam(const AdamArgs& a, float* param, float* grad, float* m, float* v, hipStream_t s) {
    if (a.n <= 0) return;
    const long long quads = (a.n + 3) / 4;
    const long long blocks = (quads + 255) / 256;
    const unsigned grid = (unsigned)(blocks < 8192 ? blocks : 8192);
    hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, s, a, param, grad, m, v);
}

}  // namespace gsd
