// gsd_densify.hip -- per-view densification statistics, fused.
//
// Reference (train.py:613-616, scene/gaussian_model.py:1252-1257), for the Gaussians with radii > 0:
//   max_radii2D = max(max_radii2D, radii)
//   xyz_gradient_accum_3vec += viewspace_grad
//   xyz_gradient_accum      += ||viewspace_grad[:, :2]||
//   denom                   += 1
// torch runs these as ~8 boolean-mask gather/scatter kernels per view; here one HBM-bound pass:
// 4 + 12 B read and 20 B read-modify-written per Gaussian.
#include "gsd_kernels.h"

namespace gsd {

__global__ __launch_bounds__(256) void k_densify_stats(int P, const float* __restrict__ vgrad,
                                                       const int* __restrict__ radii, float* __restrict__ accum,
                                                       float* __restrict__ accum3, float* __restrict__ denom,
                                                       float* __restrict__ max_radii) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    if (!(r > 0)) return;
    const float gx = vgrad[3 * i], gy = vgrad[3 * i + 1], gz = vgrad[3 * i + 2];
    max_radii[i] = fmaxf(max_radii[i], (float)r);
    accum3[3 * i] += gx;
    accum3[3 * i + 1] += gy;
    accum3[3 * i + 2] += gz;
    accum[i] += sqrtf(gx * gx + gy * gy);
    denom[i] += 1.0f;
}

void launch_densify_stats(int P, const float* vgrad, const int* radii, float* accum, float* accum3, float* denom,
                          float* max_radii, hipStream_t s) {
    if (P > 0)
        hipLaunchKernelGGL(k_densify_stats, dim3((P + 255) / 256), dim3(256), 0, s, P, vgrad, radii, accum, accum3,
                           denom, max_radii);
}

}  // namespace gsd
