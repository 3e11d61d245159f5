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

// Measured on the bench slab (59M floats, 28 B each): nontemporal loads/stores 4.9 -> 5.5 TB/s, and one quad
// per thread (a grid covering the slab) rather than a grid-stride loop over 8192 workgroups 5.5 -> 5.8 TB/s;
// more quads per thread per iteration (2, 4) did not help.
constexpr int kAdamUnroll = 1;
constexpr unsigned kAdamMaxGrid = 1u << 20;

// every byte of the state is touched once per step: nontemporal (streaming) loads and stores
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld(const float4* p) {
    const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(r.x, r.y, r.z, r.w);
}
__device__ __forceinline__ void st(float4* p, float4 v) {
    const f4v r = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(r, reinterpret_cast<f4v*>(p));
}

__device__ __forceinline__ int group_of(const AdamArgs& a, long long i) {
    int g = 0;
    while (g + 1 < a.n_groups && i >= a.begin[g + 1]) ++g;
    return g;
}

__device__ __forceinline__ void adam_quad(const AdamArgs& a, float4& p4, float4 g4, float4& m4, float4& v4, int gi) {
    const float ss = a.step_size[gi], b2 = a.bc2_sqrt[gi];
    adam_elem(p4.x, g4.x, m4.x, v4.x, a.w1, a.beta2, a.omb2, ss, b2, a.eps);
    adam_elem(p4.y, g4.y, m4.y, v4.y, a.w1, a.beta2, a.omb2, ss, b2, a.eps);
    adam_elem(p4.z, g4.z, m4.z, v4.z, a.w1, a.beta2, a.omb2, ss, b2, a.eps);
    adam_elem(p4.w, g4.w, m4.w, v4.w, a.w1, a.beta2, a.omb2, ss, b2, a.eps);
}

// Whole quads (16-B aligned, inside one group) take the vector path (kAdamUnroll per thread and iteration,
// every load issued before the first use); a quad that straddles a group boundary or the
// end goes element by element.
__global__ __launch_bounds__(256) void k_adam(AdamArgs a, float* __restrict__ param, float* __restrict__ grad,
                                              float* __restrict__ m, float* __restrict__ v) {
    const long long nq = (a.n + 3) / 4;
    const long long stride = (long long)gridDim.x * 256;
    const bool aligned = ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                           reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
    // the addend's quads line up with the slab's when its first element sits on a quad boundary of both
    const bool add_aligned = a.addend && (a.addend_lo & 3) == 0 && (reinterpret_cast<uintptr_t>(a.addend) & 15) == 0;
    const float4* A4 = reinterpret_cast<const float4*>(a.addend);
    float4* P4 = reinterpret_cast<float4*>(param);
    float4* G4 = reinterpret_cast<float4*>(grad);
    float4* M4 = reinterpret_cast<float4*>(m);
    float4* V4 = reinterpret_cast<float4*>(v);
    for (long long q0 = (long long)blockIdx.x * 256 + threadIdx.x; q0 < nq; q0 += stride * kAdamUnroll) {
        long long qs[kAdamUnroll];
        int gs[kAdamUnroll];
        bool whole[kAdamUnroll];
        float4 p4[kAdamUnroll], g4[kAdamUnroll], m4[kAdamUnroll], v4[kAdamUnroll];
#pragma unroll
        for (int u = 0; u < kAdamUnroll; ++u) {
            qs[u] = q0 + u * stride;
            const long long i0 = qs[u] * 4;
            gs[u] = group_of(a, i0);
            // a quad with addend elements takes the vector path only when all four have one (quad-aligned)
            const bool add_none = !a.addend || i0 + 4 <= a.addend_lo || i0 >= a.addend_hi;
            const bool add_all = add_aligned && i0 >= a.addend_lo && i0 + 4 <= a.addend_hi;
            whole[u] = aligned && qs[u] < nq && i0 + 4 <= a.n &&
                       (gs[u] + 1 >= a.n_groups || i0 + 4 <= a.begin[gs[u] + 1]) && (add_none || add_all);
            if (whole[u]) {
                p4[u] = ld(P4 + qs[u]);
                g4[u] = ld(G4 + qs[u]);
                m4[u] = ld(M4 + qs[u]);
                v4[u] = ld(V4 + qs[u]);
                if (add_all) {
                    const float4 e = ld(A4 + (i0 - a.addend_lo) / 4);
                    g4[u] = make_float4(g4[u].x + e.x, g4[u].y + e.y, g4[u].z + e.z, g4[u].w + e.w);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kAdamUnroll; ++u) {
            if (whole[u]) {
                adam_quad(a, p4[u], g4[u], m4[u], v4[u], gs[u]);
                st(P4 + qs[u], p4[u]);
                st(M4 + qs[u], m4[u]);
                st(V4 + qs[u], v4[u]);
                if (a.zero_grad) st(G4 + qs[u], make_float4(0.f, 0.f, 0.f, 0.f));
            } else if (qs[u] < nq) {
                const long long i0 = qs[u] * 4;
                for (long long i = i0; i < i0 + 4 && i < a.n; ++i) {
                    const int g = group_of(a, i);
                    float pp = param[i], mm = m[i], vv = v[i];
                    const float gi = a.addend && i >= a.addend_lo && i < a.addend_hi
                                         ? grad[i] + a.addend[i - a.addend_lo] : grad[i];
                    adam_elem(pp, gi, mm, vv, a.w1, a.beta2, a.omb2, a.step_size[g], a.bc2_sqrt[g], a.eps);
                    param[i] = pp;
                    m[i] = mm;
                    v[i] = vv;
                    if (a.zero_grad) grad[i] = 0.f;
                }
            }
        }
    }
}

void launch_adam(const AdamArgs& a, float* param, float* grad, float* m, float* v, hipStream_t s) {
    if (a.n <= 0) return;
    const long long quads = (a.n + 3) / 4;
    const long long blocks = (quads + 255) / 256;
    const unsigned grid = (unsigned)(blocks < kAdamMaxGrid ? blocks : kAdamMaxGrid);
    hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, s, a, param, grad, m, v);
}

}  // namespace gsd
