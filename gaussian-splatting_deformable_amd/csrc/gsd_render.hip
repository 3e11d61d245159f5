// gsd_render.hip -- per-tile front-to-back compositing (forward) and its
// back-to-front replay (backward).
//
// One 256-lane workgroup per 16x16 tile (4 wave64s, each owning 4 pixel rows);
// the tile's depth-sorted Gaussian list is streamed through LDS 256 records at
// a time (xy, conic+opacity, rgb: 40 B/record, broadcast reads).  The tile ->
// workgroup map is XCD-swizzled so neighbouring tiles, which gather the same
// Gaussian records, share one XCD's L2.
//
// Backward: the reference issues 9 float atomicAdds per (pixel, Gaussian) pair
// (backward.cu:523,545-554), all 256 lanes on the same address.  Here each
// wave computes 8 records' partials, reduces them across its 64 lanes with one
// transposed butterfly per quantity (wave_sum8: permlane32/16 swaps + DPP),
// 8 lanes add the 8 wave totals into LDS accumulators, and after each
// 256-record batch every record's 9 sums go to HBM as one set of global
// atomics: at most 9 global atomics per (Gaussian, tile) instance instead of
// 9 per (Gaussian, pixel) pair.
#include "gsd_kernels.h"

namespace gsd {

constexpr int kFwdBatch = 8;  // records whose alphas are evaluated together (ILP across the exps)

__global__ __launch_bounds__(256) void k_render_fwd(RenderParams p) {
    __shared__ float2 s_xy[kTilePix];
    __shared__ float4 s_co[kTilePix];
    __shared__ float4 s_rgb[kTilePix];
    const int tile = xcd_swizzle(blockIdx.x, p.num_tiles);
    const int tid = threadIdx.x;
    const int px = (tile % p.grid_x) * kTileX + (tid & (kTileX - 1));
    const int py = (tile / p.grid_x) * kTileY + (tid >> 4);
    const bool inside = px < p.W && py < p.H;
    bool done = !inside;
    const uint2 rg = p.ranges[tile];
    const int rounds = ((int)(rg.y - rg.x) + kTilePix - 1) / kTilePix;
    int toDo = (int)(rg.y - rg.x);
    const float pxf = (float)px, pyf = (float)py;
    float T = 1.0f;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    uint32_t contributor = 0, last_contributor = 0;

    for (int i = 0; i < rounds; ++i, toDo -= kTilePix) {
        // forward.cu:309-311: stop once every pixel of the tile is saturated
        if (__syncthreads_count(done) == kTilePix) break;
        const int k = (int)rg.x + i * kTilePix + tid;
        if (k < (int)rg.y) {
            const uint32_t g = p.point_list[k];
            s_xy[tid] = p.means2D[g];
            s_co[tid] = p.conic_opacity[g];
            s_rgb[tid] = p.rgb[g];
        }
        __syncthreads();
        const int n = min(kTilePix, toDo);
        for (int j0 = 0; j0 < n; j0 += kFwdBatch) {
            if (!__ballot(!done)) break;  // every pixel of this wave has saturated
            // branch-free alphas of kFwdBatch records (independent: the exps overlap) ...
            float a[kFwdBatch];
#pragma unroll
            for (int u = 0; u < kFwdBatch; ++u) {
                const float2 xy = s_xy[j0 + u];
                const float dx = xy.x - pxf, dy = xy.y - pyf;
                const float4 co = s_co[j0 + u];
                const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                a[u] = power > 0.0f ? 0.0f : fminf(0.99f, co.w * expf(power));  // 0 => skipped below
            }
            // ... then the sequential front-to-back recurrence (forward.cu:325-362)
#pragma unroll
            for (int u = 0; u < kFwdBatch; ++u) {
                if (done || j0 + u >= n) continue;
                contributor++;
                const float alpha = a[u];
                if (alpha < 1.0f / 255.0f) continue;
                const float test_T = T * (1 - alpha);
                if (test_T < 0.0001f) {
                    done = true;
                    continue;
                }
                const float4 c = s_rgb[j0 + u];
                C0 += c.x * alpha * T;
                C1 += c.y * alpha * T;
                C2 += c.z * alpha * T;
                T = test_T;
                last_contributor = contributor;
            }
        }
    }
    if (inside) {
        const int pid = p.W * py + px;
        const int plane = p.H * p.W;
        p.final_T[pid] = T;
        p.n_contrib[pid] = last_contributor;
        p.out_color[pid] = C0 + T * p.bg[0];
        p.out_color[plane + pid] = C1 + T * p.bg[1];
        p.out_color[2 * plane + pid] = C2 + T * p.bg[2];
    }
}

// Per-pixel state of the back-to-front replay (backward.cu:441-461).
struct BwdPixel {
    float T, T_final, last_alpha;
    float acc0, acc1, acc2, lc0, lc1, lc2;
    float dpix0, dpix1, dpix2, bg_dot;
};

constexpr int kRedBatch = 8;  // records reduced together by wave_sum8

__global__ __launch_bounds__(256) void k_render_bwd(RenderBwdParams p) {
    __shared__ uint32_t s_id[kTilePix];
    __shared__ float2 s_xy[kTilePix];
    __shared__ float4 s_co[kTilePix];
    __shared__ float4 s_rgb[kTilePix];
    __shared__ float s_acc[9][kTilePix];
    const int tile = xcd_swizzle(blockIdx.x, p.num_tiles);
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int px = (tile % p.grid_x) * kTileX + (tid & (kTileX - 1));
    const int py = (tile / p.grid_x) * kTileY + (tid >> 4);
    const bool inside = px < p.W && py < p.H;
    const uint2 rg = p.ranges[tile];
    const int rounds = ((int)(rg.y - rg.x) + kTilePix - 1) / kTilePix;
    int toDo = (int)(rg.y - rg.x);
    const int pid = p.W * py + px;
    const int plane = p.H * p.W;
    BwdPixel st;
    st.T_final = inside ? p.final_T[pid] : 0.f;
    st.T = st.T_final;
    uint32_t contributor = (uint32_t)toDo;
    const uint32_t last_contributor = inside ? p.n_contrib[pid] : 0u;
    st.dpix0 = st.dpix1 = st.dpix2 = 0.f;
    if (inside) {
        st.dpix0 = p.dL_dpix[pid];
        st.dpix1 = p.dL_dpix[plane + pid];
        st.dpix2 = p.dL_dpix[2 * plane + pid];
    }
    st.acc0 = st.acc1 = st.acc2 = 0.f;  // accum_rec
    st.lc0 = st.lc1 = st.lc2 = 0.f;     // last_color
    st.last_alpha = 0.f;
    st.bg_dot = p.bg[0] * st.dpix0 + p.bg[1] * st.dpix1 + p.bg[2] * st.dpix2;
    const float ddelx_dx = (float)(0.5 * p.W), ddely_dy = (float)(0.5 * p.H);
    const float pxf = (float)px, pyf = (float)py;

    for (int i = 0; i < rounds; ++i, toDo -= kTilePix) {
        __syncthreads();
        const int progress = i * kTilePix + tid;
        if ((int)rg.x + progress < (int)rg.y) {
            const uint32_t g = p.point_list[rg.y - progress - 1];
            s_id[tid] = g;
            s_xy[tid] = p.means2D[g];
            s_co[tid] = p.conic_opacity[g];
            s_rgb[tid] = p.rgb[g];
        }
#pragma unroll
        for (int q = 0; q < 9; ++q) s_acc[q][tid] = 0.f;
        __syncthreads();
        const int n = min(kTilePix, toDo);
        for (int j0 = 0; j0 < n; j0 += kRedBatch) {
            // branch-free G / alpha of kRedBatch records (independent: the exps overlap) ...
            float Gs[kRedBatch], As[kRedBatch];
#pragma unroll
            for (int u = 0; u < kRedBatch; ++u) {
                const float2 xy = s_xy[j0 + u];
                const float dx = xy.x - pxf, dy = xy.y - pyf;
                const float4 co = s_co[j0 + u];
                const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                const float G = expf(power);
                Gs[u] = G;
                As[u] = power > 0.0f ? 0.0f : fminf(0.99f, co.w * G);  // 0 => skipped below
            }
            // ... then the sequential back-to-front recurrence (backward.cu:482-555)
            float v[9][kRedBatch];
            bool any = false;
#pragma unroll
            for (int u = 0; u < kRedBatch; ++u) {
#pragma unroll
                for (int q = 0; q < 9; ++q) v[q][u] = 0.f;
                const int j = j0 + u;
                if (inside && j < n) {
                    contributor--;
                    if (contributor < last_contributor) {
                        const float2 xy = s_xy[j];
                        const float dx = xy.x - pxf, dy = xy.y - pyf;
                        const float4 co = s_co[j];
                        {
                            const float G = Gs[u];
                            const float alpha = As[u];
                            if (!(alpha < 1.0f / 255.0f)) {
                                any = true;
                                const float inv1ma = 1.f / (1.f - alpha);
                                st.T = st.T * inv1ma;  // backward.cu:503 (T recovered by division)
                                const float dchannel_dcolor = alpha * st.T;
                                const float4 c = s_rgb[j];
                                st.acc0 = st.last_alpha * st.lc0 + (1.f - st.last_alpha) * st.acc0;
                                st.acc1 = st.last_alpha * st.lc1 + (1.f - st.last_alpha) * st.acc1;
                                st.acc2 = st.last_alpha * st.lc2 + (1.f - st.last_alpha) * st.acc2;
                                st.lc0 = c.x;
                                st.lc1 = c.y;
                                st.lc2 = c.z;
                                float dL_dalpha = (c.x - st.acc0) * st.dpix0;
                                dL_dalpha += (c.y - st.acc1) * st.dpix1;
                                dL_dalpha += (c.z - st.acc2) * st.dpix2;
                                v[6][u] = dchannel_dcolor * st.dpix0;
                                v[7][u] = dchannel_dcolor * st.dpix1;
                                v[8][u] = dchannel_dcolor * st.dpix2;
                                dL_dalpha *= st.T;
                                st.last_alpha = alpha;
                                dL_dalpha += (-st.T_final * inv1ma) * st.bg_dot;
                                const float dL_dG = co.w * dL_dalpha;
                                const float gdx = G * dx, gdy = G * dy;
                                const float dG_ddelx = -gdx * co.x - gdy * co.y;
                                const float dG_ddely = -gdy * co.z - gdx * co.y;
                                v[0][u] = dL_dG * dG_ddelx * ddelx_dx;
                                v[1][u] = dL_dG * dG_ddely * ddely_dy;
                                v[2][u] = -0.5f * gdx * dx * dL_dG;
                                v[3][u] = -0.5f * gdx * dy * dL_dG;
                                v[4][u] = -0.5f * gdy * dy * dL_dG;
                                v[5][u] = G * dL_dalpha;
                            }
                        }
                    }
                }
            }
            if (__ballot(any)) {  // wave-uniform
#pragma unroll
                for (int q = 0; q < 9; ++q) {
                    const float r = wave_sum8(v[q]);
                    if ((lane & 7) == 0) atomicAdd(&s_acc[q][j0 + (lane >> 3)], r);
                }
            }
        }
        __syncthreads();
        if (tid < n) {
            const uint32_t g = s_id[tid];
            const float a0 = s_acc[0][tid], a1 = s_acc[1][tid], a2 = s_acc[2][tid], a3 = s_acc[3][tid],
                        a4 = s_acc[4][tid], a5 = s_acc[5][tid], a6 = s_acc[6][tid], a7 = s_acc[7][tid],
                        a8 = s_acc[8][tid];
            if (a0 != 0.f) atomicAdd(p.dL_dmean2D + 3 * g, a0);
            if (a1 != 0.f) atomicAdd(p.dL_dmean2D + 3 * g + 1, a1);
            if (a2 != 0.f) atomicAdd(p.dL_dconic + 4 * g, a2);
            if (a3 != 0.f) atomicAdd(p.dL_dconic + 4 * g + 1, a3);
            if (a4 != 0.f) atomicAdd(p.dL_dconic + 4 * g + 3, a4);
            if (a5 != 0.f) atomicAdd(p.dL_dopacity + g, a5);
            if (a6 != 0.f) atomicAdd(p.dL_dcolors + 3 * g, a6);
            if (a7 != 0.f) atomicAdd(p.dL_dcolors + 3 * g + 1, a7);
            if (a8 != 0.f) atomicAdd(p.dL_dcolors + 3 * g + 2, a8);
        }
    }
}

void launch_render_fwd(const RenderParams& p, hipStream_t s) {
    if (p.num_tiles > 0) hipLaunchKernelGGL(k_render_fwd, dim3(p.num_tiles), dim3(kTilePix), 0, s, p);
}
void launch_render_bwd(const RenderBwdParams& p, hipStream_t s) {
    if (p.num_tiles > 0) hipLaunchKernelGGL(k_render_bwd, dim3(p.num_tiles), dim3(kTilePix), 0, s, p);
}

}  // namespace gsd
