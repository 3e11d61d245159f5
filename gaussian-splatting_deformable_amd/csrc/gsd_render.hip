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
// wave reduces its 64 lanes' partials with DPP (wave_sum), one lane adds the
// wave total into an LDS accumulator per record, and after each 256-record
// batch every record's 9 sums go to HBM as one set of global atomics: at most
// 9 global atomics per (Gaussian, tile) instance instead of per pixel.
#include "gsd_kernels.h"

namespace gsd {

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
        for (int j = 0; !done && j < n; ++j) {
            contributor++;
            const float2 xy = s_xy[j];
            const float dx = xy.x - pxf, dy = xy.y - pyf;
            const float4 co = s_co[j];
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, co.w * expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = T * (1 - alpha);
            if (test_T < 0.0001f) {
                done = true;
                continue;
            }
            const float4 c = s_rgb[j];
            C0 += c.x * alpha * T;
            C1 += c.y * alpha * T;
            C2 += c.z * alpha * T;
            T = test_T;
            last_contributor = contributor;
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
    const float T_final = inside ? p.final_T[pid] : 0.f;
    float T = T_final;
    uint32_t contributor = (uint32_t)toDo;
    const uint32_t last_contributor = inside ? p.n_contrib[pid] : 0u;
    float dpix0 = 0.f, dpix1 = 0.f, dpix2 = 0.f;
    if (inside) {
        dpix0 = p.dL_dpix[pid];
        dpix1 = p.dL_dpix[plane + pid];
        dpix2 = p.dL_dpix[2 * plane + pid];
    }
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;      // accum_rec
    float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f;         // last_color
    float last_alpha = 0.f;
    const float bg_dot = p.bg[0] * dpix0 + p.bg[1] * dpix1 + p.bg[2] * dpix2;
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
        for (int j = 0; j < n; ++j) {
            float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f, v4 = 0.f, v5 = 0.f, v6 = 0.f, v7 = 0.f, v8 = 0.f;
            bool has = false;
            if (inside) {
                contributor--;
                if (contributor < last_contributor) {
                    const float2 xy = s_xy[j];
                    const float dx = xy.x - pxf, dy = xy.y - pyf;
                    const float4 co = s_co[j];
                    const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                    if (power <= 0.0f) {
                        const float G = expf(power);
                        const float alpha = fminf(0.99f, co.w * G);
                        if (!(alpha < 1.0f / 255.0f)) {
                            has = true;
                            T = T / (1.f - alpha);
                            const float dchannel_dcolor = alpha * T;
                            const float4 c = s_rgb[j];
                            // backward.cu:511-524
                            acc0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
                            acc1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
                            acc2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
                            lc0 = c.x;
                            lc1 = c.y;
                            lc2 = c.z;
                            float dL_dalpha = 0.0f;
                            dL_dalpha += (c.x - acc0) * dpix0;
                            dL_dalpha += (c.y - acc1) * dpix1;
                            dL_dalpha += (c.z - acc2) * dpix2;
                            v6 = dchannel_dcolor * dpix0;
                            v7 = dchannel_dcolor * dpix1;
                            v8 = dchannel_dcolor * dpix2;
                            dL_dalpha *= T;
                            last_alpha = alpha;
                            dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                            const float dL_dG = co.w * dL_dalpha;
                            const float gdx = G * dx, gdy = G * dy;
                            const float dG_ddelx = -gdx * co.x - gdy * co.y;
                            const float dG_ddely = -gdy * co.z - gdx * co.y;
                            v0 = dL_dG * dG_ddelx * ddelx_dx;
                            v1 = dL_dG * dG_ddely * ddely_dy;
                            v2 = -0.5f * gdx * dx * dL_dG;
                            v3 = -0.5f * gdx * dy * dL_dG;
                            v4 = -0.5f * gdy * dy * dL_dG;
                            v5 = G * dL_dalpha;
                        }
                    }
                }
            }
            if (__ballot(has)) {  // wave-uniform: reduce only when some lane of this wave contributed
                const float r0 = wave_sum(v0), r1 = wave_sum(v1), r2 = wave_sum(v2), r3 = wave_sum(v3),
                            r4 = wave_sum(v4), r5 = wave_sum(v5), r6 = wave_sum(v6), r7 = wave_sum(v7),
                            r8 = wave_sum(v8);
                if (lane == 0) {
                    atomicAdd(&s_acc[0][j], r0);
                    atomicAdd(&s_acc[1][j], r1);
                    atomicAdd(&s_acc[2][j], r2);
                    atomicAdd(&s_acc[3][j], r3);
                    atomicAdd(&s_acc[4][j], r4);
                    atomicAdd(&s_acc[5][j], r5);
                    atomicAdd(&s_acc[6][j], r6);
                    atomicAdd(&s_acc[7][j], r7);
                    atomicAdd(&s_acc[8][j], r8);
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
