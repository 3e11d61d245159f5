// gsd_render.hip -- per-tile front-to-back compositing (forward) and its
// back-to-front replay (backward).
//
// One 256-lane workgroup per 16x16 tile; each wave64 owns one 8x8 quadrant.
// The tile's depth-sorted record list (point_list) is streamed through LDS
// 256 records at a time, each staged from its Gaussian's 64-B RenderRec (xy,
// conic+opacity, rgb and the alpha bounding box the preprocess computed).
//
// Wave-level culling: a record can only change a pixel where
// alpha = o*exp(-Q/2) >= 1/255, i.e. inside the ellipse Q <= 2 ln(255 o)
// (Q = the conic's quadratic form).  Its bounding box (inflated by a safety
// margin) is computed once per record; each wave compacts, per 256-record
// batch, the list of records whose box meets its 8x8 quadrant and iterates
// only those.  Records outside the list would have been skipped by every
// lane (alpha < 1/255), so results are unchanged -- ~57% of (wave, record)
// pairs never reach the ALUs on the bench scene.  The forward culls per 4x4
// pixel block (16 lanes), each block walking its own list.
//
// Backward: the reference issues 9 float atomicAdds per (pixel, Gaussian) pair
// (backward.cu:523,545-554), all 256 lanes on the same address.  Here the work
// per record is split in two phases.  Pixel-major: each lane replays its pixel
// back to front and hands two numbers per record to LDS, o G dL/dalpha and
// alpha T.  Record-major: every one of the record's nine sums (dL/dmean2D,
// dL/dconic, dL/dopacity, dL/dcolor) is a dot product of those two with
// per-pixel factors (the pixel offsets and dL/dpixel), so a quad of lanes sums
// one record over 4 pixels each and a short transposed butterfly finishes it;
// the sums go to LDS accumulators and, after each 256-record batch, to HBM as
// one set of global atomics per (Gaussian, tile) instance.
#include <type_traits>

#include "../../include/gsd_raster.h"

#include "gsd_kernels.h"

namespace gsd {

// GSD_BWD_ABLATE (k_render_bwd timing-only builds, wrong results): 1 no phase 2, 2 no LDS accumulation, 4 no global
// flush, 8 no walk
#ifndef GSD_BWD_ABLATE
#define GSD_BWD_ABLATE 0
#endif

#ifdef GSD_COUNT_WORK
// gsd_work_counters (include/gsd_raster.h): fwd steps, fwd pairs, bwd steps, bwd pairs
__device__ unsigned long long g_work[4];
__device__ __forceinline__ void count_work(int i, unsigned long long steps, unsigned long long pairs) {
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&g_work[i], steps);
        atomicAdd(&g_work[i + 1], pairs);
    }
}
#endif


// forward: records whose alphas are evaluated together (ILP across the exps); measured 2/3/4/6/8/16 ->
// 4 is fastest (0.33 ms vs 0.38 at 8: fewer alphas wasted past a pixel's termination; re-measured with the
// uniform-skip recurrence: 2 / 4 / 8 -> 0.305 / 0.289 / 0.328 ms; with the 4x4 lane groups: 4 / 8 -> 0.252 / 0.280)
constexpr int kBatch = 4;
// (forward culling: the exact ellipse test costs the forward more than it saves -- 0.306 vs 0.289 ms per 8x8
// quadrant, 0.366 vs 0.261 per 4x4 lane group; the backward's linear bound over the 4x4 block on top of the alpha
// box pays: 0.1994 / 0.1995 ms against 0.2040 / 0.2034 with the box alone, round 5)
constexpr int kBwdGroup = 4;  // backward: records per pixel-major -> record-major hand-off through LDS

// Does the ellipse {d : Q(d) <= t} around (mx, my) meet the rectangle [x0, x1] x [y0, y1]?
// Q(d) = a dx^2 + 2 b dx dy + c dy^2 (positive definite: a, c > 0, det > 0).  Q is convex, so its minimum
// over the rectangle is 0 when the centre is inside, else it lies on an edge; on an edge x = const the
// minimiser is dy* = -b dx / c clamped to the edge (and symmetrically).  Conservative by `slack`.
// The minimiser is taken with the hardware reciprocal of c (1 ulp): an inexact dy* only moves the evaluated
// point along the edge by ~1e-7 relative, which raises Q by a second-order amount far inside the test's slack.
__device__ __forceinline__ float edge_min_x(float a, float b, float c, float rc, float dx, float dy0, float dy1) {
    const float dy = fminf(fmaxf(-b * dx * rc, dy0), dy1);
    return a * dx * dx + 2.f * b * dx * dy + c * dy * dy;
}
// ra, rc: the hardware reciprocals of a and c (RenderRec.q2, computed once per Gaussian by the preprocess).
__device__ __forceinline__ bool ellipse_meets_rect(float2 xy, float4 co, float t, float ra, float rc, float x0,
                                                   float x1, float y0, float y1) {
    const float dx0 = x0 - xy.x, dx1 = x1 - xy.x, dy0 = y0 - xy.y, dy1 = y1 - xy.y;
    if (dx0 <= 0.f && dx1 >= 0.f && dy0 <= 0.f && dy1 >= 0.f) return true;  // centre inside
    const float a = co.x, b = co.y, c = co.z;
    float q = fminf(edge_min_x(a, b, c, rc, dx0, dy0, dy1), edge_min_x(a, b, c, rc, dx1, dy0, dy1));
    q = fminf(q, fminf(edge_min_x(c, b, a, ra, dy0, dx0, dx1), edge_min_x(c, b, a, ra, dy1, dx0, dx1)));
    return !(q > t);  // NaN-safe: keeps the record
}

// Per-wave compaction of the batch: s_list receives, in increasing slot order,
// the slots whose alpha box meets [qx0, qx0+7] x [qy0, qy0+7] -- and, with kExact,
// whose alpha ellipse meets it too (-11 % of the backward's record iterations on the
// bench scene; the forward, cheaper per record and early-terminating, loses more to
// the extra test than it saves).  Returns the count.
// Slots below t_min are skipped too (the backward's last-contributor bound).
// With kCount, *below returns per lane how many list entries have a slot <= t_cut (the lane's own bound): the
// list is in slot order, so the entries with a larger slot are exactly those at list index >= *below.
template <bool kExact, int RW = 8, int RH = 8, bool kCount = false>
__device__ __forceinline__ int wave_compact(const float4* __restrict__ s_box, const float4* __restrict__ s_pc,
                                            const float4* __restrict__ s_bo, const float4* __restrict__ s_rgb,
                                            uint8_t* __restrict__ s_list, int n, float qx0, float qy0, int lane,
                                            int t_min = 0, int t_cut = 0, int* below_cut = nullptr) {
    int m = 0;
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < kTilePix / 64; ++k) {
        const int t = k * 64 + lane;
        bool hit = false;
        if (t < n && t >= t_min) {
            const float4 bx = s_box[t];
            hit = bx.y >= qx0 && bx.x <= qx0 + (float)(RW - 1) && bx.w >= qy0 && bx.z <= qy0 + (float)(RH - 1);
            if (kExact && hit) {
                const float4 pc = s_pc[t];
                const float4 bo = s_bo[t];  // (b, t_o, o, 1 / a)
                const float4 co = make_float4(-2.f * pc.z, bo.x, -2.f * pc.w, bo.z);  // exact: (a, b, c, o)
                const float det = co.x * co.z - co.y * co.y;
                // alpha >= 1/255  <=>  Q <= 2 ln(255 o) = -2 t_o, with 0.1 % + 0.05 of slack (the exact decision
                // is power >= t_o, record_alpha); the reciprocals come precomputed (RenderRec.q2)
                if (co.x > 0.f && co.z > 0.f && det > 0.f)
                    hit = ellipse_meets_rect(make_float2(pc.x, pc.y), co, fmaf(-2.002f, bo.y, 0.05f), bo.w,
                                             s_rgb[t].w, qx0, qx0 + (float)(RW - 1), qy0, qy0 + (float)(RH - 1));
            }
        }
        const unsigned long long mask = wave_ballot(hit);
        if (hit) {
            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
            s_list[m + below] = (uint8_t)t;
        }
        if (kCount) {  // hits among slots k*64 .. t_cut: the mask's lowest clamp(t_cut - 64 k + 1, 0, 64) bits
            const int nb = min(max(t_cut - k * 64 + 1, 0), 64);
            const unsigned long long le = nb >= 64 ? ~0ull : ((1ull << nb) - 1ull);
            cnt += __popcll(mask & le);
        }
        m += __popcll(mask);
    }
    if (kCount) *below_cut = cnt;
    wave_lds_handoff();
    return m;
}

// Forward lane groups: the wave's 8x8 quadrant as kFwdGroups rectangles of 64 / kFwdGroups pixels (2: the 8x4
// halves, lanes 0-31 / 32-63; 4: 4x4 blocks, lanes 16 g .. 16 g + 15), each walking its own compacted record
// list side by side with the others -- a record whose alpha box misses a group no longer occupies its lanes.
// Measured (render_fwd, bench workload): 1 group (the whole quadrant) 0.291 ms, 2 (8x4 halves) 0.288,
// 4 (4x4 blocks) 0.261, 8 (4x2 blocks) 0.268 -- finer groups waste fewer lanes on records that miss them, at
// the price of distinct LDS addresses per record read and more compaction.
constexpr int kFwdGroups = 4;
// pixel offset of `lane` inside the quadrant, and its group's rectangle [gx0, gx0 + gw) x [gy0, gy0 + gh)
__device__ __forceinline__ void fwd_lane_pixel(int lane, int& dx, int& dy) {
    if (kFwdGroups == 8) {  // 4x2 blocks
        const int g = lane >> 3;
        dx = (g & 1) * 4 + (lane & 3);
        dy = (g >> 1) * 2 + ((lane >> 2) & 1);
    } else if (kFwdGroups == 4) {
        const int g = lane >> 4;
        dx = (g & 1) * 4 + (lane & 3);
        dy = (g >> 1) * 4 + ((lane >> 2) & 3);
    } else {
        dx = lane & 7;
        dy = lane >> 3;
    }
}
__device__ __forceinline__ float4 fwd_group_rect(int g, float qx0, float qy0) {  // (x0, x1, y0, y1), inclusive
    if (kFwdGroups == 8) {
        const float x0 = qx0 + (float)((g & 1) * 4), y0 = qy0 + (float)((g >> 1) * 2);
        return make_float4(x0, x0 + 3.f, y0, y0 + 1.f);
    }
    if (kFwdGroups == 4) {
        const float x0 = qx0 + (float)((g & 1) * 4), y0 = qy0 + (float)((g >> 1) * 4);
        return make_float4(x0, x0 + 3.f, y0, y0 + 3.f);
    }
    if (kFwdGroups == 2) return make_float4(qx0, qx0 + 7.f, qy0 + (float)(4 * g), qy0 + (float)(4 * g) + 3.f);
    return make_float4(qx0, qx0 + 7.f, qy0, qy0 + 7.f);
}

// Compaction into one list per lane group: lists[g] receives, in increasing slot order, the slots whose alpha
// box meets group g's rectangle; cnt[g] its length (wave-uniform: popcounts of ballots, scalar registers).
__device__ __forceinline__ void wave_compact_groups(const float4* __restrict__ s_box, uint8_t (*lists)[kTilePix],
                                                    int n, float qx0, float qy0, int lane, int (&cnt)[kFwdGroups]) {
#pragma unroll
    for (int g = 0; g < kFwdGroups; ++g) cnt[g] = 0;
#pragma unroll
    for (int k = 0; k < kTilePix / 64; ++k) {
        const int t = k * 64 + lane;
        const float4 bx = t < n ? s_box[t] : make_float4(1e30f, -1e30f, 1e30f, -1e30f);
#pragma unroll
        for (int g = 0; g < kFwdGroups; ++g) {
            const float4 r = fwd_group_rect(g, qx0, qy0);
            const bool hit = t < n && bx.y >= r.x && bx.x <= r.y && bx.w >= r.z && bx.z <= r.w;
            const unsigned long long b = wave_ballot(hit);
            if (hit)
                lists[g][cnt[g] + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0))] = (uint8_t)t;
            cnt[g] += __popcll(b);
        }
    }
    wave_lds_handoff();
}

// Backward compaction into one list per 4x4 lane group (the forward's groups, fwd_lane_pixel): lists[g] receives, in
// increasing slot order, the slots t >= t_min[g] (the group's last-contributor cut) whose alpha box meets group g's
// block and whose alpha ellipse passes a linear bound over the block: with d the block centre minus the mean and
// h = 1.5 px the block's half-size, min over the block of Q >= Q(d) - h |grad Q(d)|_1 = Q(d) - 3 (|u| + |v|),
// (u, v) = (a dx + b dy, b dx + c dy) -- conservative for a positive-definite conic, so a culled record has
// alpha < 1/255 at every pixel of the block (the same slack as the exact test: 0.1 % + 0.05 on 2 ln(255 o)).
// Counted on the cfg4 scene (scripts/sim_bwd_lists.py): the wave then walks 0.708 of the per-quadrant lists' steps
// (the exact ellipse test per block: 0.682, the alpha box alone: 0.817).
// UNROLL: slots per lane whose loads and tests the compiler may interleave (the forward, at 64 VGPRs, takes them
// one at a time: unrolled, the extra live values spilled 24 B per lane, ~95 MB of scratch traffic per launch)
template <int NB, int UNROLL = NB / 64>
__device__ __forceinline__ void bwd_compact_groups(const float4* __restrict__ s_box, const float4* __restrict__ s_pc,
                                                   const float2* __restrict__ s_bo, uint8_t (*lists)[NB], int n,
                                                   float qx0, float qy0, int lane, const int (&t_min)[4],
                                                   int (&cnt)[4]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) cnt[g] = 0;
#pragma unroll UNROLL
    for (int k = 0; k < NB / 64; ++k) {
        const int t = k * 64 + lane;
        const bool in = t < n;
        const float4 bx = s_box[t];  // slots >= n hold stale values: every test below is masked by `in`
        const float4 pc = s_pc[t];
        const float2 bo = s_bo[t];
        const float a = -2.f * pc.z, c = -2.f * pc.w, b = bo.x;
        const float thr = fmaf(-2.002f, bo.y, 0.05f);
        const bool pd = a > 0.f && c > 0.f && a * c - b * b > 0.f;
        const float dx0 = (qx0 + 1.5f) - pc.x, dy0 = (qy0 + 1.5f) - pc.y;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float ox = (float)(4 * (g & 1)), oy = (float)(4 * (g >> 1));
            const float x0 = qx0 + ox, y0 = qy0 + oy;
            bool hit = in && t >= t_min[g] && bx.y >= x0 && bx.x <= x0 + 3.f && bx.w >= y0 && bx.z <= y0 + 3.f;
            const float dx = dx0 + ox, dy = dy0 + oy;
            const float u = a * dx + b * dy, v = b * dx + c * dy;
            const float q = dx * u + dy * v;
            const float lb = fmaf(-3.f, fabsf(u) + fabsf(v), q);
            if (pd && lb > fmaf(1e-6f, q, thr)) hit = false;  // NaN-safe: keeps the record
            const unsigned long long mask = wave_ballot(hit);
            if (hit)
                lists[g][cnt[g] + __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0))] = (uint8_t)t;
            cnt[g] += __popcll(mask);
        }
    }
    wave_lds_handoff();
}

// forward.cu:330-345 / backward.cu:490-501: the record's alpha at this pixel, shared by both passes so their
// decisions are identical.  power is evaluated exactly as the reference writes it (no contraction), so it has the
// reference's bits.  The threshold decision alpha = min(0.99, o exp(power)) >= 1/255 is taken as power >= t_o, with
// t_o = -ln(255 o) computed in double and rounded to a float by the preprocess (RenderRec.q2.y): for a float power
// that is the real comparison (up to exact ties, where alpha is within half an ulp of t_o of 1/255), so it differs
// from the reference's rounded o * expf(power) >= 1/255 only where that product lies within its own rounding of 1/255
// (the borderline pixels of the parity tests).
// A hardware exp (v_exp_f32, a few ulp) deciding on o G itself flipped decisions outside that band; recomputing
// such alphas with expf cost 5 % of both kernels.  With ln o = -t_o - ln 255 the unclamped alpha
// o G = exp(power - t_o) / 255 is one v_exp_f32 of an FMA: the value is off the reference's by a few ulp (image /
// gradient tolerances), the decisions are not.
constexpr float kLog2e = 1.44269504088896341f;
constexpr float kLog2_255 = 7.99435343685885793f;
// The render kernels stage a record as pc = (mx, my, -a/2, -c/2) and bo = (b, t_o): with the halves folded into
// the staged conic, (-a/2 dx) dx + (-c/2 dy) dy is exactly -0.5f * (a dx dx + c dy dy) (scaling by a power of
// two commutes with rounding), so power below has the reference's bits with one multiply fewer per pair.
__device__ __forceinline__ float4 stage_pc(float2 xy, float4 co) {
    return make_float4(xy.x, xy.y, -0.5f * co.x, -0.5f * co.z);
}
// Returns o G = exp(power - t_o) / 255 (alpha before the 0.99 clamp); `keep` is false where power > 0 (skipped)
// and `over` false where power < t_o (alpha < 1/255) -- the callers fold both into their take / valid masks; a NaN
// power passes both, as in the reference (alpha = fminf(0.99, NaN) = 0.99).
// kRef (gsd_raster_args.alpha_mode = GSD_ALPHA_REFERENCE, ABI 17): alpha exactly as forward.cu:343-345 writes it --
// o * expf(power) (the correctly rounded-ish library exp), skipped when min(0.99, alpha) < 1/255 -- with the
// record's opacity `o`.  Measured (profiles/round6/parity/): the oracle's decisions and final_T then agree to 1.9e-6
// relative (1.05e-5 in the default mode) and one flip remains over the five configurations (11 at cfg5 by default,
// and as many with expf in the default formula: the deviation is the formula's rounding, not the hardware exp);
// it costs render_fwd +26 % and render_bwd +18 %.
template <bool kRef = false>
__device__ __forceinline__ float record_og(float4 pc, float2 bt, float pxf, float pyf, bool& keep, bool& over,
                                           float o = 0.f) {
    const float dx = pc.x - pxf;
    const float dy = pc.y - pyf;
    const float power = (pc.z * dx * dx + pc.w * dy * dy) - bt.x * dx * dy;
    keep = !(power > 0.0f);
    if (kRef) {
        const float og = o * expf(power);
        over = !(fminf(0.99f, og) < 1.0f / 255.0f);
        return og;
    }
    const float d = power - bt.y;  // its sign is exact: a float difference is 0 only for equal operands
    over = !(d < 0.0f);
#ifdef GSD_PRECISE_EXP
    return expf(d) * (1.0f / 255.0f);
#else
    return __builtin_amdgcn_exp2f(fmaf(d, kLog2e, -kLog2_255));
#endif
}

// 1/d from v_rcp_f32 (1 ulp) -- the backward's T recovery (backward.cu:503) -- instead of the ~10 VALU ops of the
// correctly rounded division.  Round 6: without the Newton step that took it to ~0.5 ulp (-DGSD_NEWTON_RCP restores
// it): k_render_bwd is VALU-issue bound (profiles/round6/stall_cfg4/), and the two FMAs per (pixel, record) step cost
// 2.4 % of it (0.3813 / 0.3788 / 0.3759 ms against 0.3885 / 0.3901 / 0.3849, profiles/round6/render_ab/); the
// gradients stay inside the parity bars (rel L2 1e-4, tests/test_gpu_parity.py).
__device__ __forceinline__ float fast_recip(float d) {
    float r = __builtin_amdgcn_rcpf(d);
#ifdef GSD_NEWTON_RCP
    return fmaf(fmaf(-d, r, 1.0f), r, r);
#else
    return r;
#endif
}

struct TileGeom {
    int tile, wave, lane, px, py;
    float qx0, qy0;
    bool inside;
};
// fwd_map: the forward's lane -> pixel map (fwd_lane_pixel); else row-major 8x8 (the backward)
__device__ __forceinline__ TileGeom tile_geom(int num_tiles, int grid_x, int W, int H, bool fwd_map = false) {
    TileGeom g;
    g.tile = xcd_swizzle(blockIdx.x, num_tiles);
    g.wave = threadIdx.x >> 6;
    g.lane = threadIdx.x & 63;
    const int x0 = (g.tile % grid_x) * kTileX + (g.wave & 1) * 8;
    const int y0 = (g.tile / grid_x) * kTileY + (g.wave >> 1) * 8;
    int dx = g.lane & 7, dy = g.lane >> 3;
    if (fwd_map) fwd_lane_pixel(g.lane, dx, dy);
    g.px = x0 + dx;
    g.py = y0 + dy;
    g.qx0 = (float)x0;
    g.qy0 = (float)y0;
    g.inside = g.px < W && g.py < H;
    return g;
}

template <bool kRef>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_render_fwd(RenderParams p) {
    // staged records (stage_pc); (b, o) at an 8-B stride keeps the LDS at 8 workgroups per CU
    __shared__ float4 s_pc[kTilePix];
    __shared__ float2 s_bo[kTilePix];
    __shared__ float4 s_rgb[kTilePix];
    __shared__ float4 s_box[kTilePix];
    __shared__ __attribute__((aligned(4))) uint8_t s_list[4][kFwdGroups][kTilePix];
    const int tid = threadIdx.x;
    // the backward's gradient records cleared here, ahead of the capacity check (a relaunch after a short binning
    // buffer clears them again): ~2 16-B stores per lane, issued before the VALU-bound compositing and never
    // waited on, instead of a separate 64-B-per-Gaussian memset launch in the backward
    if (p.zero_rec) {
        const long long stride = (long long)gridDim.x * kTilePix;
        for (long long e = (long long)blockIdx.x * kTilePix + tid; e < p.zero_n16; e += stride)
            p.zero_rec[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (over_capacity(p.k_guard, p.k_cap)) return;
    const TileGeom tg = tile_geom(p.num_tiles, p.grid_x, p.W, p.H, true);
    // `done` (the pixel has saturated, or lies outside the image) as the wave's lane mask: the per-record
    // decisions below are lane masks combined on the scalar unit and used as select masks
    // (__builtin_amdgcn_inverse_ballot_w64), so no bool is materialised in a vector register
    unsigned long long done_m = wave_ballot(!tg.inside);
    const uint2 rg = p.ranges[tg.tile];
    const int rounds = ((int)(rg.y - rg.x) + kTilePix - 1) / kTilePix;
    int toDo = (int)(rg.y - rg.x);
    const float pxf = (float)tg.px, pyf = (float)tg.py;
    float T = 1.0f;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    uint32_t last_contributor = 0;
    uint8_t* list = s_list[tg.wave][tg.lane / (64 / kFwdGroups)];
#ifdef GSD_COUNT_WORK
    unsigned long long n_steps = 0, n_pairs = 0;
#endif

    for (int i = 0; i < rounds; ++i, toDo -= kTilePix) {
        // forward.cu:309-311: stop once every pixel of the tile is saturated
        if (__syncthreads_count(__builtin_amdgcn_inverse_ballot_w64(done_m)) == kTilePix) break;
        const int k = (int)rg.x + i * kTilePix + tid;
        if (k < (int)rg.y) {
            const RenderRec* r = p.rec + p.point_list[k];  // one 64-B record per gathered instance
            const float4 q0 = r->q0, q1 = r->q1, q2 = r->q2;
            s_pc[tid] = stage_pc(make_float2(q0.x, q0.y), make_float4(q0.z, q0.w, q1.x, q1.y));
            s_bo[tid] = make_float2(q0.w, q2.y);  // b, t_o
            s_rgb[tid] = make_float4(q1.z, q1.w, q2.x, q1.y);  // r, g, b, o (o read by the reference alpha mode)
            s_box[tid] = r->box;
        } else {  // slots past the tile's list: finite zeros (the walk below reads list bytes past a group's end)
            // (zeros built here from an opaque scalar: a float2 zero hoisted out of the round loop was a VGPR pair
            // the 64-register limit spilled)
            int zi = 0;
            asm volatile("" : "+s"(zi));
            const float z = __int_as_float(zi);
            s_pc[tid] = make_float4(z, z, z, z);
            s_bo[tid] = make_float2(z, z);
            s_rgb[tid] = make_float4(z, z, z, z);
        }
        __syncthreads();
        const int n = min(kTilePix, toDo);
        int cnt[kFwdGroups];  // the groups' list lengths (scalar)
#ifndef GSD_FWD_BOX_ONLY
        // the backward's compaction (alpha box + the linear bound of the ellipse over the 4x4 block), without its
        // contributor cut: a record it drops has alpha < 1/255 at every pixel of the block, so it is one the
        // recurrence skips anyway (forward.cu:343-345)
        {
            const int t_none[4] = {0, 0, 0, 0};
            bwd_compact_groups<kTilePix, 1>(s_box, s_pc, s_bo, s_list[tg.wave], n, tg.qx0, tg.qy0, tg.lane, t_none, cnt);
        }
#else
        wave_compact_groups(s_box, s_list[tg.wave], n, tg.qx0, tg.qy0, tg.lane, cnt);
#endif
        int m = cnt[0], mine = cnt[0];  // the longest; the calling lane's group's
#pragma unroll
        for (int g = 1; g < kFwdGroups; ++g) {
            m = max(m, cnt[g]);
            mine = tg.lane / (64 / kFwdGroups) == g ? cnt[g] : mine;
        }
        for (int j0 = 0; j0 < m; j0 += kBatch) {
            if (done_m == ~0ull) break;  // every pixel of this wave has saturated
            // branch-free alphas of kBatch records (independent: the exps overlap) ...
            float a[kBatch];
            bool keep[kBatch], over[kBatch];
            int slot[kBatch];
            static_assert(kBatch == 4, "one LDS word of list entries per batch");
            const uint32_t w4 = *reinterpret_cast<const uint32_t*>(list + j0);
            // lanes whose group list holds entry j0 + u, built on the scalar unit from the groups' lengths.  A lane
            // past its group's list reads whatever byte lies there -- a slot of this batch's staging, so every
            // value read through it is finite -- and never takes it (the mask); no per-lane bounds select.
            unsigned long long in_m[kBatch];
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
#ifdef GSD_FWD_SCALAR_MASK
                in_m[u] = 0;
#pragma unroll
                for (int g = 0; g < kFwdGroups; ++g)
                    in_m[u] |= j0 + u < cnt[g] ? (~0ull >> (64 - 64 / kFwdGroups)) << (g * (64 / kFwdGroups)) : 0ull;
#else
                in_m[u] = wave_ballot(j0 + u < mine);
#endif
                slot[u] = (int)((w4 >> (8 * u)) & 0xffu);
                a[u] = fminf(0.99f, record_og<kRef>(s_pc[slot[u]], s_bo[slot[u]], pxf, pyf, keep[u], over[u],
                                                    kRef ? s_rgb[slot[u]].w : 0.f));
            }
            // ... then the sequential front-to-back recurrence (forward.cu:325-362)
            // One wave-uniform branch per record (skipped when no lane takes it), the lane decisions as selects:
            // 0.300 -> 0.289 ms against a divergent branch per test (each an exec-mask save / restore); fully
            // branch-free (no skip) was slower, 0.335 ms.
#pragma unroll
            for (int u = 0; u < kBatch; ++u) {
                if (j0 + u >= m) break;
#ifdef GSD_COUNT_WORK
                ++n_steps;
#endif
                unsigned long long take_m = ~done_m & in_m[u] & wave_ballot(keep[u]) & wave_ballot(over[u]);
                if (!take_m) continue;
                const float alpha = a[u];
                const float test_T = T * (1 - alpha);
                const unsigned long long fin_m = take_m & wave_ballot(test_T < 0.0001f);
                done_m |= fin_m;
                take_m &= ~fin_m;
#ifdef GSD_COUNT_WORK
                n_pairs += __popcll(take_m);
#endif
                const bool take = __builtin_amdgcn_inverse_ballot_w64(take_m);
                const float4 c = s_rgb[slot[u]];
                // C += c alpha T (forward.cu:356-357) as one FMA per channel on the weight alpha T, selected to 0
                // where the lane does not take the record (C + c * 0 == C for the finite colours of staged records;
                // a non-finite colour would now poison C where the reference skips it): 5 VALU ops instead of 12.  Rounds
                // differently from ((c alpha) T) by an ulp per step (image tolerance); T -- all the
                // backward reads -- keeps the reference's operations.
                const float wgt = take ? alpha * T : 0.f;
                C0 = fmaf(c.x, wgt, C0);
                C1 = fmaf(c.y, wgt, C1);
                C2 = fmaf(c.z, wgt, C2);
                T = take ? test_T : T;
                last_contributor = take ? (uint32_t)(i * kTilePix + slot[u] + 1) : last_contributor;
            }
        }
    }
#ifdef GSD_COUNT_WORK
    count_work(0, n_steps, n_pairs);
#endif
    if (tg.inside) {
        const int pid = p.W * tg.py + tg.px;
        const int plane = p.H * p.W;
        p.final_T[pid] = T;
        p.n_contrib[pid] = last_contributor;
        p.out_color[pid] = C0 + T * p.bg[0];
        p.out_color[plane + pid] = C1 + T * p.bg[1];
        p.out_color[2 * plane + pid] = C2 + T * p.bg[2];
    }
}

// DPP row_newbcast:U -- every lane of a 16-lane row takes lane U of that row (U a compile-time constant, so the
// compiler folds the broadcast into the consuming VALU op as its DPP source)
template <int U>
__device__ __forceinline__ float row_bcast(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + U, 0xf, 0xf, true));
}
template <int U>
__device__ __forceinline__ int row_bcast_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + U, 0xf, 0xf, true);
}
// acc + (lane U of the row's v) * w as ONE v_fmac_f32_dpp (the broadcast on src0, a fused multiply-add as fmaf):
// for a v_fmac the compiler puts the broadcast in a v_mov_b32_dpp of its own.  v must not be written by a VALU
// instruction in the two before it (a DPP source hazard the compiler cannot see inside the asm): the callers pass
// record fields loaded from LDS at the start of their 16-entry block.
template <int U>
__device__ __forceinline__ float fmac_bcast(float v, float w, float acc) {
    asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "+v"(acc)
        : "v"(v), "v"(w), "n"(U));
    return acc;
}

// The round-4 backward (one record list per wave, the 8x8 quadrant, float LDS atomics): kept for A/B against the
// per-group kernel below (-DGSD_BWD_QUADRANT).
__global__ __launch_bounds__(256) void k_render_bwd_quadrant(RenderBwdParams p) {
    __shared__ uint32_t s_id[kTilePix];
    // staged records (stage_pc), all at a 16-B stride: one LDS address per record serves the three reads
    __shared__ float4 s_pc[kTilePix];
    __shared__ float4 s_bo[kTilePix];
    __shared__ float4 s_rgb[kTilePix];
    __shared__ float s_acc[9][kTilePix + 1];  // +1: a record's nine sums sit in nine different banks
    __shared__ __attribute__((aligned(4))) uint8_t s_list[4][kTilePix];
    // the alpha boxes are read only by the compaction, the (G dL/dalpha, alpha T) hand-off only after it (a
    // barrier apart): one region, 31.2 KB of LDS per workgroup in all -> 5 workgroups per CU
    __shared__ union {
        float4 box[kTilePix];
        float2 qa[4][kBwdGroup][65];  // per wave: per record and pixel; +1 pad
    } s_u;
    float4* s_box = s_u.box;
    const TileGeom tg = tile_geom(p.num_tiles, p.grid_x, p.W, p.H);
    const int tid = threadIdx.x;
    const int lane = tg.lane, u16 = lane & 15;
    __shared__ int s_tile_lc;
    const uint2 rg = p.ranges[tg.tile];
    const int pid = p.W * tg.py + tg.px;
    const int plane = p.H * p.W;
    const bool inside = tg.inside;
    // per-pixel replay state (backward.cu:441-461)
    const float T_final = inside ? p.final_T[pid] : 0.f;
    float T = T_final;
    const int last_contributor = inside ? (int)p.n_contrib[pid] : 0;
    // Every pixel skips list positions >= its last contributor (backward.cu:487-488), so the replay starts
    // at the tile's largest last contributor, and each wave compacts away positions beyond its own.
    int wave_lc = last_contributor;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wave_lc = max(wave_lc, __shfl_xor(wave_lc, off));
    if (tid == 0) s_tile_lc = 0;
    lds_barrier();
    if (lane == 0) atomicMax(&s_tile_lc, wave_lc);
    lds_barrier();
    const int total = min((int)(rg.y - rg.x), s_tile_lc);
    const uint32_t end = rg.x + (uint32_t)total;
    const int rounds = (total + kTilePix - 1) / kTilePix;
    int toDo = total;
    float dpix0 = 0.f, dpix1 = 0.f, dpix2 = 0.f;
    if (inside) {
        dpix0 = p.dL_dpix[pid];
        dpix1 = p.dL_dpix[plane + pid];
        dpix2 = p.dL_dpix[2 * plane + pid];
    }
    float2(*qa)[65] = s_u.qa[tg.wave];
    // dL/dpixel of the four pixels of the lane's quad (DPP quad broadcasts), for phase 2 below
    float3 dpq[4];
    dpq[0] = make_float3(quad_bcast<0>(dpix0), quad_bcast<0>(dpix1), quad_bcast<0>(dpix2));
    dpq[1] = make_float3(quad_bcast<1>(dpix0), quad_bcast<1>(dpix1), quad_bcast<1>(dpix2));
    dpq[2] = make_float3(quad_bcast<2>(dpix0), quad_bcast<2>(dpix1), quad_bcast<2>(dpix2));
    dpq[3] = make_float3(quad_bcast<3>(dpix0), quad_bcast<3>(dpix1), quad_bcast<3>(dpix2));
    float adot = 0.f;  // accum_rec . dL/dpixel (accum_rec with last_color / last_alpha folded in)
    const float bg_dot = p.bg[0] * dpix0 + p.bg[1] * dpix1 + p.bg[2] * dpix2;
    const float kbg = -T_final * bg_dot;
    const bool any_bg = wave_ballot(kbg != 0.f) != 0;  // wave-uniform
    const float ddelx_dx = (float)(0.5 * p.W), ddely_dy = (float)(0.5 * p.H);
    const float pxf = (float)tg.px, pyf = (float)tg.py;
    uint8_t* list = s_list[tg.wave];
#ifdef GSD_COUNT_WORK
    unsigned long long n_steps = 0, n_pairs = 0;
#endif
    // phase 2: the first pixel of the lane's half-row of four
    const float ph2_x0 = tg.qx0 + (float)(4 * ((lane >> 2) & 1)), ph2_y0 = tg.qy0 + (float)(lane >> 3);

    for (int i = 0; i < rounds; ++i, toDo -= kTilePix) {
        lds_barrier();
        const int progress = i * kTilePix + tid;
        if (progress < total) {  // loaded back to front (backward.cu:466-478)
            const uint32_t g = p.point_list[end - progress - 1];
            const RenderRec* r = p.rec + g;
            const float4 q0 = r->q0, q1 = r->q1, q2 = r->q2;
            s_id[tid] = g;
            s_pc[tid] = stage_pc(make_float2(q0.x, q0.y), make_float4(q0.z, q0.w, q1.x, q1.y));
            s_bo[tid] = make_float4(q0.w, q2.y, q1.y, q2.z);   // b, t_o, o, 1 / a
            s_rgb[tid] = make_float4(q1.z, q1.w, q2.x, q2.w);  // r, g, b, 1 / c
            s_box[tid] = r->box;
        }
#pragma unroll
        for (int q = 0; q < 9; ++q) s_acc[q][tid] = 0.f;
        lds_barrier();
        const int n = min(kTilePix, toDo);
        // slot t of this batch is list position (total - 1 - i*256 - t) counted from the front
        const int front_base = total - 1 - i * kTilePix;
        // backward.cu:487-488: a pixel replays list position front_base - t only below its last contributor, i.e.
        // slot t counts for this pixel iff t > front_base - last_contributor: iff its list index >= first_valid
        int first_valid;
        const int m = wave_compact<true, 8, 8, true>(s_box, s_pc, s_bo, s_rgb, list, n, tg.qx0, tg.qy0, lane,
                                                     front_base - wave_lc + 1, front_base - last_contributor,
                                                     &first_valid);
        lds_barrier();  // every wave is done with s_box before s_u.qa is written
        // the group loop twice: with the background term of dL/dalpha and, where it is 0 for every pixel of
        // the wave (a black background: the default of train.py), without its multiply-add
        auto walk = [&](auto with_bg) {
            constexpr bool kBg = decltype(with_bg)::value;
            // The list is the wave's, so its records are wave-uniform.  Instead of every lane reading every record
            // from LDS (36 B x 64 lanes per record: with four waves per CU doing so, the LDS array and not the VALU
            // bounded this loop), lane u of each 16-lane row loads list entry j0 + u once per 16 entries, and
            // record U reaches all lanes by DPP row_newbcast:U, folded into the consuming VALU op.
            for (int j0 = 0; j0 < m; j0 += 16) {
                const int nv = m - j0;  // entries left from j0 (wave-uniform)
                const int rslot = u16 < nv ? (int)list[j0 + u16] : 0;  // slot 0 past the list: finite, never taken
                const float4 rpc = s_pc[rslot];
                const float2 rbo = *reinterpret_cast<const float2*>(&s_bo[rslot]);
                const float4 rrgb = s_rgb[rslot];
                auto hand_off = [&](auto kc) {
                    constexpr int K = decltype(kc)::value;
                    // Phase 1 (pixel-major): entries K .. K + 3.  Each lane runs the back-to-front recurrence for
                    // its pixel and leaves two numbers per record in qa: v = o G dL/dalpha and w = alpha T.  Every
                    // one of the nine per-record sums is a dot product of these with per-pixel factors -- the pixel
                    // offsets (mean - pixel) and dL/dpixel -- so nothing else is needed from the lane.
                    const int r = lane & 3, grp = lane >> 2;
                    // phase 2's record (entry K + r) and its mean, read ahead of phase 1
                    const int rs = K + r < nv ? (int)list[j0 + K + r] : 0;
                    const float2 mrec = *reinterpret_cast<const float2*>(&s_pc[rs]);
                    unsigned long long any_m = 0;  // lanes that took any record of the hand-off
                    auto rec = [&](auto uc) {
                        constexpr int U = K + decltype(uc)::value;
                        const float4 pc = make_float4(row_bcast<U>(rpc.x), row_bcast<U>(rpc.y), row_bcast<U>(rpc.z),
                                                      row_bcast<U>(rpc.w));
                        const float2 bo = make_float2(row_bcast<U>(rbo.x), row_bcast<U>(rbo.y));
                        bool keep, over;
                        const float OG = record_og(pc, bo, pxf, pyf, keep, over);  // alpha before the 0.99 clamp
                        // backward.cu:487-488 (list position below the pixel's last contributor), :490-501
                        const unsigned long long valid_m = (U < nv ? ~0ull : 0ull) &
                                                           wave_ballot(j0 + U >= first_valid) & wave_ballot(keep) &
                                                           wave_ballot(over);
                        any_m |= valid_m;
#ifdef GSD_COUNT_WORK
                        n_steps += U < nv ? 1 : 0;
                        n_pairs += __popcll(valid_m);
#endif
                        {
#pragma clang fp contract(fast)
                            const bool valid = __builtin_amdgcn_inverse_ballot_w64(valid_m);
                            // one select: o G zeroed where the lane skips the record gives alpha = 0 (T unchanged)
                            // and a zero hand-off; the hand-off carries q = o G dL/dalpha
                            const float og = valid ? OG : 0.f;
                            const float alpha = fminf(0.99f, og);
                            const float inv1ma = fast_recip(1.f - alpha);
                            T = T * inv1ma;  // backward.cu:503 (T recovered by division)
                            const float cd = fmaf(row_bcast<U>(rrgb.z), dpix2,
                                                  fmaf(row_bcast<U>(rrgb.y), dpix1, row_bcast<U>(rrgb.x) * dpix0));
                            const float diff = cd - adot;
                            // backward.cu:512-529 (kbg = 0: fmaf(diff, T, -0) is diff * T, bit for bit)
                            const float dL_dalpha = kBg ? fmaf(diff, T, kbg * inv1ma) : diff * T;
                            qa[U & 3][lane] = make_float2(og * dL_dalpha, alpha * T);
                            adot = fmaf(alpha, diff, adot);
                        }
                    };
                    rec(std::integral_constant<int, 0>{});
                    rec(std::integral_constant<int, 1>{});
                    rec(std::integral_constant<int, 2>{});
                    rec(std::integral_constant<int, 3>{});
                    if (!any_m) return;  // wave-uniform: no pixel took any of these records
                    wave_lds_handoff();
                    // Phase 2 (record-major): lane 4 g + r sums record r over pixels 4 g + i, i = 0..3 -- the lanes of
                    // its own quad, whose dL/dpixel were broadcast into dpq once.  Pixel 4 g + i sits at (x0 + i,
                    // y0), x0 = qx0 + 4 (g & 1), y0 = qy0 + (g >> 1); relative to the record's mean ex = x0 - mx,
                    // ey = y0 - my.  With S0 = sum v, X1 = sum v i, X2 = sum v i^2 (constant offsets i):
                    // sum v (x - mx) = ex S0 + X1, sum v (x - mx)^2 = ex (ex S0 + X1) + ex X1 + X2, the y sums from
                    // the lane's constant ey, and C = sum w dL/dpixel.  The reference's dx = mx - x
                    // (backward.cu:545-554) flips the first moments' sign (the flush).  19 VALU ops for the four
                    // pixels' sums instead of 27, and no per-pixel offsets.  (Raw tile-local moments centred only
                    // in the flush need no record read here, but the centring cancels: the float-atomic order noise
                    // of the sums grew to ~1e-4 relative.)
                    const float2 q0 = qa[r][4 * grp], q1 = qa[r][4 * grp + 1], q2 = qa[r][4 * grp + 2],
                                 q3 = qa[r][4 * grp + 3];
                    float S0, Mx, Mxx, My, Mxy, Myy, C0, C1, C2;
                    {
#pragma clang fp contract(fast)
                        const float ex = ph2_x0 - mrec.x, ey = ph2_y0 - mrec.y;
                        S0 = (q0.x + q1.x) + (q2.x + q3.x);
                        const float X1 = fmaf(3.f, q3.x, fmaf(2.f, q2.x, q1.x));  // sum v i
                        const float X2 = fmaf(9.f, q3.x, fmaf(4.f, q2.x, q1.x));  // sum v i^2
                        Mx = fmaf(ex, S0, X1);                                      // sum v (x - mx)
                        Mxx = fmaf(ex, Mx + X1, X2);                                // sum v (x - mx)^2
                        My = ey * S0;
                        Myy = ey * My;
                        Mxy = ey * Mx;
                        C0 = fmaf(q3.y, dpq[3].x, fmaf(q2.y, dpq[2].x, fmaf(q1.y, dpq[1].x, q0.y * dpq[0].x)));
                        C1 = fmaf(q3.y, dpq[3].y, fmaf(q2.y, dpq[2].y, fmaf(q1.y, dpq[1].y, q0.y * dpq[0].y)));
                        C2 = fmaf(q3.y, dpq[3].z, fmaf(q2.y, dpq[2].z, fmaf(q1.y, dpq[1].z, q0.y * dpq[0].z)));
                    }
                    // the nine sums in s_acc order, summed over the 16 groups g (lane bits 5, 4 transposed; bits 3,
                    // 2 by row rotations): afterwards lane 4 g + r with bits 2-3 clear holds record r's total of
                    // quantity (bit 5) + 2 (bit 4) [+ 4 for c1, 8 for c2]
                    const float c0 = sum4(sum8(pair16(pair32(Mx, My), pair32(Mxx, Mxy))));
                    const float c1 = sum4(sum8(pair16(pair32(Myy, S0), pair32(C0, C1))));
                    const float c2 = sum4(sum8(pair16(pair32(C2, 0.f), 0.f)));
                    wave_lds_handoff();  // phase-1 writes of the next hand-off must stay behind these reads
                    if (!(lane & 12) && K + r < nv) {
                        const int qk = ((lane >> 5) & 1) + ((lane >> 3) & 2);
                        atomicAdd(&s_acc[qk][rs], c0);
                        atomicAdd(&s_acc[4 + qk][rs], c1);
                        if (qk == 0) atomicAdd(&s_acc[8][rs], c2);
                    }
                };
                hand_off(std::integral_constant<int, 0>{});
                if (nv > 4) hand_off(std::integral_constant<int, 4>{});
                if (nv > 8) hand_off(std::integral_constant<int, 8>{});
                if (nv > 12) hand_off(std::integral_constant<int, 12>{});
            }
        };
        if (any_bg)
            walk(std::true_type{});
        else
            walk(std::false_type{});
        lds_barrier();
        if (tid < n) {  // finish record tid's sums in place: moments -> dL/dmean2D, the constant factors
            const float4 pc = s_pc[tid];
            const float4 bo = s_bo[tid];
            const float4 co = make_float4(-2.f * pc.z, bo.x, -2.f * pc.w, bo.z);  // exact: (a, b, c, o)
            const float o = co.w;  // the sums are over q = o G dL/dalpha; dL/dopacity = sum G dL/dalpha = S0 / o
            // phase 2 summed the first moments over x - mx, y - my: the reference's dx = mx - x flips them
            const float m0 = -s_acc[0][tid], m1 = -s_acc[1][tid];
            s_acc[0][tid] = (co.x * m0 + co.y * m1) * -ddelx_dx;
            s_acc[1][tid] = (co.z * m1 + co.y * m0) * -ddely_dy;
            s_acc[2][tid] *= -0.5f;
            s_acc[3][tid] *= -0.5f;
            s_acc[4][tid] *= -0.5f;
            s_acc[5][tid] = o > 0.f ? s_acc[5][tid] / o : 0.f;  // o = 0: alpha = 0, the record never took a pixel
        }
        lds_barrier();
        // One lane per (record, quantity): a wave-instruction's atomics cover ~7 records' nine-float runs,
        // each inside one 64-B segment of its Gaussian's gradient record -- ~7 memory-side atomic requests
        // instead of 64 when every lane adds one quantity of a different Gaussian (0.43 of 1.16 ms).
        for (int e = tid; e < n * kRecUsed; e += kTilePix) {
            const int r = e / kRecUsed, q = e - kRecUsed * r;
            const float a = s_acc[q][r];
            if (a != 0.f) atomicAdd(p.grad_rec + (size_t)s_id[r] * kGradRec + q, a);
        }
    }
#ifdef GSD_COUNT_WORK
    count_work(2, n_steps, n_pairs);
#endif
}

// Transposed reduction steps inside a 16-lane row.  DPP bank b is lanes 4b .. 4b + 3 of each row, so a bank mask
// selects by lane bits 3:2, and a DPP move with a partial bank mask writes only those lanes (the others keep
// `old`).  row_ror:N gives lane l the value of lane (l - N) mod 16.
// tstep8: lanes with bit 3 clear return a(l) + a(l ^ 8), lanes with bit 3 set b(l) + b(l ^ 8).  Three VALU ops for
// a pair of quantities: two full-row DPP adds (row_ror:8) and a select on the lane's bit 3 -- the bank-masked moves
// of the round-5 first form needed a register copy of the masked move's `old` on top (four ops; GSD_TSTEP_BANKS)
#ifndef GSD_TSTEP_BANKS
__device__ __forceinline__ float tstep8(float a, float b) {
    const float sa = a + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x128, 0xf, 0xf, true));
    const float sb = b + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(b), 0x128, 0xf, 0xf, true));
    return (__lane_id() & 8) ? sb : sa;
}
// tstep4: lanes with bit 2 clear return a(l) + a(l ^ 4), lanes with bit 2 set b(l) + b(l ^ 4): the partner is
// l + 4 (row_ror:12) for bit 2 clear and l - 4 (row_ror:4) for bit 2 set.
__device__ __forceinline__ float tstep4(float a, float b) {
    const float sa = a + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x12c, 0xf, 0xf, true));
    const float sb = b + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(b), 0x124, 0xf, 0xf, true));
    return (__lane_id() & 4) ? sb : sa;
}
#else
__device__ __forceinline__ float tstep8(float a, float b) {
    const int u = __builtin_amdgcn_update_dpp(__float_as_int(a), __float_as_int(b), 0x128, 0xf, 0xc, false);
    const int v = __builtin_amdgcn_update_dpp(__float_as_int(b), __float_as_int(a), 0x128, 0xf, 0x3, false);
    return __int_as_float(u) + __int_as_float(v);
}
// tstep4: lanes with bit 2 clear return a(l) + a(l ^ 4), lanes with bit 2 set b(l) + b(l ^ 4): the partner is
// l - 4 (row_ror:4) for bit 2 set and l + 4 (row_ror:12) for bit 2 clear.
__device__ __forceinline__ float tstep4(float a, float b) {
    const int u = __builtin_amdgcn_update_dpp(__float_as_int(a), __float_as_int(b), 0x124, 0xf, 0xa, false);
    const int v = __builtin_amdgcn_update_dpp(__float_as_int(b), __float_as_int(a), 0x12c, 0xf, 0x5, false);
    return __int_as_float(u) + __int_as_float(v);
}
#endif

// Backward with one record list per 4x4 lane group.  The wave's four 16-lane rows are the forward's four 4x4 pixel
// blocks, and each row walks its own list (bwd_compact_groups): a wave step serves four (block, record) pairs, one per
// row, instead of one record over the 8x8 quadrant.  Everything per record stays row-local:
// - lane u of a row loads its row's list entry j0 + u, and record U reaches the row's lanes by DPP row_newbcast:U
//   (different records in different rows, one LDS read per lane per 16 entries, as in the quadrant kernel);
// - phase 1 is unchanged: each lane replays its pixel and hands (o G dL/dalpha, alpha T) of four records to LDS;
// - phase 2: lane 16 g + 4 r' + r sums record r of row g over the four pixels of block row r' (its own quad), then
//   two transposed DPP steps inside the row (tstep8, tstep4: full-row DPP adds and a lane select) leave each lane two of
//   the record's nine sums (and the ninth in the lanes with bits 3:2 clear): three LDS adds per lane and hand-off,
//   as in the quadrant kernel, into the tile's accumulators.
//   The accumulators are doubles: each (row, record) pair leaves its own nine sums (12.8M pairs at cfg4, against
//   4.9M (wave, record) pairs in the quadrant kernel), and on gfx950 ds_add_f32 costs ~3 LDS cycles per LANE (192 per
//   64-lane instruction) while ds_add_f64 costs 8 per instruction (scripts/calib/lds_rate.hip).
// LDS: 24.7 KB at 128-record batches (the Gaussian ids of a batch wait in registers and go through the hand-off
// region for the flush); five waves per SIMD (the register limit).
// Round 5, measured at cfg4 (profiles/round5/render_bwd/): 3.57M wave steps instead of 4.92M, 0.532 useful lanes
// instead of 0.386 (GSD_COUNT_WORK), parity green; 0.398 ms against 0.477 for the quadrant kernel (-DGSD_BWD_QUADRANT).
// Along the way: ds_add_f32 accumulators 0.735 ms, compare-and-swap float adds 0.489, plain stores in their place
// (timing only) 0.38.
// records staged per batch: the double accumulators below take 72 B per record, so 128 keep the workgroup's LDS at
// 24.6 KB (five workgroups per CU, the register limit)
constexpr int kGB = 128;
#ifndef GSD_BWD_GROUPS_WAVES
#define GSD_BWD_GROUPS_WAVES 5
#endif
template <bool kRef>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSD_BWD_GROUPS_WAVES))) void k_render_bwd(
    RenderBwdParams p) {
    __shared__ float4 s_pc[kGB];   // stage_pc: mx, my, -a/2, -c/2
    __shared__ float2 s_bo[kGB];   // b, t_o
    __shared__ float4 s_rgb[kGB];  // r, g, b, o
    // record t's nine sums at [9 t + q], in double: ds_add_f64 costs 8 LDS cycles per 64-lane instruction on gfx950
    // against 192 for ds_add_f32 (scripts/calib/lds_rate.hip); the odd pitch spreads a lane group's per-record
    // accesses over the banks, and the flush reads it linearly
    __shared__ double s_acc[kRecUsed * kGB];
    __shared__ __attribute__((aligned(4))) uint8_t s_list[4][4][kGB];  // [wave][group][entry]
    // the alpha boxes are read by the compaction only, the hand-off buffer by the walk only, the Gaussian ids by
    // the flush only (barriers apart)
    __shared__ union {
        float4 box[kGB];
        float2 qa[4][kBwdGroup][65];  // per wave: per record and pixel; +1 pad
        uint32_t id[kGB];
    } s_u;
    __shared__ int s_tile_lc;
    const TileGeom tg = tile_geom(p.num_tiles, p.grid_x, p.W, p.H, true);  // the forward's 4x4-group lane map
    const int tid = threadIdx.x;
    const int lane = tg.lane, u16 = lane & 15, grp = lane >> 4;
    const uint2 rg = p.ranges[tg.tile];
    const int pid = p.W * tg.py + tg.px;
    const int plane = p.H * p.W;
    const bool inside = tg.inside;
    // per-pixel replay state (backward.cu:441-461)
    const float T_final = inside ? p.final_T[pid] : 0.f;
    float T = T_final;
    const int last_contributor = inside ? (int)p.n_contrib[pid] : 0;
    // Every pixel skips list positions >= its last contributor (backward.cu:487-488): the replay starts at the
    // tile's largest last contributor, and each group's list drops positions beyond its own largest.
    int row_lc = last_contributor;
    row_lc = max(row_lc, __shfl_xor(row_lc, 8));
    row_lc = max(row_lc, __shfl_xor(row_lc, 4));
    row_lc = max(row_lc, __shfl_xor(row_lc, 2));
    row_lc = max(row_lc, __shfl_xor(row_lc, 1));
    int glc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) glc[g] = __builtin_amdgcn_readlane(row_lc, 16 * g);
    if (tid == 0) s_tile_lc = 0;
    lds_barrier();
    if (lane == 0) atomicMax(&s_tile_lc, max(max(glc[0], glc[1]), max(glc[2], glc[3])));
    lds_barrier();
    const int total = min((int)(rg.y - rg.x), s_tile_lc);
    const uint32_t end = rg.x + (uint32_t)total;
    const int rounds = (total + kGB - 1) / kGB;
    int toDo = total;
    float dpix0 = 0.f, dpix1 = 0.f, dpix2 = 0.f;
    if (inside) {
        dpix0 = p.dL_dpix[pid];
        dpix1 = p.dL_dpix[plane + pid];
        dpix2 = p.dL_dpix[2 * plane + pid];
    }
    float2(*qa)[65] = s_u.qa[tg.wave];
    // dL/dpixel of the four pixels of the lane's quad (DPP quad broadcasts), for phase 2 below
    float3 dpq[4];
    dpq[0] = make_float3(quad_bcast<0>(dpix0), quad_bcast<0>(dpix1), quad_bcast<0>(dpix2));
    dpq[1] = make_float3(quad_bcast<1>(dpix0), quad_bcast<1>(dpix1), quad_bcast<1>(dpix2));
    dpq[2] = make_float3(quad_bcast<2>(dpix0), quad_bcast<2>(dpix1), quad_bcast<2>(dpix2));
    dpq[3] = make_float3(quad_bcast<3>(dpix0), quad_bcast<3>(dpix1), quad_bcast<3>(dpix2));
    float adot = 0.f;  // accum_rec . dL/dpixel (accum_rec with last_color / last_alpha folded in)
    const float bg_dot = p.bg[0] * dpix0 + p.bg[1] * dpix1 + p.bg[2] * dpix2;
    const float kbg = -T_final * bg_dot;
    const bool any_bg = wave_ballot(kbg != 0.f) != 0;  // wave-uniform
    const float pxf = (float)tg.px, pyf = (float)tg.py;
    const uint8_t* my_list = s_list[tg.wave][grp];
#ifdef GSD_COUNT_WORK
    unsigned long long n_steps = 0, n_pairs = 0;
#endif
    // phase 2: the first pixel of the lane's block row (the quad's four pixels are x0 .. x0 + 3 on row y0)
    const float ph2_x0 = tg.qx0 + (float)(4 * (grp & 1)), ph2_y0 = tg.qy0 + (float)(4 * (grp >> 1) + ((lane >> 2) & 3));
    // phase 2's accumulator rows: lane bits 3:2 = (1, 0) -> quantity 1, (0, 1) -> 2 (tstep8 keeps a pair's first
    // member where bit 3 is clear, tstep4 where bit 2 is clear)
    const int qsel = ((lane >> 3) & 1) | ((lane >> 1) & 2);

    for (int i = 0; i < rounds; ++i, toDo -= kGB) {
        lds_barrier();
        const int progress = i * kGB + tid;
        uint32_t gid = 0;
        if (tid < kGB && progress < total) {  // loaded back to front (backward.cu:466-478)
            gid = p.point_list[end - progress - 1];
            const RenderRec* r = p.rec + gid;
            const float4 q0 = r->q0, q1 = r->q1, q2 = r->q2;
            s_pc[tid] = stage_pc(make_float2(q0.x, q0.y), make_float4(q0.z, q0.w, q1.x, q1.y));
            s_bo[tid] = make_float2(q0.w, q2.y);               // b, t_o
            s_rgb[tid] = make_float4(q1.z, q1.w, q2.x, q1.y);  // r, g, b, o
            s_u.box[tid] = r->box;
        }
        for (int e = tid; e < kRecUsed * kGB; e += kTilePix) s_acc[e] = 0.0;
        lds_barrier();
        const int n = min(kGB, toDo);
        // slot t of this batch is list position (total - 1 - i*kGB - t) counted from the front
        const int front_base = total - 1 - i * kGB;
        int t_min[4], cnt[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) t_min[g] = front_base - glc[g] + 1;
        bwd_compact_groups<kGB>(s_u.box, s_pc, s_bo, s_list[tg.wave], n, tg.qx0, tg.qy0, lane, t_min, cnt);
        const int m = max(max(cnt[0], cnt[1]), max(cnt[2], cnt[3]));  // the longest list (wave-uniform)
        const int mine = grp == 0 ? cnt[0] : grp == 1 ? cnt[1] : grp == 2 ? cnt[2] : cnt[3];
        // backward.cu:487-488: a pixel replays list position front_base - t only below its last contributor, i.e.
        // slot t counts for this pixel iff t > t_cut
        const int t_cut = front_base - last_contributor;
        lds_barrier();  // every wave is done with the boxes before s_u.qa is written
        auto walk = [&](auto with_bg) {
            constexpr bool kBg = decltype(with_bg)::value;
            for (int j0 = 0; j0 < m; j0 += 16) {
                const int nv = m - j0;      // entries left in the longest list (wave-uniform)
                const int nvm = mine - j0;  // entries left in the lane's group's list (row-uniform)
                const bool in_list = u16 < nvm;
                const int slot = (int)my_list[j0 + u16];
                const int rslot = in_list ? slot : 0;  // slot 0 past the list: finite, never taken (rkey)
                const int rkey = in_list ? slot : -__INT_MAX__ - 1;
                const float4 rpc = s_pc[rslot];
                const float2 rbo = s_bo[rslot];
                const float4 rrgb = s_rgb[rslot];
                auto hand_off = [&](auto kc) {
                    constexpr int K = decltype(kc)::value;
                    const int r = lane & 3;
                    // phase 2's record (entry K + r of the row's list) and its mean, read ahead of phase 1
                    const bool own = K + r < nvm;
                    const int rs = own ? (int)my_list[j0 + K + r] : 0;
                    const float2 mrec = *reinterpret_cast<const float2*>(&s_pc[rs]);
                    double* acc = s_acc + kRecUsed * rs;
                    unsigned long long any_m = 0;  // lanes that took any record of the hand-off
                    auto rec = [&](auto uc) {
                        constexpr int U = K + decltype(uc)::value;
                        const float4 pc = make_float4(row_bcast<U>(rpc.x), row_bcast<U>(rpc.y), row_bcast<U>(rpc.z),
                                                      row_bcast<U>(rpc.w));
                        const float2 bo = make_float2(row_bcast<U>(rbo.x), row_bcast<U>(rbo.y));
                        bool keep, over;
                        const float OG = record_og<kRef>(pc, bo, pxf, pyf, keep, over,
                                                         kRef ? row_bcast<U>(rrgb.w) : 0.f);  // before the 0.99 clamp
                        // backward.cu:487-488 (list position below the pixel's last contributor; INT_MIN past the
                        // row's list), :490-501
                        const unsigned long long valid_m =
                            wave_ballot(row_bcast_i<U>(rkey) > t_cut) & wave_ballot(keep) & wave_ballot(over);
                        any_m |= valid_m;
#ifdef GSD_COUNT_WORK
                        n_steps += U < nv ? 1 : 0;
                        n_pairs += __popcll(valid_m);
#endif
                        {
#pragma clang fp contract(fast)
                            const bool valid = __builtin_amdgcn_inverse_ballot_w64(valid_m);
                            const float og = valid ? OG : 0.f;
                            const float alpha = fminf(0.99f, og);
                            const float inv1ma = fast_recip(1.f - alpha);
                            T = T * inv1ma;  // backward.cu:503 (T recovered by division)
#ifndef GSD_BWD_NO_FMAC_DPP
                            const float cd = fmac_bcast<U>(rrgb.z, dpix2,
                                                           fmac_bcast<U>(rrgb.y, dpix1, row_bcast<U>(rrgb.x) * dpix0));
#else
                            const float cd = fmaf(row_bcast<U>(rrgb.z), dpix2,
                                                  fmaf(row_bcast<U>(rrgb.y), dpix1, row_bcast<U>(rrgb.x) * dpix0));
#endif
                            const float diff = cd - adot;
                            // backward.cu:512-529 (kbg = 0: fmaf(diff, T, -0) is diff * T, bit for bit)
                            const float dL_dalpha = kBg ? fmaf(diff, T, kbg * inv1ma) : diff * T;
                            qa[U & 3][lane] = make_float2(og * dL_dalpha, alpha * T);
                            adot = fmaf(alpha, diff, adot);
                        }
                    };
                    rec(std::integral_constant<int, 0>{});
                    rec(std::integral_constant<int, 1>{});
                    rec(std::integral_constant<int, 2>{});
                    rec(std::integral_constant<int, 3>{});
                    if (!any_m) return;  // wave-uniform: no pixel took any of these records
#if GSD_BWD_ABLATE & 1
                    return;  // timing only: no phase 2
#endif
                    wave_lds_handoff();
                    // Phase 2 (record-major), as in the quadrant kernel: lane 4 G + r sums its row's record K + r over
                    // the four pixels of its quad, (x0 + i, y0), i = 0..3, from the moments S0 = sum v,
                    // X1 = sum v i, X2 = sum v i^2 centred on the record mean (ex, ey), and C = sum w dL/dpixel.
                    const float2 q0 = qa[r][(lane & ~3)], q1 = qa[r][(lane & ~3) + 1], q2 = qa[r][(lane & ~3) + 2],
                                 q3 = qa[r][(lane & ~3) + 3];
                    float S0, Mx, Mxx, My, Mxy, Myy, C0, C1, C2;
                    {
#pragma clang fp contract(fast)
                        const float ex = ph2_x0 - mrec.x, ey = ph2_y0 - mrec.y;
                        S0 = (q0.x + q1.x) + (q2.x + q3.x);
                        const float X1 = fmaf(3.f, q3.x, fmaf(2.f, q2.x, q1.x));  // sum v i
                        const float X2 = fmaf(9.f, q3.x, fmaf(4.f, q2.x, q1.x));  // sum v i^2
                        Mx = fmaf(ex, S0, X1);                                      // sum v (x - mx)
                        Mxx = fmaf(ex, Mx + X1, X2);                                // sum v (x - mx)^2
                        My = ey * S0;
                        Myy = ey * My;
                        Mxy = ey * Mx;
                        C0 = fmaf(q3.y, dpq[3].x, fmaf(q2.y, dpq[2].x, fmaf(q1.y, dpq[1].x, q0.y * dpq[0].x)));
                        C1 = fmaf(q3.y, dpq[3].y, fmaf(q2.y, dpq[2].y, fmaf(q1.y, dpq[1].y, q0.y * dpq[0].y)));
                        C2 = fmaf(q3.y, dpq[3].z, fmaf(q2.y, dpq[2].z, fmaf(q1.y, dpq[1].z, q0.y * dpq[0].z)));
                    }
                    // the record's sums over the row's four quads: lane bits 3:2 = (b3, b2) end with quantity
                    // qsel = b3 + 2 b2 of (Mx, My, Mxx, Mxy) in ca and of (Myy, S0, C0, C1) in cb; C2 everywhere
                    float ca = tstep4(tstep8(Mx, My), tstep8(Mxx, Mxy));
                    float cb = tstep4(tstep8(Myy, S0), tstep8(C0, C1));
                    float c2 = sum4(sum8(C2));
                    // computed here, ahead of the `own` branch: sunk into it, the last adds lost their DPP sources (a
                    // broadcast stays outside the branch as a v_mov_b32_dpp of its own)
                    asm volatile("" : "+v"(ca), "+v"(cb), "+v"(c2));
                    wave_lds_handoff();  // phase-1 writes of the next hand-off must stay behind these reads
#if GSD_BWD_ABLATE & 2
                    if (own && ca == 12345.f && cb == 0.5f && c2 == 0.25f) acc[0] = 1.0;  // timing only: no accumulation
                    return;
#endif
                    if (own) {  // the record's sums into the tile's accumulators (ds_add_f64)
                        atomicAdd(acc + qsel, (double)ca);
                        atomicAdd(acc + 4 + qsel, (double)cb);
                        if (!(lane & 12)) atomicAdd(acc + 8, (double)c2);
                    }
                };
                hand_off(std::integral_constant<int, 0>{});
                if (nv > 4) hand_off(std::integral_constant<int, 4>{});
                if (nv > 8) hand_off(std::integral_constant<int, 8>{});
                if (nv > 12) hand_off(std::integral_constant<int, 12>{});
            }
        };
#if !(GSD_BWD_ABLATE & 8)
        if (any_bg)
            walk(std::true_type{});
        else
            walk(std::false_type{});
#else
        if (m == 12345 && mine == 7 && t_cut == 3) walk(std::false_type{});  // timing only: no walk
#endif
        lds_barrier();
        if (tid < n) {  // finish record tid's sums in place: moments -> dL/dmean2D, the constant factors
            const float4 pc = s_pc[tid];
            const double b = s_bo[tid].x;
            const float o = s_rgb[tid].w;  // the sums are over q = o G dL/dalpha; dL/dopacity = sum G dL/dalpha = S0 / o
            const double a = -2.f * pc.z, c = -2.f * pc.w;  // exact
            double* acc = s_acc + kRecUsed * tid;
            // phase 2 summed the first moments over x - mx, y - my: the reference's dx = mx - x flips them
            const double m0 = -acc[0], m1 = -acc[1];
            // -(double)ddelx_dx, -(double)ddely_dy (= -W/2, -H/2 exactly) rebuilt here from the scalar image size: hoisted
            // out of the batch loop they were a VGPR pair the register limit spilled (8 B of scratch stored per lane,
            // reloaded every batch)
            int wh[2] = {p.W, p.H};
            asm volatile("" : "+s"(wh[0]), "+s"(wh[1]));
            acc[0] = (a * m0 + b * m1) * (-0.5 * (double)wh[0]);
            acc[1] = (c * m1 + b * m0) * (-0.5 * (double)wh[1]);
            acc[2] *= -0.5;
            acc[3] *= -0.5;
            acc[4] *= -0.5;
            acc[5] = o > 0.f ? acc[5] / (double)o : 0.0;  // o = 0: alpha = 0, the record never took a pixel
            s_u.id[tid] = gid;
        }
        lds_barrier();
        // One lane per (record, quantity): a wave-instruction's atomics cover ~7 records' nine-float runs,
        // each inside one 64-B segment of its Gaussian's gradient record.
#if !(GSD_BWD_ABLATE & 4)
        for (int e = tid; e < n * kRecUsed; e += kTilePix) {
            const int r = e / kRecUsed, q = e - kRecUsed * r;
            const float a = (float)s_acc[e];
            if (a != 0.f) atomicAdd(p.grad_rec + (size_t)s_u.id[r] * kGradRec + q, a);
        }
#endif
    }
#ifdef GSD_COUNT_WORK
    count_work(2, n_steps, n_pairs);
#endif
}

void launch_render_fwd(const RenderParams& p, hipStream_t s) {
    if (p.num_tiles <= 0) return;
    if (p.ref_alpha)
        hipLaunchKernelGGL(k_render_fwd<true>, dim3(p.num_tiles), dim3(kTilePix), 0, s, p);
    else
        hipLaunchKernelGGL(k_render_fwd<false>, dim3(p.num_tiles), dim3(kTilePix), 0, s, p);
}
void launch_render_bwd(const RenderBwdParams& p, hipStream_t s) {
#ifdef GSD_BWD_QUADRANT
    if (p.num_tiles > 0) hipLaunchKernelGGL(k_render_bwd_quadrant, dim3(p.num_tiles), dim3(kTilePix), 0, s, p);
#else
    if (p.num_tiles <= 0) return;
    if (p.ref_alpha)
        hipLaunchKernelGGL(k_render_bwd<true>, dim3(p.num_tiles), dim3(kTilePix), 0, s, p);
    else
        hipLaunchKernelGGL(k_render_bwd<false>, dim3(p.num_tiles), dim3(kTilePix), 0, s, p);
#endif
}

}  // namespace gsd

extern "C" int gsd_work_counters(int32_t n, uint64_t* out, int32_t reset) {
    if (n < 0 || (n > 0 && !out)) return GSD_ERR_ARG;
    unsigned long long v[4] = {0, 0, 0, 0};
#ifdef GSD_COUNT_WORK
    if (hipDeviceSynchronize() != hipSuccess) return GSD_ERR_HIP;
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(gsd::g_work), sizeof(v)) != hipSuccess) return GSD_ERR_HIP;
    if (reset) {
        const unsigned long long z[4] = {0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gsd::g_work), z, sizeof(z)) != hipSuccess) return GSD_ERR_HIP;
    }
#else
    (void)reset;
#endif
    for (int i = 0; i < n && i < 4; ++i) out[i] = v[i];
    return GSD_OK;
}
