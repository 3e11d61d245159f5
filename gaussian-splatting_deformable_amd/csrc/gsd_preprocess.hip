// gsd_preprocess.hip -- per-Gaussian kernels of the hot path (forward and backward).
//
// One lane per Gaussian, 256-lane workgroups (4 waves).  These kernels are
// HBM-bound (DESIGN.md roofline table): ~60 B of position/shape/opacity +
// 12*(D+1)^2 B of SH read per Gaussian, ~50 B written.  VALU 3x3 chains are
// cheaper than packing single 3x3 products into MFMA tiles (a 16x16x4 f32 MFMA
// wastes >90% of its lanes on one Gaussian's 3x3), so there is no MFMA here.
#include "gsd_kernels.h"

namespace gsd {

// ---------------------------------------------------------------------------
// SH -> RGB, forward.cu:20-71 (per channel, identical expression tree)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sh_channel(int deg, const float* __restrict__ s, float x, float y, float z) {
    // s[3*k] is coefficient k of this channel
    float res = kSH0 * s[0];
    if (deg > 0) {
        res = res - kSH1 * y * s[3] + kSH1 * z * s[6] - kSH1 * x * s[9];
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            res = res + kSH2_0 * xy * s[12] + kSH2_1 * yz * s[15] + kSH2_2 * (2.0f * zz - xx - yy) * s[18] +
                  kSH2_3 * xz * s[21] + kSH2_4 * (xx - yy) * s[24];
            if (deg > 2) {
                res = res + kSH3_0 * y * (3.0f * xx - yy) * s[27] + kSH3_1 * xy * z * s[30] +
                      kSH3_2 * y * (4.0f * zz - xx - yy) * s[33] +
                      kSH3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * s[36] +
                      kSH3_4 * x * (4.0f * zz - xx - yy) * s[39] + kSH3_5 * z * (xx - yy) * s[42] +
                      kSH3_6 * x * (xx - 3.0f * yy) * s[45];
            }
        }
    }
    return res + 0.5f;
}

// Stage one Gaussian's active SH coefficients (3*(D+1)^2 floats, <= 48) into
// registers: from its (P,M,3) row, or from the split operand (dc | rest, plus
// the optional offset -- the same float add as the reference's
// get_features + mlp_shs, gaussian_renderer/__init__.py:134).
// Element strides of the split operand: element e of Gaussian g at [g * sg + e * se] (gsd_sh_split).
struct ShStrides {
    long long dc_sg, dc_se, rest_sg, rest_se;
};
// kStr = false: contiguous rows, strides as compile-time constants (so the row loads stay wide); the
// general strided form is a separate instantiation (launchers pick by the strides).
template <bool kStr, typename Prm>
__device__ __forceinline__ ShStrides sh_strides(const Prm& p) {
    if (kStr) return ShStrides{p.dc_sg, p.dc_se, p.rest_sg, p.rest_se};
    return ShStrides{3, 1, 3LL * (p.M - 1), 1};
}

// kSrc: which operand holds the coefficients -- -1 decided at run time, 0 shs, 1 the split operand, 2 the
// split operand plus an offset.  A compile-time source keeps the other paths' loads out of the kernel's
// register allocation (the offset path alone holds 96 loaded values).
template <int NC, int kSrc = -1>
__device__ __forceinline__ void load_sh(const float* __restrict__ shs, const float* __restrict__ dc,
                                        const float* __restrict__ rest, const float* __restrict__ off, int M,
                                        int idx, float (&s)[48], const ShStrides& st) {
    if (kSrc < 0 ? shs != nullptr : kSrc == 0) {
        const float* row = shs + (size_t)idx * M * 3;
#pragma unroll
        for (int k = 0; k < NC * 3; ++k) s[k] = row[k];
        return;
    }
    // contiguous rows (element stride 1) keep compile-time offsets (wide loads); 2x faster than the general
    // strided form on them
    const float* d = dc + idx * st.dc_sg;
    if (st.dc_se == 1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) s[k] = d[k];
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) s[k] = d[k * st.dc_se];
    }
    const float* r = rest + idx * st.rest_sg;
    if (st.rest_se == 1) {
#pragma unroll
        for (int k = 3; k < NC * 3; ++k) s[k] = r[k - 3];
    } else {
#pragma unroll
        for (int k = 3; k < NC * 3; ++k) s[k] = r[(k - 3) * st.rest_se];
    }
    if (kSrc < 0 ? off != nullptr : kSrc == 2) {
        const float* o = off + (size_t)idx * M * 3;
#pragma unroll
        for (int k = 0; k < NC * 3; ++k) s[k] = s[k] + o[k];
    }
}

// The preamble's activations, the same float operations as k_activate_fwd (gsd_activate.hip): exp(scaling),
// F.normalize(rotation) (eps 1e-12), sigmoid(opacity) -- used when the rasterizer is handed raw parameters.
__device__ __forceinline__ float3 act_scale(const float* s, int i) {
    return make_float3(expf(s[3 * i]), expf(s[3 * i + 1]), expf(s[3 * i + 2]));
}
__device__ __forceinline__ float4 act_rot(float4 q) {
    const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);
    return make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
}
__device__ __forceinline__ float act_opac(float o) { return 1.f / (1.f + expf(-o)); }

template <int DEG>
__device__ __forceinline__ float3 sh_to_rgb(const float (&s)[48], float3 pos, float3 cam, uint8_t& clamp_bits) {
    constexpr int deg = DEG;
    float3 d = make_float3(pos.x - cam.x, pos.y - cam.y, pos.z - cam.z);
    const float len = sqrtf(dot3(d, d));
    d = make_float3(d.x / len, d.y / len, d.z / len);
    float3 rgb;
    rgb.x = sh_channel(deg, s + 0, d.x, d.y, d.z);
    rgb.y = sh_channel(deg, s + 1, d.x, d.y, d.z);
    rgb.z = sh_channel(deg, s + 2, d.x, d.y, d.z);
    clamp_bits = (uint8_t)((rgb.x < 0) | ((rgb.y < 0) << 1) | ((rgb.z < 0) << 2));
    rgb.x = rgb.x < 0.0f ? 0.0f : rgb.x;
    rgb.y = rgb.y < 0.0f ? 0.0f : rgb.y;
    rgb.z = rgb.z < 0.0f ? 0.0f : rgb.z;
    return rgb;
}

// forward.cu:74-113 computeCov2D -> (a, b, c) of the low-pass-filtered 2D covariance
__device__ __forceinline__ float3 cov2d_fwd(const float3 mean, float fx, float fy, float tanx, float tany,
                                            const Cov6& c3, const Mat4& V) {
    float3 t = xform_point3(mean, V);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const M3 J = m3_cols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0,
                         0, 0);
    const M3 W = m3_cols(V.m[0], V.m[4], V.m[8], V.m[1], V.m[5], V.m[9], V.m[2], V.m[6], V.m[10]);
    const M3 T = m3_mul(W, J);
    const M3 Vk = m3_cols(c3.v[0], c3.v[1], c3.v[2], c3.v[1], c3.v[3], c3.v[4], c3.v[2], c3.v[4], c3.v[5]);
    const M3 A = m3_mul(m3_T(T), m3_T(Vk));
    const M3 cov = m3_mul(A, T);
    return make_float3(cov.c[0].x + 0.3f, cov.c[0].y, cov.c[1].y + 0.3f);
}

// ---------------------------------------------------------------------------
// Forward preprocess: forward.cu:155-256 (+ the per-tile instance count of
// the binning stage, folded in so the rect is computed once).
// ---------------------------------------------------------------------------
template <int DEG, bool kStr>
__global__ __launch_bounds__(256) void k_preprocess_fwd(PreprocessParams p) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= p.P) return;
    const Mat4 V = load_mat4(p.view);
    const Mat4 Pm = load_mat4(p.proj);
    p.radii[idx] = 0;
    const float3 mean = make_float3(p.means3D[3 * idx], p.means3D[3 * idx + 1], p.means3D[3 * idx + 2]);
    // auxiliary.h:139-164 in_frustum (near plane only)
    const float3 pv = xform_point3(mean, V);
    if (pv.z <= 0.2f) {
        if (p.prefiltered) atomicOr(p.err_flags, kErrPrefiltered);
        return;
    }
    const float4 ph = xform_point4(mean, Pm);
    const float pw = 1.0f / (ph.w + 0.0000001f);
    const float ppx = ph.x * pw, ppy = ph.y * pw;

    Cov6 c3;
    if (p.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3.v[k] = p.cov3D_precomp[6 * idx + k];
    } else {
        float3 s = make_float3(p.scales[3 * idx], p.scales[3 * idx + 1], p.scales[3 * idx + 2]);
        float4 q = reinterpret_cast<const float4*>(p.rotations)[idx];
        if (p.raw_act) {
            s = act_scale(p.scales, idx);
            q = act_rot(q);
        }
        c3 = cov3d_from_scale_rot(s, p.scale_modifier, q);
    }
    const float3 cov = cov2d_fwd(mean, p.focal_x, p.focal_y, p.tan_fovx, p.tan_fovy, c3, V);
    const float det = (cov.x * cov.z - cov.y * cov.y);
    if (det == 0.0f) return;
    const float det_inv = 1.f / det;
    const float3 conic = make_float3(cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv);
    const float mid = 0.5f * (cov.x + cov.z);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    const float2 pix = make_float2(ndc_to_pix(ppx, p.W), ndc_to_pix(ppy, p.H));
    const Rect r = tile_rect(pix.x, pix.y, (int)my_radius, p.grid_x, p.grid_y);
    if ((r.x1 - r.x0) * (r.y1 - r.y0) == 0) return;

    float4 col;
    uint8_t cl = 0;
    if (p.colors_precomp) {
        col = make_float4(p.colors_precomp[3 * idx], p.colors_precomp[3 * idx + 1], p.colors_precomp[3 * idx + 2], 0.f);
    } else {
        const float3 cam = make_float3(p.campos[0], p.campos[1], p.campos[2]);
        float sh[48];
        load_sh<(DEG + 1) * (DEG + 1)>(p.shs, p.sh_dc, p.sh_rest, p.sh_off, p.M, idx, sh, sh_strides<kStr>(p));
        const float3 rgb = sh_to_rgb<DEG>(sh, mean, cam, cl);
        col = make_float4(rgb.x, rgb.y, rgb.z, 0.f);
    }
    p.clamped[idx] = cl;
    p.depths[idx] = pv.z;
    p.radii[idx] = (int)my_radius;
    p.means2D[idx] = pix;
    const float opac = p.raw_act ? act_opac(p.opacities[idx]) : p.opacities[idx];
    const float4 co = make_float4(conic.x, conic.y, conic.z, opac);
    RenderRec* rr = p.rec + idx;  // what the render kernels gather per instance (RenderRec)
    rr->q0 = make_float4(pix.x, pix.y, co.x, co.y);
    rr->q1 = make_float4(co.z, co.w, col.x, col.y);
    // t_o = -ln(255 o) in double, rounded to the nearest float: for a float power, power >= t_o is the real
    // comparison power >= -ln(255 o), i.e. o exp(power) >= 1/255, except where power equals t_o exactly (then
    // alpha lies within half an ulp of t_o of the threshold) -- the render kernels' alpha threshold
    // (gsd_render.hip record_og) -- and, with slack, the backward's ellipse culling (Q <= -2 t_o); the hardware
    // reciprocals of a and c.  (Rounded up, t_o made the comparison exact at ties too, but biased every alpha VALUE
    // low by up to an ulp of t_o, which the transmittance accumulates: 10 instead of 1 n_contrib flips at cfg4.)
    // A negative opacity gives alpha = min(0.99, o G) < 1/255 at every pixel (forward.cu:343-345): t_o = +inf takes
    // no pixel (power >= +inf is false) and culls the record from the backward's lists; -log of a negative would be
    // NaN, which passes every decision.  A NaN opacity keeps NaN: alpha = fminf(0.99, NaN) = 0.99, as upstream.
    const double t_o = co.w < 0.f ? INFINITY : -log(255.0 * (double)co.w);
    rr->q2 = make_float4(col.z, __double2float_rn(t_o), __builtin_amdgcn_rcpf(co.x), __builtin_amdgcn_rcpf(co.z));
    rr->box = alpha_box(pix, co);
    // per-tile instance counts by global atomics -- only on the fallback path for very
    // large tile grids; normally k_tile_hist builds them from LDS histograms instead
    if (!p.tile_count) return;
    for (int y = r.y0; y < r.y1; ++y)
        for (int x = r.x0; x < r.x1; ++x)
            __hip_atomic_fetch_add(p.tile_count + (y * p.grid_x + x), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// auxiliary.h:139-164 via rasterizer_impl.cu:54-66 checkFrustum
__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* __restrict__ means3D,
                                                      const float* __restrict__ view, uint8_t* __restrict__ present) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= P) return;
    const Mat4 V = load_mat4(view);
    const float3 mean = make_float3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
    present[idx] = (uint8_t)!(xform_point3(mean, V).z <= 0.2f);
}

// ---------------------------------------------------------------------------
// Backward: computeCov2DCUDA (backward.cu:144-274) + preprocessCUDA
// (backward.cu:346-396: projective mean term, SH backward :20-139, cov3D
// backward :278-341) fused into one pass over the Gaussians.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cov2d_bwd(const float3 mean, const Cov6& c3, float hx, float hy, float tanx,
                                          float tany, const Mat4& Vm, const float3 dc, float3& dmean, Cov6& dcov) {
    float3 t = xform_point3(mean, Vm);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float xgm = txtz < -limx || txtz > limx ? 0 : 1;
    const float ygm = tytz < -limy || tytz > limy ? 0 : 1;
    const M3 J = m3_cols(hx / t.z, 0.0f, -(hx * t.x) / (t.z * t.z), 0.0f, hy / t.z, -(hy * t.y) / (t.z * t.z), 0,
                         0, 0);
    const M3 W = m3_cols(Vm.m[0], Vm.m[4], Vm.m[8], Vm.m[1], Vm.m[5], Vm.m[9], Vm.m[2], Vm.m[6], Vm.m[10]);
    const M3 V = m3_cols(c3.v[0], c3.v[1], c3.v[2], c3.v[1], c3.v[3], c3.v[4], c3.v[2], c3.v[4], c3.v[5]);
    const M3 T = m3_mul(W, J);
    const M3 cov2 = m3_mul(m3_mul(m3_T(T), m3_T(V)), T);
    const float a = cov2.c[0].x + 0.3f;
    const float b = cov2.c[0].y;
    const float c = cov2.c[1].y + 0.3f;
    const float denom = a * c - b * b;
    float dL_da = 0, dL_db = 0, dL_dc = 0;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    // T[col][row] accessors
    const float T00 = T.c[0].x, T01 = T.c[0].y, T02 = T.c[0].z, T10 = T.c[1].x, T11 = T.c[1].y, T12 = T.c[1].z;
    // backward.cu:204-228: everything stays 0 when denom2inv == 0 -- as selects, not a branch (the branch made the
    // compiler keep dcov in scratch memory)
    const bool inv_ok = denom2inv != 0;
    dL_da = inv_ok ? denom2inv * (-c * c * dc.x + 2 * b * c * dc.y + (denom - a * c) * dc.z) : 0.f;
    dL_dc = inv_ok ? denom2inv * (-a * a * dc.z + 2 * a * b * dc.y + (denom - a * c) * dc.x) : 0.f;
    dL_db = inv_ok ? denom2inv * 2 * (b * c * dc.x - (denom + 2 * b * b) * dc.y + a * b * dc.z) : 0.f;
    {
        const float v0 = (T00 * T00 * dL_da + T00 * T10 * dL_db + T10 * T10 * dL_dc);
        const float v3 = (T01 * T01 * dL_da + T01 * T11 * dL_db + T11 * T11 * dL_dc);
        const float v5 = (T02 * T02 * dL_da + T02 * T12 * dL_db + T12 * T12 * dL_dc);
        const float v1 = 2 * T00 * T01 * dL_da + (T00 * T11 + T01 * T10) * dL_db + 2 * T10 * T11 * dL_dc;
        const float v2 = 2 * T00 * T02 * dL_da + (T00 * T12 + T02 * T10) * dL_db + 2 * T10 * T12 * dL_dc;
        const float v4 = 2 * T02 * T01 * dL_da + (T01 * T12 + T02 * T11) * dL_db + 2 * T11 * T12 * dL_dc;
        dcov.v[0] = inv_ok ? v0 : 0.f;
        dcov.v[1] = inv_ok ? v1 : 0.f;
        dcov.v[2] = inv_ok ? v2 : 0.f;
        dcov.v[3] = inv_ok ? v3 : 0.f;
        dcov.v[4] = inv_ok ? v4 : 0.f;
        dcov.v[5] = inv_ok ? v5 : 0.f;
    }
    // Vrk[col][row]
    const float V00 = V.c[0].x, V01 = V.c[0].y, V02 = V.c[0].z, V10 = V.c[1].x, V11 = V.c[1].y, V12 = V.c[1].z,
                V20 = V.c[2].x, V21 = V.c[2].y, V22 = V.c[2].z;
    const float dT00 = 2 * (T00 * V00 + T01 * V01 + T02 * V02) * dL_da + (T10 * V00 + T11 * V01 + T12 * V02) * dL_db;
    const float dT01 = 2 * (T00 * V10 + T01 * V11 + T02 * V12) * dL_da + (T10 * V10 + T11 * V11 + T12 * V12) * dL_db;
    const float dT02 = 2 * (T00 * V20 + T01 * V21 + T02 * V22) * dL_da + (T10 * V20 + T11 * V21 + T12 * V22) * dL_db;
    const float dT10 = 2 * (T10 * V00 + T11 * V01 + T12 * V02) * dL_dc + (T00 * V00 + T01 * V01 + T02 * V02) * dL_db;
    const float dT11 = 2 * (T10 * V10 + T11 * V11 + T12 * V12) * dL_dc + (T00 * V10 + T01 * V11 + T02 * V12) * dL_db;
    const float dT12 = 2 * (T10 * V20 + T11 * V21 + T12 * V22) * dL_dc + (T00 * V20 + T01 * V21 + T02 * V22) * dL_db;
    // W[col][row]
    const float W00 = W.c[0].x, W01 = W.c[0].y, W02 = W.c[0].z, W10 = W.c[1].x, W11 = W.c[1].y, W12 = W.c[1].z,
                W20 = W.c[2].x, W21 = W.c[2].y, W22 = W.c[2].z;
    const float dJ00 = W00 * dT00 + W01 * dT01 + W02 * dT02;
    const float dJ02 = W20 * dT00 + W21 * dT01 + W22 * dT02;
    const float dJ11 = W10 * dT10 + W11 * dT11 + W12 * dT12;
    const float dJ12 = W20 * dT10 + W21 * dT11 + W22 * dT12;
    const float tz = 1.f / t.z;
    const float tz2 = tz * tz;
    const float tz3 = tz2 * tz;
    const float dtx = xgm * -hx * tz2 * dJ02;
    const float dty = ygm * -hy * tz2 * dJ12;
    const float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * t.x) * tz3 * dJ02 + (2 * hy * t.y) * tz3 * dJ12;
    dmean = xform_vec3_T(make_float3(dtx, dty, dtz), Vm);
}

// auxiliary.h:107-117 dnormvdv(float3)
__device__ __forceinline__ float3 dnormvdv(const float3 v, const float3 dv) {
    const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    return make_float3(((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32,
                       (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32,
                       (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32);
}

// backward.cu:20-139 for one channel: writes the channel's dL/dsh, returns its (dRGB/dx, dRGB/dy, dRGB/dz)
__device__ __forceinline__ float3 sh_channel_bwd(int deg, const float* __restrict__ s, float dRGB, float x, float y,
                                                 float z, float* __restrict__ dsh) {
    float dx = 0, dy = 0, dz = 0;
    dsh[0] = kSH0 * dRGB;
    if (deg > 0) {
        dsh[3] = (-kSH1 * y) * dRGB;
        dsh[6] = (kSH1 * z) * dRGB;
        dsh[9] = (-kSH1 * x) * dRGB;
        dx = -kSH1 * s[9];
        dy = -kSH1 * s[3];
        dz = kSH1 * s[6];
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            dsh[12] = (kSH2_0 * xy) * dRGB;
            dsh[15] = (kSH2_1 * yz) * dRGB;
            dsh[18] = (kSH2_2 * (2.f * zz - xx - yy)) * dRGB;
            dsh[21] = (kSH2_3 * xz) * dRGB;
            dsh[24] = (kSH2_4 * (xx - yy)) * dRGB;
            dx += kSH2_0 * y * s[12] + kSH2_2 * 2.f * -x * s[18] + kSH2_3 * z * s[21] + kSH2_4 * 2.f * x * s[24];
            dy += kSH2_0 * x * s[12] + kSH2_1 * z * s[15] + kSH2_2 * 2.f * -y * s[18] + kSH2_4 * 2.f * -y * s[24];
            dz += kSH2_1 * y * s[15] + kSH2_2 * 2.f * 2.f * z * s[18] + kSH2_3 * x * s[21];
            if (deg > 2) {
                dsh[27] = (kSH3_0 * y * (3.f * xx - yy)) * dRGB;
                dsh[30] = (kSH3_1 * xy * z) * dRGB;
                dsh[33] = (kSH3_2 * y * (4.f * zz - xx - yy)) * dRGB;
                dsh[36] = (kSH3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy)) * dRGB;
                dsh[39] = (kSH3_4 * x * (4.f * zz - xx - yy)) * dRGB;
                dsh[42] = (kSH3_5 * z * (xx - yy)) * dRGB;
                dsh[45] = (kSH3_6 * x * (xx - 3.f * yy)) * dRGB;
                dx += (kSH3_0 * s[27] * 3.f * 2.f * xy + kSH3_1 * s[30] * yz + kSH3_2 * s[33] * -2.f * xy +
                       kSH3_3 * s[36] * -3.f * 2.f * xz + kSH3_4 * s[39] * (-3.f * xx + 4.f * zz - yy) +
                       kSH3_5 * s[42] * 2.f * xz + kSH3_6 * s[45] * 3.f * (xx - yy));
                dy += (kSH3_0 * s[27] * 3.f * (xx - yy) + kSH3_1 * s[30] * xz +
                       kSH3_2 * s[33] * (-3.f * yy + 4.f * zz - xx) + kSH3_3 * s[36] * -3.f * 2.f * yz +
                       kSH3_4 * s[39] * -2.f * xy + kSH3_5 * s[42] * -2.f * yz + kSH3_6 * s[45] * -3.f * 2.f * xy);
                dz += (kSH3_1 * s[30] * xy + kSH3_2 * s[33] * 4.f * 2.f * yz +
                       kSH3_3 * s[36] * 3.f * (2.f * zz - xx - yy) + kSH3_4 * s[39] * 4.f * 2.f * xz +
                       kSH3_5 * s[42] * (xx - yy));
            }
        }
    }
    return make_float3(dx, dy, dz);
}

__device__ __forceinline__ void cov3d_bwd(const float3 scale, float mod, const float4 q, const Cov6& dc,
                                          float3& dscale, float4& drot) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    const M3 R = quat_to_R(q);
    M3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    const float3 s = make_float3(mod * scale.x, mod * scale.y, mod * scale.z);
    S.c[0].x = s.x;
    S.c[1].y = s.y;
    S.c[2].z = s.z;
    const M3 M = m3_mul(S, R);
    const M3 dSig = m3_cols(dc.v[0], 0.5f * dc.v[1], 0.5f * dc.v[2], 0.5f * dc.v[1], dc.v[3], 0.5f * dc.v[4],
                            0.5f * dc.v[2], 0.5f * dc.v[4], dc.v[5]);
    M3 M2;
#pragma unroll
    for (int k = 0; k < 3; ++k) M2.c[k] = make_float3(2.0f * M.c[k].x, 2.0f * M.c[k].y, 2.0f * M.c[k].z);
    const M3 dM = m3_mul(M2, dSig);
    const M3 Rt = m3_T(R);
    M3 dMt = m3_T(dM);
    dscale = make_float3(dot3(Rt.c[0], dMt.c[0]), dot3(Rt.c[1], dMt.c[1]), dot3(Rt.c[2], dMt.c[2]));
    dMt.c[0] = make_float3(dMt.c[0].x * s.x, dMt.c[0].y * s.x, dMt.c[0].z * s.x);
    dMt.c[1] = make_float3(dMt.c[1].x * s.y, dMt.c[1].y * s.y, dMt.c[1].z * s.y);
    dMt.c[2] = make_float3(dMt.c[2].x * s.z, dMt.c[2].y * s.z, dMt.c[2].z * s.z);
    const float D00 = dMt.c[0].x, D01 = dMt.c[0].y, D02 = dMt.c[0].z, D10 = dMt.c[1].x, D11 = dMt.c[1].y,
                D12 = dMt.c[1].z, D20 = dMt.c[2].x, D21 = dMt.c[2].y, D22 = dMt.c[2].z;
    drot.x = 2 * z * (D01 - D10) + 2 * y * (D20 - D02) + 2 * x * (D12 - D21);
    drot.y = 2 * y * (D10 + D01) + 2 * z * (D20 + D02) + 2 * r * (D12 - D21) - 4 * x * (D22 + D11);
    drot.z = 2 * x * (D10 + D01) + 2 * r * (D20 - D02) + 2 * z * (D12 + D21) - 4 * y * (D22 + D00);
    drot.w = 2 * r * (D01 - D10) + 2 * x * (D20 + D02) + 2 * y * (D12 + D21) - 4 * z * (D11 + D00);
}

// SH gradient entries [from, M) x 3 of one Gaussian: the coefficients above the active degree get zero
// gradients (and all of them for a skipped Gaussian), as in the reference's zero-initialised dL_dsh.
// Accumulating split sinks are left untouched.
__device__ __forceinline__ void zero_sh_tail(const PreprocessBwdParams& p, int idx, int from, const ShStrides& st) {
    if (p.dL_dsh) {
        for (int k = 3 * from; k < p.M * 3; ++k) p.dL_dsh[(size_t)idx * p.M * 3 + k] = 0.f;
    } else if (!p.sh_accumulate) {
        if (p.dsh_dc && from == 0)
            for (int k = 0; k < 3; ++k) p.dsh_dc[idx * st.dc_sg + k * st.dc_se] = 0.f;
        if (p.dsh_rest)
            for (int k = 3 * (from > 1 ? from - 1 : 0); k < (p.M - 1) * 3; ++k)
                p.dsh_rest[idx * st.rest_sg + k * st.rest_se] = 0.f;
        if (p.dsh_off)
            for (int k = 3 * from; k < p.M * 3; ++k) p.dsh_off[(size_t)idx * p.M * 3 + k] = 0.f;
    }
}

// dL/d(raw parameters) of one Gaussian from the activated-space gradients (k_activate_bwd's formulas):
// xyz: identity; scaling: * exp(scaling); rotation: (I - u u^T) / |q| (u = q / |q|); opacity: * s (1 - s).
// With the fused Adam epilogue (adam_row != nullptr) the final gradients of the parameters that have an Adam sink
// go to the lane's LDS row (columns: xyz 0-2, scaling 3-5, rotation 6-9, opacity 10), from which the wave
// applies the step to its 64 Gaussians' contiguous regions (k_preprocess_bwd).
constexpr int kGeoCol[4] = {0, 3, 6, 10};
__device__ __forceinline__ void raw_grads(const PreprocessBwdParams& p, int i, float3 dmean, float3 dscale,
                                          float3 scale, float4 drot, float dopac, float4 q, float raw_opac, bool vis,
                                          float* __restrict__ adam_row) {
    const bool acc = p.a_accumulate != 0;
    auto put = [acc, vis](float* d, float v) {  // a skipped Gaussian's gradients are zeros (+0 when accumulating)
        v = vis ? v : 0.f;
        *d = acc ? *d + v : v;
    };
    auto upd = [&](int col, float v) { adam_row[col] = vis ? v : 0.f; };
    if (adam_row && p.adam.xyz.p) {
        upd(kGeoCol[0], dmean.x);
        upd(kGeoCol[0] + 1, dmean.y);
        upd(kGeoCol[0] + 2, dmean.z);
    } else if (p.a_xyz) {
        put(p.a_xyz + 3 * i, dmean.x);
        put(p.a_xyz + 3 * i + 1, dmean.y);
        put(p.a_xyz + 3 * i + 2, dmean.z);
    }
    if (adam_row && p.adam.scaling.p) {
        upd(kGeoCol[1], dscale.x * scale.x);
        upd(kGeoCol[1] + 1, dscale.y * scale.y);
        upd(kGeoCol[1] + 2, dscale.z * scale.z);
    } else if (p.a_scaling) {
        put(p.a_scaling + 3 * i, dscale.x * scale.x);
        put(p.a_scaling + 3 * i + 1, dscale.y * scale.y);
        put(p.a_scaling + 3 * i + 2, dscale.z * scale.z);
    }
    if (p.a_rotation || (adam_row && p.adam.rotation.p)) {
        const float nraw = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
        float4 gq;
        if (nraw > 1e-12f) {
            const float inv = 1.f / nraw;
            const float4 u = make_float4(q.x * inv, q.y * inv, q.z * inv, q.w * inv);
            const float ug = u.x * drot.x + u.y * drot.y + u.z * drot.z + u.w * drot.w;
            gq = make_float4((drot.x - u.x * ug) * inv, (drot.y - u.y * ug) * inv, (drot.z - u.z * ug) * inv,
                             (drot.w - u.w * ug) * inv);
        } else {
            gq = make_float4(drot.x * 1e12f, drot.y * 1e12f, drot.z * 1e12f, drot.w * 1e12f);
        }
        if (!vis) gq = make_float4(0.f, 0.f, 0.f, 0.f);
        if (adam_row && p.adam.rotation.p) {
            upd(kGeoCol[2], gq.x);
            upd(kGeoCol[2] + 1, gq.y);
            upd(kGeoCol[2] + 2, gq.z);
            upd(kGeoCol[2] + 3, gq.w);
        } else {
            float4* d = reinterpret_cast<float4*>(p.a_rotation) + i;
            if (acc) {
                const float4 o = *d;
                gq = make_float4(o.x + gq.x, o.y + gq.y, o.z + gq.z, o.w + gq.w);
            }
            *d = gq;
        }
    }
    if (adam_row && p.adam.opacity.p) {
        const float sg = act_opac(raw_opac);
        upd(kGeoCol[3], dopac * sg * (1.f - sg));
    } else if (p.a_opacity) {
        const float sg = act_opac(raw_opac);
        put(p.a_opacity + i, dopac * sg * (1.f - sg));
    }
}

// Gradients of a Gaussian the backward skips (radii == 0): every per-Gaussian output is written, so callers need
// not zero-fill them (only the rasterizer's atomic accumulation targets must start at zero).  This is the SH
// part (the d_rgb row or the SH gradient entries; accumulating SH sinks are left untouched); the geometry half
// selects zeros for the rest.
__device__ __forceinline__ void zero_sh_outputs(const PreprocessBwdParams& p, int idx, const ShStrides& st) {
    if (p.d_rgb) {  // the SH gradient is assembled from the views' d_rgb rows (gsd_sh_grad_views)
        p.d_rgb[3 * idx] = 0.f;
        p.d_rgb[3 * idx + 1] = 0.f;
        p.d_rgb[3 * idx + 2] = 0.f;
        return;
    }
    if (p.shs || p.sh_dc) zero_sh_tail(p, idx, 0, st);
}


// The SH basis B_k of forward.cu:20-71 (the factor backward.cu:20-139 multiplies dL/dRGB by), k < (DEG+1)^2;
// the same expressions as sh_channel_bwd's, so dL/dsh_k,c = B_k dL/dRGB_c to the bit.
template <int DEG>
__device__ __forceinline__ void sh_basis(float x, float y, float z, float (&B)[16]) {
    B[0] = kSH0;
    if (DEG > 0) {
        B[1] = -kSH1 * y;
        B[2] = kSH1 * z;
        B[3] = -kSH1 * x;
    }
    if (DEG > 1) {
        const float xx = x * x, yy = y * y, zz = z * z;
        const float xy = x * y, yz = y * z, xz = x * z;
        B[4] = kSH2_0 * xy;
        B[5] = kSH2_1 * yz;
        B[6] = kSH2_2 * (2.f * zz - xx - yy);
        B[7] = kSH2_3 * xz;
        B[8] = kSH2_4 * (xx - yy);
        if (DEG > 2) {
            B[9] = kSH3_0 * y * (3.f * xx - yy);
            B[10] = kSH3_1 * xy * z;
            B[11] = kSH3_2 * y * (4.f * zz - xx - yy);
            B[12] = kSH3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
            B[13] = kSH3_4 * x * (4.f * zz - xx - yy);
            B[14] = kSH3_5 * z * (xx - yy);
            B[15] = kSH3_6 * x * (xx - 3.f * yy);
        }
    }
}

// dst[(k - K0) * se] (+)= B_k dc for coefficients k in [K0, K1), three channels each (element stride se).
// Accumulating: every old value is loaded before the first store, so the loads issue together instead of
// each waiting behind a store it might alias.
template <int K0, int K1, bool kAcc>
__device__ __forceinline__ void sink_basis(float* __restrict__ dst, const float (&B)[16], const float3 dc,
                                           long long se) {
    constexpr int n = K1 > K0 ? 3 * (K1 - K0) : 1;
    float old[n];
#pragma unroll
    for (int e = 0; e < 3 * (K1 - K0); ++e) old[e] = kAcc ? dst[e * se] : 0.f;
#pragma unroll
    for (int k = K0; k < K1; ++k) {
        const int e = 3 * (k - K0);
        dst[e * se] = old[e] + B[k] * dc.x;
        dst[(e + 1) * se] = old[e + 1] + B[k] * dc.y;
        dst[(e + 2) * se] = old[e + 2] + B[k] * dc.z;
    }
}

// The SH half of the per-Gaussian backward (backward.cu:20-139 and the view-direction term of
// backward.cu:385-392), in its own launch ahead of k_preprocess_bwd.  Together with the projection math in
// one kernel it needed 226 VGPRs (2 waves per SIMD) and streamed the SH rows at ~4 TB/s.  Here:
//  - dL/dsh_k,c = B_k dL/dRGB_c is written straight from the 16 basis values (no 48-float gradient array);
//  - the view-direction gradient sum_c dL/dRGB_c sum_k sh_k,c grad B_k is taken as sum_k w_k grad B_k with
//    w_k = sh_k . dL/dRGB (reassociated over the three channels), so the 48 loaded coefficients fold into
//    16 values as they arrive;
//  - the operand source (kSrc: 0 shs, 1 split, 2 split + offset) and accumulation (kAcc) are compile-time,
//    so no other path's loads share the register allocation.
// The view-direction term of dL/dmean3D goes to floats 9..11 of the Gaussian's gradient record, where the
// geometry half adds it.
template <int DEG, bool kStr, int kSrc, bool kAcc>
__global__ __launch_bounds__(256) void k_preprocess_bwd_sh(PreprocessBwdParams p) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= p.P) return;
    const ShStrides st = sh_strides<kStr>(p);
    if (!(p.radii[idx] > 0)) {
        zero_sh_outputs(p, idx, st);
        return;
    }
    float4* rec = reinterpret_cast<float4*>(p.grad_rec + (size_t)idx * kGradRec);
    const float4 r1 = rec[1], r2 = rec[2];  // colour gradient: r1.z, r1.w, r2.x
    constexpr int nc = (DEG + 1) * (DEG + 1);
    float s[48];
    load_sh<nc, kSrc>(p.shs, p.sh_dc, p.sh_rest, p.sh_off, p.M, idx, s, st);
    const float3 m = make_float3(p.means3D[3 * idx], p.means3D[3 * idx + 1], p.means3D[3 * idx + 2]);
    const float3 cam = make_float3(p.campos[0], p.campos[1], p.campos[2]);
    const float3 dir_orig = make_float3(m.x - cam.x, m.y - cam.y, m.z - cam.z);
    const float len = sqrtf(dot3(dir_orig, dir_orig));
    const float3 dir = make_float3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
    const uint8_t cl = p.clamped[idx];
    // backward.cu:31-34: no gradient through a clamped channel
    const float3 dc = make_float3(r1.z * ((cl & 1) ? 0 : 1), r1.w * ((cl & 2) ? 0 : 1), r2.x * ((cl & 4) ? 0 : 1));
    float B[16];
    sh_basis<DEG>(dir.x, dir.y, dir.z, B);
    if (p.d_rgb) {  // this view's factor of the SH gradient; the sinks are filled by gsd_sh_grad_views
        p.d_rgb[3 * idx] = dc.x;
        p.d_rgb[3 * idx + 1] = dc.y;
        p.d_rgb[3 * idx + 2] = dc.z;
    } else if (kSrc == 0) {
        float* drow = p.dL_dsh + (size_t)idx * p.M * 3;
        sink_basis<0, nc, false>(drow, B, dc, 1);
        for (int k = 3 * nc; k < p.M * 3; ++k) drow[k] = 0.f;
    } else {  // split sinks: dSH/d dc = dSH/d rest = dSH/d offset = identity
        if (p.dsh_dc) sink_basis<0, 1, kAcc>(p.dsh_dc + idx * st.dc_sg, B, dc, st.dc_se);
        if (p.dsh_rest) sink_basis<1, nc, kAcc>(p.dsh_rest + idx * st.rest_sg, B, dc, st.rest_se);
        if (p.dsh_off) sink_basis<0, nc, kAcc>(p.dsh_off + (size_t)idx * p.M * 3, B, dc, 1);
        if (p.M > nc && !kAcc) zero_sh_tail(p, idx, nc, st);
    }
    float w[48], unused[48];
#pragma unroll
    for (int k = 0; k < nc; ++k) w[3 * k] = s[3 * k] * dc.x + s[3 * k + 1] * dc.y + s[3 * k + 2] * dc.z;
    const float3 ddir = sh_channel_bwd(DEG, w, 1.f, dir.x, dir.y, dir.z, unused);
    const float3 dmn = dnormvdv(dir_orig, ddir);
    rec[2] = make_float4(r2.x, dmn.x, dmn.y, dmn.z);
}

// ---------------------------------------------------------------------------------------------------------
// The SH half with coalesced HBM access (contiguous rows, M = 16: every training configuration).  One wave
// per 64 consecutive Gaussians: their SH rows are one contiguous region per operand (dc 64 x 3, rest
// 64 x 45, or shs / offset 64 x 48 floats), read with lane-consecutive dword loads (256 B per
// wave-instruction) into LDS rows of 48 coefficients; each lane then works on its own row (stride 49:
// conflict-free) and leaves the gradient in the row, and the rows go back out the same way.  The per-lane
// kernel above reads each Gaussian's 180-B rows with one lane, 64 rows per wave-instruction (3.2 TB/s).
constexpr int kShWave = 64;
constexpr int kShRowStride = 49;

// region rows [0, rows) x R floats at src  <->  LDS rows, columns [c0, c0 + R).  A full wave (rows = 64, all
// but the last) has no per-element guard, so all R loads are in flight before the first LDS store (with a
// guard per element every load sat in its own branch and waited for the previous one: 2x slower).
template <int R, int kMode>  // kMode 0: lds = src, 1: lds += src (the offset operand)
__device__ __forceinline__ void sh_region_load(const float* __restrict__ src, int rows, float* __restrict__ lds,
                                               int c0) {
    const int lane = threadIdx.x, n = rows * R;
    float v[R];
    if (rows == kShWave) {
#pragma unroll
        for (int i = 0; i < R; ++i) v[i] = src[i * kShWave + lane];
    } else {
#pragma unroll
        for (int i = 0; i < R; ++i) v[i] = i * kShWave + lane < n ? src[i * kShWave + lane] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int e = i * kShWave + lane;
        const int g = e / R, j = e - g * R;
        float* d = lds + g * kShRowStride + c0 + j;  // rows >= `rows` are scratch: harmless
        *d = kMode ? *d + v[i] : v[i];
    }
}
template <int R, bool kAcc>
__device__ __forceinline__ void sh_region_store(float* __restrict__ dst, int rows, const float* __restrict__ lds,
                                                int c0) {
    const int lane = threadIdx.x, n = rows * R;
    float v[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int e = i * kShWave + lane;
        const int g = e / R, j = e - g * R;
        v[i] = lds[g * kShRowStride + c0 + j];
    }
    if (rows == kShWave) {
        float old[R];
#pragma unroll
        for (int i = 0; i < R; ++i) old[i] = kAcc ? dst[i * kShWave + lane] : 0.f;
#pragma unroll
        for (int i = 0; i < R; ++i) dst[i * kShWave + lane] = old[i] + v[i];
        return;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int e = i * kShWave + lane;
        if (e < n) dst[e] = (kAcc ? dst[e] : 0.f) + v[i];
    }
}

// The fused Adam step over a region (gsd_adam_epilogue): the gradient rows in LDS (columns [c0, c0 + R)) are
// the final gradients of the region's parameter elements; each is applied to (param, exp_avg, exp_avg_sq) in
// place -- coalesced like sh_region_store, kCh elements per lane in flight -- instead of being stored.
template <int R, int RS = kShRowStride>
__device__ __forceinline__ void sh_region_adam(const AdamSinkDev& sk, const AdamEpiDev& e, long long base, int rows,
                                               const float* __restrict__ lds, int c0, int lane = threadIdx.x) {
    constexpr int kCh = R < 15 ? R : 15;
    static_assert(R % kCh == 0, "whole chunks");
    const int n = rows * R;
    float* __restrict__ P = sk.p + base;
    float* __restrict__ Mo = sk.m + base;
    float* __restrict__ V = sk.v + base;
#pragma unroll
    for (int c = 0; c < R; c += kCh) {
        float g[kCh], pp[kCh], mm[kCh], vv[kCh];
        bool in[kCh];
#pragma unroll
        for (int i = 0; i < kCh; ++i) {
            const int el = (c + i) * kShWave + lane;
            const int gi = el / R, j = el - gi * R;
            in[i] = rows == kShWave || el < n;
            g[i] = lds[gi * RS + c0 + j];
            pp[i] = in[i] ? P[el] : 0.f;
            mm[i] = in[i] ? __builtin_nontemporal_load(Mo + el) : 0.f;
            vv[i] = in[i] ? __builtin_nontemporal_load(V + el) : 0.f;
        }
#pragma unroll
        for (int i = 0; i < kCh; ++i) {
            adam_elem(pp[i], g[i], mm[i], vv[i], e.w1, e.beta2, e.omb2, sk.step_size, sk.bc2_sqrt, e.eps);
            const int el = (c + i) * kShWave + lane;
            if (in[i]) {
                P[el] = pp[i];
                __builtin_nontemporal_store(mm[i], Mo + el);
                __builtin_nontemporal_store(vv[i], V + el);
            }
        }
    }
}

template <int DEG, int kSrc, bool kAcc, bool kAdam = false>
__global__ __launch_bounds__(kShWave) __attribute__((amdgpu_waves_per_eu(4))) void k_preprocess_bwd_sh_rows(PreprocessBwdParams p) {
    __shared__ float rows_lds[kShWave * kShRowStride];
    constexpr int M = 16;
    const int g0 = blockIdx.x * kShWave, lane = threadIdx.x, idx = g0 + lane;
    const int rows = min(kShWave, p.P - g0);
    if (kSrc == 0) {
        sh_region_load<3 * M, 0>(p.shs + (size_t)g0 * 3 * M, rows, rows_lds, 0);
    } else {
        sh_region_load<3, 0>(p.sh_dc + (size_t)g0 * 3, rows, rows_lds, 0);
        sh_region_load<3 * (M - 1), 0>(p.sh_rest + (size_t)g0 * 3 * (M - 1), rows, rows_lds, 3);
    }
    __syncthreads();
    if (kSrc == 2) {  // the same float add as load_sh (gaussian_renderer/__init__.py:134)
        sh_region_load<3 * M, 1>(p.sh_off + (size_t)g0 * 3 * M, rows, rows_lds, 0);
        __syncthreads();
    }
    float* row = rows_lds + lane * kShRowStride;
    constexpr int nc = (DEG + 1) * (DEG + 1);
    if (idx < p.P) {
        if (!(p.radii[idx] > 0)) {
            if (p.d_rgb) {
                p.d_rgb[3 * idx] = 0.f;
                p.d_rgb[3 * idx + 1] = 0.f;
                p.d_rgb[3 * idx + 2] = 0.f;
            }
#pragma unroll
            for (int k = 0; k < 3 * M; ++k) row[k] = 0.f;
        } else {
            float4* rec = reinterpret_cast<float4*>(p.grad_rec + (size_t)idx * kGradRec);
            const float4 r1 = rec[1], r2 = rec[2];  // colour gradient: r1.z, r1.w, r2.x
            const float3 m = make_float3(p.means3D[3 * idx], p.means3D[3 * idx + 1], p.means3D[3 * idx + 2]);
            const float3 cam = make_float3(p.campos[0], p.campos[1], p.campos[2]);
            const float3 dir_orig = make_float3(m.x - cam.x, m.y - cam.y, m.z - cam.z);
            const float len = sqrtf(dot3(dir_orig, dir_orig));
            const float3 dir = make_float3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
            const uint8_t cl = p.clamped[idx];
            const float3 dc =
                make_float3(r1.z * ((cl & 1) ? 0 : 1), r1.w * ((cl & 2) ? 0 : 1), r2.x * ((cl & 4) ? 0 : 1));
            float w[48], unused[48];
#pragma unroll
            for (int k = 0; k < nc; ++k) w[3 * k] = row[3 * k] * dc.x + row[3 * k + 1] * dc.y + row[3 * k + 2] * dc.z;
            const float3 ddir = sh_channel_bwd(DEG, w, 1.f, dir.x, dir.y, dir.z, unused);
            const float3 dmn = dnormvdv(dir_orig, ddir);
            rec[2] = make_float4(r2.x, dmn.x, dmn.y, dmn.z);
            if (p.d_rgb) {  // this view's factor of the SH gradient; the sinks are filled by gsd_sh_grad_views
                p.d_rgb[3 * idx] = dc.x;
                p.d_rgb[3 * idx + 1] = dc.y;
                p.d_rgb[3 * idx + 2] = dc.z;
            } else {
                float B[16];
                sh_basis<DEG>(dir.x, dir.y, dir.z, B);
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    row[3 * k] = k < nc ? B[k] * dc.x : 0.f;  // zero above the active degree
                    row[3 * k + 1] = k < nc ? B[k] * dc.y : 0.f;
                    row[3 * k + 2] = k < nc ? B[k] * dc.z : 0.f;
                }
            }
        }
    }
    if (p.d_rgb) return;
    __syncthreads();
    if (kSrc == 0) {
        sh_region_store<3 * M, false>(p.dL_dsh + (size_t)g0 * 3 * M, rows, rows_lds, 0);
        return;
    }
    if (kAdam && p.adam.dc.p) sh_region_adam<3>(p.adam.dc, p.adam, (long long)g0 * 3, rows, rows_lds, 0);
    else if (p.dsh_dc) sh_region_store<3, kAcc>(p.dsh_dc + (size_t)g0 * 3, rows, rows_lds, 0);
    if (kAdam && p.adam.rest.p)
        sh_region_adam<3 * (M - 1)>(p.adam.rest, p.adam, (long long)g0 * 3 * (M - 1), rows, rows_lds, 3);
    else if (p.dsh_rest)
        sh_region_store<3 * (M - 1), kAcc>(p.dsh_rest + (size_t)g0 * 3 * (M - 1), rows, rows_lds, 3);
    if (p.dsh_off) sh_region_store<3 * M, kAcc>(p.dsh_off + (size_t)g0 * 3 * M, rows, rows_lds, 0);
}

// The SH half with the fused Adam step for the split operand without an offset (the bench / training path:
// store mode, M = 16).  The SH parameters stay in the LDS rows they were staged into, and each lane leaves its
// Gaussian's 16 basis values and masked dL/dRGB in a short LDS row; the Adam pass then forms each gradient element
// B_k dL/dRGB_c from those (the product k_preprocess_bwd_sh_rows stores in its gradient rows, bit for bit) and
// takes the parameter from LDS.  k_preprocess_bwd_sh_rows<.., kAdam> re-reads the parameter from global memory
// instead, and that re-read missed L2: FETCH_SIZE showed ~200 MB more than the algorithmic reads per step at 1M
// Gaussians (scripts/prof_step.py PMC pass), one 192-B SH row per Gaussian.
constexpr int kBasisStride = 19;  // 16 basis values + dL/dRGB (3): odd, so the per-lane row writes are conflict-free
template <int R, int C0>
__device__ __forceinline__ float basis_grad(const float* __restrict__ bas, int el, int& gi, int& col) {
    gi = el / R;
    col = C0 + (el - gi * R);
    const int k = col / 3, ch = col - 3 * k;
    return bas[gi * kBasisStride + k] * bas[gi * kBasisStride + 16 + ch];
}
template <int R, int C0>
__device__ __forceinline__ void sh_region_adam_basis(const AdamSinkDev& sk, const AdamEpiDev& e, long long base,
                                                     int rows, const float* __restrict__ prm,
                                                     const float* __restrict__ bas) {
    constexpr int kCh = R < 15 ? R : 15;
    static_assert(R % kCh == 0, "whole chunks");
    const int lane = threadIdx.x, n = rows * R;
    float* __restrict__ P = sk.p + base;
    float* __restrict__ Mo = sk.m + base;
    float* __restrict__ V = sk.v + base;
#pragma unroll
    for (int c = 0; c < R; c += kCh) {
        float g[kCh], pp[kCh], mm[kCh], vv[kCh];
        bool in[kCh];
#pragma unroll
        for (int i = 0; i < kCh; ++i) {
            const int el = (c + i) * kShWave + lane;
            int gi, col;
            g[i] = basis_grad<R, C0>(bas, el, gi, col);
            pp[i] = prm[gi * kShRowStride + col];
            in[i] = rows == kShWave || el < n;
            mm[i] = in[i] ? __builtin_nontemporal_load(Mo + el) : 0.f;
            vv[i] = in[i] ? __builtin_nontemporal_load(V + el) : 0.f;
        }
#pragma unroll
        for (int i = 0; i < kCh; ++i) {
            adam_elem(pp[i], g[i], mm[i], vv[i], e.w1, e.beta2, e.omb2, sk.step_size, sk.bc2_sqrt, e.eps);
            const int el = (c + i) * kShWave + lane;
            if (in[i]) {
                P[el] = pp[i];
                __builtin_nontemporal_store(mm[i], Mo + el);
                __builtin_nontemporal_store(vv[i], V + el);
            }
        }
    }
}
template <int R, int C0>
__device__ __forceinline__ void sh_region_store_basis(float* __restrict__ dst, int rows, const float* __restrict__ bas) {
    const int lane = threadIdx.x, n = rows * R;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int el = i * kShWave + lane;
        int gi, col;
        const float g = basis_grad<R, C0>(bas, el, gi, col);
        if (rows == kShWave || el < n) dst[el] = g;
    }
}

template <int DEG>
__global__ __launch_bounds__(kShWave) void k_preprocess_bwd_sh_adam(PreprocessBwdParams p) {
    __shared__ float rows_lds[kShWave * kShRowStride];   // the SH parameters (dc | rest) of the 64 Gaussians
    __shared__ float basis_lds[kShWave * kBasisStride];  // per Gaussian: B_0..B_15, masked dL/dRGB
    constexpr int nc = (DEG + 1) * (DEG + 1);
    const int g0 = blockIdx.x * kShWave, lane = threadIdx.x, idx = g0 + lane;
    const int rows = min(kShWave, p.P - g0);
    sh_region_load<3, 0>(p.sh_dc + (size_t)g0 * 3, rows, rows_lds, 0);
    sh_region_load<45, 0>(p.sh_rest + (size_t)g0 * 45, rows, rows_lds, 3);
    __syncthreads();
    const float* row = rows_lds + lane * kShRowStride;
    float B[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) B[k] = 0.f;  // zero above the active degree, and for skipped Gaussians
    float3 dc = make_float3(0.f, 0.f, 0.f);
    if (idx < p.P && p.radii[idx] > 0) {
        float4* rec = reinterpret_cast<float4*>(p.grad_rec + (size_t)idx * kGradRec);
        const float4 r1 = rec[1], r2 = rec[2];  // colour gradient: r1.z, r1.w, r2.x
        const float3 m = make_float3(p.means3D[3 * idx], p.means3D[3 * idx + 1], p.means3D[3 * idx + 2]);
        const float3 cam = make_float3(p.campos[0], p.campos[1], p.campos[2]);
        const float3 dir_orig = make_float3(m.x - cam.x, m.y - cam.y, m.z - cam.z);
        const float len = sqrtf(dot3(dir_orig, dir_orig));
        const float3 dir = make_float3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
        const uint8_t cl = p.clamped[idx];
        dc = make_float3(r1.z * ((cl & 1) ? 0 : 1), r1.w * ((cl & 2) ? 0 : 1), r2.x * ((cl & 4) ? 0 : 1));
        float w[48], unused[48];
#pragma unroll
        for (int k = 0; k < nc; ++k) w[3 * k] = row[3 * k] * dc.x + row[3 * k + 1] * dc.y + row[3 * k + 2] * dc.z;
        const float3 ddir = sh_channel_bwd(DEG, w, 1.f, dir.x, dir.y, dir.z, unused);
        const float3 dmn = dnormvdv(dir_orig, ddir);
        rec[2] = make_float4(r2.x, dmn.x, dmn.y, dmn.z);
        sh_basis<DEG>(dir.x, dir.y, dir.z, B);
    }
    float* brow = basis_lds + lane * kBasisStride;
#pragma unroll
    for (int k = 0; k < 16; ++k) brow[k] = k < nc ? B[k] : 0.f;
    brow[16] = dc.x;
    brow[17] = dc.y;
    brow[18] = dc.z;
    __syncthreads();
    if (p.adam.dc.p) sh_region_adam_basis<3, 0>(p.adam.dc, p.adam, (long long)g0 * 3, rows, rows_lds, basis_lds);
    else if (p.dsh_dc) sh_region_store_basis<3, 0>(p.dsh_dc + (size_t)g0 * 3, rows, basis_lds);
    if (p.adam.rest.p)
        sh_region_adam_basis<45, 3>(p.adam.rest, p.adam, (long long)g0 * 45, rows, rows_lds, basis_lds);
    else if (p.dsh_rest)
        sh_region_store_basis<45, 3>(p.dsh_rest + (size_t)g0 * 45, rows, basis_lds);
}

// The geometry half of the per-Gaussian backward: computeCov2DCUDA + preprocessCUDA bwd without the SH
// (backward.cu:144-396); the view-direction term of dL/dmean3D comes from the record (k_preprocess_bwd_sh,
// launched first; zeros when there is no SH operand).
// One Gaussian of the geometry half; with the fused Adam epilogue its final raw-parameter gradients go to
// adam_row instead (raw_grads).
__device__ __forceinline__ void preprocess_bwd_one(const PreprocessBwdParams& p, int idx, float* adam_row) {
    // Every per-Gaussian load is issued up front, before the visibility test: a Gaussian the backward skips
    // (radii == 0, backward.cu:359-360) is computed like the others and its outputs are replaced by the zeros
    // torch::zeros holds -- one latency instead of two, and no divergent branch.
    const int rad = p.radii[idx];
    const bool vis = rad > 0;
    const float3 m = make_float3(p.means3D[3 * idx], p.means3D[3 * idx + 1], p.means3D[3 * idx + 2]);
    const float4* rec4 = reinterpret_cast<const float4*>(p.grad_rec + (size_t)idx * kGradRec);
    const float4 r0 = rec4[0], r1 = rec4[1], r2 = rec4[2];
    // r0 = (mean2D x, mean2D y, conic a, conic b), r1 = (conic c, opacity, color r, color g), r2.x = color b,
    // r2.yzw = the SH half's dL/dmean3D term
    Cov6 c3;
    float3 scale = make_float3(0, 0, 0);
    float4 q_in = make_float4(0, 0, 0, 0), q = q_in;
    const float raw_opac = p.raw_act && p.a_opacity ? p.raw_opacity[idx] : 0.f;
    if (p.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3.v[k] = p.cov3D_precomp[6 * idx + k];
    } else {
        scale = make_float3(p.scales[3 * idx], p.scales[3 * idx + 1], p.scales[3 * idx + 2]);
        q_in = reinterpret_cast<const float4*>(p.rotations)[idx];
        q = q_in;
        if (p.raw_act) {
            scale = act_scale(p.scales, idx);
            q = act_rot(q_in);
        }
        // the 3D covariance the forward used (recomputed: cheaper than storing 24 B/G)
        c3 = cov3d_from_scale_rot(scale, p.scale_modifier, q);
    }
    const Mat4 Vm = load_mat4(p.view);
    const Mat4 Pm = load_mat4(p.proj);
    auto z = [vis](float v) { return vis ? v : 0.f; };
    // the rasterizer's per-Gaussian record: unpack the API outputs (rasterize_points.cu:180-188) and use it
    if (p.dL_dmean2D) {
        p.dL_dmean2D[3 * idx] = z(r0.x);
        p.dL_dmean2D[3 * idx + 1] = z(r0.y);
        p.dL_dmean2D[3 * idx + 2] = 0.f;
    }
    if (p.dens_accum && vis) {  // gsd_densify_stats for this view, the same float operations (gsd_densify.hip)
        const float gx = r0.x, gy = r0.y;
        p.dens_max_radii[idx] = fmaxf(p.dens_max_radii[idx], (float)rad);
        p.dens_accum3[3 * idx] += gx;
        p.dens_accum3[3 * idx + 1] += gy;
        p.dens_accum3[3 * idx + 2] += 0.f;  // dL/dmean2D.z, stored as 0 above
        p.dens_accum[idx] += sqrtf(gx * gx + gy * gy);
        p.dens_denom[idx] += 1.0f;
    }
    if (p.dL_dopacity) p.dL_dopacity[idx] = z(r1.y);
    if (p.dL_dcolor) {
        p.dL_dcolor[3 * idx] = z(r1.z);
        p.dL_dcolor[3 * idx + 1] = z(r1.w);
        p.dL_dcolor[3 * idx + 2] = z(r2.x);
    }
    if (p.defer_view_dir) {  // no SH half ran: this view's row of the exchanged SH factor, masked as it masks it
        const uint8_t cl = p.clamped[idx];
        p.d_rgb[3 * idx] = (cl & 1) ? 0.f : z(r1.z);
        p.d_rgb[3 * idx + 1] = (cl & 2) ? 0.f : z(r1.w);
        p.d_rgb[3 * idx + 2] = (cl & 4) ? 0.f : z(r2.x);
    }
    float3 dmean;
    Cov6 dcov;
    cov2d_bwd(m, c3, p.focal_x, p.focal_y, p.tan_fovx, p.tan_fovy, Vm, make_float3(r0.z, r0.w, r1.x), dmean, dcov);
    if (p.dL_dcov3D) {
#pragma unroll
        for (int k = 0; k < 6; ++k) p.dL_dcov3D[6 * idx + k] = z(dcov.v[k]);
    }

    // backward.cu:373-387 projective term from dL/dmean2D
    const float4 mh = xform_point4(m, Pm);
    const float mw = 1.0f / (mh.w + 0.0000001f);
    const float* P = Pm.m;
    const float mul1 = (P[0] * m.x + P[4] * m.y + P[8] * m.z + P[12]) * mw * mw;
    const float mul2 = (P[1] * m.x + P[5] * m.y + P[9] * m.z + P[13]) * mw * mw;
    const float d2x = r0.x, d2y = r0.y;
    float3 dm2;
    dm2.x = (P[0] * mw - P[3] * mul1) * d2x + (P[1] * mw - P[3] * mul2) * d2y;
    dm2.y = (P[4] * mw - P[7] * mul1) * d2x + (P[5] * mw - P[7] * mul2) * d2y;
    dm2.z = (P[8] * mw - P[11] * mul1) * d2x + (P[9] * mw - P[11] * mul2) * d2y;
    dmean = make_float3(dmean.x + dm2.x, dmean.y + dm2.y, dmean.z + dm2.z);

    dmean = make_float3(dmean.x + r2.y, dmean.y + r2.z, dmean.z + r2.w);  // backward.cu:390-392 (SH half)
    float3 dscale = make_float3(0.f, 0.f, 0.f);
    float4 drot = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.scales) cov3d_bwd(scale, p.scale_modifier, q, dcov, dscale, drot);
    dmean = make_float3(z(dmean.x), z(dmean.y), z(dmean.z));
    dscale = make_float3(z(dscale.x), z(dscale.y), z(dscale.z));
    drot = make_float4(z(drot.x), z(drot.y), z(drot.z), z(drot.w));
    if (p.raw_act) {  // through the activations into the raw parameters' sinks (k_activate_bwd's formulas)
        raw_grads(p, idx, dmean, dscale, scale, drot, r1.y, q_in, raw_opac, vis, adam_row);
        return;
    }
    p.dL_dmeans3D[3 * idx] = dmean.x;
    p.dL_dmeans3D[3 * idx + 1] = dmean.y;
    p.dL_dmeans3D[3 * idx + 2] = dmean.z;
    if (p.dL_dscales) {
        p.dL_dscales[3 * idx] = dscale.x;
        p.dL_dscales[3 * idx + 1] = dscale.y;
        p.dL_dscales[3 * idx + 2] = dscale.z;
    }
    if (p.dL_drotations) reinterpret_cast<float4*>(p.dL_drotations)[idx] = drot;
}

// The geometry half, one lane per Gaussian.  With the fused Adam epilogue (gsd_adam_epilogue) each wave then
// steps its 64 Gaussians' xyz / scaling / rotation / opacity as contiguous regions: lane-consecutive dword
// accesses to (param, exp_avg, exp_avg_sq), the gradients read from the lanes' LDS rows (sh_region_adam), in
// place of one lane reading and writing its own 3- or 4-float rows at a 12- / 16-B lane stride.
constexpr int kGeoRowStride = 11;  // odd: the lanes' row writes are bank-conflict free
__global__ __launch_bounds__(256) void k_preprocess_bwd(PreprocessBwdParams p) {
    __shared__ float s_geo[256 / kShWave][kShWave * kGeoRowStride];
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (!p.adam_on) {
        if (idx < p.P) preprocess_bwd_one(p, idx, nullptr);
        return;
    }
    const int lane = threadIdx.x & (kShWave - 1);
    const float* rows_lds = s_geo[threadIdx.x / kShWave];
    if (idx < p.P) preprocess_bwd_one(p, idx, s_geo[threadIdx.x / kShWave] + lane * kGeoRowStride);
    wave_lds_handoff();
    const int g0 = idx - lane, rows = min(kShWave, p.P - g0);
    if (rows <= 0) return;
    if (p.adam.xyz.p)
        sh_region_adam<3, kGeoRowStride>(p.adam.xyz, p.adam, 3LL * g0, rows, rows_lds, kGeoCol[0], lane);
    if (p.adam.scaling.p)
        sh_region_adam<3, kGeoRowStride>(p.adam.scaling, p.adam, 3LL * g0, rows, rows_lds, kGeoCol[1], lane);
    if (p.adam.rotation.p)
        sh_region_adam<4, kGeoRowStride>(p.adam.rotation, p.adam, 4LL * g0, rows, rows_lds, kGeoCol[2], lane);
    if (p.adam.opacity.p)
        sh_region_adam<1, kGeoRowStride>(p.adam.opacity, p.adam, (long long)g0, rows, rows_lds, kGeoCol[3], lane);
}

}  // namespace gsd

namespace gsd {

// dL/dsh_k = sum_v B_k(dir_v) dL/dRGB_v (the per-view SH backward of backward.cu:20-139, summed over the views
// whose masked dL/dRGB rows were exchanged) for Gaussian idx: the 3 (D+1)^2 sums in acc.
template <int DEG>
__device__ __forceinline__ void sh_views_sum(const ShViewsParams& p, int idx, float (&acc)[48]) {
    constexpr int nc = (DEG + 1) * (DEG + 1);
    const float3 m = make_float3(p.means3D[3 * idx], p.means3D[3 * idx + 1], p.means3D[3 * idx + 2]);
#pragma unroll
    for (int k = 0; k < 48; ++k) acc[k] = 0.f;
    for (int v = 0; v < p.n_views; ++v) {
        const float* row = p.views + (size_t)v * (size_t)p.view_stride;
        const float* cam = row + (size_t)p.P * 3;
        const float3 g = make_float3(row[3 * idx], row[3 * idx + 1], row[3 * idx + 2]);
        const float3 d0 = make_float3(m.x - cam[0], m.y - cam[1], m.z - cam[2]);
        const float len = sqrtf(dot3(d0, d0));
        // a view that culled this Gaussian handed over a zero row: its term is exactly zero, and is skipped
        // rather than evaluated (a mean at that camera's centre would give a NaN basis, and NaN * 0 = NaN)
        if ((g.x == 0.f && g.y == 0.f && g.z == 0.f) || !(len > 0.f)) continue;
        const float x = d0.x / len, y = d0.y / len, z = d0.z / len;
        float b[16];
        b[0] = kSH0;
        if (DEG > 0) {
            b[1] = -kSH1 * y;
            b[2] = kSH1 * z;
            b[3] = -kSH1 * x;
        }
        if (DEG > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            b[4] = kSH2_0 * (x * y);
            b[5] = kSH2_1 * (y * z);
            b[6] = kSH2_2 * (2.f * zz - xx - yy);
            b[7] = kSH2_3 * (x * z);
            b[8] = kSH2_4 * (xx - yy);
            if (DEG > 2) {
                b[9] = kSH3_0 * y * (3.f * xx - yy);
                b[10] = kSH3_1 * (x * y) * z;
                b[11] = kSH3_2 * y * (4.f * zz - xx - yy);
                b[12] = kSH3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
                b[13] = kSH3_4 * x * (4.f * zz - xx - yy);
                b[14] = kSH3_5 * z * (xx - yy);
                b[15] = kSH3_6 * x * (xx - 3.f * yy);
            }
        }
#pragma unroll
        for (int k = 0; k < nc; ++k) {
            acc[3 * k] += b[k] * g.x;
            acc[3 * k + 1] += b[k] * g.y;
            acc[3 * k + 2] += b[k] * g.z;
        }
    }
}

// One lane per Gaussian, writing its own rows (any sink layout).
template <int DEG>
__global__ __launch_bounds__(256) void k_sh_grad_views(ShViewsParams p) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= p.P) return;
    constexpr int nc = (DEG + 1) * (DEG + 1);
    float acc[48];
    sh_views_sum<DEG>(p, idx, acc);
    const bool add = p.accumulate != 0;
    if (p.d_dc) {
        float* d = p.d_dc + idx * p.dc_sg;
#pragma unroll
        for (int c = 0; c < 3; ++c) d[c * p.dc_se] = (add ? d[c * p.dc_se] : 0.f) + acc[c];
    }
    if (p.d_rest) {
        float* d = p.d_rest + idx * p.rest_sg;
        const long long se = p.rest_se;
        if (se == 1) {
#pragma unroll
            for (int k = 3; k < nc * 3; ++k) d[k - 3] = (add ? d[k - 3] : 0.f) + acc[k];
        } else {
#pragma unroll
            for (int k = 3; k < nc * 3; ++k) d[(k - 3) * se] = (add ? d[(k - 3) * se] : 0.f) + acc[k];
        }
        if (!add)
            for (int k = nc * 3; k < p.M * 3; ++k) d[(k - 3) * se] = 0.f;
    }
    if (p.d_off) {
        float* d = p.d_off + (size_t)idx * p.M * 3;
#pragma unroll
        for (int k = 0; k < nc * 3; ++k) d[k] = (add ? d[k] : 0.f) + acc[k];
        if (!add)
            for (int k = nc * 3; k < p.M * 3; ++k) d[k] = 0.f;
    }
}

// With d_means (gsd_sh_grad_views_ex; store mode, contiguous pieces, M = 16): the views' summed view-direction
// term of the SH colour, which the backwards of a defer_view_dir exchange left out of dL/dmeans3D -- per view v,
// dnormvdv(m - campos_v, sum_k w_k grad B_k(dir_v)) with w_k = sh_k . d_rgb_v (k_preprocess_bwd_sh_rows's
// expressions).  The coefficients are staged once into the LDS rows; before the rows take the assembled
// gradient, every lane copies the coefficients of the region elements it will step into registers, so the Adam
// pass reads no parameter from HBM and one 12.5-KB LDS buffer serves both (a second buffer for the gradient
// halved the workgroups per CU: 0.242 ms against 0.197 for k_sh_grad_views_rows at one view).
template <int R, int C0>
__device__ __forceinline__ void region_params_to_regs(const float* __restrict__ prm, float (&pre)[R]) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int el = i * kShWave + (int)threadIdx.x;
        const int gi = el / R, j = el - gi * R;
        pre[i] = prm[gi * kShRowStride + C0 + j];
    }
}
template <int R>
__device__ __forceinline__ void sh_region_adam_regs(const AdamSinkDev& sk, const AdamEpiDev& e, long long base,
                                                    int rows, const float (&pre)[R], const float* __restrict__ grd,
                                                    int c0) {
    constexpr int kCh = R < 15 ? R : 15;
    static_assert(R % kCh == 0, "whole chunks");
    const int lane = threadIdx.x, n = rows * R;
    float* __restrict__ P = sk.p + base;
    float* __restrict__ Mo = sk.m + base;
    float* __restrict__ V = sk.v + base;
#pragma unroll
    for (int c = 0; c < R; c += kCh) {
        float g[kCh], pp[kCh], mm[kCh], vv[kCh];
        bool in[kCh];
#pragma unroll
        for (int i = 0; i < kCh; ++i) {
            const int el = (c + i) * kShWave + lane;
            const int gi = el / R, j = el - gi * R;
            in[i] = rows == kShWave || el < n;
            g[i] = grd[gi * kShRowStride + c0 + j];
            pp[i] = pre[c + i];
            mm[i] = in[i] ? __builtin_nontemporal_load(Mo + el) : 0.f;
            vv[i] = in[i] ? __builtin_nontemporal_load(V + el) : 0.f;
        }
#pragma unroll
        for (int i = 0; i < kCh; ++i) {
            adam_elem(pp[i], g[i], mm[i], vv[i], e.w1, e.beta2, e.omb2, sk.step_size, sk.bc2_sqrt, e.eps);
            const int el = (c + i) * kShWave + lane;
            if (in[i]) {
                P[el] = pp[i];
                __builtin_nontemporal_store(mm[i], Mo + el);
                __builtin_nontemporal_store(vv[i], V + el);
            }
        }
    }
}
template <int DEG>
__global__ __launch_bounds__(kShWave) void k_sh_grad_views_dir(ShViewsParams p) {
    __shared__ float rows_lds[kShWave * kShRowStride];  // the SH coefficients (dc | rest), then the gradient
    constexpr int M = 16, nc = (DEG + 1) * (DEG + 1);
    const int g0 = blockIdx.x * kShWave, lane = threadIdx.x, idx = g0 + lane;
    const int rows = min(kShWave, p.P - g0);
    sh_region_load<3, 0>(p.sh_dc + (size_t)g0 * 3, rows, rows_lds, 0);
    sh_region_load<3 * (M - 1), 0>(p.sh_rest + (size_t)g0 * 3 * (M - 1), rows, rows_lds, 3);
    __syncthreads();
    float* row = rows_lds + lane * kShRowStride;
    float acc[48];
#pragma unroll
    for (int k = 0; k < 48; ++k) acc[k] = 0.f;
    if (idx < p.P) {
        sh_views_sum<DEG>(p, idx, acc);
        const float* s = row;  // the coefficients straight from the LDS row (48 registers fewer: occupancy)
        const float3 m = make_float3(p.means3D[3 * idx], p.means3D[3 * idx + 1], p.means3D[3 * idx + 2]);
        float3 dm = make_float3(0.f, 0.f, 0.f);
        for (int v = 0; v < p.n_views; ++v) {
            const float* vrow = p.views + (size_t)v * (size_t)p.view_stride;
            const float* cam = vrow + (size_t)p.P * 3;
            const float3 g = make_float3(vrow[3 * idx], vrow[3 * idx + 1], vrow[3 * idx + 2]);
            const float3 d0 = make_float3(m.x - cam[0], m.y - cam[1], m.z - cam[2]);
            const float len = sqrtf(dot3(d0, d0));
            // a view that culled this Gaussian (zero row) adds nothing (and a mean at its centre no NaN)
            if ((g.x == 0.f && g.y == 0.f && g.z == 0.f) || !(len > 0.f)) continue;
            const float3 dir = make_float3(d0.x / len, d0.y / len, d0.z / len);
            float w[48], unused[48];
#pragma unroll
            for (int k = 0; k < nc; ++k) w[3 * k] = s[3 * k] * g.x + s[3 * k + 1] * g.y + s[3 * k + 2] * g.z;
            const float3 ddir = sh_channel_bwd(DEG, w, 1.f, dir.x, dir.y, dir.z, unused);
            const float3 dmn = dnormvdv(d0, ddir);
            dm = make_float3(dm.x + dmn.x, dm.y + dmn.y, dm.z + dmn.z);
        }
        p.d_means[3 * idx] = dm.x;
        p.d_means[3 * idx + 1] = dm.y;
        p.d_means[3 * idx + 2] = dm.z;
    }
    const bool adam_dc = p.adam.dc.p != nullptr, adam_rest = p.adam.rest.p != nullptr;
    float pre_dc[3], pre_rest[3 * (M - 1)];
    if (adam_dc) region_params_to_regs<3, 0>(rows_lds, pre_dc);
    if (adam_rest) region_params_to_regs<3 * (M - 1), 3>(rows_lds, pre_rest);
    __syncthreads();  // every coefficient read: the rows take the gradient
#pragma unroll
    for (int k = 0; k < 3 * M; ++k) row[k] = k < 3 * nc ? acc[k] : 0.f;  // zero above the active degree
    __syncthreads();
    if (adam_dc) sh_region_adam_regs<3>(p.adam.dc, p.adam, (long long)g0 * 3, rows, pre_dc, rows_lds, 0);
    else if (p.d_dc) sh_region_store<3, false>(p.d_dc + (size_t)g0 * 3, rows, rows_lds, 0);
    if (adam_rest)
        sh_region_adam_regs<3 * (M - 1)>(p.adam.rest, p.adam, (long long)g0 * 3 * (M - 1), rows, pre_rest, rows_lds, 3);
    else if (p.d_rest)
        sh_region_store<3 * (M - 1), false>(p.d_rest + (size_t)g0 * 3 * (M - 1), rows, rows_lds, 3);
}

// The same with coalesced sinks (contiguous rows, M = 16): one wave per 64 Gaussians, the sums through LDS rows
// and out as lane-consecutive region stores (the SH half of the backward's scheme).
template <int DEG, bool kAcc>
__global__ __launch_bounds__(kShWave) void k_sh_grad_views_rows(ShViewsParams p) {
    __shared__ float rows_lds[kShWave * kShRowStride];
    constexpr int M = 16, nc = (DEG + 1) * (DEG + 1);
    const int g0 = blockIdx.x * kShWave, lane = threadIdx.x, idx = g0 + lane;
    const int rows = min(kShWave, p.P - g0);
    if (idx < p.P) {
        float acc[48];
        sh_views_sum<DEG>(p, idx, acc);
        float* row = rows_lds + lane * kShRowStride;
#pragma unroll
        for (int k = 0; k < 3 * M; ++k) row[k] = k < 3 * nc ? acc[k] : 0.f;  // zero above the active degree
    }
    __syncthreads();
    if (!kAcc && p.adam.dc.p) sh_region_adam<3>(p.adam.dc, p.adam, (long long)g0 * 3, rows, rows_lds, 0);
    else if (p.d_dc) sh_region_store<3, kAcc>(p.d_dc + (size_t)g0 * 3, rows, rows_lds, 0);
    if (!kAcc && p.adam.rest.p)
        sh_region_adam<3 * (M - 1)>(p.adam.rest, p.adam, (long long)g0 * 3 * (M - 1), rows, rows_lds, 3);
    else if (p.d_rest)
        sh_region_store<3 * (M - 1), kAcc>(p.d_rest + (size_t)g0 * 3 * (M - 1), rows, rows_lds, 3);
    if (p.d_off) sh_region_store<3 * M, kAcc>(p.d_off + (size_t)g0 * 3 * M, rows, rows_lds, 0);
}

template <bool kAcc>
static void launch_sh_views_rows(const ShViewsParams& p, hipStream_t s) {
    const dim3 g((p.P + kShWave - 1) / kShWave), b(kShWave);
    switch (p.D <= 0 ? 0 : (p.D >= 3 ? 3 : p.D)) {
        case 0: hipLaunchKernelGGL((k_sh_grad_views_rows<0, kAcc>), g, b, 0, s, p); break;
        case 1: hipLaunchKernelGGL((k_sh_grad_views_rows<1, kAcc>), g, b, 0, s, p); break;
        case 2: hipLaunchKernelGGL((k_sh_grad_views_rows<2, kAcc>), g, b, 0, s, p); break;
        default: hipLaunchKernelGGL((k_sh_grad_views_rows<3, kAcc>), g, b, 0, s, p); break;
    }
}
void launch_sh_grad_views(const ShViewsParams& p, hipStream_t s) {
    if (p.P <= 0) return;
    if (p.d_means) {  // gsd_sh_grad_views_ex checked the layout (contiguous, M = 16, store mode)
        const dim3 g((p.P + kShWave - 1) / kShWave), b(kShWave);
        switch (p.D <= 0 ? 0 : (p.D >= 3 ? 3 : p.D)) {
            case 0: hipLaunchKernelGGL(k_sh_grad_views_dir<0>, g, b, 0, s, p); break;
            case 1: hipLaunchKernelGGL(k_sh_grad_views_dir<1>, g, b, 0, s, p); break;
            case 2: hipLaunchKernelGGL(k_sh_grad_views_dir<2>, g, b, 0, s, p); break;
            default: hipLaunchKernelGGL(k_sh_grad_views_dir<3>, g, b, 0, s, p); break;
        }
        return;
    }
#ifndef GSD_SH_VIEWS_LANE
    const bool rows = p.M == 16 && (!p.d_dc || (p.dc_sg == 3 && p.dc_se == 1)) &&
                      (!p.d_rest || (p.rest_sg == 3LL * (p.M - 1) && p.rest_se == 1));
    if (rows) {
        if (p.accumulate) launch_sh_views_rows<true>(p, s);
        else launch_sh_views_rows<false>(p, s);
        return;
    }
#endif
    const dim3 g((p.P + 255) / 256), b(256);
    switch (p.D <= 0 ? 0 : (p.D >= 3 ? 3 : p.D)) {
        case 0: hipLaunchKernelGGL(k_sh_grad_views<0>, g, b, 0, s, p); break;
        case 1: hipLaunchKernelGGL(k_sh_grad_views<1>, g, b, 0, s, p); break;
        case 2: hipLaunchKernelGGL(k_sh_grad_views<2>, g, b, 0, s, p); break;
        default: hipLaunchKernelGGL(k_sh_grad_views<3>, g, b, 0, s, p); break;
    }
}

}  // namespace gsd

namespace gsd {
template <typename Prm>
static bool strided_sh(const Prm& p) {
    return p.sh_dc && !(p.dc_sg == 3 && p.dc_se == 1 && p.rest_sg == 3LL * (p.M - 1) && p.rest_se == 1);
}
template <bool kStr>
static void launch_fwd(const PreprocessParams& p, hipStream_t s) {
    const dim3 g((p.P + 255) / 256), b(256);
    switch (p.D <= 0 ? 0 : (p.D >= 3 ? 3 : p.D)) {  // degrees > 3 evaluate as 3, like forward.cu:32-60
        case 0: hipLaunchKernelGGL((k_preprocess_fwd<0, kStr>), g, b, 0, s, p); break;
        case 1: hipLaunchKernelGGL((k_preprocess_fwd<1, kStr>), g, b, 0, s, p); break;
        case 2: hipLaunchKernelGGL((k_preprocess_fwd<2, kStr>), g, b, 0, s, p); break;
        default: hipLaunchKernelGGL((k_preprocess_fwd<3, kStr>), g, b, 0, s, p); break;
    }
}
void launch_preprocess_fwd(const PreprocessParams& p, hipStream_t s) {
    if (p.P <= 0) return;
    if (strided_sh(p)) launch_fwd<true>(p, s);
    else launch_fwd<false>(p, s);
}
template <bool kStr, int kSrc, bool kAcc>
static void launch_bwd_sh(const PreprocessBwdParams& p, dim3 g, dim3 b, hipStream_t s) {
    if (!kStr && !kAcc && kSrc == 1 && p.M == 16 && (p.adam.dc.p || p.adam.rest.p)) {  // fused Adam, params in LDS
        const dim3 gw((p.P + kShWave - 1) / kShWave), bw(kShWave);
        switch (p.D <= 0 ? 0 : (p.D >= 3 ? 3 : p.D)) {
            case 0: hipLaunchKernelGGL(k_preprocess_bwd_sh_adam<0>, gw, bw, 0, s, p); break;
            case 1: hipLaunchKernelGGL(k_preprocess_bwd_sh_adam<1>, gw, bw, 0, s, p); break;
            case 2: hipLaunchKernelGGL(k_preprocess_bwd_sh_adam<2>, gw, bw, 0, s, p); break;
            default: hipLaunchKernelGGL(k_preprocess_bwd_sh_adam<3>, gw, bw, 0, s, p); break;
        }
        return;
    }
    if (!kStr && !kAcc && kSrc != 0 && p.M == 16 && (p.adam.dc.p || p.adam.rest.p)) {  // fused Adam epilogue
        const dim3 gw((p.P + kShWave - 1) / kShWave), bw(kShWave);
        switch (p.D <= 0 ? 0 : (p.D >= 3 ? 3 : p.D)) {
            case 0: hipLaunchKernelGGL((k_preprocess_bwd_sh_rows<0, kSrc, false, true>), gw, bw, 0, s, p); break;
            case 1: hipLaunchKernelGGL((k_preprocess_bwd_sh_rows<1, kSrc, false, true>), gw, bw, 0, s, p); break;
            case 2: hipLaunchKernelGGL((k_preprocess_bwd_sh_rows<2, kSrc, false, true>), gw, bw, 0, s, p); break;
            default: hipLaunchKernelGGL((k_preprocess_bwd_sh_rows<3, kSrc, false, true>), gw, bw, 0, s, p); break;
        }
        return;
    }
    if (!kStr && p.M == 16) {  // coalesced rows (every training configuration)
        const dim3 gw((p.P + kShWave - 1) / kShWave), bw(kShWave);
        switch (p.D <= 0 ? 0 : (p.D >= 3 ? 3 : p.D)) {
            case 0: hipLaunchKernelGGL((k_preprocess_bwd_sh_rows<0, kSrc, kAcc>), gw, bw, 0, s, p); break;
            case 1: hipLaunchKernelGGL((k_preprocess_bwd_sh_rows<1, kSrc, kAcc>), gw, bw, 0, s, p); break;
            case 2: hipLaunchKernelGGL((k_preprocess_bwd_sh_rows<2, kSrc, kAcc>), gw, bw, 0, s, p); break;
            default: hipLaunchKernelGGL((k_preprocess_bwd_sh_rows<3, kSrc, kAcc>), gw, bw, 0, s, p); break;
        }
        return;
    }
    switch (p.D <= 0 ? 0 : (p.D >= 3 ? 3 : p.D)) {
        case 0: hipLaunchKernelGGL((k_preprocess_bwd_sh<0, kStr, kSrc, kAcc>), g, b, 0, s, p); break;
        case 1: hipLaunchKernelGGL((k_preprocess_bwd_sh<1, kStr, kSrc, kAcc>), g, b, 0, s, p); break;
        case 2: hipLaunchKernelGGL((k_preprocess_bwd_sh<2, kStr, kSrc, kAcc>), g, b, 0, s, p); break;
        default: hipLaunchKernelGGL((k_preprocess_bwd_sh<3, kStr, kSrc, kAcc>), g, b, 0, s, p); break;
    }
}
// With SH: the SH half (k_preprocess_bwd_sh<DEG>) then the geometry half (degree-independent); without
// (colors_precomp): the geometry half alone.
template <bool kStr>
static void launch_bwd(const PreprocessBwdParams& p, hipStream_t s) {
    const dim3 g((p.P + 255) / 256), b(256);
    if ((p.shs || p.sh_dc) && !p.defer_view_dir) {
        const int src = p.shs ? 0 : (p.sh_off ? 2 : 1);
        const bool acc = p.sh_accumulate != 0 && !p.shs;
        if (src == 0) launch_bwd_sh<kStr, 0, false>(p, g, b, s);
        else if (src == 1) acc ? launch_bwd_sh<kStr, 1, true>(p, g, b, s) : launch_bwd_sh<kStr, 1, false>(p, g, b, s);
        else acc ? launch_bwd_sh<kStr, 2, true>(p, g, b, s) : launch_bwd_sh<kStr, 2, false>(p, g, b, s);
    }
    hipLaunchKernelGGL(k_preprocess_bwd, g, b, 0, s, p);
}
void launch_preprocess_bwd(const PreprocessBwdParams& p, hipStream_t s) {
    if (p.P <= 0) return;
    if (strided_sh(p)) launch_bwd<true>(p, s);
    else launch_bwd<false>(p, s);
}
void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t s) {
    if (P > 0) hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, view, present);
}
}  // namespace gsd
