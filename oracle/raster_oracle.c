/*
 * raster_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A float32 CPU restatement of the reference rasterizer
 * (Heng14/gaussian-splatting_deformable, submodules/diff-gaussian-rasterization).
 * It is the checker the parity tests, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg compare the HIP path against.  Nothing in the product path
 * (gaussian-splatting_deformable_amd/) may link, load or call this file.
 *
 * Every routine follows one reference function; the citation is given above it.
 * Expression trees are written in the reference's evaluation order (glm
 * column-major products expanded explicitly), and the file is compiled with
 * -ffp-contract=off, so the results are exactly the un-contracted IEEE-754
 * float32 values of the reference's arithmetic.  That no-FMA contract is the
 * parity contract for the bit-exact outputs (depth, xy, radii, rect, keys,
 * ranges, point_list); the real CUDA build (nvcc contracts to FMA) cannot be
 * run here (no nvcc, no NVIDIA GPU), see DESIGN.md "Oracle".
 *
 * Atomic-accumulated gradients (backward render) are summed here in double
 * and rounded once, i.e. the order-free value the float atomics approximate.
 *
 * Threads (OpenMP, orc_set_threads): the per-Gaussian loops split over
 * Gaussians, the render loops over tiles, the instance emission over Gaussians
 * at their scanned offsets; each result element has one writer, so the
 * outputs do not depend on the thread count, except the backward render's
 * double sums, which each thread keeps in its own buffer and which are added
 * in thread order (differences at the 1e-16 level before the float rounding).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TILE_X 16 /* config.h:16 BLOCK_X */
#define TILE_Y 16 /* config.h:17 BLOCK_Y */

/* thread count of every parallel loop below; 0 = OpenMP's default (OMP_NUM_THREADS or all cores) */
static int g_threads = 0;
void orc_set_threads(int n) { g_threads = n > 0 ? n : 0; }
int orc_get_threads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}
#define NT orc_get_threads()

/* auxiliary.h:22-39 */
static const float C0 = 0.28209479177387814f;
static const float C1 = 0.4886025119029199f;
static const float C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                            -1.0925484305920792f, 0.5462742152960396f};
static const float C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                            0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                            -0.5900435899266435f};

static inline float fminf_(float a, float b) { return a < b ? a : b; }
static inline float fmaxf_(float a, float b) { return a > b ? a : b; }

/* glm 3x3, column-major: m[c][r] */
typedef struct { float m[3][3]; } mat3;

/* glm type_mat3x3.inl operator*(mat3, mat3): R[c][r] = (A[0][r]B[c][0] + A[1][r]B[c][1]) + A[2][r]B[c][2] */
static mat3 mmul(const mat3* A, const mat3* B) {
    mat3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r)
            R.m[c][r] = A->m[0][r] * B->m[c][0] + A->m[1][r] * B->m[c][1] + A->m[2][r] * B->m[c][2];
    return R;
}
static mat3 mtrans(const mat3* A) {
    mat3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) R.m[c][r] = A->m[r][c];
    return R;
}
/* glm::mat3(a..i) takes columns: (a,b,c) is column 0 */
static mat3 mcols(float a, float b, float c, float d, float e, float f, float g, float h, float i) {
    mat3 R;
    R.m[0][0] = a; R.m[0][1] = b; R.m[0][2] = c;
    R.m[1][0] = d; R.m[1][1] = e; R.m[1][2] = f;
    R.m[2][0] = g; R.m[2][1] = h; R.m[2][2] = i;
    return R;
}
/* glm::dot(vec3,vec3) = (x*x' + y*y') + z*z' (func_geometric.inl compute_dot) */
static inline float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

/* auxiliary.h:58-66 transformPoint4x3 */
static void xform4x3(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
/* auxiliary.h:68-77 transformPoint4x4 */
static void xform4x4(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}
/* auxiliary.h:89-97 transformVec4x3Transpose */
static void xvec4x3T(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[1] * p[1] + m[2] * p[2];
    o[1] = m[4] * p[0] + m[5] * p[1] + m[6] * p[2];
    o[2] = m[8] * p[0] + m[9] * p[1] + m[10] * p[2];
}

/* auxiliary.h:41-44 ndc2Pix -- the literals 1.0 / 0.5 make this a double expression */
static inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

/* auxiliary.h:46-56 getRect (grid clamp; int truncation of float quotients) */
static void get_rect(float px, float py, int max_radius, int gx, int gy, int* rmin, int* rmax) {
    int a;
    float r = (float)max_radius;
    a = (int)((px - r) / (float)TILE_X); a = a > 0 ? a : 0; rmin[0] = a < gx ? a : gx;
    a = (int)((py - r) / (float)TILE_Y); a = a > 0 ? a : 0; rmin[1] = a < gy ? a : gy;
    a = (int)((px + r + (float)TILE_X - 1.0f) / (float)TILE_X); a = a > 0 ? a : 0; rmax[0] = a < gx ? a : gx;
    a = (int)((py + r + (float)TILE_Y - 1.0f) / (float)TILE_Y); a = a > 0 ? a : 0; rmax[1] = a < gy ? a : gy;
}

/* auxiliary.h:139-164 in_frustum (near plane only; the lateral test is commented out upstream) */
static int in_frustum(const float* p, const float* view, const float* proj, float* p_view) {
    float ph[4];
    xform4x4(p, proj, ph);   /* computed upstream, result unused */
    (void)ph;
    xform4x3(p, view, p_view);
    return !(p_view[2] <= 0.2f);
}

/* rasterizer_impl.cu:54-66 checkFrustum / rasterize_points.cu:198-217 markVisible */
void orc_mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present) {
    for (int i = 0; i < P; ++i) {
        float pv[3];
        present[i] = (uint8_t)in_frustum(means3D + 3 * i, view, proj, pv);
    }
}

/* forward.cu:118-152 computeCov3D (no quaternion normalisation, forward.cu:127) */
static void cov3d_fwd(const float* s, float mod, const float* q, float* cov) {
    mat3 S = mcols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * s[0];
    S.m[1][1] = mod * s[1];
    S.m[2][2] = mod * s[2];
    float r = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R = mcols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                   2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                   2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 M = mmul(&S, &R);
    mat3 Mt = mtrans(&M);
    mat3 Sig = mmul(&Mt, &M);
    cov[0] = Sig.m[0][0]; cov[1] = Sig.m[0][1]; cov[2] = Sig.m[0][2];
    cov[3] = Sig.m[1][1]; cov[4] = Sig.m[1][2]; cov[5] = Sig.m[2][2];
}

/* forward.cu:74-113 computeCov2D (EWA: J W Sigma W^T J^T + 0.3 I) */
static void cov2d_fwd(const float* mean, float fx, float fy, float tanx, float tany, const float* c3,
                      const float* view, float* out) {
    float t[3];
    xform4x3(mean, view, t);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = fminf_(limx, fmaxf_(-limx, txtz)) * t[2];
    t[1] = fminf_(limy, fmaxf_(-limy, tytz)) * t[2];
    mat3 J = mcols(fx / t[2], 0.0f, -(fx * t[0]) / (t[2] * t[2]), 0.0f, fy / t[2], -(fy * t[1]) / (t[2] * t[2]), 0, 0, 0);
    mat3 W = mcols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    mat3 T = mmul(&W, &J);
    mat3 V = mcols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    mat3 Tt = mtrans(&T), Vt = mtrans(&V);
    mat3 A = mmul(&Tt, &Vt);
    mat3 cov = mmul(&A, &T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    out[0] = cov.m[0][0]; out[1] = cov.m[0][1]; out[2] = cov.m[1][1];
}

/* forward.cu:20-71 computeColorFromSH (vec3 ops expanded per component, same tree) */
static void sh_fwd(int deg, const float* pos, const float* campos, const float* sh, float* rgb, uint8_t* clamp) {
    float d[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    float len = sqrtf(dot3(d, d));
    d[0] = d[0] / len; d[1] = d[1] / len; d[2] = d[2] / len;
    float x = d[0], y = d[1], z = d[2];
    for (int ch = 0; ch < 3; ++ch) {
        const float* s = sh + ch; /* s[3*k] is coefficient k of channel ch */
        float res = C0 * s[0];
        if (deg > 0) {
            res = res - C1 * y * s[3] + C1 * z * s[6] - C1 * x * s[9];
            if (deg > 1) {
                float xx = x * x, yy = y * y, zz = z * z;
                float xy = x * y, yz = y * z, xz = x * z;
                res = res + C2[0] * xy * s[12] + C2[1] * yz * s[15] + C2[2] * (2.0f * zz - xx - yy) * s[18] +
                      C2[3] * xz * s[21] + C2[4] * (xx - yy) * s[24];
                if (deg > 2) {
                    res = res + C3[0] * y * (3.0f * xx - yy) * s[27] + C3[1] * xy * z * s[30] +
                          C3[2] * y * (4.0f * zz - xx - yy) * s[33] +
                          C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * s[36] +
                          C3[4] * x * (4.0f * zz - xx - yy) * s[39] + C3[5] * z * (xx - yy) * s[42] +
                          C3[6] * x * (xx - 3.0f * yy) * s[45];
                }
            }
        }
        res += 0.5f;
        clamp[ch] = (uint8_t)(res < 0);
        rgb[ch] = res < 0.0f ? 0.0f : res; /* glm::max(result, 0) */
    }
}

/*
 * forward.cu:155-256 preprocessCUDA.  Culled Gaussians get radii=0,
 * tiles_touched=0 and (unlike the reference, which leaves them untouched)
 * zeros in every other output.
 */
void orc_preprocess(int P, int D, int M, const float* means3D, const float* scales, float scale_mod,
                    const float* rots, const float* opac, const float* shs, const float* cov3D_precomp,
                    const float* colors_precomp, const float* view, const float* proj, const float* campos,
                    int W, int H, float tanx, float tany,
                    int* radii, float* means2D, float* depths, float* cov3D, float* rgb,
                    float* conic_opacity, uint32_t* tiles_touched, uint8_t* clamped) {
    const float fy = (float)H / (2.0f * tany); /* rasterizer_impl.cu:222-223 */
    const float fx = (float)W / (2.0f * tanx);
    const int gx = (W + TILE_X - 1) / TILE_X, gy = (H + TILE_Y - 1) / TILE_Y;
    (void)M;
#pragma omp parallel for schedule(static) num_threads(NT)
    for (int i = 0; i < P; ++i) {
        radii[i] = 0; tiles_touched[i] = 0;
        depths[i] = 0; means2D[2 * i] = means2D[2 * i + 1] = 0;
        for (int k = 0; k < 4; ++k) conic_opacity[4 * i + k] = 0;
        for (int k = 0; k < 3; ++k) { rgb[3 * i + k] = 0; clamped[3 * i + k] = 0; }
        for (int k = 0; k < 6; ++k) cov3D[6 * i + k] = 0;
        const float* p = means3D + 3 * i;
        float pv[3];
        if (!in_frustum(p, view, proj, pv)) continue;
        float ph[4];
        xform4x4(p, proj, ph);
        float pw = 1.0f / (ph[3] + 0.0000001f);
        float pp[3] = {ph[0] * pw, ph[1] * pw, ph[2] * pw};
        const float* c3;
        if (cov3D_precomp) {
            c3 = cov3D_precomp + 6 * i;
        } else {
            cov3d_fwd(scales + 3 * i, scale_mod, rots + 4 * i, cov3D + 6 * i);
            c3 = cov3D + 6 * i;
        }
        float cov[3];
        cov2d_fwd(p, fx, fy, tanx, tany, c3, view, cov);
        float det = (cov[0] * cov[2] - cov[1] * cov[1]);
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
        float mid = 0.5f * (cov[0] + cov[2]);
        float l1 = mid + sqrtf(fmaxf_(0.1f, mid * mid - det));
        float l2 = mid - sqrtf(fmaxf_(0.1f, mid * mid - det));
        float my_radius = ceilf(3.f * sqrtf(fmaxf_(l1, l2)));
        float pix[2] = {ndc2pix(pp[0], W), ndc2pix(pp[1], H)};
        int rmin[2], rmax[2];
        get_rect(pix[0], pix[1], (int)my_radius, gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        if (!colors_precomp) sh_fwd(D, p, campos, shs + (size_t)i * M * 3, rgb + 3 * i, clamped + 3 * i);
        depths[i] = pv[2];
        radii[i] = (int)my_radius;
        means2D[2 * i] = pix[0]; means2D[2 * i + 1] = pix[1];
        conic_opacity[4 * i + 0] = conic[0]; conic_opacity[4 * i + 1] = conic[1];
        conic_opacity[4 * i + 2] = conic[2]; conic_opacity[4 * i + 3] = opac[i];
        tiles_touched[i] = (uint32_t)((rmax[1] - rmin[1]) * (rmax[0] - rmin[0]));
    }
}

/* rasterizer_impl.cu:35-50 getHigherMsb */
uint32_t orc_higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4, step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step; else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

/*
 * rasterizer_impl.cu:275-318: InclusiveSum of tiles_touched, duplicateWithKeys
 * (:70-111), stable radix SortPairs over bits [0, 32+msb) (:300-308),
 * identifyTileRanges (:116-138).  The radix sort is a stable LSD counting sort
 * with 8-bit digits, i.e. the order cub::DeviceRadixSort::SortPairs defines.
 * Returns num_rendered; keys/vals/ranges must hold K / K / tiles entries
 * (call with keys==NULL first to size).
 */
int64_t orc_binning(int P, int W, int H, const float* means2D, const float* depths, const int* radii,
                    const uint32_t* tiles_touched, uint32_t* point_offsets, uint64_t* keys_out,
                    uint32_t* vals_out, uint32_t* ranges) {
    const int gx = (W + TILE_X - 1) / TILE_X, gy = (H + TILE_Y - 1) / TILE_Y;
    uint32_t acc = 0;
    for (int i = 0; i < P; ++i) { acc += tiles_touched[i]; if (point_offsets) point_offsets[i] = acc; }
    int64_t K = acc;
    if (!keys_out) return K;
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (K ? K : 1));
    uint32_t* vals = (uint32_t*)malloc(sizeof(uint32_t) * (K ? K : 1));
    /* duplicateWithKeys: Gaussian i writes from offsets[i-1] (rasterizer_impl.cu:84) */
    uint32_t* starts = (uint32_t*)malloc(sizeof(uint32_t) * (P ? P : 1));
    acc = 0;
    for (int i = 0; i < P; ++i) { starts[i] = acc; acc += tiles_touched[i]; }
#pragma omp parallel for schedule(dynamic, 4096) num_threads(NT)
    for (int i = 0; i < P; ++i) {
        if (!(radii[i] > 0)) continue;
        uint64_t off = starts[i];
        int rmin[2], rmax[2];
        get_rect(means2D[2 * i], means2D[2 * i + 1], radii[i], gx, gy, rmin, rmax);
        uint32_t dbits;
        memcpy(&dbits, depths + i, 4);
        for (int y = rmin[1]; y < rmax[1]; ++y)
            for (int x = rmin[0]; x < rmax[0]; ++x) {
                uint64_t key = (uint64_t)(uint32_t)(y * gx + x);
                key <<= 32;
                key |= dbits;
                keys[off] = key; vals[off] = (uint32_t)i; ++off;
            }
    }
    free(starts);
    int end_bit = 32 + (int)orc_higher_msb((uint32_t)(gx * gy));
    uint64_t* k2 = (uint64_t*)malloc(sizeof(uint64_t) * (K ? K : 1));
    uint32_t* v2 = (uint32_t*)malloc(sizeof(uint32_t) * (K ? K : 1));
    for (int bit = 0; bit < end_bit; bit += 8) {
        int nb = end_bit - bit < 8 ? end_bit - bit : 8;
        uint64_t mask = (1ull << nb) - 1;
        int64_t cnt[257];
        memset(cnt, 0, sizeof(cnt));
        for (int64_t k = 0; k < K; ++k) cnt[((keys[k] >> bit) & mask) + 1]++;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (int64_t k = 0; k < K; ++k) {
            int64_t dst = cnt[(keys[k] >> bit) & mask]++;
            k2[dst] = keys[k]; v2[dst] = vals[k];
        }
        uint64_t* tk = keys; keys = k2; k2 = tk;
        uint32_t* tv = vals; vals = v2; v2 = tv;
    }
    memset(ranges, 0, sizeof(uint32_t) * 2 * (size_t)gx * gy);
    for (int64_t k = 0; k < K; ++k) {
        uint32_t cur = (uint32_t)(keys[k] >> 32);
        if (k == 0) ranges[2 * cur] = 0;
        else {
            uint32_t prev = (uint32_t)(keys[k - 1] >> 32);
            if (cur != prev) { ranges[2 * prev + 1] = (uint32_t)k; ranges[2 * cur] = (uint32_t)k; }
        }
        if (k == K - 1) ranges[2 * cur + 1] = (uint32_t)K;
    }
    memcpy(keys_out, keys, sizeof(uint64_t) * K);
    memcpy(vals_out, vals, sizeof(uint32_t) * K);
    free(keys); free(vals); free(k2); free(v2);
    return K;
}

/* forward.cu:261-374 renderCUDA (per pixel; the 256-wide batching does not change results) */
void orc_render_fwd(int W, int H, const uint32_t* ranges, const uint32_t* point_list, const float* means2D,
                    const float* features, const float* conic_opacity, const float* bg,
                    float* out_color, float* final_T, uint32_t* n_contrib, float* margin) {
    const int gx = (W + TILE_X - 1) / TILE_X, gy = (H + TILE_Y - 1) / TILE_Y;
#pragma omp parallel for collapse(2) schedule(dynamic, 1) num_threads(NT)
    for (int ty = 0; ty < gy; ++ty)
        for (int tx = 0; tx < gx; ++tx) {
            const uint32_t r0 = ranges[2 * (ty * gx + tx)], r1 = ranges[2 * (ty * gx + tx) + 1];
            for (int py = ty * TILE_Y; py < ty * TILE_Y + TILE_Y && py < H; ++py)
                for (int px = tx * TILE_X; px < tx * TILE_X + TILE_X && px < W; ++px) {
                    float T = 1.0f, C[3] = {0, 0, 0};
                    uint32_t contributor = 0, last = 0;
                    /* decision margins (test infrastructure, not the reference): the smallest relative distance of
                     * an evaluated alpha from 1/255 and of a tested T (1 - alpha) from 1e-4 -- where either is within
                     * the exp's rounding, an implementation with another expf may decide the other way */
                    float m_alpha = INFINITY, m_T = INFINITY;
                    const float fx = (float)px, fy = (float)py;
                    for (uint32_t k = r0; k < r1; ++k) {
                        contributor++;
                        const uint32_t g = point_list[k];
                        const float dx = means2D[2 * g] - fx, dy = means2D[2 * g + 1] - fy;
                        const float* co = conic_opacity + 4 * g;
                        float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                        if (power > 0.0f) continue;
                        /* CUDA's min(float, float) is fminf: a NaN product gives 0.99 (IEEE minNum) */
                        float alpha = fminf(0.99f, co[3] * expf(power));
                        if (margin) m_alpha = fminf(m_alpha, fabsf((float)((double)alpha * 255.0 - 1.0)));
                        if (alpha < 1.0f / 255.0f) continue;
                        float test_T = T * (1 - alpha);
                        if (margin) m_T = fminf(m_T, fabsf((float)((double)test_T * 1e4 - 1.0)));
                        if (test_T < 0.0001f) break;
                        for (int ch = 0; ch < 3; ++ch) C[ch] += features[3 * g + ch] * alpha * T;
                        T = test_T;
                        last = contributor;
                    }
                    const int pid = W * py + px;
                    final_T[pid] = T;
                    n_contrib[pid] = last;
                    if (margin) { margin[2 * pid] = m_alpha; margin[2 * pid + 1] = m_T; }
                    for (int ch = 0; ch < 3; ++ch) out_color[ch * H * W + pid] = C[ch] + T * bg[ch];
                }
        }
}

/*
 * backward.cu:399-557 renderCUDA (backward).  Per pixel, back to front; the
 * nine atomicAdd targets are accumulated in double, in pixel order.
 * dL_dmean2D is (P,3) (z stays 0), dL_dconic is the float4 view of (P,2,2).
 */
void orc_render_bwd(int P, int W, int H, const uint32_t* ranges, const uint32_t* point_list, const float* bg,
                    const float* means2D, const float* conic_opacity, const float* colors, const float* final_Ts,
                    const uint32_t* n_contrib, const float* dL_dpix, float* dL_dmean2D, float* dL_dconic,
                    float* dL_dopacity, float* dL_dcolors) {
    const int gx = (W + TILE_X - 1) / TILE_X, gy = (H + TILE_Y - 1) / TILE_Y;
    /* one double accumulator set per thread: m2x m2y cx cy cw op r g b.  The thread count is capped so the sets
     * stay within 2 GiB (72 B per Gaussian each: many-core hosts would otherwise ask for tens of GB), and an
     * allocation failure halves it down to one thread before failing loudly. */
    const size_t per_thread = ((size_t)P * 9 + 1) * sizeof(double);
    int nt = NT;
    const size_t budget = (size_t)2 << 30;
    if ((size_t)nt * per_thread > budget) nt = (int)(budget / per_thread) > 1 ? (int)(budget / per_thread) : 1;
    double* accs = NULL;
    for (;;) {
        accs = (double*)calloc((size_t)nt * per_thread / sizeof(double), sizeof(double));
        if (accs || nt == 1) break;
        nt /= 2;
    }
    if (!accs) {
        fprintf(stderr, "orc_render_bwd: cannot allocate %zu bytes of accumulators\n", per_thread);
        abort();
    }
    const float ddelx_dx = (float)(0.5 * W), ddely_dy = (float)(0.5 * H);
#pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
    double* acc = accs + ((size_t)P * 9 + 1) * omp_get_thread_num();
#else
    double* acc = accs;
#endif
#pragma omp for collapse(2) schedule(dynamic, 1)
    for (int ty = 0; ty < gy; ++ty)
        for (int tx = 0; tx < gx; ++tx) {
            const uint32_t r0 = ranges[2 * (ty * gx + tx)], r1 = ranges[2 * (ty * gx + tx) + 1];
            for (int py = ty * TILE_Y; py < ty * TILE_Y + TILE_Y && py < H; ++py)
                for (int px = tx * TILE_X; px < tx * TILE_X + TILE_X && px < W; ++px) {
                    const int pid = W * py + px;
                    const float T_final = final_Ts[pid];
                    float T = T_final;
                    uint32_t contributor = r1 - r0;
                    const uint32_t last_contributor = n_contrib[pid];
                    float accum_rec[3] = {0, 0, 0}, last_color[3] = {0, 0, 0}, last_alpha = 0;
                    float dpix[3];
                    for (int ch = 0; ch < 3; ++ch) dpix[ch] = dL_dpix[ch * H * W + pid];
                    const float fxp = (float)px, fyp = (float)py;
                    for (uint32_t k = r1; k-- > r0;) {
                        contributor--;
                        if (contributor >= last_contributor) continue;
                        const uint32_t g = point_list[k];
                        const float dx = means2D[2 * g] - fxp, dy = means2D[2 * g + 1] - fyp;
                        const float* co = conic_opacity + 4 * g;
                        const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                        if (power > 0.0f) continue;
                        const float G = expf(power);
                        const float alpha = fminf(0.99f, co[3] * G);  /* minNum, as forward */
                        if (alpha < 1.0f / 255.0f) continue;
                        T = T / (1.f - alpha);
                        const float dchannel_dcolor = alpha * T;
                        float dL_dalpha = 0.0f;
                        for (int ch = 0; ch < 3; ++ch) {
                            const float c = colors[3 * g + ch];
                            accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                            last_color[ch] = c;
                            dL_dalpha += (c - accum_rec[ch]) * dpix[ch];
                            acc[9 * (size_t)g + 6 + ch] += (double)(dchannel_dcolor * dpix[ch]);
                        }
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        float bg_dot = 0;
                        for (int ch = 0; ch < 3; ++ch) bg_dot += bg[ch] * dpix[ch];
                        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                        const float dL_dG = co[3] * dL_dalpha;
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_ddelx = -gdx * co[0] - gdy * co[1];
                        const float dG_ddely = -gdy * co[2] - gdx * co[1];
                        acc[9 * (size_t)g + 0] += (double)(dL_dG * dG_ddelx * ddelx_dx);
                        acc[9 * (size_t)g + 1] += (double)(dL_dG * dG_ddely * ddely_dy);
                        acc[9 * (size_t)g + 2] += (double)(-0.5f * gdx * dx * dL_dG);
                        acc[9 * (size_t)g + 3] += (double)(-0.5f * gdx * dy * dL_dG);
                        acc[9 * (size_t)g + 4] += (double)(-0.5f * gdy * dy * dL_dG);
                        acc[9 * (size_t)g + 5] += (double)(G * dL_dalpha);
                    }
                }
        }
    }
    for (int t = 1; t < nt; ++t) {
        const double* a = accs + ((size_t)P * 9 + 1) * t;
#pragma omp parallel for schedule(static) num_threads(nt)
        for (size_t j = 0; j < (size_t)P * 9; ++j) accs[j] += a[j];
    }
    const double* acc = accs;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int g = 0; g < P; ++g) {
        const double* a = acc + 9 * (size_t)g;
        dL_dmean2D[3 * g + 0] = (float)a[0]; dL_dmean2D[3 * g + 1] = (float)a[1]; dL_dmean2D[3 * g + 2] = 0.0f;
        dL_dconic[4 * g + 0] = (float)a[2]; dL_dconic[4 * g + 1] = (float)a[3];
        dL_dconic[4 * g + 2] = 0.0f; dL_dconic[4 * g + 3] = (float)a[4];
        dL_dopacity[g] = (float)a[5];
        for (int ch = 0; ch < 3; ++ch) dL_dcolors[3 * g + ch] = (float)a[6 + ch];
    }
    free(accs);
}

/* backward.cu:144-274 computeCov2DCUDA -- dL_dmeans is ASSIGNED (backward.cu:273) */
static void cov2d_bwd(const float* mean, const float* c3, float hx, float hy, float tanx, float tany,
                      const float* view, const float* dconic4, float* dmean, float* dcov) {
    float dc[3] = {dconic4[0], dconic4[1], dconic4[3]};
    float t[3];
    xform4x3(mean, view, t);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = fminf_(limx, fmaxf_(-limx, txtz)) * t[2];
    t[1] = fminf_(limy, fmaxf_(-limy, tytz)) * t[2];
    const float xgm = txtz < -limx || txtz > limx ? 0 : 1;
    const float ygm = tytz < -limy || tytz > limy ? 0 : 1;
    mat3 J = mcols(hx / t[2], 0.0f, -(hx * t[0]) / (t[2] * t[2]), 0.0f, hy / t[2], -(hy * t[1]) / (t[2] * t[2]), 0, 0, 0);
    mat3 Wm = mcols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    mat3 V = mcols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    mat3 T = mmul(&Wm, &J);
    mat3 Tt = mtrans(&T), Vt = mtrans(&V);
    mat3 A = mmul(&Tt, &Vt);
    mat3 cov2 = mmul(&A, &T);
    float a = cov2.m[0][0] += 0.3f;
    float b = cov2.m[0][1];
    float c = cov2.m[1][1] += 0.3f;
    float denom = a * c - b * b;
    float dL_da = 0, dL_db = 0, dL_dc = 0;
    float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float (*Tm)[3] = T.m;
    if (denom2inv != 0) {
        dL_da = denom2inv * (-c * c * dc[0] + 2 * b * c * dc[1] + (denom - a * c) * dc[2]);
        dL_dc = denom2inv * (-a * a * dc[2] + 2 * a * b * dc[1] + (denom - a * c) * dc[0]);
        dL_db = denom2inv * 2 * (b * c * dc[0] - (denom + 2 * b * b) * dc[1] + a * b * dc[2]);
        dcov[0] = (Tm[0][0] * Tm[0][0] * dL_da + Tm[0][0] * Tm[1][0] * dL_db + Tm[1][0] * Tm[1][0] * dL_dc);
        dcov[3] = (Tm[0][1] * Tm[0][1] * dL_da + Tm[0][1] * Tm[1][1] * dL_db + Tm[1][1] * Tm[1][1] * dL_dc);
        dcov[5] = (Tm[0][2] * Tm[0][2] * dL_da + Tm[0][2] * Tm[1][2] * dL_db + Tm[1][2] * Tm[1][2] * dL_dc);
        dcov[1] = 2 * Tm[0][0] * Tm[0][1] * dL_da + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_db + 2 * Tm[1][0] * Tm[1][1] * dL_dc;
        dcov[2] = 2 * Tm[0][0] * Tm[0][2] * dL_da + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_db + 2 * Tm[1][0] * Tm[1][2] * dL_dc;
        dcov[4] = 2 * Tm[0][2] * Tm[0][1] * dL_da + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_db + 2 * Tm[1][1] * Tm[1][2] * dL_dc;
    } else {
        for (int i = 0; i < 6; ++i) dcov[i] = 0;
    }
    float (*Vm)[3] = V.m;
    float dT00 = 2 * (Tm[0][0] * Vm[0][0] + Tm[0][1] * Vm[0][1] + Tm[0][2] * Vm[0][2]) * dL_da +
                 (Tm[1][0] * Vm[0][0] + Tm[1][1] * Vm[0][1] + Tm[1][2] * Vm[0][2]) * dL_db;
    float dT01 = 2 * (Tm[0][0] * Vm[1][0] + Tm[0][1] * Vm[1][1] + Tm[0][2] * Vm[1][2]) * dL_da +
                 (Tm[1][0] * Vm[1][0] + Tm[1][1] * Vm[1][1] + Tm[1][2] * Vm[1][2]) * dL_db;
    float dT02 = 2 * (Tm[0][0] * Vm[2][0] + Tm[0][1] * Vm[2][1] + Tm[0][2] * Vm[2][2]) * dL_da +
                 (Tm[1][0] * Vm[2][0] + Tm[1][1] * Vm[2][1] + Tm[1][2] * Vm[2][2]) * dL_db;
    float dT10 = 2 * (Tm[1][0] * Vm[0][0] + Tm[1][1] * Vm[0][1] + Tm[1][2] * Vm[0][2]) * dL_dc +
                 (Tm[0][0] * Vm[0][0] + Tm[0][1] * Vm[0][1] + Tm[0][2] * Vm[0][2]) * dL_db;
    float dT11 = 2 * (Tm[1][0] * Vm[1][0] + Tm[1][1] * Vm[1][1] + Tm[1][2] * Vm[1][2]) * dL_dc +
                 (Tm[0][0] * Vm[1][0] + Tm[0][1] * Vm[1][1] + Tm[0][2] * Vm[1][2]) * dL_db;
    float dT12 = 2 * (Tm[1][0] * Vm[2][0] + Tm[1][1] * Vm[2][1] + Tm[1][2] * Vm[2][2]) * dL_dc +
                 (Tm[0][0] * Vm[2][0] + Tm[0][1] * Vm[2][1] + Tm[0][2] * Vm[2][2]) * dL_db;
    float (*Wq)[3] = Wm.m;
    float dJ00 = Wq[0][0] * dT00 + Wq[0][1] * dT01 + Wq[0][2] * dT02;
    float dJ02 = Wq[2][0] * dT00 + Wq[2][1] * dT01 + Wq[2][2] * dT02;
    float dJ11 = Wq[1][0] * dT10 + Wq[1][1] * dT11 + Wq[1][2] * dT12;
    float dJ12 = Wq[2][0] * dT10 + Wq[2][1] * dT11 + Wq[2][2] * dT12;
    float tz = 1.f / t[2];
    float tz2 = tz * tz;
    float tz3 = tz2 * tz;
    float dtx = xgm * -hx * tz2 * dJ02;
    float dty = ygm * -hy * tz2 * dJ12;
    float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * t[0]) * tz3 * dJ02 + (2 * hy * t[1]) * tz3 * dJ12;
    float dt[3] = {dtx, dty, dtz};
    xvec4x3T(dt, view, dmean);
}

/* auxiliary.h:107-117 dnormvdv(float3) */
static void dnormvdv3(const float* v, const float* dv, float* o) {
    float sum2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    o[0] = ((+sum2 - v[0] * v[0]) * dv[0] - v[1] * v[0] * dv[1] - v[2] * v[0] * dv[2]) * invsum32;
    o[1] = (-v[0] * v[1] * dv[0] + (sum2 - v[1] * v[1]) * dv[1] - v[2] * v[1] * dv[2]) * invsum32;
    o[2] = (-v[0] * v[2] * dv[0] - v[1] * v[2] * dv[1] + (sum2 - v[2] * v[2]) * dv[2]) * invsum32;
}

/* backward.cu:20-139 computeColorFromSH (backward); vec3 ops per component, same trees */
static void sh_bwd(int deg, int M, const float* pos, const float* campos, const float* sh, const uint8_t* clamped,
                   const float* dcolor, float* dmean, float* dsh) {
    float dir_orig[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    float len = sqrtf(dot3(dir_orig, dir_orig));
    float dir[3] = {dir_orig[0] / len, dir_orig[1] / len, dir_orig[2] / len};
    float dRGB[3];
    for (int c = 0; c < 3; ++c) dRGB[c] = dcolor[c] * (clamped[c] ? 0 : 1);
    float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
    float x = dir[0], y = dir[1], z = dir[2];
    (void)M;
#define SH(k, c) sh[3 * (k) + (c)]
#define DSH(k, c) dsh[3 * (k) + (c)]
    float d0 = C0;
    for (int c = 0; c < 3; ++c) DSH(0, c) = d0 * dRGB[c];
    if (deg > 0) {
        float d1 = -C1 * y, d2 = C1 * z, d3 = -C1 * x;
        for (int c = 0; c < 3; ++c) {
            DSH(1, c) = d1 * dRGB[c]; DSH(2, c) = d2 * dRGB[c]; DSH(3, c) = d3 * dRGB[c];
            dx[c] = -C1 * SH(3, c); dy[c] = -C1 * SH(1, c); dz[c] = C1 * SH(2, c);
        }
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            float d4 = C2[0] * xy, d5 = C2[1] * yz, d6 = C2[2] * (2.f * zz - xx - yy), d7 = C2[3] * xz,
                  d8 = C2[4] * (xx - yy);
            for (int c = 0; c < 3; ++c) {
                DSH(4, c) = d4 * dRGB[c]; DSH(5, c) = d5 * dRGB[c]; DSH(6, c) = d6 * dRGB[c];
                DSH(7, c) = d7 * dRGB[c]; DSH(8, c) = d8 * dRGB[c];
                /* glm: scalar*scalar*...*vec3 products associate left to right */
                dx[c] += C2[0] * y * SH(4, c) + C2[2] * 2.f * -x * SH(6, c) + C2[3] * z * SH(7, c) + C2[4] * 2.f * x * SH(8, c);
                dy[c] += C2[0] * x * SH(4, c) + C2[1] * z * SH(5, c) + C2[2] * 2.f * -y * SH(6, c) + C2[4] * 2.f * -y * SH(8, c);
                dz[c] += C2[1] * y * SH(5, c) + C2[2] * 2.f * 2.f * z * SH(6, c) + C2[3] * x * SH(7, c);
            }
            if (deg > 2) {
                float d9 = C3[0] * y * (3.f * xx - yy), d10 = C3[1] * xy * z, d11 = C3[2] * y * (4.f * zz - xx - yy),
                      d12 = C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy), d13 = C3[4] * x * (4.f * zz - xx - yy),
                      d14 = C3[5] * z * (xx - yy), d15 = C3[6] * x * (xx - 3.f * yy);
                for (int c = 0; c < 3; ++c) {
                    DSH(9, c) = d9 * dRGB[c]; DSH(10, c) = d10 * dRGB[c]; DSH(11, c) = d11 * dRGB[c];
                    DSH(12, c) = d12 * dRGB[c]; DSH(13, c) = d13 * dRGB[c]; DSH(14, c) = d14 * dRGB[c];
                    DSH(15, c) = d15 * dRGB[c];
                    dx[c] += (C3[0] * SH(9, c) * 3.f * 2.f * xy + C3[1] * SH(10, c) * yz + C3[2] * SH(11, c) * -2.f * xy +
                              C3[3] * SH(12, c) * -3.f * 2.f * xz + C3[4] * SH(13, c) * (-3.f * xx + 4.f * zz - yy) +
                              C3[5] * SH(14, c) * 2.f * xz + C3[6] * SH(15, c) * 3.f * (xx - yy));
                    dy[c] += (C3[0] * SH(9, c) * 3.f * (xx - yy) + C3[1] * SH(10, c) * xz +
                              C3[2] * SH(11, c) * (-3.f * yy + 4.f * zz - xx) + C3[3] * SH(12, c) * -3.f * 2.f * yz +
                              C3[4] * SH(13, c) * -2.f * xy + C3[5] * SH(14, c) * -2.f * yz + C3[6] * SH(15, c) * -3.f * 2.f * xy);
                    dz[c] += (C3[1] * SH(10, c) * xy + C3[2] * SH(11, c) * 4.f * 2.f * yz +
                              C3[3] * SH(12, c) * 3.f * (2.f * zz - xx - yy) + C3[4] * SH(13, c) * 4.f * 2.f * xz +
                              C3[5] * SH(14, c) * (xx - yy));
                }
            }
        }
    }
#undef SH
#undef DSH
    float ddir[3] = {dot3(dx, dRGB), dot3(dy, dRGB), dot3(dz, dRGB)};
    float dm[3];
    dnormvdv3(dir_orig, ddir, dm);
    dmean[0] += dm[0]; dmean[1] += dm[1]; dmean[2] += dm[2];
}

/* backward.cu:278-341 computeCov3D (backward): dL/dscale (no modifier factor), dL/dq (unnormalised q) */
static void cov3d_bwd(const float* scale, float mod, const float* q, const float* dcov, float* dscale, float* drot) {
    float r = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R = mcols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                   2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                   2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 S = mcols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2];
    mat3 M = mmul(&S, &R);
    mat3 dSig = mcols(dcov[0], 0.5f * dcov[1], 0.5f * dcov[2], 0.5f * dcov[1], dcov[3], 0.5f * dcov[4],
                      0.5f * dcov[2], 0.5f * dcov[4], dcov[5]);
    mat3 M2;
    for (int c = 0; c < 3; ++c)
        for (int rr = 0; rr < 3; ++rr) M2.m[c][rr] = 2.0f * M.m[c][rr];
    mat3 dM = mmul(&M2, &dSig);
    mat3 Rt = mtrans(&R), dMt = mtrans(&dM);
    dscale[0] = dot3(Rt.m[0], dMt.m[0]);
    dscale[1] = dot3(Rt.m[1], dMt.m[1]);
    dscale[2] = dot3(Rt.m[2], dMt.m[2]);
    for (int k = 0; k < 3; ++k) { dMt.m[0][k] *= s[0]; dMt.m[1][k] *= s[1]; dMt.m[2][k] *= s[2]; }
    float (*D)[3] = dMt.m;
    drot[0] = 2 * z * (D[0][1] - D[1][0]) + 2 * y * (D[2][0] - D[0][2]) + 2 * x * (D[1][2] - D[2][1]);
    drot[1] = 2 * y * (D[1][0] + D[0][1]) + 2 * z * (D[2][0] + D[0][2]) + 2 * r * (D[1][2] - D[2][1]) - 4 * x * (D[2][2] + D[1][1]);
    drot[2] = 2 * x * (D[1][0] + D[0][1]) + 2 * r * (D[2][0] - D[0][2]) + 2 * z * (D[1][2] + D[2][1]) - 4 * y * (D[2][2] + D[0][0]);
    drot[3] = 2 * r * (D[0][1] - D[1][0]) + 2 * x * (D[2][0] + D[0][2]) + 2 * y * (D[1][2] + D[2][1]) - 4 * z * (D[1][1] + D[0][0]);
}

/*
 * backward.cu:559-622 BACKWARD::preprocess = computeCov2DCUDA (:144-274) then
 * preprocessCUDA (:346-396).  Only Gaussians with radii > 0 are touched.
 */
void orc_preprocess_bwd(int P, int D, int M, const float* means3D, const int* radii, const float* shs,
                        const uint8_t* clamped, const float* scales, const float* rots, float scale_mod,
                        const float* cov3D, const float* view, const float* proj, int W, int H, float tanx,
                        float tany, const float* campos, const float* dL_dmean2D, const float* dL_dconic,
                        const float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh,
                        float* dL_dscale, float* dL_drot) {
    const float fy = (float)H / (2.0f * tany), fx = (float)W / (2.0f * tanx);
#pragma omp parallel for schedule(static) num_threads(NT)
    for (int i = 0; i < P; ++i) {
        if (!(radii[i] > 0)) continue;
        const float* m = means3D + 3 * i;
        cov2d_bwd(m, cov3D + 6 * i, fx, fy, tanx, tany, view, dL_dconic + 4 * i, dL_dmean3D + 3 * i, dL_dcov3D + 6 * i);
        float mh[4];
        xform4x4(m, proj, mh);
        float mw = 1.0f / (mh[3] + 0.0000001f);
        float mul1 = (proj[0] * m[0] + proj[4] * m[1] + proj[8] * m[2] + proj[12]) * mw * mw;
        float mul2 = (proj[1] * m[0] + proj[5] * m[1] + proj[9] * m[2] + proj[13]) * mw * mw;
        const float* d2 = dL_dmean2D + 3 * i;
        float dm[3];
        dm[0] = (proj[0] * mw - proj[3] * mul1) * d2[0] + (proj[1] * mw - proj[3] * mul2) * d2[1];
        dm[1] = (proj[4] * mw - proj[7] * mul1) * d2[0] + (proj[5] * mw - proj[7] * mul2) * d2[1];
        dm[2] = (proj[8] * mw - proj[11] * mul1) * d2[0] + (proj[9] * mw - proj[11] * mul2) * d2[1];
        float* out = dL_dmean3D + 3 * i;
        out[0] += dm[0]; out[1] += dm[1]; out[2] += dm[2];
        if (shs)
            sh_bwd(D, M, m, campos, shs + (size_t)i * M * 3, clamped + 3 * i, dL_dcolor + 3 * i, out,
                   dL_dsh + (size_t)i * M * 3);
        if (scales) cov3d_bwd(scales + 3 * i, scale_mod, rots + 4 * i, dL_dcov3D + 6 * i, dL_dscale + 3 * i, dL_drot + 4 * i);
    }
}

/* Exported single-stage helpers for pinning against the reference's Python modules. */
void orc_sh_to_rgb(int N, int deg, int M, const float* pos, const float* campos, const float* sh, float* rgb,
                   uint8_t* clamped) {
    for (int i = 0; i < N; ++i) sh_fwd(deg, pos + 3 * i, campos, sh + (size_t)i * M * 3, rgb + 3 * i, clamped + 3 * i);
}
void orc_cov3d(int N, const float* scales, float mod, const float* rots, float* cov) {
    for (int i = 0; i < N; ++i) cov3d_fwd(scales + 3 * i, mod, rots + 4 * i, cov + 6 * i);
}
