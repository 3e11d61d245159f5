// gsd_kernels.h -- kernel parameter blocks and launch declarations.
//
// State layout in HBM (one view; all arrays SoA, 256-B aligned; see
// gsd_capi.hip "carve" functions and DESIGN.md "Data layout"):
//   geometry (per Gaussian):  means2D float2 | conic_opacity float4 | rgb float4 (a=0) |
//                             depth f32 | clamped u8 (bit c = channel c clamped) | radii i32
//   image (per pixel / tile): final_T f32 [Npix] | n_contrib u32 [Npix] |
//                             ranges uint2 [T] | tile_count u32 [T] | tile_cursor u32 [T] |
//                             counters u32 [4] (num_rendered, error flags)
//   binning (per instance):   bucket_keys u64 [K] ((depth bits << 32) | gaussian id, grouped by
//                             tile) | merge scratch u64 [K] | point_list u32 [K]
#pragma once
#include "gsd_device.h"

namespace gsd {

enum : uint32_t { kErrPrefiltered = 1u };

// What the render kernels stage per gathered instance, one 64-B record per Gaussian (k_preprocess_fwd writes it
// for the visible ones; point_list references no other): one 64-B fetch per instance instead of three from the
// separate xy, conic + opacity and rgb arrays (the render kernels' FETCH_SIZE was 3.4x their algorithmic bytes),
// and the alpha box computed once per Gaussian instead of per instance in both passes.
// Bounding box (x0, x1, y0, y1) of {d : alpha(d) >= 1/255} for a record, inflated for safety.
// Q(d) = a dx^2 + 2 b dx dy + c dy^2 <= t = 2 ln(255 o); half-widths sqrt(t c/det), sqrt(t a/det).
__device__ __forceinline__ float4 alpha_box(float2 xy, float4 co) {
    const float a = co.x, b = co.y, c = co.z, o = co.w;
    const float det = a * c - b * b;
    const float lo = 255.0f * o;
    // a NaN opacity composites at alpha = fminf(0.99, NaN) = 0.99 wherever power <= 0 (forward.cu:343): never cull
    if (lo != lo) return make_float4(-1e30f, 1e30f, -1e30f, 1e30f);
    if (!(lo >= 0.999f)) return make_float4(1e30f, -1e30f, 1e30f, -1e30f);  // alpha < 1/255 everywhere
    if (!(det > 0.0f)) return make_float4(-1e30f, 1e30f, -1e30f, 1e30f); // degenerate: never cull
    const float t = 2.0f * 0.69314718f * __builtin_amdgcn_logf(lo);     // 2 ln(255 o), v_log_f32 = log2
    // hardware sqrt / reciprocal (1 ulp): far inside the 0.1 % inflation
    const float rdet = __builtin_amdgcn_rcpf(det);
    const float ex = __builtin_amdgcn_sqrtf(fmaxf(t, 0.f) * c * rdet) * 1.001f + 0.02f;
    const float ey = __builtin_amdgcn_sqrtf(fmaxf(t, 0.f) * a * rdet) * 1.001f + 0.02f;
    if (!(ex < 1e30f) || !(ey < 1e30f)) return make_float4(-1e30f, 1e30f, -1e30f, 1e30f);
    return make_float4(xy.x - ex, xy.x + ex, xy.y - ey, xy.y + ey);
}

struct RenderRec {
    float4 q0;   // mean2D x, y, conic a, b
    float4 q1;   // conic c, opacity, r, g
    float4 q2;   // b, the backward culling's ellipse threshold (slack included), 1 / a, 1 / c
    float4 box;  // alpha_box(): x0, x1, y0, y1
};
static_assert(sizeof(RenderRec) == 64, "one 64-B segment per record");

struct PreprocessParams {
    int P, D, M, W, H, grid_x, grid_y, prefiltered;
    float scale_modifier, tan_fovx, tan_fovy, focal_x, focal_y;
    const float* means3D;
    const float* scales;
    const float* rotations;
    const float* opacities;
    const float* shs;
    const float* sh_dc;    // split SH operand (gsd_sh_split), used when shs == nullptr
    const float* sh_rest;
    const float* sh_off;
    long long dc_sg, dc_se, rest_sg, rest_se;  // split SH element strides (Gaussian, element)
    const float* cov3D_precomp;
    const float* colors_precomp;
    const float* view;
    const float* proj;
    const float* campos;
    int* radii;
    float2* means2D;
    float* depths;
    RenderRec* rec;        // what the render kernels gather per instance (written for visible Gaussians)
    uint8_t* clamped;
    uint32_t* tile_count;
    uint32_t* err_flags;
    int raw_act;           // scales / rotations / opacities are raw parameters (gsd_activation)
};

// Per-Gaussian gradient record of the rasterizer backward: 16 floats (one 64-B segment, the memory-side
// unit of a global atomic) holding dL/dmean2D x,y | dL/dconic a,b,c | dL/dopacity | dL/dcolor r,g,b.
constexpr int kGradRec = 16;
enum GradRecField { kRecMean2D = 0, kRecConic = 2, kRecOpacity = 5, kRecColor = 6, kRecUsed = 9 };
// floats 9..11 of a record: the view-direction term of dL/dmean3D, left there by k_preprocess_bwd_sh for
// k_preprocess_bwd (the two halves of the per-Gaussian backward)
constexpr int kRecShMean = 9;

// The Adam step of one fused sink (gsd_adam_sink after the host's double-precision coefficients); p == nullptr:
// not fused, the gradient goes to the sink.
struct AdamSinkDev {
    float* p;
    float* m;
    float* v;
    float step_size, bc2_sqrt;  // -lr / (1 - beta1^t), sqrt(1 - beta2^t)
};
struct AdamEpiDev {
    AdamSinkDev dc, rest, xyz, scaling, rotation, opacity;
    float w1, beta2, omb2, eps;  // 1 - beta1, beta2, 1 - beta2, eps
};

// torch.optim.Adam's per-element update in torch's foreach order (torch/optim/adam.py _multi_tensor_adam):
//   m = lerp(m, g, 1 - beta1); v = v * beta2 + (1 - beta2) * g * g; p += step_size * (m / (sqrt(v) / bc2 + eps))
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float w1, float beta2, float omb2,
                                          float step_size, float bc2_sqrt, float eps) {
    m = w1 < 0.5f ? m + w1 * (g - m) : g - (g - m) * (1.f - w1);
    v = v * beta2;
    v = v + omb2 * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p + step_size * (m / denom);
}
__device__ __forceinline__ void adam_at(const AdamSinkDev& s, const AdamEpiDev& e, long long i, float g) {
    float pp = s.p[i], mm = s.m[i], vv = s.v[i];
    adam_elem(pp, g, mm, vv, e.w1, e.beta2, e.omb2, s.step_size, s.bc2_sqrt, e.eps);
    s.p[i] = pp;
    s.m[i] = mm;
    s.v[i] = vv;
}

struct PreprocessBwdParams {
    int P, D, M;
    float scale_modifier, tan_fovx, tan_fovy, focal_x, focal_y;
    const float* means3D;
    const int* radii;
    const float* shs;
    const float* sh_dc;    // split SH operand, used when shs == nullptr
    const float* sh_rest;
    const float* sh_off;
    long long dc_sg, dc_se, rest_sg, rest_se;  // strides of sh_dc / dsh_dc and sh_rest / dsh_rest
    const uint8_t* clamped;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    const float* view;
    const float* proj;
    const float* campos;
    float* grad_rec;          // (P, kGradRec) per-Gaussian gradient records accumulated by k_render_bwd
    float* dL_dmean2D;        // (P,3) outputs unpacked from the records (written for every Gaussian)
    float* dL_dopacity;       // (P)
    float* dL_dcolor;         // (P,3)
    float* dL_dmeans3D;
    float* dL_dcov3D;
    float* dL_dsh;
    float* dsh_dc;         // split SH sinks (when dL_dsh == nullptr)
    float* dsh_rest;
    float* dsh_off;
    int sh_accumulate;
    float* d_rgb;          // (P,3) masked dL/dRGB instead of the SH sinks (gsd_sh_split.d_rgb), or NULL
    int defer_view_dir;    // with d_rgb: no SH half; the geometry half writes d_rgb, without the view-dir term
    int raw_act;           // raw parameters: gradients go to the sinks below (gsd_activation)
    const float* raw_opacity;
    float *a_xyz, *a_scaling, *a_rotation, *a_opacity;
    int a_accumulate;
    float* dL_dscales;
    float* dL_drotations;
    int adam_on;           // fused Adam epilogue (any of its sinks set)
    AdamEpiDev adam;
    // the view's densification statistics (gsd_densify_stats, train.py:613-616) folded into the geometry half,
    // which holds dL/dmean2D and radii in registers; NULL: not here (gsd_train_step sets them)
    float *dens_accum, *dens_accum3, *dens_denom, *dens_max_radii;
};

struct BinParams {
    int P, grid_x, grid_y, num_tiles;
    const int* radii;
    const float2* means2D;
    const float* depths;
    uint32_t* tile_cursor;
    unsigned long long* bucket_keys;
    const uint32_t* k_guard;  // optional: skip the launch when *k_guard (num_rendered) > k_cap
    uint32_t k_cap;
};

// LDS-histogram binning (gsd_binning.hip): block b owns Gaussians [b*chunk, (b+1)*chunk)
struct HistParams {
    int P, chunk, num_blocks, num_tiles, grid_x, grid_y;
    const int* radii;
    const float2* means2D;
    uint32_t* hist;  // [num_blocks][num_tiles]
    uint32_t* part;  // [ceil(num_blocks / kColSeg)][num_tiles]
    const uint32_t* k_guard;  // optional: k_scatter_hist does nothing when *k_guard (num_rendered) > k_cap
    uint32_t k_cap;
};

struct RenderParams {
    int W, H, grid_x, num_tiles;
    const uint2* ranges;
    const uint32_t* point_list;
    const RenderRec* rec;
    const float* bg;
    float* final_T;
    uint32_t* n_contrib;
    float* out_color;
    const uint32_t* k_guard;  // optional: skip the launch when *k_guard (num_rendered) > k_cap
    uint32_t k_cap;
    float4* zero_rec;         // optional: the backward's gradient records, zeroed by this launch (n16 float4s)
    long long zero_n16;
    int ref_alpha;            // gsd_raster_args.alpha_mode (ABI 17): 1 = the reference's alpha expression
};

struct RenderBwdParams {
    int W, H, grid_x, num_tiles;
    const uint2* ranges;
    const uint32_t* point_list;
    const RenderRec* rec;
    const float* bg;
    const float* final_T;
    const uint32_t* n_contrib;
    const float* dL_dpix;
    float* grad_rec;    // (P, kGradRec), zeroed before the launch
    int ref_alpha;      // as RenderParams.ref_alpha (the forward's mode)
};

struct ActivateParams {
    int P, R;  // R = rest SH coefficients per Gaussian (f_rest is (P,R,3))
    const float* xyz;
    const float* dxyz;     // optional offsets (NULL = 0)
    const float* scaling;
    const float* dscale;
    const float* rotation;
    const float* drot;
    const float* opacity;
    const float* f_dc;
    const float* f_rest;
    const float* dsh;      // (P,1+R,3) or NULL
    float* means_out;
    float* scales_out;
    float* rot_out;
    float* opac_out;
    float* shs_out;
};

struct ActivateBwdParams {
    int P, R, accumulate;
    const float* scaling;
    const float* dscale;
    const float* rotation;
    const float* drot;
    const float* opacity;
    const float* g_means;
    const float* g_scales;
    const float* g_rot;
    const float* g_opac;
    const float* g_shs;
    float* g_xyz;        // parameter grads: written, or added to when accumulate != 0 (NULL = skip)
    float* g_scaling;
    float* g_rotation;
    float* g_opacity;
    float* g_fdc;
    float* g_frest;
    float* g_dxyz;       // offset grads: always written (NULL = skip)
    float* g_dscale;
    float* g_drot;
    float* g_dsh;
};

// Host-side launchers (one per kernel; each lives in the .hip file that defines the kernel).
void launch_activate_fwd(const ActivateParams& p, hipStream_t s);
void launch_activate_bwd(const ActivateBwdParams& p, hipStream_t s);
void launch_preprocess_fwd(const PreprocessParams& p, hipStream_t s);
void launch_preprocess_bwd(const PreprocessBwdParams& p, hipStream_t s);
struct ShViewsParams {
    int P, D, M, n_views;
    long long view_stride;
    const float* means3D;
    const float* views;
    float *d_dc, *d_rest, *d_off;
    long long dc_sg, dc_se, rest_sg, rest_se;
    int accumulate;
    AdamEpiDev adam;  // fused Adam epilogue for dc / rest (rows kernel, store mode), p == nullptr: off
    const float* sh_dc;    // the SH coefficients (contiguous, M = 16) for d_means, else unused
    const float* sh_rest;
    float* d_means;        // (P,3): the views' summed view-direction term (gsd_sh_grad_views_ex), or nullptr
};
void launch_sh_grad_views(const ShViewsParams& p, hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t s);
void launch_tile_scan(int num_tiles, const uint32_t* tile_count, uint2* ranges, uint32_t* tile_cursor,
                      uint32_t* counters, hipStream_t s);
void launch_scatter_keys(const BinParams& p, hipStream_t s);
void launch_tile_sort(int num_tiles, const uint2* ranges, unsigned long long* keys, unsigned long long* scratch,
                      uint32_t* point_list, hipStream_t s, const uint32_t* k_guard = nullptr, uint32_t k_cap = 0);
void launch_render_fwd(const RenderParams& p, hipStream_t s);
void launch_render_bwd(const RenderBwdParams& p, hipStream_t s);
void launch_se3_fwd(int P, const float* twist, const float* means_in, const float* rot_in, float* means_out,
                    float* rot_out, hipStream_t s);
void launch_se3_bwd(int P, const float* twist, const float* means_in, const float* rot_in, const float* dmeans_out,
                    const float* drot_out, float* dtwist, float* dmeans_in, float* drot_in, hipStream_t s);

void launch_tile_hist(const HistParams& p, uint32_t* tile_count, hipStream_t s);
void launch_scatter_hist(const HistParams& p, const uint32_t* tile_base, const float* depths,
                         unsigned long long* keys, hipStream_t s);

void launch_densify_stats(int P, const float* vgrad, const int* radii, float* accum, float* accum3, float* denom,
                          float* max_radii, hipStream_t s);

size_t knn_workspace(int P, size_t* sort_bytes);
int launch_knn(int P, const float* pts, float* out, void* ws, hipStream_t s);

// deformation network forward on the bf16 matrix cores (gsd_mlp.hip)
constexpr int kMlpLayers = 9;      // 8 hidden + the four heads as one
constexpr int kMlpFrags = 64512;   // 16-B A fragments of all layers (1008 KB)
constexpr int kMlpBias = 2112;     // packed biases (32 per row block)
struct MlpParams {
    int P;
    const float* x;      // (P,3) canonical means
    const float* t;      // (P) time
    const void* frags;   // kMlpFrags x 16 B, fragment-major (gsd_amd.deform_mlp.pack_fused_mlp)
    const float* bias;   // kMlpBias floats, [layer][row block][lane half][register]
    float* d_xyz;        // (P,3)
    float* d_scale;      // (P,3)
    float* d_rot;        // (P,4)
    float* d_sh;         // (P,48)
};
void launch_mlp_fwd(const MlpParams& p, hipStream_t s);
int relu_bwd_bias_blocks(long long P, int rows);
void launch_relu_bwd_bias(long long P, int N, int bf16, const void* gy, const void* y, void* g, float* part,
                          int rows, hipStream_t s);

// the deformation network's f32-accurate training path (gsd_mlp_train.hip)
// A layer's weight as the reference stores it: up to 4 row pieces (the four heads) of ldw columns each; `map` names
// the padded input layout: 0 identity, 1 layer 0 [enc(x) 63 | 0 | enc(t) 21 | 0 x 11], 2 layer 5 [enc(x) 63 | 0 | h 256]
struct MlpWeightRef {
    float* W[4];
    int row_off[5];      // piece i holds rows [row_off[i], row_off[i + 1])
    int n_pieces, ldw, map;
};
struct MlpPackParams {
    MlpWeightRef w;
    int M, K;              // packed A is M x K (multiples of 32 / 16); forward A = W, backward A = W^T
    int transpose;
    void* out;             // (K / 16) x (M / 32) x 3 x 64 fragments of 16 B
    // k-steps >= perm_from take their 16 columns in the accumulator order of the layer before (element j of lane
    // half h is column 8 (j >> 2) + 4 h + (j & 3) of the step), for a B operand read straight from the previous
    // layer's accumulators (k_mlp_fwd_fused); natural order below it
    int perm_from;
    int m_off;             // transpose: A row m is W^T row m + m_off (layer 5's h rows for the backward chain)
    // m16: fragments of v_mfma_f32_16x16x32_bf16 (k_mlp_fwd_fused16): (K / 32) x (M / 16) x 3 x 64 of 16 B, lane l
    // holding row 16 rb + (l & 15) and columns 32 ks + 8 (l >> 4) + j (natural) or 32 ks + 16 (j >> 2) + 4 (l >> 4) +
    // (j & 3) (k-steps >= perm_from: the 16 x 16 accumulator order)
    int m16;
};
struct MlpPackBatch {   // up to 12 packs in one launch
    MlpPackParams job[12];
    int n;
};
void launch_mlp_pack_batch(const MlpPackBatch& b, hipStream_t s);
// The layer-fused training forward (k_mlp_fwd_fused): the encoding in, every hidden layer's output, its ReLU words
// and the heads out; the weights packed with the accumulator-order k permutation (perm_from 0; layer 5: 4; layer 0:
// natural).
// The four heads' outputs (dx 3, d log-scale 3, d quaternion 4, dSH 48: columns [0,3) [3,6) [6,10) [10,58) of the
// 58-wide head layer), each a row-major (P, ld[k]) array: separate tensors (ld = width), or views into one (P, 58)
// array (ld = 58, out[k] offset by the head's first column).  Inputs (the backward's incoming gradients) likewise,
// NULL: a zero gradient.
constexpr int kMlpHeadCol[5] = {0, 3, 6, 10, 58};
struct MlpHeads {
    float* out[4];
    int ld[4];
};
struct MlpHeadsIn {
    const float* src[4];
    int ld[4];
};
__device__ __forceinline__ void mlp_store_head(const MlpHeads& o, long long g, int n, float v) {
    const int k = n < 3 ? 0 : (n < 6 ? 1 : (n < 10 ? 2 : 3));
    const int c0 = k == 0 ? 0 : (k == 1 ? 3 : (k == 2 ? 6 : 10));
    o.out[k][g * o.ld[k] + (n - c0)] = v;
}
struct MlpFusedParams {
    int P, ldp;
    const float* E;          // [64][ldp]: enc(x), row 63 zero
    const float* ET;         // [32][ldp]: enc(t), rows 21.. zero
    const void* frags[9];    // packed W of the eight hidden layers and the heads
    const float* bias[8];    // the hidden layers' biases (256)
    const float* bias_heads; // 64 (58 used)
    float* H[8];             // layer l's output: [256][ldp]
    unsigned short* bits[8]; // its ReLU words: [(rb * 2 + h) * ldp + g]
    MlpHeads heads;          // the four heads' outputs
};
// The backward's dX chain (k_mlp_bwd_chain): step i = layer 8 - i multiplies W^T by g_{8-i} (frags[i]: W8^T natural
// k order, K = 64; then W7^T .. W1^T in the accumulator order, layer 5's rows 64-319), masks by the forward's ReLU
// words of h_{8-i} (bits[i]) and stores its input g_{8-i} to G[i] (G[0]: [64][ldp], the rest [256][ldp]); the final
// step stores g0 to G[8] and the encoding's gradient W5^T[enc rows] g5 + W0^T[enc rows] g0 to dE ([64][ldp]).
struct MlpChainParams {
    int P, ldp;
    MlpHeadsIn heads;                 // the heads' incoming gradients
    const void* frags[8];
    const void* frags_e;              // W0^T rows 0-63 (accumulator order, K = 256)
    const void* frags_e5;             // W5^T rows 0-63 (the enc(x) rows of the skip layer; accumulator order)
    const unsigned short* bits[8];
    float* G[9];
    float* dE;
};
void launch_mlp_bwd_chain(const MlpChainParams& p, hipStream_t s);
// the same chain at two waves per SIMD, 16 Gaussians per wave (k_mlp_bwd_chain16: every W^T packed with m16; reads
// the ReLU words either forward writes)
void launch_mlp_bwd_chain16(const MlpChainParams& p, hipStream_t s);
enum { kMlpFwdRelu = 0, kMlpFwdHeads = 1, kMlpBwdMask = 2 };
struct MlpGemmParams {
    int P, ldp;                     // Gaussians; row stride of the feature-major matrices (P rounded up to 256)
    const float* src0;              // X^T rows 0 .. 16 ks0 - 1: [16 ks0][ldp]
    int ks0;
    const float* src1;              // the rest: [16 ks1][ldp] (the concatenated inputs of layers 0 and 5)
    int ks1;
    const void* frags;              // k_mlp_pack output: [ks][rb][split][lane]
    int rb;                         // output row blocks of 32 (of the packed A)
    int rb_off;                     // launch-internal: first row block of this workgroup row (grid.y)
    const float* bias;              // forward: 32 rb floats
    float* dst;                     // forward hidden: [32 rb][ldp]; backward: g rows
    MlpHeads heads;                 // heads: the four outputs (58 columns)
    int n_a;                        // backward: rows below n_a go to dst_a (the encoding's gradient, no ReLU)
    float* dst_a;
    int accumulate_a;
    const float* mask;              // backward: h of the rows >= n_a ([rows - n_a][ldp]); NULL: those rows dropped
    // the ReLU masks as bits in the accumulator layout: word [(rb * 2 + h) * ldp + g] holds bit q of row
    // 32 rb + 8 (q >> 2) + 4 h + (q & 3) of Gaussian g (h > 0).  Forward: written when mask_out != NULL; backward:
    // read instead of mask when mask_in != NULL (row block rb >= n_a / 32 uses word rb - n_a / 32)
    unsigned short* mask_out;
    const unsigned short* mask_in;
};
struct MlpWgradParams {
    int P, ldp;
    const float* G;                 // [32 n_rb][ldp]
    int n_rb;
    const float* X0;                // [32 k_rb0][ldp], then X1: [32 (k_rb - k_rb0)][ldp]
    const float* X1;
    int k_rb, k_rb0;
    int k_off;                      // padded input column of this call's first k (a layer's k range in pieces)
    int tiles_n, tiles_k;           // 128 x 128 output tiles
    int chunk;                      // Gaussians per wave (multiple of 16)
    float* partial;                 // [chunks][32 n_rb][32 k_rb]
    float* bias_partial;            // [chunks][32 n_rb]
    int accumulate;                 // the reduction adds into the destination pieces instead of storing
    int skip_bias;                  // the bias gradient is another call's (layer 5's second column range)
};
void launch_mlp_pack(const MlpPackParams& p, hipStream_t s);
void launch_mlp_encode(int P, int ldp, const float* x, const float* t, float* E, float* ET, hipStream_t s);
void launch_mlp_encode_bwd(int P, int ldp, const float* E, const float* dE, float* dx, int accumulate, hipStream_t s);
void launch_mlp_gemm(const MlpGemmParams& p, int mode, hipStream_t s);
void launch_mlp_fwd_fused(const MlpFusedParams& p, hipStream_t s, bool store = true);
// the same forward at two waves per SIMD, 16 Gaussians per wave (weights packed with m16; the same outputs)
void launch_mlp_fwd_fused16(const MlpFusedParams& p, hipStream_t s, bool store = true);
// dW scattered into the reference-shaped weight pieces (dst.W; map/rows as the forward weight), db into dst_b
void launch_mlp_wgrad(const MlpWgradParams& p, const MlpWeightRef& dst, const MlpWeightRef& dst_b, hipStream_t s);
void launch_mlp_rows_to_features(int P, int ldp, const MlpHeadsIn& src, float* dst, int dst_rows, hipStream_t s);
void launch_mlp_gather_bias(const MlpWeightRef& b, float* dst, int n_pad, hipStream_t s);

constexpr int kAdamMaxGroups = 16;
struct AdamArgs {
    long long n;                        // elements in the slabs
    int n_groups;
    int zero_grad;                      // also clear the gradient slab
    long long begin[kAdamMaxGroups];    // first element of each group (begin[0] == 0, increasing)
    float step_size[kAdamMaxGroups];    // -lr / (1 - beta1^t)
    float bc2_sqrt[kAdamMaxGroups];     // sqrt(1 - beta2^t)
    float w1, beta2, omb2, eps;         // 1 - beta1, beta2, 1 - beta2, eps
    const float* addend;                // nullptr, or elements [addend_lo, addend_hi) step on grad + addend
    long long addend_lo, addend_hi;
};
void launch_adam(const AdamArgs& a, float* param, float* grad, float* m, float* v, hipStream_t s);

void ssim_tiles(int H, int W, int* tiles_x, int* tiles_y);
void launch_l1_ssim(int C, int H, int W, const float* w11, float lambda, const float* img, const float* gt,
                    float* gmaps, float* partial, float* out3, float* dimg, hipStream_t s);
void launch_l1_ssim_bwd(int C, int H, int W, const float* w11, float lambda, const float* img, const float* gt,
                        const float* gmaps, const float* gscale, float sign, float* dimg, hipStream_t s);
int offnorm_blocks(long long P);
void launch_offset_norm(long long P, const float* off, float scale, float* partial, float* out, hipStream_t s);
void launch_offset_norm_bwd(long long P, const float* off, const float* gscale, float scale, float* d_off,
                            hipStream_t s);

constexpr int kHistThreads = 512;       // LDS-histogram binning workgroup
constexpr int kHistMaxTiles = 40960;    // 160 KiB of u32 bins; larger grids use global-atomic binning
constexpr int kHistTargetBlocks = 512;  // Gaussian chunks per view
constexpr int kColSeg = 32;             // histogram rows per column-scan segment
constexpr int kScanThreads = 1024;
// Instances sorted in one LDS pass (8 B of LDS per key).  Round 5: 2048 instead of 4096 -- the LDS and the
// 16-key register network of the 4096 class held k_tile_sort at five waves per SIMD with 144 B of scratch per
// lane; at 2048 it runs eight waves with none (0.0395 -> 0.0367 ms at cfg4, profiles/round5/binning/r5al/), and
// buckets of 2049-4096 keys take the LDS-chunk + global-merge path of the larger ones.
#ifndef GSD_SORT_CAP
#define GSD_SORT_CAP 2048
#endif
constexpr int kSortCap = GSD_SORT_CAP;

}  // namespace gsd
