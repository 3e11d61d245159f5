/*
 * gsd_raster.h -- C-ABI of the MI355X-native deformable Gaussian-splatting
 * rasterizer (libgsd_hip.so, built from gaussian-splatting_deformable_amd/csrc).
 *
 * Plain pointers and sizes only: every tensor argument is a device pointer to
 * contiguous float32/int32/uint8 memory owned by the caller, every `stream` is a
 * hipStream_t (NULL = legacy default stream).  The library never allocates
 * device memory on the data path and never frees caller memory; the three
 * opaque state buffers are sized by the *_bytes() queries and allocated by the
 * caller (the two-phase protocol that replaces the reference's resizable
 * std::function<char*(size_t)> byte tensors, rasterize_points.cu:27-33).
 *
 * Every entry point returns GSD_OK (0) or an error code; gsd_last_error()
 * returns the message (thread-local), using the reference's wording where the
 * reference raises (rasterize_points.cu:57-59, rasterizer_impl.cu:242-245).
 *
 * Reference interfaces replaced (Heng14/gaussian-splatting_deformable):
 *   gsd_rasterize_forward_bin + gsd_rasterize_forward_render
 *        <- _C.rasterize_gaussians  / RasterizeGaussiansCUDA
 *           (submodules/diff-gaussian-rasterization/rasterize_points.cu:35-115,
 *            bound at ext.cpp:16) and CudaRasterizer::Rasterizer::forward
 *           (cuda_rasterizer/rasterizer_impl.cu:198-336)
 *   gsd_rasterize_backward
 *        <- _C.rasterize_gaussians_backward / RasterizeGaussiansBackwardCUDA
 *           (rasterize_points.cu:117-196, ext.cpp:17) and Rasterizer::backward
 *           (rasterizer_impl.cu:340-434)
 *   gsd_mark_visible
 *        <- _C.mark_visible / markVisible (rasterize_points.cu:198-217, ext.cpp:18)
 *           and Rasterizer::markVisible (rasterizer_impl.cu:141-153)
 *   gsd_se3_deform_forward / gsd_se3_deform_backward
 *        <- scene/rigid_body.py exp_se3 (:86-93) applied per Gaussian as in
 *           gaussian_renderer/__init__.py:90-95 (commented out upstream), with
 *           the twist normalisation of scene/gaussian_model.py:161-165 and
 *           torch autograd as the reference backward.
 */
#ifndef GSD_RASTER_H
#define GSD_RASTER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSD_ABI_VERSION 17

enum {
    GSD_OK = 0,
    GSD_ERR_ARG = 1,     /* invalid argument (AT_ERROR / std::runtime_error upstream) */
    GSD_ERR_HIP = 2,     /* HIP runtime error (CHECK_CUDA upstream, auxiliary.h:166-173) */
    GSD_ERR_STATE = 3,   /* inconsistent state buffers (wrong size / wrong call order) */
    GSD_NEED_BINNING = 4 /* gsd_rasterize_forward: binning_buffer smaller than gsd_binning_buffer_bytes(
                            *num_rendered); phase 1 is done -- allocate and call gsd_rasterize_forward_render */
};

/* Split SH operand (optional, ABI 3).  The reference's render() materialises
 * shs = cat(features_dc, features_rest) + dSH (gaussian_renderer/__init__.py:129-134,
 * scene/gaussian_model.py:647-650) before calling the rasterizer.  A caller that
 * sets gsd_raster_args.sh_split instead hands over the pieces: the rasterizer
 * reads them in place (dc + offset is the same float add torch does) and the
 * backward writes dL/dSH straight into the pieces' gradient buffers.  With
 * sh_split set, args.shs must be NULL and args.M = 1 + rest coefficients. */
typedef struct gsd_sh_split {
    const float* dc;       /* (P,1,3) */
    const float* rest;     /* (P,M-1,3); may be NULL when M == 1 */
    const float* offset;   /* (P,M,3) additive SH offset, or NULL */
    float* d_dc;           /* backward sink dL/d dc (P,1,3), or NULL */
    float* d_rest;         /* backward sink dL/d rest (P,M-1,3), or NULL */
    float* d_offset;       /* backward sink dL/d offset (P,M,3), or NULL */
    int32_t accumulate;    /* backward: 1 = add into the sinks (entries of Gaussians with radii == 0 and of
                              coefficients above the active degree are then left as they are), 0 = store
                              (every entry written, zeros included) */
    float* d_rgb;          /* backward: NULL, or (P,3): then dL/dRGB masked by the colour clamp -- the view's
                              factor of the SH gradient, dL/dsh_k = B_k(dir) dL/dRGB -- is written here for every
                              Gaussian (zeros where radii == 0) instead of the SH gradient into the sinks;
                              gsd_sh_grad_views sums such rows of several views into the SH gradient */
    int64_t dc_stride_g, dc_stride_e;     /* element e (= 3 k + channel) of Gaussian g of dc and d_dc at
                                             [g * stride_g + e * stride_e]; 0, 0 = contiguous (P,1,3) */
    int64_t rest_stride_g, rest_stride_e; /* the same for rest / d_rest; 0, 0 = contiguous (P,M-1,3).
                                             Coefficient-major storage (stride_g 1, stride_e P: what
                                             gsd_amd.optim.FusedAdam lays out) makes every SH access of a
                                             wave one contiguous 256-B run instead of 64 rows */
    int32_t defer_view_dir;  /* ABI 9, with d_rgb: 1 = the backward reads no SH coefficient at all -- it writes
                                the d_rgb row and leaves the view-direction term of the SH colour
                                (backward.cu:385-392) out of dL/dmeans3D; gsd_sh_grad_views_ex supplies that
                                term summed over the exchanged views (d_means).  0 = the term is included. */
} gsd_sh_split;

/* Optional activation of the per-Gaussian inputs inside the rasterizer (the render() preamble without
 * offsets, gaussian_renderer/__init__.py:79-140 with scene/gaussian_model.py:761-797): with
 * gsd_raster_args.activation set, args->scales, ->rotations and ->opacities are the RAW parameters
 * (_scaling, _rotation, _opacity) and the rasterizer uses exp(scaling), normalize(rotation) (F.normalize,
 * eps 1e-12) and sigmoid(opacity) -- the same float operations as gsd_activate_forward.  The backward then
 * writes the raw-parameter gradients into the sinks below instead of dL_dmeans3D / dL_dscales /
 * dL_drotations / dL_dopacity (which may be NULL). */
typedef struct gsd_activation {
    float* d_xyz;          /* (P,3) dL/d means3D (= dL/d _xyz), or NULL */
    float* d_scaling;      /* (P,3) dL/d _scaling, or NULL */
    float* d_rotation;     /* (P,4) dL/d _rotation, or NULL */
    float* d_opacity;      /* (P,1) dL/d _opacity, or NULL */
    int32_t accumulate;    /* 1 = add into the sinks, 0 = store (every Gaussian written) */
} gsd_activation;

/* Optional Adam step fused into the backward (ABI 8): torch.optim.Adam's update (the same per-element
 * arithmetic as gsd_adam_step) applied where the backward would store a parameter's gradient -- the gradient
 * is final there when this backward is its only producer and nothing sums it over ranks -- instead of writing
 * it into the sink.  That is backward + step without the gradient's round trip through HBM (8 B per float).
 * A sink with param == NULL is not fused: its gradient is written as usual.  Fusion needs the store mode
 * (accumulate == 0) of its sink and contiguous (P,K,3) SH pieces; sh_split.d_rgb excludes the SH sinks. */
typedef struct gsd_adam_sink {
    float* param;          /* the parameter the rasterizer read (features_dc / _rest, _xyz, _scaling, ...) */
    float* exp_avg;        /* Adam moments, the parameter's layout */
    float* exp_avg_sq;
    double lr;             /* its group's learning rate */
    int64_t step;          /* its 1-based step count after this update */
} gsd_adam_sink;
typedef struct gsd_adam_epilogue {
    double beta1, beta2, eps;
    gsd_adam_sink dc, rest;                          /* the split SH pieces (gsd_sh_split) */
    gsd_adam_sink xyz, scaling, rotation, opacity;   /* the raw parameters (gsd_activation) */
} gsd_adam_epilogue;

/* Raster settings + per-Gaussian inputs of one view.  Mirrors the 19 arguments
 * of _C.rasterize_gaussians (rasterize_points.cu:36-55).  Absent optional
 * inputs are NULL (the reference passes empty tensors -> nullptr). */
typedef struct gsd_raster_args {
    int32_t P;                  /* number of Gaussians */
    int32_t D;                  /* active SH degree (0..3) */
    int32_t M;                  /* SH coefficients per Gaussian (sh.size(1)); 0 if shs == NULL */
    int32_t width, height;      /* image size in pixels */
    float scale_modifier;
    float tan_fovx, tan_fovy;
    int32_t prefiltered;        /* bool */
    int32_t debug;              /* bool: synchronise + check after every kernel */
    const float* background;    /* (3) */
    const float* means3D;       /* (P,3) */
    const float* shs;           /* (P,M,3) or NULL */
    const float* colors_precomp;/* (P,3) or NULL (exactly one of shs / colors_precomp) */
    const float* opacities;     /* (P,1) */
    const float* scales;        /* (P,3) or NULL */
    const float* rotations;     /* (P,4) or NULL (quaternion r,x,y,z; NOT normalised here) */
    const float* cov3D_precomp; /* (P,6) or NULL (exactly one of scales+rotations / cov3D_precomp) */
    const float* viewmatrix;    /* (4,4), column-major as stored by scene/cameras.py:55 */
    const float* projmatrix;    /* (4,4) full projection, scene/cameras.py:57 */
    const float* campos;        /* (3) */
    const gsd_sh_split* sh_split; /* NULL, or the split SH operand above (then shs == NULL) */
    const gsd_activation* activation; /* NULL, or: scales / rotations / opacities are raw parameters */
    const gsd_adam_epilogue* adam;    /* backward only: NULL, or the fused Adam step above (ABI 8) */
    void* grad_scratch;         /* ABI 14.  Forward: NULL, or a buffer of gsd_backward_scratch_bytes(P) bytes that
                                   the compositing kernel zeroes (under its VALU-bound work, instead of a separate
                                   64-B-per-Gaussian memset in the backward).  Backward: when it equals the
                                   backward's `scratch` argument, that scratch is taken as zeroed by the forward
                                   that was given it and is not cleared again (pass it to ONE backward only);
                                   NULL or any other value: the backward zeroes its scratch itself. */
    int32_t alpha_mode;         /* ABI 17: GSD_ALPHA_FAST (0, default) decides alpha >= 1/255 as power >= t_o (the
                                   exact real comparison) and forms alpha = exp(power - t_o) / 255 with the hardware
                                   exp; GSD_ALPHA_REFERENCE (1) evaluates forward.cu:343-345 as written,
                                   min(0.99, o * expf(power)) < 1/255 -- the oracle's decisions and final_T to ~2e-6
                                   (DESIGN.md 4), ~20 % slower compositing.  A backward must use its forward's mode. */
} gsd_raster_args;

enum { GSD_ALPHA_FAST = 0, GSD_ALPHA_REFERENCE = 1 };

int gsd_abi_version(void);
const char* gsd_last_error(void);
/* ABI 16, build provenance (no reference counterpart): the SHA-256 (64 hex digits) of the sources this library
 * was compiled from -- the csrc .hip and .h sources in name order, this header, csrc/Makefile -- and the extra compiler
 * flags of the build (HIPFLAGS_EXTRA, "" for the product build).  gsd_amd/_native.py recomputes the hash from its
 * tree and refuses a library built from other sources. */
const char* gsd_build_id(void);
const char* gsd_build_flags(void);

/* State-buffer sizes in bytes (GeometryState / ImageState / BinningState,
 * rasterizer_impl.h:29-73; layouts are private to this library). */
size_t gsd_geom_buffer_bytes(int32_t P, int32_t width, int32_t height);
size_t gsd_image_buffer_bytes(int32_t width, int32_t height);
size_t gsd_binning_buffer_bytes(int64_t num_rendered);

/* Introspection (tests / debugging; the reference exposes none): byte offsets,
 * from the state buffer's first 256-B aligned address, of
 *   geom[6]  = means2D float2; conic_opacity (4 floats) and rgb (3 floats) of Gaussian 0 -- both inside the
 *              64-B render records (x, y, a, b | c, opacity, r, g | b, culling threshold, 1/a, 1/c |
 *              alpha box), so Gaussian i's
 *              are 64 i bytes further; depths f32, radii i32, clamped u8
 *   image[6] = final_T f32, n_contrib u32, ranges uint2, tile_count u32, tile_cursor u32, counters u32
 *   bin[3]   = bucket keys u64, merge scratch u64, point_list u32 (point_list first in memory) */
void gsd_state_layout(int32_t P, int32_t width, int32_t height, int64_t num_rendered, size_t* geom_offsets,
                      size_t* image_offsets, size_t* binning_offsets);

/* Forward, phase 1: preprocess (EWA projection, SH -> RGB, radii) and per-tile
 * binning counts.  Writes radii (P) and *num_rendered (the sum of tiles
 * touched; one blocking device->host read, as rasterizer_impl.cu:281). */
int gsd_rasterize_forward_bin(const gsd_raster_args* args, void* geom_buffer, void* image_buffer,
                              int32_t* radii, int64_t* num_rendered, void* stream);

/* Forward, phase 2: emit (tile, depth) instances, order them (bit-exact with a
 * stable sort on the reference key |tile|depth bits|), composite front to
 * back.  binning_buffer holds gsd_binning_buffer_bytes(num_rendered) bytes.
 * out_color is (3,H,W). */
int gsd_rasterize_forward_render(const gsd_raster_args* args, void* geom_buffer, void* image_buffer,
                                 void* binning_buffer, int64_t num_rendered, const int32_t* radii,
                                 float* out_color, void* stream);

/* Both forward phases in one call, for a caller that allocates the binning buffer before num_rendered is
 * known (e.g. from the previous view's count plus headroom).  Phase 2 is queued behind phase 1 before the
 * host waits for the num_rendered read-back (its kernels compare the device-side count with what
 * binning_bytes holds and do nothing when it does not fit), so the device never idles on the read-back.
 * Returns GSD_NEED_BINNING (phase 1 done, *num_rendered set, phase 2 not done) when the buffer is too
 * small: allocate gsd_binning_buffer_bytes(*num_rendered) and call gsd_rasterize_forward_render.  The
 * backward only needs the buffer's point_list, which sits at an offset independent of the capacity. */
int gsd_rasterize_forward(const gsd_raster_args* args, void* geom_buffer, void* image_buffer, void* binning_buffer,
                          size_t binning_bytes, int32_t* radii, float* out_color, int64_t* num_rendered,
                          void* stream);

/* Backward (rasterizer_impl.cu:340-434).  Every output is written for every
 * Gaussian (zeros where radii == 0 and above the active SH degree), so none
 * needs a fill: dL_dmeans2D (P,3), dL_dcolors (P,3), dL_dopacity (P,1),
 * dL_dmeans3D (P,3), dL_dcov3D (P,6), dL_dsh (P,M,3) (may be NULL if M == 0),
 * dL_dscales (P,3), dL_drotations (P,4).  scratch holds
 * gsd_backward_scratch_bytes(P) bytes of device memory (replacing the
 * reference's dL_dconic2D temporary, rasterize_points.cu:153): the call zeroes
 * it and accumulates the per-pixel gradients there, one 64-B record per
 * Gaussian (dL/dmean2D, dL/dconic, dL/dopacity, dL/dcolor).
 * With args->sh_split set, dL_dsh is not used (the split sinks receive dL/dSH;
 * with accumulate != 0 only visible Gaussians' entries change); dL_dcov3D may
 * be NULL when cov3D_precomp is NULL (it is then not written). */
size_t gsd_backward_scratch_bytes(int32_t P);
int gsd_rasterize_backward(const gsd_raster_args* args, const int32_t* radii, const void* geom_buffer,
                           const void* binning_buffer, const void* image_buffer, int64_t num_rendered,
                           const float* dL_dout_color, float* dL_dmeans2D, void* scratch,
                           float* dL_dopacity, float* dL_dcolors, float* dL_dmeans3D, float* dL_dcov3D,
                           float* dL_dsh, float* dL_dscales, float* dL_drotations, void* stream);

/* (layout: NULL, or a gsd_sh_split whose stride fields describe d_dc / d_rest; its pointers are ignored.)
 * SH gradient of several views from their gsd_sh_split.d_rgb rows (data-parallel training: each rank
 * exchanges its view's (P,3) row, 12 B per Gaussian, instead of all-reducing the 192-B SH gradient):
 *   dL/dsh_k[c] = sum_v B_k(normalize(means3D - campos_v)) * d_rgb_v[c]    (backward.cu:20-139 per view)
 * views: n_views rows of view_stride floats, row v = [d_rgb_v (P*3) | campos_v (3)].  means3D (P,3) must be
 * the positions every view rendered (the same on every rank).  Sinks as in gsd_sh_split (any may be NULL);
 * accumulate 0 stores every entry (coefficients above degree D as zeros), 1 adds.  adam (ABI 8): NULL, or a
 * gsd_adam_epilogue whose dc / rest sinks are fused -- the assembled SH gradient is final here (every view
 * summed), so with accumulate 0, M = 16 and contiguous layouts the Adam step of those pieces is applied in
 * place instead of storing d_dc / d_rest (its other slots are ignored). */
int gsd_sh_grad_views(int32_t P, int32_t D, int32_t M, int32_t n_views, const float* means3D, const float* views,
                      int64_t view_stride, float* d_dc, float* d_rest, float* d_offset, int32_t accumulate,
                      const gsd_sh_split* layout, const gsd_adam_epilogue* adam, void* stream);
/* gsd_sh_grad_views plus, when d_means != NULL, the view-direction term of the SH colour that a backward with
 * gsd_sh_split.defer_view_dir left out of dL/dmeans3D, summed over the views (ABI 9):
 *   d_means[g] = sum_v dnormvdv(means3D[g] - campos_v, sum_c d_rgb_v[g][c] dRGB_c/ddir_v)   (backward.cu:385-392)
 * stored (P,3).  It needs the SH coefficients every view rendered: sh_dc (P,1,3) and sh_rest (P,M-1,3),
 * contiguous, M = 16, accumulate 0 (the layout of the training path); with the fused Adam step the coefficients
 * are read once for both uses. */
int gsd_sh_grad_views_ex(int32_t P, int32_t D, int32_t M, int32_t n_views, const float* means3D, const float* views,
                         int64_t view_stride, const float* sh_dc, const float* sh_rest, float* d_dc, float* d_rest,
                         float* d_offset, float* d_means, int32_t accumulate, const gsd_sh_split* layout,
                         const gsd_adam_epilogue* adam, void* stream);

/* Near-plane visibility test (auxiliary.h:139-164): present[i] = 1/0. */
int gsd_mark_visible(int32_t P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream);

/* Per-Gaussian SE(3) deform.  twist (P,6) = raw [w, v] as produced by the
 * deformation network (scene/gaussian_model.py:156); theta = |w|,
 * R = exp_so3(w/theta, theta), p = (theta I + (1-cos) W^ + (theta-sin) W^2) v/theta
 * (rigid_body.py:61-93), evaluated through series near theta = 0 so a zero
 * twist is the identity (the reference NaNs there).  means_out = R x + p;
 * rot_out = normalize(q_R (x) q) with q_R = (cos theta/2, sin theta/2 * w/theta)
 * (Hamilton product, helpers.py:63-70).  rot_in / rot_out may be NULL. */
int gsd_se3_deform_forward(int32_t P, const float* twist, const float* means_in, const float* rot_in,
                           float* means_out, float* rot_out, void* stream);

/* Backward of gsd_se3_deform_forward: overwrites dL_dtwist (P,6), dL_dmeans_in
 * (P,3) and (if rot_in != NULL) dL_drot_in (P,4). */
int gsd_se3_deform_backward(int32_t P, const float* twist, const float* means_in, const float* rot_in,
                            const float* dL_dmeans_out, const float* dL_drot_out, float* dL_dtwist,
                            float* dL_dmeans_in, float* dL_drot_in, void* stream);

/* Fused render() preamble (gaussian_renderer/__init__.py:79-140, gaussian_model.py:761-797):
 *   means = xyz + dxyz, scales = exp(scaling + dscale), rotations = normalize(rotation + drot),
 *   opacities = sigmoid(opacity), shs = cat(f_dc, f_rest) + dsh.
 * Offsets (dxyz (P,3), dscale (P,3), drot (P,4), dsh (P,1+R,3)) may be NULL = zero; f_rest is (P,R,3).
 * shs_out may be NULL: the SH stay split and go to the rasterizer as a gsd_sh_split. */
int gsd_activate_forward(int32_t P, int32_t R, const float* xyz, const float* dxyz, const float* scaling,
                         const float* dscale, const float* rotation, const float* drot, const float* opacity,
                         const float* f_dc, const float* f_rest, const float* dsh, float* means_out,
                         float* scales_out, float* rot_out, float* opac_out, float* shs_out, void* stream);

/* Backward of gsd_activate_forward.  Parameter gradients (g_xyz .. g_frest) are written, or added into the
 * existing values when accumulate != 0; offset gradients (g_dxyz .. g_dsh) are written.  Any output may be NULL.
 * g_shs may be NULL (split SH: the SH gradients were written by gsd_rasterize_backward). */
int gsd_activate_backward(int32_t P, int32_t R, int32_t accumulate, const float* scaling, const float* dscale,
                          const float* rotation, const float* drot, const float* opacity, const float* g_means,
                          const float* g_scales, const float* g_rot, const float* g_opac, const float* g_shs,
                          float* g_xyz, float* g_scaling, float* g_rotation, float* g_opacity, float* g_fdc,
                          float* g_frest, float* g_dxyz, float* g_dscale, float* g_drot, float* g_dsh, void* stream);

/* Training loss of one view, fused (utils/loss_utils.py:17-63 combined as train.py:529):
 *   loss = (1 - lambda_dssim) * mean|img - gt| + lambda_dssim * (1 - SSIM(img, gt))
 * with the reference's 11x11 Gaussian window (sigma 1.5, zero padding 5, C1 = 0.01^2, C2 = 0.03^2).
 * img, gt: (C,H,W) device float32.  out3 (device, 3 floats) receives {loss, L1, SSIM}; dL_dimg (C,H,W)
 * receives d loss / d img (NULL: value only).  workspace: gsd_l1_ssim_workspace_bytes(C,H,W) bytes of
 * device memory, owned by the caller. */
size_t gsd_l1_ssim_workspace_bytes(int32_t C, int32_t H, int32_t W);
int gsd_l1_ssim(int32_t C, int32_t H, int32_t W, const float* img, const float* gt, float lambda_dssim,
                float* out3, float* dL_dimg, void* workspace, void* stream);

/* Backward of gsd_l1_ssim, split from it so the incoming autograd gradient scales d loss / d img inside the
 * kernel: dL_dimg = sign * grad_out[0] * d out3[0] / d img (grad_out: one device float, NULL => 1).  workspace
 * must hold what gsd_l1_ssim wrote for the same (img, gt, lambda_dssim) (its window adjoints).  sign = -1 turns
 * the loss gradient at lambda_dssim = 1 into the gradient of SSIM itself (utils/loss_utils.py:33 ssim). */
int gsd_l1_ssim_backward(int32_t C, int32_t H, int32_t W, const float* img, const float* gt, float lambda_dssim,
                         const float* grad_out, float sign, float* dL_dimg, const void* workspace, void* stream);

/* Offset-norm regulariser of the training loss (ABI 12; train.py:329-332, added to L1 before the SSIM mix of
 * :529):  out[0] = mean over the P rows of ||offset[g]||_2, i.e. torch.norm(means3D_offset, dim=-1).mean().
 * offset (P,3) contiguous float32; out one device float; workspace gsd_offset_norm_workspace_bytes(P) bytes.
 * The row norms are summed per workgroup and then in a fixed order (deterministic). */
size_t gsd_offset_norm_workspace_bytes(int64_t P);
int gsd_offset_norm(int64_t P, const float* offset, float scale, float* out, void* workspace, void* stream);
/* Backward: d_offset[g] = grad_out[0] * scale * offset[g] / ||offset[g]|| (grad_out: one device float, NULL => 1;
 * scale = the forward's), zero where the norm is zero (torch's norm backward).  d_offset (P,3) is written. */
int gsd_offset_norm_backward(int64_t P, const float* offset, const float* grad_out, float scale, float* d_offset,
                             void* stream);

/* One Adam step (torch.optim.Adam semantics as configured in scene/gaussian_model.py:839-856: per-group
 * learning rate, betas, eps 1e-15, no weight decay / amsgrad) over flat slabs of n floats: param, grad,
 * exp_avg, exp_avg_sq.  Segment g covers elements [group_begin[g], group_begin[g+1]) (group_begin[0] = 0;
 * host arrays, n_groups <= 16) with learning rate group_lr[g] and its own 1-based step count group_step[g]
 * after this update (torch keeps state['step'] per parameter: bias corrections 1 - beta^step).  The betas
 * and eps are the Python doubles: 1 - beta1, 1 - beta2 and the bias corrections are formed in double, as
 * torch forms them, and rounded to float once.  Elements whose parameter had no gradient this step (torch
 * skips grad-None parameters) must be left out of [0, n) by the caller.  zero_grad != 0 also clears the
 * gradient slab.  (ABI 7: per-segment steps, double betas.) */
int gsd_adam_step(int64_t n, float* param, float* grad, float* exp_avg, float* exp_avg_sq, int32_t n_groups,
                  const int64_t* group_begin, const float* group_lr, const int64_t* group_step, double beta1,
                  double beta2, double eps, int32_t zero_grad, void* stream);
/* gsd_adam_step with an addend (ABI 9): elements i in [addend_begin, addend_end) of this call step on
 * grad[i] + addend[i - addend_begin] -- a gradient term that arrives already summed over the data-parallel
 * ranks (gsd_sh_grad_views_ex's d_means) and so must not go through their all-reduce.  addend NULL: as
 * gsd_adam_step. */
int gsd_adam_step_ex(int64_t n, float* param, float* grad, float* exp_avg, float* exp_avg_sq, int32_t n_groups,
                     const int64_t* group_begin, const float* group_lr, const int64_t* group_step, double beta1,
                     double beta2, double eps, int32_t zero_grad, const float* addend, int64_t addend_begin,
                     int64_t addend_end, void* stream);

/* One training step of the reference's loop for one view, as ONE call (ABI 17; no reference counterpart -- the
 * reference's step is train.py:138-683's Python sequence render() -> loss -> backward() -> optimizer.step() ->
 * add_densification_stats, each a pybind / autograd hop):
 *   gsd_rasterize_forward(raster)                       (both phases, one num_rendered read-back)
 *   gsd_l1_ssim + gsd_l1_ssim_backward                  (0.8 L1 + 0.2 (1 - SSIM), train.py:529; d loss / d image
 *                                                        scaled by *grad_seed, NULL = 1)
 *   gsd_rasterize_backward(raster)                      (raster.adam: the Adam step fused where it applies;
 *                                                        dL/dmeans2D and dL/dcolors written, the parameter
 *                                                        gradients to raster.activation / raster.sh_split sinks)
 *   the densification statistics of gsd_densify_stats   (skipped when grad_accum is NULL; folded into the
 *                                                        backward's per-Gaussian pass, which holds dL/dmean2D and
 *                                                        radii in registers -- the same float operations)
 * -- the same kernels with the same arguments as the per-op calls, so the same results.  The raster args serve
 * both passes (the forward ignores the backward-only fields: sinks, adam).  GSD_NEED_BINNING: binning_bytes was
 * short -- phase 1 ran, *num_rendered is set, nothing else was done and no state was modified (the caller grows
 * the buffer to gsd_binning_buffer_bytes(*num_rendered) and calls again).  raster.grad_scratch must equal
 * scratch (the forward zeroes it for the backward). */
typedef struct gsd_train_step_args {
    gsd_raster_args raster;
    void* geom_buffer;          /* gsd_geom_buffer_bytes(P, W, H) */
    void* image_buffer;         /* gsd_image_buffer_bytes(W, H) */
    void* binning_buffer;       /* binning_bytes */
    size_t binning_bytes;
    int32_t* radii;             /* (P) out */
    float* out_color;           /* (3,H,W) out: the rendered image */
    const float* gt;            /* (3,H,W) the view's ground truth */
    float lambda_dssim;
    float* loss_out3;           /* (3) device out: {loss, L1, SSIM} */
    void* loss_workspace;       /* gsd_l1_ssim_workspace_bytes(3, H, W) */
    float* dL_dimg;             /* (3,H,W) device scratch: d loss / d image */
    const float* grad_seed;     /* one device float (autograd's seed gradient), or NULL = 1 */
    float* dL_dmeans2D;         /* (P,3) out: the viewspace_points gradient */
    float* dL_dcolors;          /* (P,3) out */
    void* scratch;              /* gsd_backward_scratch_bytes(P) */
    float* grad_accum;          /* densification statistics (gsd_densify_stats), or NULL: skipped */
    float* grad_accum_3vec;
    float* denom;
    float* max_radii2D;
} gsd_train_step_args;
int gsd_train_step(const gsd_train_step_args* args, int64_t* num_rendered, void* stream);

/* Per-view densification statistics (train.py:613-616, scene/gaussian_model.py:1252-1257): for every
 * Gaussian with radii > 0, max_radii2D = max(max_radii2D, radii); grad_accum_3vec += viewspace_grad;
 * grad_accum += ||viewspace_grad[:2]||; denom += 1.  viewspace_grad (P,3) is dL/d means2D of the view. */
int gsd_densify_stats(int32_t P, const float* viewspace_grad, const int32_t* radii, float* grad_accum,
                      float* grad_accum_3vec, float* denom, float* max_radii2D, void* stream);

/* Initial scales (simple-knn distCUDA2, submodules/simple-knn/simple_knn.cu:165-219, used by
 * create_from_pcd, scene/gaussian_model.py:817): mean_dist2[i] = mean of the squared distances from point i
 * to its 3 nearest other points.  points (P,3); workspace: gsd_knn_workspace_bytes(P) bytes of device memory
 * (256-B aligned). */
size_t gsd_knn_workspace_bytes(int32_t P);
int gsd_knn_mean_dist2(int32_t P, const float* points, float* mean_dist2, void* workspace, void* stream);

/* Deformation network forward on the bf16 matrix cores (ABI 10; gsd_mlp.hip): DirectTemporalNeRF
 * (scene/gaussian_model.py:242-316, the positional encoding :33-82) evaluated as the module does under
 * autocast-bf16, one kernel, every activation in registers.  Replaces the module's forward call
 * (gaussian_model.py:290-316) when no gradient is needed.  x (P,3), t (P) float32; frags:
 * gsd_deform_mlp_fragments() 16-byte A-operand fragments (bf16 weights, K-permuted and fragment-major, packed by
 * gsd_amd.deform_mlp.pack_fused_mlp); bias: gsd_deform_mlp_biases() float32 (bf16-rounded, packed per lane);
 * both 16-B aligned.  Outputs float32 (P,3) / (P,3) / (P,4) / (P,48): dx, d log-scale, d quaternion, dSH. */
int32_t gsd_deform_mlp_fragments(void);
int32_t gsd_deform_mlp_biases(void);
int gsd_deform_mlp_forward_bf16(int32_t P, const float* x, const float* t, const void* frags, const float* bias,
                                float* d_xyz, float* d_scale, float* d_rot, float* d_sh, void* stream);

/* The deformation network's backward between its GEMMs (ABI 11): grad_in = grad_out where out > 0 (ReLU
 * backward, torch.ops.aten.threshold_backward; every element when out is NULL, the heads) and, in the same pass, the
 * bias gradient's column sums per block of rows_per_block rows: bias_partial[(blocks, N)] float32, blocks =
 * gsd_relu_backward_bias_blocks(P, rows_per_block); the caller sums them over the blocks (the bias gradient,
 * gaussian_model.py:242-316 under autograd).  (P, N) row-major, N even and <= 512, float32 (bf16 = 0) or bf16. */
int32_t gsd_relu_backward_bias_blocks(int64_t P, int32_t rows_per_block);
int gsd_relu_backward_bias(int64_t P, int32_t N, int32_t bf16, const void* grad_out, const void* out, void* grad_in,
                           float* bias_partial, int32_t rows_per_block, void* stream);

/* The deformation network's TRAINING path at float32 accuracy (ABI 13; gsd_mlp_train.hip): DirectTemporalNeRF
 * (scene/gaussian_model.py:242-316, positional encoding :33-82) forward and backward as the reference trains it
 * (float32, autograd), on the bf16 matrix cores with every f32 operand split into three bf16 terms and the six
 * leading partial products accumulated in f32 ("BF16x6": f32-level accuracy; gfx950 has no TF32 and its f32 MFMA
 * runs at 1/16 of the bf16 rate).  weights[12] / biases[12]: device float32, the reference's parameters in order
 * _time.0 .. _time.7, _time_out, _time_out_scale, _time_out_rot, _time_out_shs (shapes (256,84), (256,256) x 4,
 * (256,319), (256,256) x 2, (3,256), (3,256), (4,256), (48,256) and their biases).  x (P,3), t (P) float32.
 * out (P,58) = [dx 3 | d log-scale 3 | d quaternion 4 | dSH 48] row-major.  workspace:
 * gsd_deform_mlp_train_workspace_bytes(P) bytes; the forward leaves in it what the backward of the same call
 * reads (the encoding and every hidden activation and, for the backward's dX chain, every layer's gradient,
 * feature-major: ~17 KB per Gaussian).  Replaces the module's forward + autograd backward (torch GEMMs). */
size_t gsd_deform_mlp_train_workspace_bytes(int64_t P);
int gsd_deform_mlp_train_forward(int64_t P, const float* x, const float* t, const float* const* weights,
                                 const float* const* biases, void* workspace, float* out, void* stream);
/* Backward: grad_out (P,58) = dL/d out.  Writes dL/dx (P,3) when dx != NULL and every weight / bias gradient
 * (d_weights[12], d_biases[12], the parameters' shapes; stored, not accumulated).  weights: the forward's. */
int gsd_deform_mlp_train_backward(int64_t P, const float* grad_out, const float* const* weights, void* workspace,
                                  float* dx, float* const* d_weights, float* const* d_biases, void* stream);

/* The same with the four heads as separate row-major outputs (dx (P,3), d log-scale (P,3), d quaternion (P,4),
 * dSH (P,48)) instead of one (P,58) array: what render() consumes, with no split copies. */
int gsd_deform_mlp_train_forward_heads(int64_t P, const float* x, const float* t, const float* const* weights,
                                       const float* const* biases, void* workspace, float* const* heads, void* stream);
/* Backward from the four heads' gradients (grad_heads[4], same shapes; a NULL entry is a zero gradient).  dx: stored,
 * or added to when dx_accumulate != 0; the weight / bias gradients likewise with accumulate != 0 (a parameter's
 * existing .grad as the destination, as autograd's accumulation would leave it). */
int gsd_deform_mlp_train_backward_heads(int64_t P, const float* const* grad_heads, const float* const* weights,
                                        void* workspace, float* dx, int32_t dx_accumulate, float* const* d_weights,
                                        float* const* d_biases, int32_t accumulate, void* stream);

/* ABI 16: the same network's float32 EVALUATION without autograd -- the reference evaluates it under torch.no_grad()
 * when rendering (render.py:46 -> gaussian_renderer/__init__.py:79 -> gaussian_model.py:290-316) -- at the training
 * path's accuracy (BF16x6), in the training forward's layer-fused kernel without its hidden-output and ReLU-word
 * stores.  Same arguments as gsd_deform_mlp_train_forward_heads; workspace: gsd_deform_mlp_eval_workspace_bytes(P)
 * bytes (the packed weights and the encoding, ~0.4 KB per Gaussian), free after the call. */
size_t gsd_deform_mlp_eval_workspace_bytes(int64_t P);
int gsd_deform_mlp_eval_forward_heads(int64_t P, const float* x, const float* t, const float* const* weights,
                                      const float* const* biases, void* workspace, float* const* heads, void* stream);

/* Per-kernel device timing.  While enabled, every kernel this library
 * launches is bracketed by hipEvents on its own stream (a few us of overhead
 * per launch); gsd_timing_collect() synchronises on the last recorded event
 * and writes, for up to max_kernels kernels, the name (NUL-terminated, 32 B
 * per slot), the summed device time in ms and the launch count; it returns
 * the number of kernels written and keeps accumulating.  gsd_timing_reset()
 * clears the totals. */
int gsd_timing_enable(int32_t on);
int gsd_timing_collect(int32_t max_kernels, char* names, double* total_ms, int64_t* launches);
void gsd_timing_reset(void);

/* Work counters of the compositing kernels (the roofline's useful-work figures; no reference counterpart).
 * Counted only by a library built with -DGSD_COUNT_WORK -- otherwise the kernels carry no counting code and
 * every counter reads 0:
 *   [0] render_fwd (wave, record) steps    [1] render_fwd (pixel, record) pairs composited
 *   [2] render_bwd (wave, record) steps    [3] render_bwd (pixel, record) pairs replayed
 * Copies min(n, 4) counters into out after synchronising the device; zeroes them when reset != 0.
 * Returns GSD_OK, or GSD_ERR_ARG for n < 0 or a NULL out with n > 0. */
int gsd_work_counters(int32_t n, uint64_t* out, int32_t reset);

#ifdef __cplusplus
}
#endif
#endif /* GSD_RASTER_H */
