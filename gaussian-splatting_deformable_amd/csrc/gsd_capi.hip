// gsd_capi.hip -- the extern "C" boundary (include/gsd_raster.h).
//
// Orchestration of Rasterizer::forward / ::backward (rasterizer_impl.cu:198-434)
// over caller-owned state buffers.  No device allocation, no hipFree, and one
// host synchronisation per forward (the num_rendered read the reference also
// does, rasterizer_impl.cu:281); everything else is stream-ordered on the
// caller's stream, so one process per GPU can run views back to back.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gsd_raster.h"
#include "gsd_kernels.h"

namespace {

thread_local std::string g_err;
thread_local uint32_t* g_pinned = nullptr;  // 16 B of pinned host memory for the counter read-back
constexpr int kMaxDevices = 64;
thread_local hipEvent_t g_kevent[kMaxDevices] = {};  // per device: "the read-back copy has landed"

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define GSD_HIP(expr)                                                                                    \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) return fail(GSD_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// CHECK_CUDA(..., debug) equivalent (auxiliary.h:166-173)
#define GSD_CHECK(debug, stream)                                                                      \
    do {                                                                                              \
        hipError_t e_ = hipGetLastError();                                                            \
        if (e_ == hipSuccess && (debug)) e_ = hipStreamSynchronize(stream);                           \
        if (e_ != hipSuccess) return fail(GSD_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)

constexpr size_t kAlign = 256;
size_t up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }
char* align_ptr(void* p) { return reinterpret_cast<char*>(up(reinterpret_cast<uintptr_t>(p))); }

struct Geom {
    float2* means2D;
    gsd::RenderRec* rec;
    float* depths;
    int* radii;
    uint8_t* clamped;
    uint32_t* hist;  // LDS-histogram binning workspace [num_blocks][T] + [segments][T]
    uint32_t* part;
    int chunk, num_blocks;
};

bool hist_binning(size_t T) { return T <= (size_t)gsd::kHistMaxTiles; }

void hist_shape(size_t P, int* chunk, int* nblocks) {
    static const size_t target = [] {  // GSD_HIST_BLOCKS: experiment override of kHistTargetBlocks
        const char* e = getenv("GSD_HIST_BLOCKS");
        const int v = e ? atoi(e) : 0;
        return (size_t)(v > 0 ? v : gsd::kHistTargetBlocks);
    }();
    const size_t c = (P + target - 1) / target;
    *chunk = (int)(c < 256 ? 256 : c);
    *nblocks = (int)((P + *chunk - 1) / *chunk);
}
// GeometryState (rasterizer_impl.h:29-41), re-laid out: what render gathers per
// instance (xy, conic/opacity, rgb, and the alpha box) is one 64-B record per
// Gaussian; means2D stays a separate array for the binning; cov3D is recomputed
// in the backward instead of stored; no P-wide scan space is needed.
size_t carve_geom(void* base, size_t P, size_t T, Geom* g) {
    char* p = base ? align_ptr(base) : nullptr;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* r = p ? p + off : nullptr;
        off += up(bytes);
        return r;
    };
    Geom v;
    v.means2D = reinterpret_cast<float2*>(take(P * sizeof(float2)));
    v.rec = reinterpret_cast<gsd::RenderRec*>(take(P * sizeof(gsd::RenderRec)));
    v.depths = reinterpret_cast<float*>(take(P * sizeof(float)));
    v.radii = reinterpret_cast<int*>(take(P * sizeof(int)));
    v.clamped = reinterpret_cast<uint8_t*>(take(P));
    hist_shape(P, &v.chunk, &v.num_blocks);
    const size_t segs = ((size_t)v.num_blocks + gsd::kColSeg - 1) / gsd::kColSeg;
    const bool use_hist = hist_binning(T) && P > 0;
    v.hist = reinterpret_cast<uint32_t*>(take(use_hist ? (size_t)v.num_blocks * T * sizeof(uint32_t) : 0));
    v.part = reinterpret_cast<uint32_t*>(take(use_hist ? segs * T * sizeof(uint32_t) : 0));
    if (g) *g = v;
    return off + kAlign;
}

size_t grid_tiles(int W, int H) {
    return (size_t)((W + gsd::kTileX - 1) / gsd::kTileX) * (size_t)((H + gsd::kTileY - 1) / gsd::kTileY);
}

struct Img {
    float* final_T;
    uint32_t* n_contrib;
    uint2* ranges;
    uint32_t* tile_count;
    uint32_t* tile_cursor;
    uint32_t* counters;
};
size_t carve_img(void* base, size_t npix, size_t T, Img* g) {
    char* p = base ? align_ptr(base) : nullptr;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* r = p ? p + off : nullptr;
        off += up(bytes);
        return r;
    };
    Img v;
    v.final_T = reinterpret_cast<float*>(take(npix * sizeof(float)));
    v.n_contrib = reinterpret_cast<uint32_t*>(take(npix * sizeof(uint32_t)));
    v.ranges = reinterpret_cast<uint2*>(take(T * sizeof(uint2)));
    v.tile_count = reinterpret_cast<uint32_t*>(take(T * sizeof(uint32_t)));
    v.tile_cursor = reinterpret_cast<uint32_t*>(take(T * sizeof(uint32_t)));
    v.counters = reinterpret_cast<uint32_t*>(take(4 * sizeof(uint32_t)));
    if (g) *g = v;
    return off + kAlign;
}

struct Bin {
    unsigned long long* keys;
    unsigned long long* scratch;
    uint32_t* point_list;
};
size_t carve_bin(void* base, size_t K, Bin* g) {
    char* p = base ? align_ptr(base) : nullptr;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* r = p ? p + off : nullptr;
        off += up(bytes);
        return r;
    };
    Bin v;
    // point_list first: the only part the backward reads, so its offset does not depend on K (a forward
    // may carve the buffer by its capacity before K is known, gsd_rasterize_forward)
    v.point_list = reinterpret_cast<uint32_t*>(take(K * 4));
    v.keys = reinterpret_cast<unsigned long long*>(take(K * 8));
    v.scratch = reinterpret_cast<unsigned long long*>(take(K * 8));
    if (g) *g = v;
    return off + kAlign;
}

int grid_x(const gsd_raster_args* a) { return (a->width + gsd::kTileX - 1) / gsd::kTileX; }
int grid_y(const gsd_raster_args* a) { return (a->height + gsd::kTileY - 1) / gsd::kTileY; }

gsd::HistParams hist_params(const gsd_raster_args* a, const Geom& g, int T) {
    gsd::HistParams hp{};
    hp.P = a->P; hp.chunk = g.chunk; hp.num_blocks = g.num_blocks; hp.num_tiles = T;
    hp.grid_x = grid_x(a); hp.grid_y = grid_y(a);
    hp.radii = g.radii; hp.means2D = g.means2D; hp.hist = g.hist; hp.part = g.part;
    return hp;
}

// element strides of the split SH operand (0, 0 = contiguous rows)
template <typename Prm>
void set_sh_strides(Prm& p, const gsd_sh_split* sp, int M) {
    const bool dc_set = sp && (sp->dc_stride_g || sp->dc_stride_e);
    const bool rest_set = sp && (sp->rest_stride_g || sp->rest_stride_e);
    p.dc_sg = dc_set ? sp->dc_stride_g : 3;
    p.dc_se = dc_set ? sp->dc_stride_e : 1;
    p.rest_sg = rest_set ? sp->rest_stride_g : 3LL * (M > 1 ? M - 1 : 0);
    p.rest_se = rest_set ? sp->rest_stride_e : 1;
}

// gsd_adam_epilogue -> the kernels' float coefficients, formed in double as gsd_adam_step forms them; checks
// that every fused sink is one the backward stores into with the layout the fused kernels walk.
gsd::AdamSinkDev adam_sink(const gsd_adam_sink& k, double beta1, double beta2) {
    gsd::AdamSinkDev d{};
    if (!k.param) return d;
    const double bc1 = 1.0 - std::pow(beta1, (double)k.step), bc2 = 1.0 - std::pow(beta2, (double)k.step);
    d.p = k.param; d.m = k.exp_avg; d.v = k.exp_avg_sq;
    d.step_size = (float)((k.lr / bc1) * -1.0);
    d.bc2_sqrt = (float)std::pow(bc2, 0.5);
    return d;
}
int adam_epilogue(const gsd_raster_args* a, const gsd_activation* act, const gsd_adam_epilogue* ad,
                  gsd::AdamEpiDev* out) {
    const gsd_adam_sink* all[6] = {&ad->dc, &ad->rest, &ad->xyz, &ad->scaling, &ad->rotation, &ad->opacity};
    for (const gsd_adam_sink* k : all)
        if (k->param && (!k->exp_avg || !k->exp_avg_sq || k->step < 1))
            return fail(GSD_ERR_ARG, "adam epilogue: a fused sink needs both moments and a step count >= 1");
    const gsd_sh_split* sp = a->sh_split;
    if (ad->dc.param || ad->rest.param) {
        if (!sp || sp->accumulate || sp->d_rgb || a->M != 16 || sp->dc_stride_g || sp->dc_stride_e ||
            sp->rest_stride_g || sp->rest_stride_e)
            return fail(GSD_ERR_ARG, "adam epilogue: the SH pieces need sh_split in store mode (accumulate 0, no "
                                     "d_rgb), M = 16 and contiguous (P,K,3) layouts");
        if ((ad->dc.param && ad->dc.param != sp->dc) || (ad->rest.param && ad->rest.param != sp->rest))
            return fail(GSD_ERR_ARG, "adam epilogue: dc / rest params must be the sh_split pieces themselves");
    }
    if (ad->xyz.param || ad->scaling.param || ad->rotation.param || ad->opacity.param) {
        if (!act || act->accumulate)
            return fail(GSD_ERR_ARG, "adam epilogue: the raw parameters need gsd_activation in store mode");
        if ((ad->xyz.param && ad->xyz.param != a->means3D) || (ad->scaling.param && ad->scaling.param != a->scales) ||
            (ad->rotation.param && ad->rotation.param != a->rotations) ||
            (ad->opacity.param && ad->opacity.param != a->opacities))
            return fail(GSD_ERR_ARG, "adam epilogue: raw params must be the tensors the rasterizer reads");
    }
    out->dc = adam_sink(ad->dc, ad->beta1, ad->beta2);
    out->rest = adam_sink(ad->rest, ad->beta1, ad->beta2);
    out->xyz = adam_sink(ad->xyz, ad->beta1, ad->beta2);
    out->scaling = adam_sink(ad->scaling, ad->beta1, ad->beta2);
    out->rotation = adam_sink(ad->rotation, ad->beta1, ad->beta2);
    out->opacity = adam_sink(ad->opacity, ad->beta1, ad->beta2);
    out->w1 = (float)(1.0 - ad->beta1);
    out->beta2 = (float)ad->beta2;
    out->omb2 = (float)(1.0 - ad->beta2);
    out->eps = (float)ad->eps;
    return GSD_OK;
}

int validate(const gsd_raster_args* a, bool forward) {
    if (!a) return fail(GSD_ERR_ARG, "null gsd_raster_args");
    if (a->P < 0) return fail(GSD_ERR_ARG, "means3D must have dimensions (num_points, 3)");
    if (a->width <= 0 || a->height <= 0) return fail(GSD_ERR_ARG, "image_width and image_height must be positive");
    if (a->P == 0) return GSD_OK;
    if (!a->means3D || (forward && !a->opacities) || !a->viewmatrix || !a->projmatrix || !a->background)
        return fail(GSD_ERR_ARG, "means3D, opacities, viewmatrix, projmatrix and bg are required");
    if (a->shs && a->sh_split) return fail(GSD_ERR_ARG, "shs and sh_split are mutually exclusive");
    const bool have_sh = a->shs || a->sh_split;
    if (have_sh == (a->colors_precomp != nullptr))
        return fail(GSD_ERR_ARG, "Please provide excatly one of either SHs or precomputed colors!");
    if (a->sh_split && (!a->sh_split->dc || (a->M > 1 && !a->sh_split->rest)))
        return fail(GSD_ERR_ARG, "sh_split needs dc, and rest when M > 1");
    if (a->activation && !(a->scales && a->rotations && a->opacities))
        return fail(GSD_ERR_ARG, "activation needs the raw scaling, rotation and opacity");
    const bool have_sr = a->scales && a->rotations;
    if (have_sr == (a->cov3D_precomp != nullptr) || ((a->scales == nullptr) != (a->rotations == nullptr)))
        return fail(GSD_ERR_ARG,
                    "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (have_sh) {
        if (!a->campos) return fail(GSD_ERR_ARG, "campos is required with SHs");
        const int d = a->D < 0 ? 0 : (a->D > 3 ? 3 : a->D);
        if (a->D < 0) return fail(GSD_ERR_ARG, "sh_degree must be >= 0");
        if (a->M < (d + 1) * (d + 1))
            return fail(GSD_ERR_ARG, "sh has fewer coefficients than (sh_degree+1)^2");
    }
    return GSD_OK;
}

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- optional per-kernel device timing (gsd_timing_*) ----
enum KernelId { kPreFwd, kTileHist, kTileScan, kScatter, kTileSort, kRenderFwd, kRenderBwd, kPreBwd, kSe3Fwd,
                kSe3Bwd, kMarkVis, kActFwd, kActBwd, kLoss, kLossBwd, kShViews, kAdam, kDensify, kKnn, kMlp, kMlpBwd,
                kOffNorm, kOffNormBwd, kMlpTrainFwd, kMlpTrainBwd, kNumKernels };
const char* const kKernelNames[kNumKernels] = {"preprocess_fwd", "tile_hist",    "tile_scan",    "scatter_keys",
                                               "tile_sort",      "render_fwd",   "render_bwd",   "preprocess_bwd",
                                               "se3_fwd",        "se3_bwd",      "mark_visible", "activate_fwd",
                                               "activate_bwd",   "l1_ssim",      "l1_ssim_bwd",  "sh_grad_views", "adam",         "densify_stats",
                                               "knn",            "deform_mlp",   "deform_mlp_relu_bias",
                                               "offset_norm",    "offset_norm_bwd", "deform_mlp_train_fwd", "deform_mlp_train_bwd"};
struct TimingState {
    bool on = false;
    struct Rec {
        int id;
        hipEvent_t a, b;
    };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    double total_ms[kNumKernels] = {};
    int64_t launches[kNumKernels] = {};
    std::mutex mu;
};
TimingState g_timing;

hipEvent_t pooled_event() {
    if (!g_timing.pool.empty()) {
        hipEvent_t e = g_timing.pool.back();
        g_timing.pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

template <class F>
void timed(int id, hipStream_t s, F&& launch) {
    if (!g_timing.on) {
        launch();
        return;
    }
    std::lock_guard<std::mutex> lk(g_timing.mu);
    TimingState::Rec r{id, pooled_event(), pooled_event()};
    (void)hipEventRecord(r.a, s);
    launch();
    (void)hipEventRecord(r.b, s);
    g_timing.pending.push_back(r);
}

}  // namespace

extern "C" {

int gsd_abi_version(void) { return GSD_ABI_VERSION; }
const char* gsd_last_error(void) { return g_err.c_str(); }

size_t gsd_geom_buffer_bytes(int32_t P, int32_t width, int32_t height) {
    return carve_geom(nullptr, (size_t)(P < 0 ? 0 : P), grid_tiles(width, height), nullptr);
}
size_t gsd_backward_scratch_bytes(int32_t P) {
    return up(sizeof(float) * gsd::kGradRec * (size_t)(P < 0 ? 0 : P)) + kAlign;
}
size_t gsd_image_buffer_bytes(int32_t width, int32_t height) {
    const size_t gx = (size_t)(width + gsd::kTileX - 1) / gsd::kTileX, gy = (size_t)(height + gsd::kTileY - 1) / gsd::kTileY;
    return carve_img(nullptr, (size_t)width * (size_t)height, gx * gy, nullptr);
}
size_t gsd_binning_buffer_bytes(int64_t K) { return carve_bin(nullptr, (size_t)(K < 0 ? 0 : K), nullptr); }

namespace {
// the largest K whose binning layout fits in `bytes`
int64_t binning_capacity(size_t bytes) {
    int64_t k = (int64_t)(bytes / 20);
    while (k > 0 && gsd_binning_buffer_bytes(k) > bytes) k -= 1 + k / 4096;
    return k;
}
}  // namespace

void gsd_state_layout(int32_t P, int32_t width, int32_t height, int64_t K, size_t* go, size_t* io, size_t* bo) {
    // carve from a fake, 256-aligned base so the returned pointers are the offsets
    char* const base = reinterpret_cast<char*>(uintptr_t(1) << 20);
    auto off = [&](const void* p) { return (size_t)(reinterpret_cast<const char*>(p) - base); };
    const size_t gx = (size_t)(width + gsd::kTileX - 1) / gsd::kTileX, gy = (size_t)(height + gsd::kTileY - 1) / gsd::kTileY;
    Geom g;
    Img im;
    Bin b;
    carve_geom(base, (size_t)(P < 0 ? 0 : P), gx * gy, &g);
    carve_img(base, (size_t)width * (size_t)height, gx * gy, &im);
    carve_bin(base, (size_t)(K < 0 ? 0 : K), &b);
    if (go) {
        // conic + opacity and rgb live in the 64-B render records: offsets of the first record's fields
        go[0] = off(g.means2D); go[1] = off(g.rec) + 8; go[2] = off(g.rec) + 24;
        go[3] = off(g.depths); go[4] = off(g.radii); go[5] = off(g.clamped);
    }
    if (io) {
        io[0] = off(im.final_T); io[1] = off(im.n_contrib); io[2] = off(im.ranges);
        io[3] = off(im.tile_count); io[4] = off(im.tile_cursor); io[5] = off(im.counters);
    }
    if (bo) {
        bo[0] = off(b.keys); bo[1] = off(b.scratch); bo[2] = off(b.point_list);
    }
}

// Phase 1 on the stream: preprocess, tile counts, ranges, and the copy of num_rendered (+ the error flags)
// into pinned host memory, followed by an event the host can wait on (read_back below).  No host wait.
static int enqueue_bin(const gsd_raster_args* a, void* geom_buffer, void* image_buffer, int32_t* radii, hipStream_t s,
                uint32_t** counters_dev, hipEvent_t* done) {
    Geom g;
    Img im;
    const int gx = grid_x(a), gy = grid_y(a), T = gx * gy;
    carve_geom(geom_buffer, a->P, T, &g);
    carve_img(image_buffer, (size_t)a->width * a->height, T, &im);
    const bool use_hist = hist_binning(T);
    if (!use_hist) GSD_HIP(hipMemsetAsync(im.tile_count, 0, sizeof(uint32_t) * T, s));
    // counters[1] collects the prefiltered-culling error flag (set only when prefiltered, forward.cu:174-175);
    // counters[0] is written by the tile scan
    if (a->prefiltered) GSD_HIP(hipMemsetAsync(im.counters, 0, 16, s));

    gsd::PreprocessParams p{};
    p.P = a->P; p.D = a->D; p.M = a->M; p.W = a->width; p.H = a->height; p.grid_x = gx; p.grid_y = gy;
    p.prefiltered = a->prefiltered;
    p.scale_modifier = a->scale_modifier; p.tan_fovx = a->tan_fovx; p.tan_fovy = a->tan_fovy;
    p.focal_y = a->height / (2.0f * a->tan_fovy);  // rasterizer_impl.cu:222-223
    p.focal_x = a->width / (2.0f * a->tan_fovx);
    p.means3D = a->means3D; p.scales = a->scales; p.rotations = a->rotations; p.opacities = a->opacities;
    p.shs = a->shs; p.cov3D_precomp = a->cov3D_precomp; p.colors_precomp = a->colors_precomp;
    if (const gsd_sh_split* sp = a->sh_split) {
        p.sh_dc = sp->dc; p.sh_rest = sp->rest; p.sh_off = sp->offset;
    }
    set_sh_strides(p, a->sh_split, a->M);
    p.view = a->viewmatrix; p.proj = a->projmatrix; p.campos = a->campos;
    p.raw_act = a->activation != nullptr;
    p.radii = radii ? radii : g.radii;
    p.means2D = g.means2D; p.depths = g.depths; p.rec = g.rec;
    p.clamped = g.clamped; p.tile_count = use_hist ? nullptr : im.tile_count; p.err_flags = im.counters + 1;
    timed(kPreFwd, s, [&] { gsd::launch_preprocess_fwd(p, s); });
    GSD_CHECK(a->debug, s);
    if (use_hist) {
        gsd::HistParams hp = hist_params(a, g, T);
        hp.radii = p.radii;
        timed(kTileHist, s, [&] { gsd::launch_tile_hist(hp, im.tile_count, s); });
        GSD_CHECK(a->debug, s);
    }
    timed(kTileScan, s, [&] { gsd::launch_tile_scan(T, im.tile_count, im.ranges, im.tile_cursor, im.counters, s); });
    GSD_CHECK(a->debug, s);
    if (!g_pinned) GSD_HIP(hipHostMalloc(reinterpret_cast<void**>(&g_pinned), 16, hipHostMallocDefault));
    GSD_HIP(hipMemcpyAsync(g_pinned, im.counters, 8, hipMemcpyDeviceToHost, s));
    int dev = 0;
    GSD_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDevices) return fail(GSD_ERR_ARG, "device ordinal out of range");
    if (!g_kevent[dev]) GSD_HIP(hipEventCreateWithFlags(&g_kevent[dev], hipEventDisableTiming));
    GSD_HIP(hipEventRecord(g_kevent[dev], s));
    *counters_dev = im.counters;
    *done = g_kevent[dev];
    return GSD_OK;
}

// Waits for phase 1's read-back (not for anything queued after it) -> *num_rendered; the prefiltered check.
static int read_back(const gsd_raster_args* a, hipEvent_t done, int64_t* num_rendered) {
    GSD_HIP(hipEventSynchronize(done));
    if (a->prefiltered && (g_pinned[1] & gsd::kErrPrefiltered))
        return fail(GSD_ERR_ARG, "Point is filtered although prefiltered is set. This shouldn't happen!");
    *num_rendered = (int64_t)g_pinned[0];
    return GSD_OK;
}

int gsd_rasterize_forward_bin(const gsd_raster_args* a, void* geom_buffer, void* image_buffer, int32_t* radii,
                              int64_t* num_rendered, void* stream) {
    int rc = validate(a, true);
    if (rc) return rc;
    if (!num_rendered) return fail(GSD_ERR_ARG, "num_rendered must not be null");
    *num_rendered = 0;
    if (a->P == 0) return GSD_OK;
    if (!geom_buffer || !image_buffer) return fail(GSD_ERR_STATE, "state buffers must be allocated");
    uint32_t* counters = nullptr;
    hipEvent_t done = nullptr;
    rc = enqueue_bin(a, geom_buffer, image_buffer, radii, as_stream(stream), &counters, &done);
    if (rc) return rc;
    return read_back(a, done, num_rendered);
}

// Phase 2 on the stream.  With k_guard (the device copy of num_rendered) the launches are queued before
// the host knows K: the buffer is carved for K = capacity and every kernel exits when *k_guard > K.
static int enqueue_render(const gsd_raster_args* a, void* geom_buffer, void* image_buffer, void* binning_buffer, int64_t K,
                   const int32_t* radii, float* out_color, hipStream_t s, const uint32_t* k_guard) {
    Geom g;
    Img im;
    Bin b;
    const int gx = grid_x(a), gy = grid_y(a), T = gx * gy;
    carve_geom(geom_buffer, a->P, T, &g);
    carve_img(image_buffer, (size_t)a->width * a->height, T, &im);
    carve_bin(binning_buffer, (size_t)K, &b);
    const uint32_t cap = (uint32_t)std::min<int64_t>(K, UINT32_MAX);
    if (K > 0) {
        if (hist_binning(T)) {
            gsd::HistParams hp = hist_params(a, g, T);
            hp.radii = radii ? radii : g.radii;
            hp.k_guard = k_guard; hp.k_cap = cap;
            timed(kScatter, s, [&] { gsd::launch_scatter_hist(hp, im.tile_cursor, g.depths, b.keys, s); });
        } else {
            gsd::BinParams bp{};
            bp.P = a->P; bp.grid_x = gx; bp.grid_y = gy; bp.num_tiles = T;
            bp.radii = radii ? radii : g.radii;
            bp.means2D = g.means2D; bp.depths = g.depths; bp.tile_cursor = im.tile_cursor; bp.bucket_keys = b.keys;
            bp.k_guard = k_guard; bp.k_cap = cap;
            timed(kScatter, s, [&] { gsd::launch_scatter_keys(bp, s); });
        }
        GSD_CHECK(a->debug, s);
        timed(kTileSort, s,
              [&] { gsd::launch_tile_sort(T, im.ranges, b.keys, b.scratch, b.point_list, s, k_guard, cap); });
        GSD_CHECK(a->debug, s);
    }
    gsd::RenderParams rp{};
    rp.W = a->width; rp.H = a->height; rp.grid_x = gx; rp.num_tiles = T;
    rp.ranges = im.ranges; rp.point_list = b.point_list; rp.rec = g.rec;
    rp.bg = a->background; rp.final_T = im.final_T; rp.n_contrib = im.n_contrib;
    rp.out_color = out_color;
    rp.k_guard = k_guard; rp.k_cap = cap;
    if (a->grad_scratch) {  // the backward's gradient records (gsd_rasterize_backward's scratch layout)
        rp.zero_rec = reinterpret_cast<float4*>(align_ptr(a->grad_scratch));
        rp.zero_n16 = (long long)gsd::kGradRec * a->P / 4;
    }
    timed(kRenderFwd, s, [&] { gsd::launch_render_fwd(rp, s); });
    GSD_CHECK(a->debug, s);
    return GSD_OK;
}

int gsd_rasterize_forward_render(const gsd_raster_args* a, void* geom_buffer, void* image_buffer,
                                 void* binning_buffer, int64_t K, const int32_t* radii, float* out_color,
                                 void* stream) {
    int rc = validate(a, true);
    if (rc) return rc;
    if (a->P == 0) return GSD_OK;
    if (!geom_buffer || !image_buffer || (K > 0 && !binning_buffer) || !out_color)
        return fail(GSD_ERR_STATE, "state buffers / out_color must be allocated");
    return enqueue_render(a, geom_buffer, image_buffer, binning_buffer, K, radii, out_color, as_stream(stream),
                          nullptr);
}

int gsd_rasterize_forward(const gsd_raster_args* a, void* geom_buffer, void* image_buffer, void* binning_buffer,
                          size_t binning_bytes, int32_t* radii, float* out_color, int64_t* num_rendered,
                          void* stream) {
    int rc = validate(a, true);
    if (rc) return rc;
    if (!num_rendered) return fail(GSD_ERR_ARG, "num_rendered must not be null");
    *num_rendered = 0;
    if (a->P == 0) return GSD_OK;
    if (!geom_buffer || !image_buffer || !out_color)
        return fail(GSD_ERR_STATE, "state buffers / out_color must be allocated");
    hipStream_t s = as_stream(stream);
    uint32_t* counters = nullptr;
    hipEvent_t done = nullptr;
    rc = enqueue_bin(a, geom_buffer, image_buffer, radii, s, &counters, &done);
    if (rc) return rc;
    // Phase 2 goes behind phase 1 on the stream before the host waits for num_rendered, so the device never
    // idles on the read-back; its kernels check the device count against what the buffer holds.
    const int64_t cap = binning_buffer ? binning_capacity(binning_bytes) : 0;
    if (cap > 0) {
        rc = enqueue_render(a, geom_buffer, image_buffer, binning_buffer, cap, radii, out_color, s, counters);
        if (rc) return rc;
    }
    rc = read_back(a, done, num_rendered);
    if (rc) return rc;
    if (*num_rendered > cap || (cap == 0 && *num_rendered == 0)) {
        if (*num_rendered == 0)  // nothing to bin: the render phase still writes the background image
            return enqueue_render(a, geom_buffer, image_buffer, binning_buffer, 0, radii, out_color, s, nullptr);
        g_err = "binning buffer too small for num_rendered: allocate gsd_binning_buffer_bytes(num_rendered)";
        return GSD_NEED_BINNING;
    }
    return GSD_OK;
}

int gsd_rasterize_backward(const gsd_raster_args* a, const int32_t* radii, const void* geom_buffer,
                           const void* binning_buffer, const void* image_buffer, int64_t K,
                           const float* dL_dout_color, float* dL_dmeans2D, void* scratch, float* dL_dopacity,
                           float* dL_dcolors, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                           float* dL_dscales, float* dL_drotations, void* stream) {
    int rc = validate(a, false);
    if (rc) return rc;
    if (a->P == 0) return GSD_OK;
    if (!geom_buffer || !image_buffer || (K > 0 && !binning_buffer))
        return fail(GSD_ERR_STATE, "state buffers from the matching forward are required");
    const gsd_activation* act = a->activation;
    if (!dL_dout_color || !dL_dmeans2D || !scratch || (a->cov3D_precomp && !dL_dcov3D))
        return fail(GSD_ERR_ARG, "gradient outputs must be allocated");
    if (!act && (!dL_dopacity || !dL_dcolors || !dL_dmeans3D || (a->scales && (!dL_dscales || !dL_drotations))))
        return fail(GSD_ERR_ARG, "gradient outputs must be allocated");
    if (a->shs && !dL_dsh) return fail(GSD_ERR_ARG, "gradient outputs must be allocated");
    if (act && a->cov3D_precomp) return fail(GSD_ERR_ARG, "activation needs scales/rotations, not cov3D_precomp");
    hipStream_t s = as_stream(stream);
    Geom g;
    Img im;
    Bin b;
    const int gx = grid_x(a), gy = grid_y(a), T = gx * gy;
    carve_geom(const_cast<void*>(geom_buffer), a->P, T, &g);
    carve_img(const_cast<void*>(image_buffer), (size_t)a->width * a->height, T, &im);
    carve_bin(const_cast<void*>(binning_buffer), (size_t)K, &b);

    gsd::RenderBwdParams rp{};
    rp.W = a->width; rp.H = a->height; rp.grid_x = gx; rp.num_tiles = T;
    rp.ranges = im.ranges; rp.point_list = b.point_list; rp.rec = g.rec;
    rp.bg = a->background; rp.final_T = im.final_T; rp.n_contrib = im.n_contrib;
    rp.dL_dpix = dL_dout_color;
    // the per-Gaussian gradient records (scratch) start at zero; render_bwd adds into them.  A scratch the forward
    // was given as args.grad_scratch was zeroed by its compositing kernel (ABI 14)
    float* rec = reinterpret_cast<float*>(align_ptr(scratch));
    rp.grad_rec = rec;
    if (a->grad_scratch != scratch)
        GSD_HIP(hipMemsetAsync(rec, 0, sizeof(float) * gsd::kGradRec * (size_t)a->P, s));
    if (K > 0) {
        timed(kRenderBwd, s, [&] { gsd::launch_render_bwd(rp, s); });
        GSD_CHECK(a->debug, s);
    }
    gsd::PreprocessBwdParams p{};
    p.P = a->P; p.D = a->D; p.M = a->M;
    p.scale_modifier = a->scale_modifier; p.tan_fovx = a->tan_fovx; p.tan_fovy = a->tan_fovy;
    p.focal_y = a->height / (2.0f * a->tan_fovy);
    p.focal_x = a->width / (2.0f * a->tan_fovx);
    p.means3D = a->means3D; p.radii = radii ? radii : g.radii; p.shs = a->shs; p.clamped = g.clamped;
    p.scales = a->scales; p.rotations = a->rotations; p.cov3D_precomp = a->cov3D_precomp;
    p.view = a->viewmatrix; p.proj = a->projmatrix; p.campos = a->campos;
    p.grad_rec = rec; p.dL_dmean2D = dL_dmeans2D; p.dL_dopacity = dL_dopacity; p.dL_dcolor = dL_dcolors;
    p.dL_dmeans3D = dL_dmeans3D; p.dL_dcov3D = dL_dcov3D; p.dL_dsh = dL_dsh; p.dL_dscales = dL_dscales;
    p.dL_drotations = dL_drotations;
    if (const gsd_sh_split* sp = a->sh_split) {
        p.sh_dc = sp->dc; p.sh_rest = sp->rest; p.sh_off = sp->offset;
        p.dL_dsh = nullptr; p.dsh_dc = sp->d_dc; p.dsh_rest = sp->d_rest; p.dsh_off = sp->d_offset;
        p.sh_accumulate = sp->accumulate;
        p.d_rgb = sp->d_rgb;
        p.defer_view_dir = sp->d_rgb && sp->defer_view_dir;
    }
    set_sh_strides(p, a->sh_split, a->M);
    if (act) {
        p.raw_act = 1; p.raw_opacity = a->opacities;
        p.a_xyz = act->d_xyz; p.a_scaling = act->d_scaling; p.a_rotation = act->d_rotation;
        p.a_opacity = act->d_opacity; p.a_accumulate = act->accumulate;
    }
    if (const gsd_adam_epilogue* ad = a->adam) {
        if (int e = adam_epilogue(a, act, ad, &p.adam)) return e;
        p.adam_on = 1;
    }
    timed(kPreBwd, s, [&] { gsd::launch_preprocess_bwd(p, s); });
    GSD_CHECK(a->debug, s);
    return GSD_OK;
}

int gsd_sh_grad_views(int32_t P, int32_t D, int32_t M, int32_t n_views, const float* means3D, const float* views,
                      int64_t view_stride, float* d_dc, float* d_rest, float* d_offset, int32_t accumulate,
                      const gsd_sh_split* layout, const gsd_adam_epilogue* adam, void* stream) {
    return gsd_sh_grad_views_ex(P, D, M, n_views, means3D, views, view_stride, nullptr, nullptr, d_dc, d_rest,
                                d_offset, nullptr, accumulate, layout, adam, stream);
}

int gsd_sh_grad_views_ex(int32_t P, int32_t D, int32_t M, int32_t n_views, const float* means3D, const float* views,
                         int64_t view_stride, const float* sh_dc, const float* sh_rest, float* d_dc, float* d_rest,
                         float* d_offset, float* d_means, int32_t accumulate, const gsd_sh_split* layout,
                         const gsd_adam_epilogue* adam, void* stream) {
    if (P < 0 || n_views < 0 || M < 1 || M < (D + 1) * (D + 1))
        return fail(GSD_ERR_ARG, "sh_grad_views: need P >= 0, n_views >= 0, M >= (D+1)^2");
    if (view_stride < 3 * (int64_t)P + 3) return fail(GSD_ERR_ARG, "sh_grad_views: view_stride < 3 P + 3");
    if (P == 0) return GSD_OK;
    if (!means3D || (n_views > 0 && !views)) return fail(GSD_ERR_ARG, "null pointer argument");
    gsd::ShViewsParams p{};
    p.P = P; p.D = D; p.M = M; p.n_views = n_views; p.view_stride = view_stride;
    p.means3D = means3D; p.views = views; p.d_dc = d_dc; p.d_rest = d_rest; p.d_off = d_offset;
    p.accumulate = accumulate;
    set_sh_strides(p, layout, M);
    if (d_means) {
        const bool contiguous = p.dc_sg == 3 && p.dc_se == 1 && p.rest_sg == 3LL * (M - 1) && p.rest_se == 1;
        if (!sh_dc || !sh_rest || M != 16 || accumulate || !contiguous || d_offset)
            return fail(GSD_ERR_ARG, "sh_grad_views d_means: needs sh_dc and sh_rest, M = 16, accumulate 0, "
                                     "contiguous pieces and no offset sink");
        p.sh_dc = sh_dc; p.sh_rest = sh_rest; p.d_means = d_means;
    }
    if (adam && (adam->dc.param || adam->rest.param)) {
        const bool contiguous = p.dc_sg == 3 && p.dc_se == 1 && p.rest_sg == 3LL * (M - 1) && p.rest_se == 1;
        if (accumulate || M != 16 || !contiguous)
            return fail(GSD_ERR_ARG, "sh_grad_views adam epilogue: needs accumulate 0, M = 16, contiguous pieces");
        for (const gsd_adam_sink* k : {&adam->dc, &adam->rest})
            if (k->param && (!k->exp_avg || !k->exp_avg_sq || k->step < 1))
                return fail(GSD_ERR_ARG, "adam epilogue: a fused sink needs both moments and a step count >= 1");
        p.adam.dc = adam_sink(adam->dc, adam->beta1, adam->beta2);
        p.adam.rest = adam_sink(adam->rest, adam->beta1, adam->beta2);
        p.adam.w1 = (float)(1.0 - adam->beta1);
        p.adam.beta2 = (float)adam->beta2;
        p.adam.omb2 = (float)(1.0 - adam->beta2);
        p.adam.eps = (float)adam->eps;
    }
    hipStream_t s = as_stream(stream);
    timed(kShViews, s, [&] { gsd::launch_sh_grad_views(p, s); });
    GSD_CHECK(false, s);
    return GSD_OK;
}

int gsd_mark_visible(int32_t P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream) {
    (void)projmatrix;  // in_frustum computes the projection but only tests the view-space depth
    if (P < 0) return fail(GSD_ERR_ARG, "means3D must have dimensions (num_points, 3)");
    if (P == 0) return GSD_OK;
    if (!means3D || !viewmatrix || !present) return fail(GSD_ERR_ARG, "null pointer argument");
    timed(kMarkVis, as_stream(stream), [&] { gsd::launch_mark_visible(P, means3D, viewmatrix, present, as_stream(stream)); });
    GSD_CHECK(false, as_stream(stream));
    return GSD_OK;
}

int gsd_se3_deform_forward(int32_t P, const float* twist, const float* means_in, const float* rot_in,
                           float* means_out, float* rot_out, void* stream) {
    if (P < 0) return fail(GSD_ERR_ARG, "twist must have dimensions (num_points, 6)");
    if (P == 0) return GSD_OK;
    if (!twist || !means_in || !means_out || (rot_in && !rot_out)) return fail(GSD_ERR_ARG, "null pointer argument");
    timed(kSe3Fwd, as_stream(stream), [&] { gsd::launch_se3_fwd(P, twist, means_in, rot_in, means_out, rot_out, as_stream(stream)); });
    GSD_CHECK(false, as_stream(stream));
    return GSD_OK;
}

int gsd_se3_deform_backward(int32_t P, const float* twist, const float* means_in, const float* rot_in,
                            const float* dL_dmeans_out, const float* dL_drot_out, float* dL_dtwist,
                            float* dL_dmeans_in, float* dL_drot_in, void* stream) {
    if (P < 0) return fail(GSD_ERR_ARG, "twist must have dimensions (num_points, 6)");
    if (P == 0) return GSD_OK;
    if (!twist || !means_in || !dL_dmeans_out || !dL_dtwist || !dL_dmeans_in ||
        (rot_in && (!dL_drot_out || !dL_drot_in)))
        return fail(GSD_ERR_ARG, "null pointer argument");
    timed(kSe3Bwd, as_stream(stream), [&] {
        gsd::launch_se3_bwd(P, twist, means_in, rot_in, dL_dmeans_out, dL_drot_out, dL_dtwist, dL_dmeans_in,
                            dL_drot_in, as_stream(stream));
    });
    GSD_CHECK(false, as_stream(stream));
    return GSD_OK;
}

int gsd_activate_forward(int32_t P, int32_t R, const float* xyz, const float* dxyz, const float* scaling,
                         const float* dscale, const float* rotation, const float* drot, const float* opacity,
                         const float* f_dc, const float* f_rest, const float* dsh, float* means_out,
                         float* scales_out, float* rot_out, float* opac_out, float* shs_out, void* stream) {
    if (P < 0 || R < 0) return fail(GSD_ERR_ARG, "invalid P / R");
    if (P == 0) return GSD_OK;
    if ((unsigned long long)P * 3ull * (1ull + R) >= (1ull << 32)) return fail(GSD_ERR_ARG, "P too large");
    if (!xyz || !scaling || !rotation || !opacity || !means_out || !scales_out || !rot_out || !opac_out ||
        (shs_out && (!f_dc || (R > 0 && !f_rest))))
        return fail(GSD_ERR_ARG, "null pointer argument");
    gsd::ActivateParams p{};
    p.P = P; p.R = R; p.xyz = xyz; p.dxyz = dxyz; p.scaling = scaling; p.dscale = dscale; p.rotation = rotation;
    p.drot = drot; p.opacity = opacity; p.f_dc = f_dc; p.f_rest = f_rest; p.dsh = dsh; p.means_out = means_out;
    p.scales_out = scales_out; p.rot_out = rot_out; p.opac_out = opac_out; p.shs_out = shs_out;
    hipStream_t s = as_stream(stream);
    timed(kActFwd, s, [&] { gsd::launch_activate_fwd(p, s); });
    GSD_CHECK(false, s);
    return GSD_OK;
}

int gsd_activate_backward(int32_t P, int32_t R, int32_t accumulate, const float* scaling, const float* dscale,
                          const float* rotation, const float* drot, const float* opacity, const float* g_means,
                          const float* g_scales, const float* g_rot, const float* g_opac, const float* g_shs,
                          float* g_xyz, float* g_scaling, float* g_rotation, float* g_opacity, float* g_fdc,
                          float* g_frest, float* g_dxyz, float* g_dscale, float* g_drot, float* g_dsh, void* stream) {
    if (P < 0 || R < 0) return fail(GSD_ERR_ARG, "invalid P / R");
    if (P == 0) return GSD_OK;
    if ((unsigned long long)P * 3ull * (1ull + R) >= (1ull << 32)) return fail(GSD_ERR_ARG, "P too large");
    if (!scaling || !rotation || !opacity || !g_means || !g_scales || !g_rot || !g_opac)
        return fail(GSD_ERR_ARG, "null pointer argument");
    gsd::ActivateBwdParams p{};
    p.P = P; p.R = R; p.accumulate = accumulate; p.scaling = scaling; p.dscale = dscale; p.rotation = rotation;
    p.drot = drot; p.opacity = opacity; p.g_means = g_means; p.g_scales = g_scales; p.g_rot = g_rot;
    p.g_opac = g_opac; p.g_shs = g_shs; p.g_xyz = g_xyz; p.g_scaling = g_scaling; p.g_rotation = g_rotation;
    p.g_opacity = g_opacity; p.g_fdc = g_fdc; p.g_frest = g_frest; p.g_dxyz = g_dxyz; p.g_dscale = g_dscale;
    p.g_drot = g_drot; p.g_dsh = g_dsh;
    hipStream_t s = as_stream(stream);
    timed(kActBwd, s, [&] { gsd::launch_activate_bwd(p, s); });
    GSD_CHECK(false, s);
    return GSD_OK;
}

// ---- training loss (gsd_loss.hip) ----
namespace {
struct LossWs {
    float* gmaps;    // 3 x (C,H,W)
    float* partial;  // 2 per workgroup
    float* out3;     // unused slot (callers pass their own out3)
};
size_t carve_loss(void* base, int C, int H, int W, LossWs* w) {
    char* p = base ? align_ptr(base) : nullptr;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* r = p ? p + off : nullptr;
        off += up(bytes);
        return r;
    };
    int tx, ty;
    gsd::ssim_tiles(H, W, &tx, &ty);
    LossWs v;
    v.gmaps = reinterpret_cast<float*>(take((size_t)3 * C * H * W * sizeof(float)));
    v.partial = reinterpret_cast<float*>(take((size_t)2 * C * tx * ty * sizeof(float)));
    v.out3 = nullptr;
    if (w) *w = v;
    return off + kAlign;
}
}  // namespace

size_t gsd_l1_ssim_workspace_bytes(int32_t C, int32_t H, int32_t W) {
    if (C <= 0 || H <= 0 || W <= 0) return kAlign;
    return carve_loss(nullptr, C, H, W, nullptr);
}

static void ssim_window(float (&w)[11]) {
    // utils/loss_utils.py:23-25: gaussian(11, 1.5), float32 exp values normalised by their float32 sum
    float sum = 0.f;
    for (int k = 0; k < 11; ++k) {
        w[k] = (float)std::exp(-(double)((k - 5) * (k - 5)) / (2.0 * 1.5 * 1.5));
        sum += w[k];
    }
    for (int k = 0; k < 11; ++k) w[k] = w[k] / sum;
}

int gsd_l1_ssim(int32_t C, int32_t H, int32_t W, const float* img, const float* gt, float lambda_dssim, float* out3,
                float* dL_dimg, void* workspace, void* stream) {
    if (C <= 0 || H <= 0 || W <= 0) return fail(GSD_ERR_ARG, "image must be (C,H,W) with positive sizes");
    if (!img || !gt || !out3 || !workspace) return fail(GSD_ERR_ARG, "null pointer argument");
    if ((size_t)C * H * W >= (1ull << 31)) return fail(GSD_ERR_ARG, "image too large");
    float w[11];
    ssim_window(w);
    LossWs ws;
    carve_loss(workspace, C, H, W, &ws);
    hipStream_t s = as_stream(stream);
    timed(kLoss, s, [&] { gsd::launch_l1_ssim(C, H, W, w, lambda_dssim, img, gt, ws.gmaps, ws.partial, out3, dL_dimg, s); });
    GSD_CHECK(false, s);
    return GSD_OK;
}

int gsd_l1_ssim_backward(int32_t C, int32_t H, int32_t W, const float* img, const float* gt, float lambda_dssim,
                         const float* grad_out, float sign, float* dL_dimg, const void* workspace, void* stream) {
    if (C <= 0 || H <= 0 || W <= 0) return fail(GSD_ERR_ARG, "image must be (C,H,W) with positive sizes");
    if (!img || !gt || !dL_dimg || !workspace) return fail(GSD_ERR_ARG, "null pointer argument");
    if ((size_t)C * H * W >= (1ull << 31)) return fail(GSD_ERR_ARG, "image too large");
    float w[11];
    ssim_window(w);
    LossWs ws;
    carve_loss(const_cast<void*>(workspace), C, H, W, &ws);
    hipStream_t s = as_stream(stream);
    timed(kLossBwd, s, [&] {
        gsd::launch_l1_ssim_bwd(C, H, W, w, lambda_dssim, img, gt, ws.gmaps, grad_out, sign, dL_dimg, s);
    });
    GSD_CHECK(false, s);
    return GSD_OK;
}

size_t gsd_offset_norm_workspace_bytes(int64_t P) {
    return P > 0 ? (size_t)gsd::offnorm_blocks(P) * sizeof(float) : sizeof(float);
}

int gsd_offset_norm(int64_t P, const float* offset, float scale, float* out, void* workspace, void* stream) {
    if (P <= 0) return fail(GSD_ERR_ARG, "offset_norm: need P > 0 (the mean of no rows is undefined)");
    if (P >= (1ll << 40)) return fail(GSD_ERR_ARG, "P too large");
    if (!offset || !out || !workspace) return fail(GSD_ERR_ARG, "null pointer argument");
    hipStream_t s = as_stream(stream);
    timed(kOffNorm, s, [&] { gsd::launch_offset_norm(P, offset, scale, static_cast<float*>(workspace), out, s); });
    GSD_CHECK(false, s);
    return GSD_OK;
}

int gsd_offset_norm_backward(int64_t P, const float* offset, const float* grad_out, float scale, float* d_offset,
                             void* stream) {
    if (P < 0) return fail(GSD_ERR_ARG, "invalid P");
    if (P == 0) return GSD_OK;
    if (P >= (1ll << 40)) return fail(GSD_ERR_ARG, "P too large");
    if (!offset || !d_offset) return fail(GSD_ERR_ARG, "null pointer argument");
    hipStream_t s = as_stream(stream);
    timed(kOffNormBwd, s, [&] { gsd::launch_offset_norm_bwd(P, offset, grad_out, scale, d_offset, s); });
    GSD_CHECK(false, s);
    return GSD_OK;
}

int gsd_adam_step(int64_t n, float* param, float* grad, float* exp_avg, float* exp_avg_sq, int32_t n_groups,
                  const int64_t* group_begin, const float* group_lr, const int64_t* group_step, double beta1,
                  double beta2, double eps, int32_t zero_grad, void* stream) {
    return gsd_adam_step_ex(n, param, grad, exp_avg, exp_avg_sq, n_groups, group_begin, group_lr, group_step, beta1,
                            beta2, eps, zero_grad, nullptr, 0, 0, stream);
}

int gsd_adam_step_ex(int64_t n, float* param, float* grad, float* exp_avg, float* exp_avg_sq, int32_t n_groups,
                     const int64_t* group_begin, const float* group_lr, const int64_t* group_step, double beta1,
                     double beta2, double eps, int32_t zero_grad, const float* addend, int64_t addend_begin,
                     int64_t addend_end, void* stream) {
    if (n < 0 || n_groups < 1 || n_groups > gsd::kAdamMaxGroups)
        return fail(GSD_ERR_ARG, "adam: need n >= 0 and 1 <= n_groups <= 16");
    if (addend && (addend_begin < 0 || addend_end < addend_begin || addend_end > n))
        return fail(GSD_ERR_ARG, "adam: need 0 <= addend_begin <= addend_end <= n");
    if (n == 0) return GSD_OK;
    if (!param || !grad || !exp_avg || !exp_avg_sq || !group_begin || !group_lr || !group_step)
        return fail(GSD_ERR_ARG, "null pointer argument");
    gsd::AdamArgs a{};
    a.n = n;
    a.n_groups = n_groups;
    a.zero_grad = zero_grad != 0;
    // torch/optim/adam.py _multi_tensor_adam: bias_correction1 = 1 - beta1 ** step, step_size = -(lr / bc1),
    // bias_correction2_sqrt = bc2 ** 0.5, all Python doubles; the foreach kernels take them as float scalars
    for (int g = 0; g < n_groups; ++g) {
        if (group_begin[g] < (g ? group_begin[g - 1] : 0) || group_begin[g] > n || (g == 0 && group_begin[0] != 0))
            return fail(GSD_ERR_ARG, "adam: group_begin must start at 0 and be non-decreasing");
        if (group_step[g] < 1) return fail(GSD_ERR_ARG, "adam: every step count must be >= 1");
        const double bc1 = 1.0 - std::pow(beta1, (double)group_step[g]);
        const double bc2 = 1.0 - std::pow(beta2, (double)group_step[g]);
        a.begin[g] = group_begin[g];
        a.step_size[g] = (float)(((double)group_lr[g] / bc1) * -1.0);
        a.bc2_sqrt[g] = (float)std::pow(bc2, 0.5);  // bc2 ** 0.5
    }
    a.w1 = (float)(1.0 - beta1);     // _foreach_lerp_(exp_avgs, grads, 1 - beta1)
    a.beta2 = (float)beta2;          // _foreach_mul_(exp_avg_sqs, beta2)
    a.omb2 = (float)(1.0 - beta2);   // _foreach_addcmul_(exp_avg_sqs, grads, grads, 1 - beta2)
    a.eps = (float)eps;
    if (addend && addend_end > addend_begin) {
        a.addend = addend;
        a.addend_lo = addend_begin;
        a.addend_hi = addend_end;
    }
    hipStream_t s = as_stream(stream);
    timed(kAdam, s, [&] { gsd::launch_adam(a, param, grad, exp_avg, exp_avg_sq, s); });
    GSD_CHECK(false, s);
    return GSD_OK;
}

int gsd_densify_stats(int32_t P, const float* viewspace_grad, const int32_t* radii, float* grad_accum,
                      float* grad_accum_3vec, float* denom, float* max_radii2D, void* stream) {
    if (P < 0) return fail(GSD_ERR_ARG, "invalid P");
    if (P == 0) return GSD_OK;
    if (!viewspace_grad || !radii || !grad_accum || !grad_accum_3vec || !denom || !max_radii2D)
        return fail(GSD_ERR_ARG, "null pointer argument");
    hipStream_t s = as_stream(stream);
    timed(kDensify, s, [&] {
        gsd::launch_densify_stats(P, viewspace_grad, radii, grad_accum, grad_accum_3vec, denom, max_radii2D, s);
    });
    GSD_CHECK(false, s);
    return GSD_OK;
}

size_t gsd_knn_workspace_bytes(int32_t P) { return P > 0 ? gsd::knn_workspace(P, nullptr) : kAlign; }

int gsd_knn_mean_dist2(int32_t P, const float* points, float* mean_dist2, void* workspace, void* stream) {
    if (P < 0) return fail(GSD_ERR_ARG, "invalid P");
    if (P == 0) return GSD_OK;
    if (!points || !mean_dist2 || !workspace) return fail(GSD_ERR_ARG, "null pointer argument");
    hipStream_t s = as_stream(stream);
    int e = 0;
    timed(kKnn, s, [&] { e = gsd::launch_knn(P, points, mean_dist2, workspace, s); });
    if (e) return fail(GSD_ERR_HIP, std::string("knn sort: ") + hipGetErrorString((hipError_t)e));
    GSD_CHECK(false, s);
    return GSD_OK;
}

int32_t gsd_deform_mlp_fragments(void) { return gsd::kMlpFrags; }
int32_t gsd_deform_mlp_biases(void) { return gsd::kMlpBias; }

int gsd_deform_mlp_forward_bf16(int32_t P, const float* x, const float* t, const void* frags, const float* bias,
                                float* d_xyz, float* d_scale, float* d_rot, float* d_sh, void* stream) {
    if (P < 0) return fail(GSD_ERR_ARG, "invalid P");
    if (P == 0) return GSD_OK;
    if (!x || !t || !frags || !bias || !d_xyz || !d_scale || !d_rot || !d_sh)
        return fail(GSD_ERR_ARG, "null pointer argument");
    if ((reinterpret_cast<uintptr_t>(frags) | reinterpret_cast<uintptr_t>(bias)) & 15)
        return fail(GSD_ERR_ARG, "deform_mlp: frags and bias must be 16-B aligned");
    gsd::MlpParams p{P, x, t, frags, bias, d_xyz, d_scale, d_rot, d_sh};
    hipStream_t s = as_stream(stream);
    timed(kMlp, s, [&] { gsd::launch_mlp_fwd(p, s); });
    GSD_CHECK(false, s);
    return GSD_OK;
}

int32_t gsd_relu_backward_bias_blocks(int64_t P, int32_t rows_per_block) {
    return (P < 0 || rows_per_block <= 0) ? 0 : gsd::relu_bwd_bias_blocks(P, rows_per_block);
}

int gsd_relu_backward_bias(int64_t P, int32_t N, int32_t bf16, const void* grad_out, const void* out, void* grad_in,
                           float* bias_partial, int32_t rows_per_block, void* stream) {
    if (P < 0 || N <= 0 || (N & 1) || N > 512 || rows_per_block <= 0)
        return fail(GSD_ERR_ARG, "relu_backward_bias: need P >= 0, even 0 < N <= 512, rows_per_block > 0");
    if (P == 0) return GSD_OK;
    if (!grad_out || !grad_in || !bias_partial) return fail(GSD_ERR_ARG, "null pointer argument");
    hipStream_t s = as_stream(stream);
    timed(kMlpBwd, s, [&] {
        gsd::launch_relu_bwd_bias(P, N, bf16, grad_out, out, grad_in, bias_partial, rows_per_block, s);
    });
    GSD_CHECK(false, s);
    return GSD_OK;
}

// ---- the deformation network's f32-accurate training path (gsd_mlp_train.hip) ----
}  // extern "C"
namespace {
// padded input / output widths of the nine layers (8 hidden + the heads) and the reference's weight widths
constexpr int kMlpIn[9] = {96, 256, 256, 256, 256, 320, 256, 256, 256};
constexpr int kMlpOut[9] = {256, 256, 256, 256, 256, 256, 256, 256, 64};
constexpr int kMlpLdw[9] = {84, 256, 256, 256, 256, 319, 256, 256, 256};
constexpr int kMlpMap[9] = {1, 0, 0, 0, 0, 2, 0, 0, 0};
constexpr int kMlpChunk = 2048;   // Gaussians per wave of the weight-gradient kernel

size_t mlp_frag_bytes(int M, int K) { return (size_t)(K / 16) * (M / 32) * 3 * 64 * 16; }

struct MlpWs {
    int64_t ldp;
    void* ffrag[9];   // forward A = W
    void* bfrag[9];   // backward A = W^T
    void* cfrag[8];   // the backward chain's W^T in the accumulator k order: layers 1-7 (layer 5: rows 64-319), [0]: W0^T's enc(x) rows
    void* cfrag_e5;   // W5^T's enc(x) rows, accumulator k order
    float* bias_heads;
    float *E, *ET, *H[9];   // H[1..8]: the hidden layers' outputs
    float *Gh, *ga, *gb, *dE;
    float* G[9];      // the backward chain's gradients: G[0] = g8 (Gh), G[i] = g_{8-i} (G[1], G[2] = ga, gb)
    float *partial, *bias_partial;
    unsigned short* bits[9];   // bits[1..8]: the ReLU masks of H[1..8] (16 row blocks x 2 halves x ldp words)
};
size_t carve_mlp(void* base, int64_t P, MlpWs* w) {
    char* p = base ? align_ptr(base) : nullptr;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* r = p ? p + off : nullptr;
        off += up(bytes);
        return r;
    };
    MlpWs v{};
    v.ldp = (P + 255) / 256 * 256;
    const size_t row = sizeof(float) * (size_t)v.ldp;
    for (int l = 0; l < 9; ++l) v.ffrag[l] = take(mlp_frag_bytes(kMlpOut[l], kMlpIn[l]));
    for (int l = 0; l < 9; ++l) v.bfrag[l] = take(mlp_frag_bytes(kMlpIn[l], kMlpOut[l]));
    for (int l = 0; l < 8; ++l) v.cfrag[l] = take(mlp_frag_bytes(l == 0 ? 64 : 256, 256));
    v.cfrag_e5 = take(mlp_frag_bytes(64, 256));
    v.bias_heads = reinterpret_cast<float*>(take(64 * sizeof(float)));
    v.E = reinterpret_cast<float*>(take(64 * row));
    v.ET = reinterpret_cast<float*>(take(32 * row));
    v.H[0] = nullptr;
    for (int l = 1; l <= 8; ++l) v.H[l] = reinterpret_cast<float*>(take(256 * row));
    v.Gh = reinterpret_cast<float*>(take(64 * row));
    v.ga = reinterpret_cast<float*>(take(256 * row));
    v.gb = reinterpret_cast<float*>(take(256 * row));
    v.dE = reinterpret_cast<float*>(take(64 * row));
    v.G[0] = v.Gh;
    v.G[1] = v.ga;
    v.G[2] = v.gb;
    for (int i = 3; i < 9; ++i) v.G[i] = reinterpret_cast<float*>(take(256 * row));
    const int64_t chunks = (P + kMlpChunk - 1) / kMlpChunk;
    v.partial = reinterpret_cast<float*>(take(sizeof(float) * (size_t)chunks * 256 * 320));
    v.bias_partial = reinterpret_cast<float*>(take(sizeof(float) * (size_t)chunks * 256));
    v.bits[0] = nullptr;
    for (int l = 1; l <= 8; ++l) v.bits[l] = reinterpret_cast<unsigned short*>(take(2 * 16 * sizeof(short) * (size_t)v.ldp));
    if (w) *w = v;
    return off + kAlign;
}

gsd::MlpWeightRef mlp_weight(int l, float* const* w, int ldw_override = -1) {
    gsd::MlpWeightRef r{};
    if (l < 8) {
        r.W[0] = w[l];
        r.row_off[0] = 0;
        r.row_off[1] = 256;
        r.n_pieces = 1;
    } else {   // the heads: dx 3 | d log-scale 3 | d quaternion 4 | dSH 48
        const int off[5] = {0, 3, 6, 10, 58};
        for (int i = 0; i < 4; ++i) r.W[i] = w[8 + i];
        for (int i = 0; i < 5; ++i) r.row_off[i] = off[i];
        r.n_pieces = 4;
    }
    r.ldw = ldw_override >= 0 ? ldw_override : kMlpLdw[l];
    r.map = ldw_override >= 0 ? 0 : kMlpMap[l];
    return r;
}

// fused: the forward's weights for k_mlp_fwd_fused, whose B operands past the encoding are the layer before's
// accumulators (the accumulator-order k permutation: layer 0 none, layer 5 from k-step 4, the rest from 0)
void mlp_pack_all(float* const* weights, const MlpWs& ws, bool backward, bool fused, hipStream_t s) {
    gsd::MlpPackBatch b{};
    for (int l = 0; l < 9; ++l) {
        gsd::MlpPackParams& pp = b.job[b.n++];
        pp.perm_from = !fused || l == 0 ? 1 << 30 : (l == 5 ? 4 : 0);
        pp.w = mlp_weight(l, weights);
        pp.transpose = backward ? 1 : 0;
        pp.M = backward ? kMlpIn[l] : kMlpOut[l];
        pp.K = backward ? kMlpOut[l] : kMlpIn[l];
        pp.out = backward ? ws.bfrag[l] : ws.ffrag[l];
    }
    gsd::launch_mlp_pack_batch(b, s);
}
// the backward chain's W^T packs (k_mlp_bwd_chain) and the natural-order W8^T of its first step
void mlp_pack_chain(float* const* weights, const MlpWs& ws, hipStream_t s) {
    gsd::MlpPackBatch b{};
    for (int l = 0; l < 8; ++l) {
        gsd::MlpPackParams& pp = b.job[b.n++];
        pp.w = mlp_weight(l, weights);
        pp.transpose = 1;
        pp.perm_from = 0;
        pp.M = l == 0 ? 64 : 256;
        pp.m_off = l == 5 ? 64 : 0;
        pp.K = 256;
        pp.out = ws.cfrag[l];
    }
    {   // W5^T's enc(x) rows for the chain's layer-5 pass
        gsd::MlpPackParams& pp = b.job[b.n++];
        pp.w = mlp_weight(5, weights);
        pp.transpose = 1;
        pp.perm_from = 0;
        pp.M = 64;
        pp.K = 256;
        pp.out = ws.cfrag_e5;
    }
    for (int l : {8}) {
        gsd::MlpPackParams& pp = b.job[b.n++];
        pp.perm_from = 1 << 30;
        pp.w = mlp_weight(l, weights);
        pp.transpose = 1;
        pp.M = kMlpIn[l];
        pp.K = kMlpOut[l];
        pp.out = ws.bfrag[l];
    }
    gsd::launch_mlp_pack_batch(b, s);
}
}  // namespace
extern "C" {

size_t gsd_deform_mlp_train_workspace_bytes(int64_t P) { return P > 0 ? carve_mlp(nullptr, P, nullptr) : kAlign; }

static gsd::MlpHeads heads_of(float* out) {   // the (P, 58) layout of the heads as four views
    gsd::MlpHeads h{};
    for (int k = 0; k < 4; ++k) {
        h.out[k] = out + gsd::kMlpHeadCol[k];
        h.ld[k] = 58;
    }
    return h;
}

static int mlp_train_forward(int64_t P, const float* x, const float* t, const float* const* weights,
                             const float* const* biases, void* workspace, const gsd::MlpHeads& heads, void* stream);

int gsd_deform_mlp_train_forward(int64_t P, const float* x, const float* t, const float* const* weights,
                                 const float* const* biases, void* workspace, float* out, void* stream) {
    if (!out) return fail(GSD_ERR_ARG, "null pointer argument");
    return mlp_train_forward(P, x, t, weights, biases, workspace, heads_of(out), stream);
}

int gsd_deform_mlp_train_forward_heads(int64_t P, const float* x, const float* t, const float* const* weights,
                                       const float* const* biases, void* workspace, float* const* heads, void* stream) {
    if (!heads) return fail(GSD_ERR_ARG, "null pointer argument");
    gsd::MlpHeads h{};
    for (int k = 0; k < 4; ++k) {
        if (!heads[k]) return fail(GSD_ERR_ARG, "deform_mlp_train: 4 head outputs needed");
        h.out[k] = heads[k];
        h.ld[k] = gsd::kMlpHeadCol[k + 1] - gsd::kMlpHeadCol[k];
    }
    return mlp_train_forward(P, x, t, weights, biases, workspace, h, stream);
}

static int mlp_train_forward(int64_t P, const float* x, const float* t, const float* const* weights,
                             const float* const* biases, void* workspace, const gsd::MlpHeads& heads, void* stream) {
    if (P <= 0 || P >= (1ll << 31) - 256) return fail(GSD_ERR_ARG, "deform_mlp_train: need 0 < P < 2^31 - 256");
    if (!x || !t || !weights || !biases || !workspace) return fail(GSD_ERR_ARG, "null pointer argument");
    for (int i = 0; i < 12; ++i)
        if (!weights[i] || !biases[i]) return fail(GSD_ERR_ARG, "deform_mlp_train: 12 weights and 12 biases needed");
    MlpWs ws;
    carve_mlp(workspace, P, &ws);
    hipStream_t s = as_stream(stream);
    float* const* W = const_cast<float* const*>(weights);
    float* const* B = const_cast<float* const*>(biases);
    // GSD_MLP_FWD=gemm: the layer-by-layer GEMMs (k_mlp_gemm_dma) instead of the layer-fused kernel, for comparison
    static const bool fused = [] {
        const char* e = getenv("GSD_MLP_FWD");
        return !(e && strcmp(e, "gemm") == 0);
    }();
    timed(kMlpTrainFwd, s, [&] {
        mlp_pack_all(W, ws, false, fused, s);
        gsd::launch_mlp_gather_bias(mlp_weight(8, B, 1), ws.bias_heads, 64, s);
        gsd::launch_mlp_encode((int)P, (int)ws.ldp, x, t, ws.E, ws.ET, s);
        if (fused) {
            gsd::MlpFusedParams f{};
            f.P = (int)P;
            f.ldp = (int)ws.ldp;
            f.E = ws.E;
            f.ET = ws.ET;
            for (int l = 0; l < 9; ++l) f.frags[l] = ws.ffrag[l];
            for (int l = 0; l < 8; ++l) {
                f.bias[l] = B[l];
                f.H[l] = ws.H[l + 1];
                f.bits[l] = ws.bits[l + 1];
            }
            f.bias_heads = ws.bias_heads;
            f.heads = heads;
            gsd::launch_mlp_fwd_fused(f, s);
            return;
        }
        for (int l = 0; l < 9; ++l) {
            gsd::MlpGemmParams g{};
            g.P = (int)P;
            g.ldp = (int)ws.ldp;
            g.frags = ws.ffrag[l];
            g.rb = kMlpOut[l] / 32;
            if (l == 0) {
                g.src0 = ws.E; g.ks0 = 4; g.src1 = ws.ET; g.ks1 = 2;
            } else if (l == 5) {
                g.src0 = ws.E; g.ks0 = 4; g.src1 = ws.H[5]; g.ks1 = 16;
            } else {
                g.src0 = ws.H[l]; g.ks0 = 16;
            }
            if (l < 8) {
                g.bias = B[l];
                g.dst = ws.H[l + 1];
                g.mask_out = ws.bits[l + 1];
                gsd::launch_mlp_gemm(g, gsd::kMlpFwdRelu, s);
            } else {
                g.bias = ws.bias_heads;
                g.heads = heads;
                gsd::launch_mlp_gemm(g, gsd::kMlpFwdHeads, s);
            }
        }
    });
    GSD_CHECK(false, s);
    return GSD_OK;
}

static int mlp_train_backward(int64_t P, const gsd::MlpHeadsIn& gin, const float* const* weights, void* workspace,
                              float* dx, int dx_accumulate, float* const* d_weights, float* const* d_biases,
                              int accumulate, void* stream);

int gsd_deform_mlp_train_backward(int64_t P, const float* grad_out, const float* const* weights, void* workspace,
                                  float* dx, float* const* d_weights, float* const* d_biases, void* stream) {
    if (!grad_out) return fail(GSD_ERR_ARG, "null pointer argument");
    gsd::MlpHeadsIn g{};
    for (int k = 0; k < 4; ++k) {
        g.src[k] = grad_out + gsd::kMlpHeadCol[k];
        g.ld[k] = 58;
    }
    return mlp_train_backward(P, g, weights, workspace, dx, 0, d_weights, d_biases, 0, stream);
}

int gsd_deform_mlp_train_backward_heads(int64_t P, const float* const* grad_heads, const float* const* weights,
                                        void* workspace, float* dx, int32_t dx_accumulate, float* const* d_weights,
                                        float* const* d_biases, int32_t accumulate, void* stream) {
    if (!grad_heads) return fail(GSD_ERR_ARG, "null pointer argument");
    gsd::MlpHeadsIn g{};
    for (int k = 0; k < 4; ++k) {
        g.src[k] = grad_heads[k];   // NULL: a zero gradient
        g.ld[k] = gsd::kMlpHeadCol[k + 1] - gsd::kMlpHeadCol[k];
    }
    return mlp_train_backward(P, g, weights, workspace, dx, dx_accumulate, d_weights, d_biases, accumulate, stream);
}

static int mlp_train_backward(int64_t P, const gsd::MlpHeadsIn& gin, const float* const* weights, void* workspace,
                              float* dx, int dx_accumulate, float* const* d_weights, float* const* d_biases,
                              int accumulate, void* stream) {
    if (P <= 0 || P >= (1ll << 31) - 256) return fail(GSD_ERR_ARG, "deform_mlp_train: need 0 < P < 2^31 - 256");
    if (!weights || !workspace || !d_weights || !d_biases) return fail(GSD_ERR_ARG, "null pointer argument");
    for (int i = 0; i < 12; ++i)
        if (!weights[i] || !d_weights[i] || !d_biases[i])
            return fail(GSD_ERR_ARG, "deform_mlp_train: 12 weights and 12 weight / bias gradients needed");
    MlpWs ws;
    carve_mlp(workspace, P, &ws);
    hipStream_t s = as_stream(stream);
    float* const* W = const_cast<float* const*>(weights);
    const int ldp = (int)ws.ldp;
    const int chunks = (int)((P + kMlpChunk - 1) / kMlpChunk);
    auto wgrad = [&](int l, const float* G, int n_rb, const float* X0, const float* X1, int k_rb, int k_rb0,
                     int k_off = 0, int skip_bias = 0) {
        gsd::MlpWgradParams q{};
        q.P = (int)P; q.ldp = ldp; q.G = G; q.n_rb = n_rb; q.X0 = X0; q.X1 = X1; q.k_rb = k_rb; q.k_rb0 = k_rb0;
        q.k_off = k_off; q.accumulate = accumulate; q.skip_bias = skip_bias;
        q.tiles_n = (n_rb + 3) / 4; q.tiles_k = (k_rb + 3) / 4; q.chunk = kMlpChunk;
        q.partial = ws.partial; q.bias_partial = ws.bias_partial;
        gsd::launch_mlp_wgrad(q, mlp_weight(l, d_weights), mlp_weight(l, d_biases, 1), s);
    };
    auto dgemm = [&](int l, const float* G, int ks, int mask_layer, float* dst, int n_a, int acc_a) {
        gsd::MlpGemmParams g{};
        g.P = (int)P; g.ldp = ldp; g.src0 = G; g.ks0 = ks; g.frags = ws.bfrag[l]; g.rb = kMlpIn[l] / 32;
        g.mask = mask_layer > 0 ? ws.H[mask_layer] : nullptr;
        g.mask_in = mask_layer > 0 ? ws.bits[mask_layer] : nullptr;   // the forward's ReLU bits of that layer
        g.dst = dst; g.n_a = n_a; g.dst_a = ws.dE; g.accumulate_a = acc_a;
        gsd::launch_mlp_gemm(g, gsd::kMlpBwdMask, s);
    };
    (void)chunks;
    // GSD_MLP_BWD=gemm: the layer-by-layer dX GEMMs (k_mlp_gemm_dma) instead of the fused chain, for comparison
    static const bool chain = [] {
        const char* e = getenv("GSD_MLP_BWD");
        return !(e && strcmp(e, "gemm") == 0);
    }();
    if (chain) {
        timed(kMlpTrainBwd, s, [&] {
            mlp_pack_chain(W, ws, s);
            gsd::MlpChainParams c{};
            c.P = (int)P;
            c.ldp = ldp;
            c.heads = gin;
            c.frags[0] = ws.bfrag[8];
            for (int i = 1; i < 8; ++i) c.frags[i] = ws.cfrag[8 - i];
            c.frags_e = ws.cfrag[0];
            c.frags_e5 = ws.cfrag_e5;
            for (int i = 0; i < 8; ++i) c.bits[i] = ws.bits[8 - i];
            for (int i = 0; i < 9; ++i) c.G[i] = ws.G[i];
            c.dE = ws.dE;
            gsd::launch_mlp_bwd_chain(c, s);
            if (dx) gsd::launch_mlp_encode_bwd((int)P, ldp, ws.E, ws.dE, dx, dx_accumulate, s);
            wgrad(8, ws.G[0], 2, ws.H[8], nullptr, 8, 8);
            for (int l = 7; l >= 0; --l) {
                const float* g = ws.G[8 - l];
                if (l == 0) wgrad(0, g, 8, ws.E, ws.ET, 3, 2);
                else if (l == 5) {
                    wgrad(5, g, 8, ws.E, nullptr, 2, 2, 0);
                    wgrad(5, g, 8, ws.H[5], nullptr, 8, 8, 64, 1);
                } else wgrad(l, g, 8, ws.H[l], nullptr, 8, 8);
            }
        });
        GSD_CHECK(false, s);
        return GSD_OK;
    }
    timed(kMlpTrainBwd, s, [&] {
        mlp_pack_all(W, ws, true, false, s);
        gsd::launch_mlp_rows_to_features((int)P, ldp, gin, ws.Gh, 64, s);
        wgrad(8, ws.Gh, 2, ws.H[8], nullptr, 8, 8);
        dgemm(8, ws.Gh, 4, 8, ws.ga, 0, 0);   // g of layer 7's pre-activation
        float* g = ws.ga;
        float* other = ws.gb;
        for (int l = 7; l >= 0; --l) {
            if (l == 0) wgrad(0, g, 8, ws.E, ws.ET, 3, 2);
            else if (l == 5) {   // columns 0-63 (enc(x)) and 64-319 (h5) as two calls (both bias gradients equal)
                wgrad(5, g, 8, ws.E, nullptr, 2, 2, 0);
                wgrad(5, g, 8, ws.H[5], nullptr, 8, 8, 64, 1);
            }
            else wgrad(l, g, 8, ws.H[l], nullptr, 8, 8);
            if (l == 5) dgemm(5, g, 16, 5, other, 64, 0);   // rows 0-63: d enc(x); the rest masked by h5
            else if (l > 0) dgemm(l, g, 16, l, other, 0, 0);
            else if (dx) dgemm(0, g, 16, 0, nullptr, 64, 1);   // d enc(x) += W0^T g (the t rows dropped)
            float* tmp = g;
            g = other;
            other = tmp;
        }
        if (dx) gsd::launch_mlp_encode_bwd((int)P, ldp, ws.E, ws.dE, dx, dx_accumulate, s);
    });
    GSD_CHECK(false, s);
    return GSD_OK;
}

int gsd_timing_enable(int32_t on) {
    std::lock_guard<std::mutex> lk(g_timing.mu);
    g_timing.on = on != 0;
    return GSD_OK;
}

int gsd_timing_collect(int32_t max_kernels, char* names, double* total_ms, int64_t* launches) {
    std::lock_guard<std::mutex> lk(g_timing.mu);
    for (const auto& r : g_timing.pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            g_timing.total_ms[r.id] += ms;
            g_timing.launches[r.id] += 1;
        }
        g_timing.pool.push_back(r.a);
        g_timing.pool.push_back(r.b);
    }
    g_timing.pending.clear();
    int n = 0;
    for (int k = 0; k < kNumKernels && n < max_kernels; ++k) {
        if (!g_timing.launches[k]) continue;
        if (names) {
            std::strncpy(names + 32 * n, kKernelNames[k], 31);
            names[32 * n + 31] = 0;
        }
        if (total_ms) total_ms[n] = g_timing.total_ms[k];
        if (launches) launches[n] = g_timing.launches[k];
        ++n;
    }
    return n;
}

void gsd_timing_reset(void) {
    std::lock_guard<std::mutex> lk(g_timing.mu);
    for (int k = 0; k < kNumKernels; ++k) {
        g_timing.total_ms[k] = 0;
        g_timing.launches[k] = 0;
    }
}

}  // extern "C"
