// gsd_loss.hip -- the training loss of one view, fused: (1-l) L1 + l (1 - SSIM), value and dL/dimage.
//
// Reference: utils/loss_utils.py:17-63 (l1_loss, ssim with an 11x11 sigma 1.5 Gaussian window, zero
// padding 5, C1 = 0.01^2, C2 = 0.03^2, mean over C*H*W) combined as in train.py:529 with
// lambda_dssim = 0.2 (arguments/__init__.py:83).  torch evaluates it as 5 grouped conv2d + ~20
// elementwise kernels forward and as many again backward.  Here:
//
//   k_ssim_fwd   one workgroup per (32x32 tile, channel): x, y and a 5-px halo staged in LDS, the five
//                window sums A = w*x, B = w*y, C = w*x^2, D = w*y^2, E = w*xy by a separable
//                11-tap pass (horizontal into LDS, then vertical), the SSIM map f, and the three
//                per-pixel adjoints df/dA, df/dC, df/dE (scaled by -l/N) written to HBM;
//                per-workgroup partial sums of f and |x - y| (deterministic, no float atomics).
//   k_ssim_bwd   dL/dx = w * gA + 2x (w * gC) + y (w * gE) + (1-l)/N sign(x - y), the same
//                separable window (it is symmetric, so the transposed correlation is itself).
//   k_loss_sum   sums the partials in a fixed order -> loss, L1, SSIM (device scalars).
//
// dA/dx etc.: sigma1 = C - A^2, sigma12 = E - AB, f = (2AB + C1)(2 sigma12 + C2) /
// ((A^2 + B^2 + C1)(sigma1 + sigma2 + C2)); with n1, n2, d1, d2 the four factors and D = d1 d2:
//   df/dA = (2B (n2 - n1) - 2A f (d2 - d1)) / D,  df/dC = -f / d2,  df/dE = 2 n1 / D
// (quotient-rule form: no division by n2, which can vanish).  HBM per pixel and channel: forward
// reads 8 B and writes 12 B, backward reads 20 B and writes 4 B.
#include "gsd_kernels.h"

// the loss has no bit-exact contract: multiply-adds fuse to (packed) FMA
#pragma clang fp contract(fast)

namespace gsd {

constexpr int kSsimTile = 32;                        // output tile edge
constexpr int kSsimHalo = 5;                         // window radius
constexpr int kSsimIn = kSsimTile + 2 * kSsimHalo;   // 42: staged edge
constexpr int kSsimThreads = 256;
constexpr int kSsimRows = kSsimTile * kSsimTile / kSsimThreads;  // 4 output rows per thread (one column)
#ifndef GSD_SSIM_FWD_THREADS
// k_ssim_fwd's workgroup size: 512 threads, two output rows each (54 VGPRs, six waves per SIMD) -- 50.3 us at
// 1080p against 54.2 for 256 threads with four rows each (146 VGPRs, three waves); profiles/round4/r4k3/
#define GSD_SSIM_FWD_THREADS 512
#endif
constexpr int kSsimFwdThreads = GSD_SSIM_FWD_THREADS;
constexpr int kSsimFwdRows = kSsimTile * kSsimTile / kSsimFwdThreads;

// 1/d from v_rcp_f32 plus one Newton step (the loss has no bit-exact contract)
__device__ __forceinline__ float fast_rcp(float d) {
    const float r = __builtin_amdgcn_rcpf(d);
    return fmaf(fmaf(-d, r, 1.0f), r, r);
}

typedef float f2 __attribute__((ext_vector_type(2)));

struct SsimArgs {
    int C, H, W, tiles_x, tiles_y;
    float w[11];        // 1-D window (the 2-D window is its outer product)
    float wp[24];       // (w[m], w[m-1]) for m = 0..11, zero outside 0..10: two output rows per packed FMA
    float coef_ssim;    // -lambda / N
    float coef_l1;      // (1 - lambda) / N
};

// Stage a 42x42 window of one channel of `a` around the tile, zero outside the image.  Fixed trip
// counts, fully unrolled: all 12 loads of a thread are in flight before the first LDS store.
template <int RS = kSsimIn>
__device__ __forceinline__ void stage(const float* __restrict__ a, float (*sa)[RS], int H, int W, int ox,
                                      int oy) {
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    constexpr int kRowIt = (kSsimIn + 7) / 8, kColIt = 2;  // 6 x 2 slots of a 8 x 32 thread grid
    float v[kRowIt][kColIt];
#pragma unroll
    for (int i = 0; i < kRowIt; ++i) {
        const int r = ty + 8 * i, gy = oy - kSsimHalo + r;
#pragma unroll
        for (int j = 0; j < kColIt; ++j) {
            const int c = tx + 32 * j, gx = ox - kSsimHalo + c;
            const bool ok = r < kSsimIn && c < kSsimIn && gy >= 0 && gy < H && gx >= 0 && gx < W;
            v[i][j] = ok ? a[(size_t)gy * W + gx] : 0.f;
        }
    }
#pragma unroll
    for (int i = 0; i < kRowIt; ++i)
#pragma unroll
        for (int j = 0; j < kColIt; ++j) {
            const int r = ty + 8 * i, c = tx + 32 * j;
            if (r < kSsimIn && c < kSsimIn) sa[r][c] = v[i][j];
        }
}

// stage() for the image and the ground truth at once, interleaved as (x, y) pairs, by NT threads
template <int NT>
__device__ __forceinline__ void stage_pair(const float* __restrict__ a, const float* __restrict__ b,
                                           f2 (*sab)[kSsimIn], int H, int W, int ox, int oy) {
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    constexpr int kTy = NT / 32;
    constexpr int kRowIt = (kSsimIn + kTy - 1) / kTy, kColIt = 2;
    f2 v[kRowIt][kColIt];
#pragma unroll
    for (int i = 0; i < kRowIt; ++i) {
        const int r = ty + kTy * i, gy = oy - kSsimHalo + r;
#pragma unroll
        for (int j = 0; j < kColIt; ++j) {
            const int c = tx + 32 * j, gx = ox - kSsimHalo + c;
            const bool ok = r < kSsimIn && c < kSsimIn && gy >= 0 && gy < H && gx >= 0 && gx < W;
            const size_t o = ok ? (size_t)gy * W + gx : 0;
            v[i][j] = ok ? f2{a[o], b[o]} : f2{0.f, 0.f};
        }
    }
#pragma unroll
    for (int i = 0; i < kRowIt; ++i)
#pragma unroll
        for (int j = 0; j < kColIt; ++j) {
            const int r = ty + kTy * i, c = tx + 32 * j;
            if (r < kSsimIn && c < kSsimIn) sab[r][c] = v[i][j];
        }
}

// Vertical 11-tap pass over the horizontal sums: output rows 2 jp and 2 jp + 1 of the thread's four take one
// packed FMA (v_pk_fma_f32) per staged row, weights (w[m], w[m-1]) with m = t - 2 jp.  With the packed
// horizontal pass below: k_ssim_fwd 0.0756 -> 0.0705 ms at 1080p; with x and y interleaved in LDS (one 8-B
// read per tap, stage_pair) 0.0623 ms.  In k_ssim_bwd (three quantities, so one stays scalar) neither helps:
// packed arithmetic 0.0592 -> 0.0599 ms; (g0, g1) interleaved in LDS 0.0595 -> 0.0600, with the packed vertical
// pass 0.0606 -- not used there.
template <int NQ, int R>
__device__ __forceinline__ void vertical_pass(const SsimArgs& p, const float (*sh)[kSsimIn][kSsimTile], int r0,
                                              int c, float (&acc)[NQ][R]) {
    static_assert(R % 2 == 0, "row pairs per thread");
    f2 a2[NQ][R / 2];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int jp = 0; jp < R / 2; ++jp) a2[q][jp] = f2{0.f, 0.f};
#pragma unroll
    for (int t = 0; t < R + 10; ++t) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const float h = sh[q][r0 + t][c];
            const f2 hh = {h, h};
#pragma unroll
            for (int jp = 0; jp < R / 2; ++jp) {
                const int m = t - 2 * jp;
                if (m >= 0 && m <= 11)
                    a2[q][jp] = __builtin_elementwise_fma(f2{p.wp[2 * m], p.wp[2 * m + 1]}, hh, a2[q][jp]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int jp = 0; jp < R / 2; ++jp) {
            acc[q][2 * jp] = a2[q][jp].x;
            acc[q][2 * jp + 1] = a2[q][jp].y;
        }
}

__global__ __launch_bounds__(kSsimFwdThreads) void k_ssim_fwd(SsimArgs p, const float* __restrict__ img,
                                                             const float* __restrict__ gt, float* __restrict__ gmaps,
                                                             float* __restrict__ partial) {
    __shared__ f2 sxy[kSsimIn][kSsimIn];  // (x, y) interleaved: one 8-B LDS read per window tap
    __shared__ float sh[5][kSsimIn][kSsimTile];  // horizontal sums of x, y, x^2, y^2, xy
    __shared__ float red[2][kSsimFwdThreads / 64];
    const int ch = blockIdx.z;
    const int ox = blockIdx.x * kSsimTile, oy = blockIdx.y * kSsimTile;
    const size_t plane = (size_t)p.H * p.W;
    stage_pair<kSsimFwdThreads>(img + ch * plane, gt + ch * plane, sxy, p.H, p.W, ox, oy);
    __syncthreads();
    // horizontal pass: thread = (column c, row group); no integer division.  (x, y) as one packed pair: w x and
    // w y in one multiply, their sums and the squares' sums in two packed FMAs, xy scalar
    for (int r = threadIdx.x >> 5; r < kSsimIn; r += kSsimFwdThreads / 32) {
        const int c = threadIdx.x & 31;
        f2 ab = {0.f, 0.f}, cd = {0.f, 0.f};
        float e = 0.f;
#pragma unroll
        for (int k = 0; k < 11; ++k) {
            const f2 v = sxy[r][c + k];
            const f2 wv = p.w[k] * v;
            ab += wv;
            cd = __builtin_elementwise_fma(wv, v, cd);
            e = fmaf(wv.x, v.y, e);
        }
        sh[0][r][c] = ab.x;
        sh[1][r][c] = ab.y;
        sh[2][r][c] = cd.x;
        sh[3][r][c] = cd.y;
        sh[4][r][c] = e;
    }
    __syncthreads();
    constexpr float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
    float fsum = 0.f, l1sum = 0.f;
    // vertical pass: thread (c, g) produces rows 4g..4g+3 of column c from 14 staged rows (register reuse)
    const int c = threadIdx.x & (kSsimTile - 1), r0 = (threadIdx.x >> 5) * kSsimFwdRows;
    float acc[5][kSsimFwdRows];
    vertical_pass<5, kSsimFwdRows>(p, sh, r0, c, acc);
    const size_t map = (size_t)p.C * plane;  // gmaps = [dL/dA | dL/dC | dL/dE], each (C,H,W)
#pragma unroll
    for (int j = 0; j < kSsimFwdRows; ++j) {
        const int r = r0 + j, gy = oy + r, gx = ox + c;
        if (gy >= p.H || gx >= p.W) continue;
        const float A = acc[0][j], B = acc[1][j], Cx = acc[2][j], Dy = acc[3][j], E = acc[4][j];
        const float s1 = Cx - A * A, s2 = Dy - B * B, s12 = E - A * B;
        const float n1 = 2.f * A * B + C1, n2 = 2.f * s12 + C2;
        const float d1 = A * A + B * B + C1, d2 = s1 + s2 + C2;
        const float inv = fast_rcp(d1 * d2);
        const float f = (n1 * n2) * inv;
        const size_t o = ch * plane + (size_t)gy * p.W + gx;
        gmaps[o] = p.coef_ssim * ((2.f * B * (n2 - n1) - 2.f * A * f * (d2 - d1)) * inv);
        gmaps[map + o] = p.coef_ssim * (-f * fast_rcp(d2));
        gmaps[2 * map + o] = p.coef_ssim * (2.f * n1 * inv);
        fsum += f;
        const f2 v = sxy[r + kSsimHalo][c + kSsimHalo];
        l1sum += fabsf(v.x - v.y);
    }
    fsum = wave_sum(fsum);
    l1sum = wave_sum(l1sum);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = fsum;
        red[1][threadIdx.x >> 6] = l1sum;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int blk = (ch * p.tiles_y + blockIdx.y) * p.tiles_x + blockIdx.x;
        float fs = 0.f, ls = 0.f;
#pragma unroll
        for (int w = 0; w < kSsimFwdThreads / 64; ++w) {
            fs += red[0][w];
            ls += red[1][w];
        }
        partial[2 * blk] = fs;
        partial[2 * blk + 1] = ls;
    }
}

__global__ __launch_bounds__(kSsimThreads) void k_ssim_bwd(SsimArgs p, const float* __restrict__ img,
                                                             const float* __restrict__ gt,
                                                             const float* __restrict__ gmaps,
                                                             const float* __restrict__ gscale, float sign,
                                                             float* __restrict__ dimg) {
#ifndef GSD_SSIM_BWD_SCALAR_H
    // rows padded to 44 floats (176 B): the horizontal pass below reads each thread's 16-float window as four
    // 16-B-aligned ds_read_b128
    constexpr int kSgStride = 44;
#else
    constexpr int kSgStride = kSsimIn;
#endif
    __shared__ __attribute__((aligned(16))) float sg[3][kSsimIn][kSgStride];
    __shared__ __attribute__((aligned(16))) float sh[3][kSsimIn][kSsimTile];
    const int ch = blockIdx.z;
    const int ox = blockIdx.x * kSsimTile, oy = blockIdx.y * kSsimTile;
    const size_t plane = (size_t)p.H * p.W;
    const int c = threadIdx.x & (kSsimTile - 1), r0 = (threadIdx.x >> 5) * kSsimRows;
    // the thread's own image and ground-truth pixels, loaded with the staging loads (not after the window
    // passes, where their latency was exposed)
    float xs[kSsimRows], ys[kSsimRows];
#pragma unroll
    for (int j = 0; j < kSsimRows; ++j) {
        const int gy = oy + r0 + j, gx = ox + c;
        const bool ok = gy < p.H && gx < p.W;
        const size_t o = ch * plane + (ok ? (size_t)gy * p.W + gx : 0);
        xs[j] = ok ? img[o] : 0.f;
        ys[j] = ok ? gt[o] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) stage<kSgStride>(gmaps + ((size_t)q * p.C + ch) * plane, sg[q], p.H, p.W, ox, oy);
    __syncthreads();
#ifndef GSD_SSIM_BWD_SCALAR_H
    // horizontal pass, four output columns per thread: the 14-float window from four b128 reads per map instead of
    // 11 scalar reads per column (the same products and sums in the same order per output)
    for (int it = threadIdx.x; it < kSsimIn * (kSsimTile / 4); it += kSsimThreads) {
        const int r = it >> 3, c4 = (it & 7) * 4;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            float v[16];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const float4 f = *reinterpret_cast<const float4*>(&sg[q][r][c4 + 4 * b]);
                v[4 * b] = f.x; v[4 * b + 1] = f.y; v[4 * b + 2] = f.z; v[4 * b + 3] = f.w;
            }
            float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 11; ++k) {
                const float w = p.w[k];
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] += w * v[j + k];
            }
            *reinterpret_cast<float4*>(&sh[q][r][c4]) = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
#else
    for (int r = threadIdx.x >> 5; r < kSsimIn; r += kSsimThreads / 32) {
        float a = 0.f, cc = 0.f, e = 0.f;
#pragma unroll
        for (int k = 0; k < 11; ++k) {
            const float w = p.w[k];
            a += w * sg[0][r][c + k];
            cc += w * sg[1][r][c + k];
            e += w * sg[2][r][c + k];
        }
        sh[0][r][c] = a;
        sh[1][r][c] = cc;
        sh[2][r][c] = e;
    }
#endif
    __syncthreads();
    const float g = gscale ? sign * gscale[0] : sign;  // d out / d loss (autograd's incoming gradient)
    float acc[3][kSsimRows];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int j = 0; j < kSsimRows; ++j) acc[q][j] = 0.f;
#pragma unroll
    for (int t = 0; t < kSsimRows + 10; ++t) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const float h = sh[q][r0 + t][c];
#pragma unroll
            for (int j = 0; j < kSsimRows; ++j)
                if (t - j >= 0 && t - j < 11) acc[q][j] += p.w[t - j] * h;
        }
    }
#pragma unroll
    for (int j = 0; j < kSsimRows; ++j) {
        const int gy = oy + r0 + j, gx = ox + c;
        if (gy >= p.H || gx >= p.W) continue;
        const size_t o = ch * plane + (size_t)gy * p.W + gx;
        const float x = xs[j], y = ys[j];
        const float diff = x - y;
        const float sgn = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);  // torch.abs backward: sign, 0 at 0
        dimg[o] = g * (acc[0][j] + 2.f * x * acc[1][j] + y * acc[2][j] + p.coef_l1 * sgn);
    }
}

// Fixed-order sum of the per-workgroup partials (one workgroup): out = {loss, L1, SSIM}.  The partials are
// (f, l1) pairs, read two blocks per 16-B load, four loads in flight per lane per round (a strided scalar loop
// over the 6120 pairs of a 1080p view was ~24 dependent L2 round trips: 7.0 us).
constexpr int kSumThreads = 1024;
__global__ __launch_bounds__(kSumThreads) void k_loss_sum(int nblk, const float* __restrict__ partial, float inv_n,
                                                          float lambda, float* __restrict__ out) {
    __shared__ float red[2][kSumThreads / 64];
    const float4* p4 = reinterpret_cast<const float4*>(partial);
    const int n4 = nblk >> 1;
    float f = 0.f, l = 0.f;
    for (int b = threadIdx.x; b < n4; b += 4 * kSumThreads) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = b + u * kSumThreads;
            v[u] = i < n4 ? p4[i] : float4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            f += v[u].x + v[u].z;
            l += v[u].y + v[u].w;
        }
    }
    if ((nblk & 1) && threadIdx.x == 0) {
        f += partial[2 * (nblk - 1)];
        l += partial[2 * (nblk - 1) + 1];
    }
    f = wave_sum(f);
    l = wave_sum(l);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = f;
        red[1][threadIdx.x >> 6] = l;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float fs = 0.f, ls = 0.f;
#pragma unroll
        for (int w = 0; w < kSumThreads / 64; ++w) {
            fs += red[0][w];
            ls += red[1][w];
        }
        const float ssim = fs * inv_n;
        const float l1 = ls * inv_n;
        out[0] = (1.f - lambda) * l1 + lambda * (1.f - ssim);
        out[1] = l1;
        out[2] = ssim;
    }
}

void ssim_tiles(int H, int W, int* tx, int* ty) {
    *tx = (W + kSsimTile - 1) / kSsimTile;
    *ty = (H + kSsimTile - 1) / kSsimTile;
}

static SsimArgs ssim_args(int C, int H, int W, const float* w11, float lambda) {
    SsimArgs p{};
    p.C = C; p.H = H; p.W = W;
    ssim_tiles(H, W, &p.tiles_x, &p.tiles_y);
    for (int k = 0; k < 11; ++k) p.w[k] = w11[k];
    for (int m = 0; m < 12; ++m) {
        p.wp[2 * m] = m <= 10 ? w11[m] : 0.f;
        p.wp[2 * m + 1] = m >= 1 ? w11[m - 1] : 0.f;
    }
    const double n = (double)C * H * W;
    p.coef_ssim = (float)(-lambda / n);
    p.coef_l1 = (float)((1.0 - lambda) / n);
    return p;
}

void launch_l1_ssim(int C, int H, int W, const float* w11, float lambda, const float* img, const float* gt,
                    float* gmaps, float* partial, float* out3, float* dimg, hipStream_t s) {
    const SsimArgs p = ssim_args(C, H, W, w11, lambda);
    const double n = (double)C * H * W;
    const dim3 grid(p.tiles_x, p.tiles_y, C);
    hipLaunchKernelGGL(k_ssim_fwd, grid, dim3(kSsimFwdThreads), 0, s, p, img, gt, gmaps, partial);
    hipLaunchKernelGGL(k_loss_sum, dim3(1), dim3(kSumThreads), 0, s, p.tiles_x * p.tiles_y * C, partial, (float)(1.0 / n),
                       lambda, out3);
    if (dimg)
        hipLaunchKernelGGL(k_ssim_bwd, grid, dim3(kSsimThreads), 0, s, p, img, gt, gmaps, (const float*)nullptr, 1.0f,
                           dimg);
}

void launch_l1_ssim_bwd(int C, int H, int W, const float* w11, float lambda, const float* img, const float* gt,
                        const float* gmaps, const float* gscale, float sign, float* dimg, hipStream_t s) {
    const SsimArgs p = ssim_args(C, H, W, w11, lambda);
    const dim3 grid(p.tiles_x, p.tiles_y, C);
    hipLaunchKernelGGL(k_ssim_bwd, grid, dim3(kSsimThreads), 0, s, p, img, gt, gmaps, gscale, sign, dimg);
}

// ---- offset-norm regulariser (train.py:329-332): R = mean_g ||off_g||, the per-Gaussian 3-D offsets of the
// deformation.  Forward: per-workgroup partial sums of the row norms, then one workgroup sums them in a fixed order
// (deterministic, no float atomics).  Backward: dR/doff_g = g * scale * off_g / ||off_g||, zero where the norm is
// zero (torch's norm backward masks the division there).  HBM: 12 B per row read, 12 B written backward.
constexpr int kOffThreads = 256;
constexpr int kOffMaxBlocks = 1024;

int offnorm_blocks(long long P) {
    const long long b = (P + kOffThreads * 4 - 1) / (kOffThreads * 4);
    return (int)(b < 1 ? 1 : (b > kOffMaxBlocks ? kOffMaxBlocks : b));
}

__device__ __forceinline__ float row_norm(const float* __restrict__ off, long long g) {
    const float x = off[3 * g], y = off[3 * g + 1], z = off[3 * g + 2];
    return sqrtf(x * x + y * y + z * z);
}

__global__ __launch_bounds__(kOffThreads) void k_offnorm_partial(long long P, const float* __restrict__ off,
                                                                 float* __restrict__ partial) {
    __shared__ float red[kOffThreads / 64];
    float acc = 0.f;
    for (long long g = (long long)blockIdx.x * kOffThreads + threadIdx.x; g < P; g += (long long)gridDim.x * kOffThreads)
        acc += row_norm(off, g);
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(kOffMaxBlocks) void k_offnorm_final(int nblk, const float* __restrict__ partial,
                                                                 float scale, float* __restrict__ out) {
    __shared__ float red[kOffMaxBlocks / 64];
    float v = threadIdx.x < (unsigned)nblk ? partial[threadIdx.x] : 0.f;
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kOffMaxBlocks / 64; ++w) t += red[w];
        out[0] = t * scale;
    }
}

__global__ __launch_bounds__(kOffThreads) void k_offnorm_bwd(long long P, const float* __restrict__ off,
                                                             const float* __restrict__ gscale, float scale,
                                                             float* __restrict__ d_off) {
    const long long g = (long long)blockIdx.x * kOffThreads + threadIdx.x;
    if (g >= P) return;
    const float c = (gscale ? gscale[0] : 1.f) * scale;
    const float x = off[3 * g], y = off[3 * g + 1], z = off[3 * g + 2];
    const float n = sqrtf(x * x + y * y + z * z);
    const float k = n > 0.f ? c / n : 0.f;
    d_off[3 * g] = x * k;
    d_off[3 * g + 1] = y * k;
    d_off[3 * g + 2] = z * k;
}

void launch_offset_norm(long long P, const float* off, float scale, float* partial, float* out, hipStream_t s) {
    const int nb = offnorm_blocks(P);
    hipLaunchKernelGGL(k_offnorm_partial, dim3(nb), dim3(kOffThreads), 0, s, P, off, partial);
    hipLaunchKernelGGL(k_offnorm_final, dim3(1), dim3(kOffMaxBlocks), 0, s, nb, (const float*)partial, scale, out);
}

void launch_offset_norm_bwd(long long P, const float* off, const float* gscale, float scale, float* d_off,
                            hipStream_t s) {
    const long long nb = (P + kOffThreads - 1) / kOffThreads;
    hipLaunchKernelGGL(k_offnorm_bwd, dim3((unsigned)nb), dim3(kOffThreads), 0, s, P, off, gscale, scale, d_off);
}

}  // namespace gsd
