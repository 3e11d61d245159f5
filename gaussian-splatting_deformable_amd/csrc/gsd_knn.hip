// gsd_knn.hip -- initial Gaussian scales: mean squared distance to the 3 nearest neighbours.
//
// Reference: submodules/simple-knn/simple_knn.cu (SimpleKNN::knn, :165-219, distCUDA2), used by
// GaussianModel.create_from_pcd (scene/gaussian_model.py:817).  Same algorithm:
//   1. bounding box of the points together with the origin (the reference's cub reductions start
//      from init = {0,0,0}, :171-178, so the origin is always inside it);
//   2. 30-bit Morton code per point on a 1024^3 grid over that box (:45-61);
//   3. stable radix sort of (code, index) -- here hipcub (rocPRIM), the reference cub;
//   4. boxes of 1024 consecutive sorted points with their bounding boxes (:77-111);
//   5. per point: the 3rd-best squared distance among its +-3 sorted neighbours bounds the search;
//      every box not farther than that bound (and than the running 3rd best) is scanned
//      exhaustively (:139-163).  Since a box's distance is a lower bound for its points', the result
//      is the exact mean of the 3 smallest squared distances to other points.
// Float expressions keep the reference's order (dx*dx + dy*dy + dz*dz, (b0 + b1 + b2) / 3).
#include <cfloat>

#include <hipcub/hipcub.hpp>

#include "gsd_kernels.h"

namespace gsd {

constexpr int kKnnBox = 1024;

struct KnnBox {
    float3 minn, maxx;
};

__device__ __forceinline__ uint32_t prep_morton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}

// block min/max over a grid-stride range, one result pair per block (the origin included)
__global__ __launch_bounds__(256) void k_knn_bounds(int P, const float* __restrict__ pts, float* __restrict__ part) {
    __shared__ float s[6][256];
    float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // init = {0,0,0} for both reductions, like the reference
    for (int i = blockIdx.x * 256 + threadIdx.x; i < P; i += gridDim.x * 256) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float x = pts[3 * i + c];
            v[c] = fminf(v[c], x);
            v[3 + c] = fmaxf(v[3 + c], x);
        }
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) s[c][threadIdx.x] = v[c];
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                s[c][threadIdx.x] = fminf(s[c][threadIdx.x], s[c][threadIdx.x + off]);
                s[3 + c][threadIdx.x] = fmaxf(s[3 + c][threadIdx.x], s[3 + c][threadIdx.x + off]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[6 * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void k_knn_morton(int P, int nparts, const float* __restrict__ pts,
                                                    const float* __restrict__ part, uint32_t* __restrict__ codes,
                                                    uint32_t* __restrict__ idx) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    float mn[3] = {part[0], part[1], part[2]}, mx[3] = {part[3], part[4], part[5]};
    for (int b = 1; b < nparts; ++b)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            mn[c] = fminf(mn[c], part[6 * b + c]);
            mx[c] = fmaxf(mx[c], part[6 * b + 3 + c]);
        }
    uint32_t code = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float f = ((pts[3 * i + c] - mn[c]) / (mx[c] - mn[c])) * (float)((1 << 10) - 1);
        code |= prep_morton((uint32_t)f) << c;
    }
    codes[i] = code;
    idx[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_knn_boxes(int P, const float* __restrict__ pts,
                                                   const uint32_t* __restrict__ order, KnnBox* __restrict__ boxes) {
    __shared__ float s[6][256];
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int k = threadIdx.x; k < kKnnBox; k += 256) {
        const int i = blockIdx.x * kKnnBox + k;
        if (i < P) {
            const uint32_t g = order[i];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float x = pts[3 * g + c];
                v[c] = fminf(v[c], x);
                v[3 + c] = fmaxf(v[3 + c], x);
            }
        }
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) s[c][threadIdx.x] = v[c];
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                s[c][threadIdx.x] = fminf(s[c][threadIdx.x], s[c][threadIdx.x + off]);
                s[3 + c][threadIdx.x] = fmaxf(s[3 + c][threadIdx.x], s[3 + c][threadIdx.x + off]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        boxes[blockIdx.x] = KnnBox{make_float3(s[0][0], s[1][0], s[2][0]), make_float3(s[3][0], s[4][0], s[5][0])};
}

__device__ __forceinline__ float dist_box_point(const KnnBox& b, float3 p) {  // simple_knn.cu:113-123
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (p.x < b.minn.x || p.x > b.maxx.x) dx = fminf(fabsf(p.x - b.minn.x), fabsf(p.x - b.maxx.x));
    if (p.y < b.minn.y || p.y > b.maxx.y) dy = fminf(fabsf(p.y - b.minn.y), fabsf(p.y - b.maxx.y));
    if (p.z < b.minn.z || p.z > b.maxx.z) dz = fminf(fabsf(p.z - b.minn.z), fabsf(p.z - b.maxx.z));
    return dx * dx + dy * dy + dz * dz;
}

__device__ __forceinline__ void update_best3(float3 ref, float3 q, float (&best)[3]) {  // :125-139
    const float ex = q.x - ref.x, ey = q.y - ref.y, ez = q.z - ref.z;
    float d = ex * ex + ey * ey + ez * ez;
#pragma unroll
    for (int j = 0; j < 3; ++j)
        if (best[j] > d) {
            const float t = best[j];
            best[j] = d;
            d = t;
        }
}

__device__ __forceinline__ float3 load3(const float* p, uint32_t g) {
    return make_float3(p[3 * g], p[3 * g + 1], p[3 * g + 2]);
}

__global__ __launch_bounds__(256) void k_knn_mean_dist(int P, const float* __restrict__ pts,
                                                       const uint32_t* __restrict__ order,
                                                       const KnnBox* __restrict__ boxes, float* __restrict__ out) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= P) return;
    const float3 p = load3(pts, order[idx]);
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    for (int i = max(0, idx - 3); i <= min(P - 1, idx + 3); ++i)
        if (i != idx) update_best3(p, load3(pts, order[i]), best);
    const float reject = best[2];
    best[0] = best[1] = best[2] = FLT_MAX;
    const int nboxes = (P + kKnnBox - 1) / kKnnBox;
    for (int b = 0; b < nboxes; ++b) {
        const float d = dist_box_point(boxes[b], p);
        if (d > reject || d > best[2]) continue;
        const int e = min(P, (b + 1) * kKnnBox);
        for (int i = b * kKnnBox; i < e; ++i)
            if (i != idx) update_best3(p, load3(pts, order[i]), best);
    }
    out[order[idx]] = (best[0] + best[1] + best[2]) / 3.0f;
}

size_t knn_workspace(int P, size_t* sort_bytes) {
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (uint32_t*)nullptr, P);
    if (sort_bytes) *sort_bytes = tb;
    const size_t nboxes = (size_t)(P + kKnnBox - 1) / kKnnBox;
    return 4 * (size_t)P * sizeof(uint32_t) + nboxes * sizeof(KnnBox) + 6 * 256 * sizeof(float) + tb + 6 * 256;
}

int launch_knn(int P, const float* pts, float* out, void* ws, hipStream_t s) {
    size_t tb = 0;
    knn_workspace(P, &tb);
    char* w = static_cast<char*>(ws);
    auto take = [&](size_t bytes) {
        char* r = w;
        w += (bytes + 255) & ~size_t(255);
        return r;
    };
    uint32_t* codes = reinterpret_cast<uint32_t*>(take(P * sizeof(uint32_t)));
    uint32_t* codes_sorted = reinterpret_cast<uint32_t*>(take(P * sizeof(uint32_t)));
    uint32_t* idx = reinterpret_cast<uint32_t*>(take(P * sizeof(uint32_t)));
    uint32_t* order = reinterpret_cast<uint32_t*>(take(P * sizeof(uint32_t)));
    const int nboxes = (P + kKnnBox - 1) / kKnnBox;
    KnnBox* boxes = reinterpret_cast<KnnBox*>(take(nboxes * sizeof(KnnBox)));
    const int nparts = 256;
    float* part = reinterpret_cast<float*>(take(6 * nparts * sizeof(float)));
    void* tmp = take(tb);
    hipLaunchKernelGGL(k_knn_bounds, dim3(nparts), dim3(256), 0, s, P, pts, part);
    hipLaunchKernelGGL(k_knn_morton, dim3((P + 255) / 256), dim3(256), 0, s, P, nparts, pts, part, codes, idx);
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, codes, codes_sorted, idx, order, P, 0, 32, s);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_knn_boxes, dim3(nboxes), dim3(256), 0, s, P, pts, order, boxes);
    hipLaunchKernelGGL(k_knn_mean_dist, dim3((P + 255) / 256), dim3(256), 0, s, P, pts, order, boxes, out);
    return 0;
}

}  // namespace gsd
