// gsd_binning.hip -- tile binning: per-tile scan, bucketed scatter, per-tile sort.
//
// The reference (rasterizer_impl.cu:275-318) scans tiles_touched over all P
// Gaussians, emits K (u64 |tile|depth|, u32 id) pairs and radix-sorts all K
// of them with cub over 32+msb bits (6 LSD passes, ~24 B/instance/pass).
// Here the tile id is never sorted: the per-tile instance counts (histogram,
// accumulated by k_preprocess_fwd) are scanned over T tiles, which yields the
// reference's `ranges` directly; each instance is scattered into its tile's
// bucket, and each bucket is sorted independently in LDS by the 64-bit key
// (depth bits << 32 | gaussian id).  Because the reference's sort is stable
// and its input is emitted in gaussian-id order, its output order inside a
// tile is exactly ascending (depth bits, id) -- a total order on unique keys,
// so this produces the identical point_list.  HBM traffic: ~8 B (scatter) +
// 8 B read + 4 B write (sort) per instance, vs ~150 B for 6 global passes.
#include <type_traits>

#include "gsd_kernels.h"

namespace gsd {

// Exclusive scan of tile_count over T tiles (one 1024-lane workgroup; T <= a few 1e5): each lane owns `per`
// consecutive tiles (held in registers up to kScanKeep), wave-level shuffle scans of the lane sums, one LDS
// exchange of the 16 wave totals -- two barriers (an LDS Hillis-Steele over 1024 partials took 20).
constexpr int kScanKeep = 16;
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(v, off);
        if (lane >= off) v += t;
    }
    return v;
}
// kLds (T <= kScanLdsTiles): the counts are loaded tile-interleaved (coalesced) into LDS, each thread scans its
// run of `per` consecutive tiles there and leaves each tile's exclusive base in place, and the ranges / cursors go
// out in a second tile-interleaved pass (end = the next tile's base).  Loaded and written straight from each
// thread's run, every memory instruction touched 64 separate segments: 11.0 us at 1080p, 8.5 with the LDS passes
// (the rest is the one workgroup's launch and barrier latency).
constexpr int kScanLdsTiles = 32767;
template <bool kLds>
__global__ __launch_bounds__(kScanThreads) void k_tile_scan(int T, const uint32_t* __restrict__ tile_count,
                                                            uint2* __restrict__ ranges, uint32_t* __restrict__ cursor,
                                                            uint32_t* __restrict__ counters) {
    extern __shared__ uint32_t s_base[];  // kLds: [T + 1], the counts (coalesced loads), then each tile's base
    __shared__ uint32_t s_wave[kScanThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int per = (T + kScanThreads - 1) / kScanThreads;
    const int b0 = min(T, tid * per), b1 = min(T, b0 + per);
    if constexpr (kLds) {
        for (int t = tid; t < T; t += kScanThreads) s_base[t] = tile_count[t];
        __syncthreads();
        uint32_t local = 0;
        for (int i = b0; i < b1; ++i) local += s_base[i];
        const uint32_t incl = wave_incl_scan(local, lane);
        if (lane == 63) s_wave[wid] = incl;
        __syncthreads();
        if (wid == 0) {
            uint32_t v = lane < kScanThreads / 64 ? s_wave[lane] : 0u;
            v = wave_incl_scan(v, lane);
            if (lane < kScanThreads / 64) s_wave[lane] = v;
        }
        __syncthreads();
        uint32_t run = incl - local + (wid ? s_wave[wid - 1] : 0u);
        for (int i = b0; i < b1; ++i) {  // the thread's own tiles only: count read, base written in place
            const uint32_t c = s_base[i];
            s_base[i] = run;
            run += c;
        }
        if (tid == kScanThreads - 1) {
            s_base[T] = s_wave[kScanThreads / 64 - 1];
            counters[0] = s_wave[kScanThreads / 64 - 1];
        }
        __syncthreads();
        // empty tiles keep (0,0) as after the reference's memset (rasterizer_impl.cu:310)
        for (int t = tid; t < T; t += kScanThreads) {
            const uint32_t b = s_base[t], e = s_base[t + 1];
            ranges[t] = e > b ? make_uint2(b, e) : make_uint2(0u, 0u);
            cursor[t] = b;
        }
        return;
    }
    uint32_t keep[kScanKeep];
    uint32_t local = 0;
    if (per <= kScanKeep) {
#pragma unroll
        for (int i = 0; i < kScanKeep; ++i) {
            keep[i] = b0 + i < b1 ? tile_count[b0 + i] : 0u;
            local += keep[i];
        }
    } else {
        for (int i = b0; i < b1; ++i) local += tile_count[i];
    }
    const uint32_t incl = wave_incl_scan(local, lane);
    if (lane == 63) s_wave[wid] = incl;
    __syncthreads();
    if (wid == 0) {
        uint32_t v = lane < kScanThreads / 64 ? s_wave[lane] : 0u;
        v = wave_incl_scan(v, lane);
        if (lane < kScanThreads / 64) s_wave[lane] = v;
    }
    __syncthreads();
    uint32_t run = incl - local + (wid ? s_wave[wid - 1] : 0u);
    // empty tiles keep (0,0) as after the reference's memset (rasterizer_impl.cu:310)
    if (per <= kScanKeep) {
#pragma unroll
        for (int i = 0; i < kScanKeep; ++i) {
            if (b0 + i < b1) {
                const uint32_t c = keep[i];
                ranges[b0 + i] = c ? make_uint2(run, run + c) : make_uint2(0u, 0u);
                cursor[b0 + i] = run;
                run += c;
            }
        }
    } else {
        for (int i = b0; i < b1; ++i) {
            const uint32_t c = tile_count[i];
            ranges[i] = c ? make_uint2(run, run + c) : make_uint2(0u, 0u);
            cursor[i] = run;
            run += c;
        }
    }
    if (tid == kScanThreads - 1) counters[0] = s_wave[kScanThreads / 64 - 1];
}

// duplicateWithKeys (rasterizer_impl.cu:70-111), scattered straight into tile buckets.
__global__ __launch_bounds__(256) void k_scatter_keys(BinParams p) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= p.P || over_capacity(p.k_guard, p.k_cap)) return;
    const int rad = p.radii[idx];
    if (!(rad > 0)) return;
    const float2 xy = p.means2D[idx];
    const Rect r = tile_rect(xy.x, xy.y, rad, p.grid_x, p.grid_y);
    const unsigned long long key =
        ((unsigned long long)__float_as_uint(p.depths[idx]) << 32) | (unsigned long long)(uint32_t)idx;
    for (int y = r.y0; y < r.y1; ++y)
        for (int x = r.x0; x < r.x1; ++x) {
            const uint32_t pos = __hip_atomic_fetch_add(p.tile_cursor + (y * p.grid_x + x), 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            p.bucket_keys[pos] = key;
        }
}

// ---------------------------------------------------------------------------
// Atomic-free binning (tile grids up to kHistMaxTiles): global atomics on tile
// counters serialise at the memory side (~0.35 ms per view at 3.2M instances),
// so the histogram is built per block in LDS and combined by column scans.
// Block b owns Gaussians [b*chunk, (b+1)*chunk).
//   k_tile_hist:       hist[b][t] = instances of block b in tile t        (LDS atomics)
//   k_colscan_partial: part[s][t] = sum of hist rows of segment s
//   k_colscan_final:   hist[b][t] <- exclusive prefix over b; tile_count[t] = column total
//   k_tile_scan:       ranges / tile base (as before)
//   k_scatter_hist:    slot = tile base + hist[b][t] + LDS fetch-add      (LDS atomics)
// ---------------------------------------------------------------------------
// The Gaussian chunk a workgroup takes (its row of the histogram): chunks are grouped by XCD -- workgroups are dealt
// round-robin over the 8 XCDs, so workgroups b and b + 8 share one -- giving each XCD a contiguous range of chunks.
// The column scan stacks the chunks' runs inside each tile's bucket in chunk order, so each XCD's workgroups write
// one contiguous sub-range of every bucket (-18 % scatter time at cfg4).  Scanning the rows in that permuted order
// instead cost the column scans as much as it saved.  The sort downstream orders each bucket by key, so the order
// of the runs inside it does not change point_list.
__device__ __forceinline__ int hist_chunk(int b, int nb) {
    if (nb & 7) return b;
    return (b & 7) * (nb >> 3) + (b >> 3);
}

__global__ __launch_bounds__(kHistThreads) void k_tile_hist(HistParams p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_bins[];
    const int T = p.num_tiles;
    for (int t = threadIdx.x; t < T; t += kHistThreads) s_bins[t] = 0u;
    __syncthreads();
    const int c = hist_chunk(blockIdx.x, p.num_blocks);
    const int g0 = c * p.chunk, g1 = min(p.P, g0 + p.chunk);
    for (int g = g0 + threadIdx.x; g < g1; g += kHistThreads) {
        const int rad = p.radii[g];
        if (!(rad > 0)) continue;
        const float2 xy = p.means2D[g];
        const Rect r = tile_rect(xy.x, xy.y, rad, p.grid_x, p.grid_y);
        for (int y = r.y0; y < r.y1; ++y)
            for (int x = r.x0; x < r.x1; ++x) atomicAdd(&s_bins[y * p.grid_x + x], 1u);
    }
    __syncthreads();
    uint32_t* out = p.hist + (size_t)c * T;
    for (int t = threadIdx.x; t < T; t += kHistThreads) out[t] = s_bins[t];
}

__global__ __launch_bounds__(256) void k_colscan_partial(HistParams p) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= p.num_tiles) return;
    const int b0 = blockIdx.y * kColSeg, b1 = min(p.num_blocks, b0 + kColSeg);
    uint32_t s = 0;
#pragma unroll 8
    for (int b = b0; b < b1; ++b) s += p.hist[(size_t)b * p.num_tiles + t];
    p.part[(size_t)blockIdx.y * p.num_tiles + t] = s;
}

__global__ __launch_bounds__(256) void k_colscan_final(HistParams p, uint32_t* __restrict__ tile_count) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= p.num_tiles) return;
    const int T = p.num_tiles;
    uint32_t base = 0;
#pragma unroll 8
    for (int s = 0; s < (int)blockIdx.y; ++s) base += p.part[(size_t)s * T + t];
    const int b0 = blockIdx.y * kColSeg, b1 = min(p.num_blocks, b0 + kColSeg);
    // the segment's rows loaded together (independent of the running base), then the exclusive prefix written:
    // one round of load latency instead of one per row
    if (b1 - b0 == kColSeg) {
        uint32_t v[kColSeg];
#pragma unroll
        for (int i = 0; i < kColSeg; ++i) v[i] = p.hist[(size_t)(b0 + i) * T + t];
#pragma unroll
        for (int i = 0; i < kColSeg; ++i) {
            p.hist[(size_t)(b0 + i) * T + t] = base;
            base += v[i];
        }
    } else {
        for (int b = b0; b < b1; ++b) {
            uint32_t* h = p.hist + (size_t)b * T + t;
            const uint32_t v = *h;
            *h = base;
            base += v;
        }
    }
    if ((int)blockIdx.y == (int)gridDim.y - 1) tile_count[t] = base;
}

__global__ __launch_bounds__(kHistThreads) void k_scatter_hist(HistParams p, const uint32_t* __restrict__ tile_base,
                                                              const float* __restrict__ depths,
                                                              unsigned long long* __restrict__ bucket_keys) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_bins[];
    if (over_capacity(p.k_guard, p.k_cap)) return;
    const int T = p.num_tiles;
    const int c = hist_chunk(blockIdx.x, p.num_blocks);
    const uint32_t* row = p.hist + (size_t)c * T;
    for (int t = threadIdx.x; t < T; t += kHistThreads) s_bins[t] = tile_base[t] + row[t];
    __syncthreads();
    const int g0 = c * p.chunk, g1 = min(p.P, g0 + p.chunk);
    for (int g = g0 + threadIdx.x; g < g1; g += kHistThreads) {
        const int rad = p.radii[g];
        if (!(rad > 0)) continue;
        const float2 xy = p.means2D[g];
        const Rect r = tile_rect(xy.x, xy.y, rad, p.grid_x, p.grid_y);
        const unsigned long long key =
            ((unsigned long long)__float_as_uint(depths[g]) << 32) | (unsigned long long)(uint32_t)g;
        for (int y = r.y0; y < r.y1; ++y)
            for (int x = r.x0; x < r.x1; ++x) bucket_keys[atomicAdd(&s_bins[y * p.grid_x + x], 1u)] = key;
    }
}

void launch_tile_hist(const HistParams& p, uint32_t* tile_count, hipStream_t s) {
    if (p.num_blocks <= 0) return;
    const size_t lds = sizeof(uint32_t) * (size_t)p.num_tiles;
    if (lds > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_tile_hist),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_tile_hist, dim3(p.num_blocks), dim3(kHistThreads), lds, s, p);
    const dim3 g((p.num_tiles + 255) / 256, (p.num_blocks + kColSeg - 1) / kColSeg);
    hipLaunchKernelGGL(k_colscan_partial, g, dim3(256), 0, s, p);
    hipLaunchKernelGGL(k_colscan_final, g, dim3(256), 0, s, p, tile_count);
}

void launch_scatter_hist(const HistParams& p, const uint32_t* tile_base, const float* depths,
                         unsigned long long* keys, hipStream_t s) {
    if (p.num_blocks <= 0) return;
    const size_t lds = sizeof(uint32_t) * (size_t)p.num_tiles;
    if (lds > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_scatter_hist),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_scatter_hist, dim3(p.num_blocks), dim3(kHistThreads), lds, s, p, tile_base, depths, keys);
}

// In-LDS bitonic sort of N (power of two) u64 keys by the whole workgroup.
__device__ __forceinline__ void bitonic_lds(unsigned long long* s, int N) {
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < (N >> 1); i += blockDim.x) {
                const int lo = 2 * j * (i / j) + (i % j);
                const int hi = lo + j;
                const bool asc = (lo & k) == 0;
                const unsigned long long a = s[lo], b = s[hi];
                if ((a > b) == asc) {
                    s[lo] = b;
                    s[hi] = a;
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ int next_pow2(int n) {
    int v = 1;
    while (v < n) v <<= 1;
    return v;
}

// Sort [base, base+n) of `src` (n <= kSortCap) in LDS; write keys to kdst (if
// non-null) and the gaussian ids to pdst (if non-null).
__device__ void sort_chunk(unsigned long long* s, const unsigned long long* __restrict__ src, int n,
                           unsigned long long* kdst, uint32_t* pdst) {
    const int N = next_pow2(n);
    for (int i = threadIdx.x; i < N; i += blockDim.x) s[i] = i < n ? src[i] : ~0ull;
    __syncthreads();
    bitonic_lds(s, N);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (kdst) kdst[i] = s[i];
        if (pdst) pdst[i] = (uint32_t)s[i];
    }
    __syncthreads();
}

// Merge-path split: number of elements taken from A among the first d outputs.
__device__ __forceinline__ int merge_split(const unsigned long long* A, int la, const unsigned long long* B, int lb,
                                           int d) {
    int lo = max(0, d - lb), hi = min(d, la);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (A[mid] > B[d - mid - 1]) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// Register bitonic sort of one tile's bucket (n <= 256 E keys, padded with ~0 to N = 256 E): thread t holds
// keys t E .. t E + E - 1.  Of the log2(N)(log2(N)+1)/2 compare-exchange passes, those with partner distance
// j < E stay inside a thread, E <= j < 64 E cross lanes of one wave (shuffles, no barrier), and only the
// j >= 64 E ones (3 of 45 at N = 512) go through LDS with barriers -- instead of every pass.
// v of lane ^ d.  For the distances of the unrolled passes (constants) as VALU cross-lane ops instead of
// ds_bpermute (an LDS-pipe instruction plus an address, 412 of them in the 512-key network): DPP quad_perm for
// 1 and 2, two row rotations and a select for 4 (rotating a 16-lane row by 8 is xor 8), v_permlane16/32_swap
// and a select for 16 and 32.
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int d, int lane) {
    switch (d) {
        case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
        case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
        case 4: {
            const uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
            const uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12c, 0xf, 0xf, false);  // row_ror:12
            return (lane & 4) ? a : b;
        }
        case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
        case 16: {
            const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            return (lane & 16) ? r[0] : r[1];
        }
        case 32: {
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return (lane & 32) ? r[0] : r[1];
        }
        default: return (uint32_t)__shfl_xor((int)v, d);
    }
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int d) {
    const int lane = threadIdx.x & 63;
    const uint32_t lo = xor_lane((uint32_t)v, d, lane), hi = xor_lane((uint32_t)(v >> 32), d, lane);
    return ((unsigned long long)hi << 32) | lo;
}
template <int E>
__device__ void sort_tile_regs(const unsigned long long* __restrict__ src, int n, unsigned long long* s,
                               uint32_t* __restrict__ pdst) {
    constexpr int N = 256 * E;
    const int t = threadIdx.x;
    unsigned long long x[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int e = t * E + r;
        x[r] = e < n ? src[e] : ~0ull;
    }
    // a pass inside the thread, its distance J a compile-time constant: x[r | J] a register, not a scratch access
    // (with a run-time j the looped E = 8 / 16 networks kept x in scratch memory)
    auto intra = [&](auto jc, int k) {
        constexpr int J = decltype(jc)::value;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            if ((r & J) == 0) {
                const bool asc = (((t * E + r) & k) == 0);
                const unsigned long long a = x[r], b = x[r | J];
                const bool swap = (b < a) == asc;
                x[r] = swap ? b : a;
                x[r | J] = swap ? a : b;
            }
        }
    };
    auto pass = [&](int k, int j) {
        if (E == 16 && j < E) {   // (the 4096-key network keeps the looped form: its registers would cut occupancy)
#pragma unroll
            for (int r = 0; r < E; ++r) {
                if ((r & j) == 0) {
                    const bool asc = (((t * E + r) & k) == 0);
                    const unsigned long long a = x[r], b = x[r | j];
                    const bool swap = (b < a) == asc;
                    x[r] = swap ? b : a;
                    x[r | j] = swap ? a : b;
                }
            }
        } else if (j < E) {
            if (j == 1) intra(std::integral_constant<int, 1>{}, k);
            if constexpr (E > 2) if (j == 2) intra(std::integral_constant<int, 2>{}, k);
            if constexpr (E > 4) if (j == 4) intra(std::integral_constant<int, 4>{}, k);
            if constexpr (E > 8) if (j == 8) intra(std::integral_constant<int, 8>{}, k);
        } else {
            const bool lds = j >= 64 * E;
            if (lds) {
                __syncthreads();
#pragma unroll
                for (int r = 0; r < E; ++r) s[t * E + r] = x[r];
                __syncthreads();
            }
#pragma unroll
            for (int r = 0; r < E; ++r) {
                const int e = t * E + r;
                const unsigned long long p = lds ? s[e ^ j] : shfl_xor_u64(x[r], j / E);
                const bool keep_min = (((e & j) == 0) == ((e & k) == 0));
                x[r] = ((x[r] < p) == keep_min) ? x[r] : p;  // equal keys are identical (padding)
            }
        }
    };
    // fully unrolled for the common bucket sizes: every partner distance is then a compile-time constant
    // (DPP / swizzle shuffles, no index arithmetic); 0.103 -> 0.062 ms on the bench's 512-key buckets
    if constexpr (E <= 4) {
#pragma unroll
        for (int k = 2; k <= N; k <<= 1)
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1) pass(k, j);
    } else {
        for (int k = 2; k <= N; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) pass(k, j);
    }
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int e = t * E + r;
        if (e < n) pdst[e] = (uint32_t)x[r];
    }
}

__global__ __launch_bounds__(256) void k_tile_sort(int T, const uint2* __restrict__ ranges,
                                                   unsigned long long* __restrict__ keys,
                                                   unsigned long long* __restrict__ scratch,
                                                   uint32_t* __restrict__ point_list,
                                                   const uint32_t* __restrict__ k_guard, uint32_t k_cap) {
    __shared__ unsigned long long s[kSortCap];
    if (over_capacity(k_guard, k_cap)) return;
    const int tile = xcd_swizzle(blockIdx.x, T);
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    if (n <= 0) return;
    const size_t base = rg.x;
    static_assert(kSortCap >= 512 && (kSortCap & (kSortCap - 1)) == 0, "a power of two of at least 512");
    if (n <= 512) return sort_tile_regs<2>(keys + base, n, s, point_list + base);
    if constexpr (kSortCap >= 1024) if (n <= 1024) return sort_tile_regs<4>(keys + base, n, s, point_list + base);
    if constexpr (kSortCap >= 2048) if (n <= 2048) return sort_tile_regs<8>(keys + base, n, s, point_list + base);
    if constexpr (kSortCap >= 4096) if (n <= 4096) return sort_tile_regs<16>(keys + base, n, s, point_list + base);
    // Large bucket: sort kSortCap chunks in LDS, then merge runs pairwise in
    // global memory (ping-pong keys <-> scratch), the whole workgroup per merge.
    for (int c0 = 0; c0 < n; c0 += kSortCap) {
        const int len = min(kSortCap, n - c0);
        sort_chunk(s, keys + base + c0, len, keys + base + c0, nullptr);
    }
    unsigned long long* src = keys + base;
    unsigned long long* dst = scratch + base;
    for (int w = kSortCap; w < n; w <<= 1) {
        for (int a0 = 0; a0 < n; a0 += 2 * w) {
            const int a1 = min(a0 + w, n), b1 = min(a0 + 2 * w, n);
            const int la = a1 - a0, lb = b1 - a1, tot = b1 - a0;
            const int chunk = (tot + blockDim.x - 1) / blockDim.x;
            const int d0 = min(tot, (int)threadIdx.x * chunk), d1 = min(tot, d0 + chunk);
            int i = merge_split(src + a0, la, src + a1, lb, d0);
            int j = d0 - i;
            for (int d = d0; d < d1; ++d) {
                const bool takeA = j >= lb || (i < la && src[a0 + i] <= src[a1 + j]);
                dst[a0 + d] = takeA ? src[a0 + i++] : src[a1 + j++];
            }
        }
        __syncthreads();
        unsigned long long* t = src;
        src = dst;
        dst = t;
    }
    for (int i = threadIdx.x; i < n; i += blockDim.x) point_list[base + i] = (uint32_t)src[i];
}

void launch_tile_scan(int T, const uint32_t* tile_count, uint2* ranges, uint32_t* cursor, uint32_t* counters,
                      hipStream_t s) {
    if (T <= kScanLdsTiles) {
        const size_t lds = sizeof(uint32_t) * ((size_t)T + 1);
        if (lds > 65536)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_tile_scan<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_tile_scan<true>, dim3(1), dim3(kScanThreads), lds, s, T, tile_count, ranges, cursor,
                           counters);
    } else {
        hipLaunchKernelGGL(k_tile_scan<false>, dim3(1), dim3(kScanThreads), 0, s, T, tile_count, ranges, cursor,
                           counters);
    }
}
void launch_scatter_keys(const BinParams& p, hipStream_t s) {
    if (p.P > 0) hipLaunchKernelGGL(k_scatter_keys, dim3((p.P + 255) / 256), dim3(256), 0, s, p);
}
void launch_tile_sort(int T, const uint2* ranges, unsigned long long* keys, unsigned long long* scratch,
                      uint32_t* point_list, hipStream_t s, const uint32_t* k_guard, uint32_t k_cap) {
    if (T > 0)
        hipLaunchKernelGGL(k_tile_sort, dim3(T), dim3(256), 0, s, T, ranges, keys, scratch, point_list, k_guard,
                           k_cap);
}

}  // namespace gsd
