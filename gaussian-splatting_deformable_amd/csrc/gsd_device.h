// gsd_device.h -- device-side building blocks shared by the gfx950 kernels.
//
// Numerics contract: the library is compiled with -ffp-contract=off and every
// expression below keeps the evaluation order of the reference's glm/CUDA
// code (cited per function), so preprocess outputs are bit-identical to the
// un-contracted float32 arithmetic of the reference (DESIGN.md "Numerics").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsd {

constexpr int kTileX = 16;  // config.h:16 -- part of the bit-exact key contract
constexpr int kTileY = 16;  // config.h:17
constexpr int kTilePix = kTileX * kTileY;

// auxiliary.h:22-39
constexpr float kSH0 = 0.28209479177387814f;
constexpr float kSH1 = 0.4886025119029199f;
constexpr float kSH2_0 = 1.0925484305920792f, kSH2_1 = -1.0925484305920792f, kSH2_2 = 0.31539156525252005f,
                kSH2_3 = -1.0925484305920792f, kSH2_4 = 0.5462742152960396f;
constexpr float kSH3_0 = -0.5900435899266435f, kSH3_1 = 2.890611442640554f, kSH3_2 = -0.4570457994644658f,
                kSH3_3 = 0.3731763325901154f, kSH3_4 = -0.4570457994644658f, kSH3_5 = 1.445305721320277f,
                kSH3_6 = -0.5900435899266435f;

// F.relu as torch computes it (clamp_min): NaN propagates -- fmaxf(NaN, 0) would return 0 and hide a diverging
// network behind finite outputs and zero gradients
__device__ __forceinline__ float relu_nan(float v) { return __builtin_elementwise_maximum(v, 0.f); }

// The 4x4 camera matrices, read once per block into SGPR-resident registers.
struct Mat4 {
    float m[16];
};

__device__ __forceinline__ Mat4 load_mat4(const float* __restrict__ p) {
    Mat4 r;
#pragma unroll
    for (int i = 0; i < 16; ++i) r.m[i] = p[i];
    return r;
}

// auxiliary.h:58-66 transformPoint4x3
__device__ __forceinline__ float3 xform_point3(const float3 p, const Mat4& m) {
    return make_float3(m.m[0] * p.x + m.m[4] * p.y + m.m[8] * p.z + m.m[12],
                       m.m[1] * p.x + m.m[5] * p.y + m.m[9] * p.z + m.m[13],
                       m.m[2] * p.x + m.m[6] * p.y + m.m[10] * p.z + m.m[14]);
}
// auxiliary.h:68-77 transformPoint4x4
__device__ __forceinline__ float4 xform_point4(const float3 p, const Mat4& m) {
    return make_float4(m.m[0] * p.x + m.m[4] * p.y + m.m[8] * p.z + m.m[12],
                       m.m[1] * p.x + m.m[5] * p.y + m.m[9] * p.z + m.m[13],
                       m.m[2] * p.x + m.m[6] * p.y + m.m[10] * p.z + m.m[14],
                       m.m[3] * p.x + m.m[7] * p.y + m.m[11] * p.z + m.m[15]);
}
// auxiliary.h:89-97 transformVec4x3Transpose
__device__ __forceinline__ float3 xform_vec3_T(const float3 p, const Mat4& m) {
    return make_float3(m.m[0] * p.x + m.m[1] * p.y + m.m[2] * p.z, m.m[4] * p.x + m.m[5] * p.y + m.m[6] * p.z,
                       m.m[8] * p.x + m.m[9] * p.y + m.m[10] * p.z);
}

// auxiliary.h:41-44 ndc2Pix (a double expression upstream: literals 1.0 / 0.5)
__device__ __forceinline__ float ndc_to_pix(float v, int S) {
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

// auxiliary.h:46-56 getRect, clamped to the tile grid
struct Rect {
    int x0, y0, x1, y1;
};
__device__ __forceinline__ Rect tile_rect(float px, float py, int radius, int gx, int gy) {
    const float r = (float)radius;
    Rect o;
    o.x0 = min(gx, max(0, (int)((px - r) / (float)kTileX)));
    o.y0 = min(gy, max(0, (int)((py - r) / (float)kTileY)));
    o.x1 = min(gx, max(0, (int)((px + r + (float)kTileX - 1.0f) / (float)kTileX)));
    o.y1 = min(gy, max(0, (int)((py + r + (float)kTileY - 1.0f) / (float)kTileY)));
    return o;
}

// Column-major 3x3 (glm convention): c[k] is column k.
struct M3 {
    float3 c[3];
};
// glm operator*(mat3,mat3) (type_mat3x3.inl:486-520): R[c][r] = (A0r*Bc0 + A1r*Bc1) + A2r*Bc2
__device__ __forceinline__ float3 m3_col(const M3& A, const float3 b) {
    return make_float3(A.c[0].x * b.x + A.c[1].x * b.y + A.c[2].x * b.z,
                       A.c[0].y * b.x + A.c[1].y * b.y + A.c[2].y * b.z,
                       A.c[0].z * b.x + A.c[1].z * b.y + A.c[2].z * b.z);
}
__device__ __forceinline__ M3 m3_mul(const M3& A, const M3& B) {
    M3 R;
    R.c[0] = m3_col(A, B.c[0]);
    R.c[1] = m3_col(A, B.c[1]);
    R.c[2] = m3_col(A, B.c[2]);
    return R;
}
__device__ __forceinline__ M3 m3_T(const M3& A) {
    M3 R;
    R.c[0] = make_float3(A.c[0].x, A.c[1].x, A.c[2].x);
    R.c[1] = make_float3(A.c[0].y, A.c[1].y, A.c[2].y);
    R.c[2] = make_float3(A.c[0].z, A.c[1].z, A.c[2].z);
    return R;
}
__device__ __forceinline__ M3 m3_cols(float a, float b, float c, float d, float e, float f, float g, float h,
                                      float i) {
    M3 R;
    R.c[0] = make_float3(a, b, c);
    R.c[1] = make_float3(d, e, f);
    R.c[2] = make_float3(g, h, i);
    return R;
}
__device__ __forceinline__ float dot3(const float3 a, const float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// Quaternion (r,x,y,z) -> glm rotation matrix of forward.cu:134-138 / backward.cu:287-291
__device__ __forceinline__ M3 quat_to_R(const float4 q) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    return m3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                   2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                   2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
}

// forward.cu:118-152 computeCov3D (no quaternion normalisation, :127)
struct Cov6 {
    float v[6];
};
__device__ __forceinline__ Cov6 cov3d_from_scale_rot(const float3 s, float mod, const float4 q) {
    M3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.c[0].x = mod * s.x;
    S.c[1].y = mod * s.y;
    S.c[2].z = mod * s.z;
    const M3 R = quat_to_R(q);
    const M3 M = m3_mul(S, R);
    const M3 Sig = m3_mul(m3_T(M), M);
    Cov6 o;
    o.v[0] = Sig.c[0].x; o.v[1] = Sig.c[0].y; o.v[2] = Sig.c[0].z;
    o.v[3] = Sig.c[1].y; o.v[4] = Sig.c[1].z; o.v[5] = Sig.c[2].z;
    return o;
}

// ---- wave64 reductions (DPP; full sum lands in lane 63, returned wave-uniform) ----
template <int CTRL, int ROWMASK, int BANKMASK>
__device__ __forceinline__ float dpp_step(float v) {
    const int t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, BANKMASK, false);
    return v + __int_as_float(t);
}
// quad_perm[1,0,3,2] -> quad_perm[2,3,0,1] -> row_shr:4 -> row_shr:8 -> row_bcast:15 -> row_bcast:31
__device__ __forceinline__ float wave_sum(float v) {
    v = dpp_step<0xb1, 0xf, 0xf>(v);
    v = dpp_step<0x4e, 0xf, 0xf>(v);
    v = dpp_step<0x114, 0xf, 0xe>(v);
    v = dpp_step<0x118, 0xf, 0xc>(v);
    v = dpp_step<0x142, 0xa, 0xf>(v);
    v = dpp_step<0x143, 0xc, 0xf>(v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Ballot of a bool straight from its lane mask.  HIP's __ballot(int) converts the bool to an int and back,
// which the compiler emits as v_cndmask 0/1 + v_cmp_ne (two VALU ops per ballot in the render loops).
__device__ __forceinline__ unsigned long long wave_ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Four-column variant: returns, in every lane l, the 64-lane total of column (l >> 4).
// permlane32 swap (distance 32), permlane16 swap (16), then a full 16-lane row reduction by DPP:
// ~10 VALU ops for 4 sums, with half the live registers of wave_sum8's inputs.
__device__ __forceinline__ float wave_sum4(const float (&c)[4]) {
    float s[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // low half keeps column k, high half column k+2
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(c[k]), __float_as_uint(c[k + 2]), false,
                                                        false);
        s[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s[0]), __float_as_uint(s[1]), false, false);
    float t = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // row q of the wave now holds column q
    t = dpp_step<0xb1, 0xf, 0xf>(t);   // quad_perm [1,0,3,2]
    t = dpp_step<0x4e, 0xf, 0xf>(t);   // quad_perm [2,3,0,1]
    t = dpp_step<0x141, 0xf, 0xf>(t);  // row_half_mirror
    t = dpp_step<0x140, 0xf, 0xf>(t);  // row_mirror
    return t;
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup
// release/acquire fence plus s_barrier, and the release makes every wave wait
// for its outstanding global stores and atomics (s_waitcnt vmcnt(0)) before it
// may arrive -- a full memory round trip after each flush of gradient atomics.
// Here only the LDS traffic is drained (lgkmcnt(0)); global writes stay in
// flight across the barrier (nothing in the workgroup reads them back).
__device__ __forceinline__ void lds_barrier() {
    // the "memory" clobber keeps the compiler from moving LDS accesses across it
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Hand-off of LDS data between lanes of one wave.  The wave's LDS instructions execute in issue order, so
// only the compiler has to be stopped from reordering them: it reasons per lane, and a load of another lane's
// slot whose address provably differs from this lane's stores may otherwise be hoisted above them
// (__builtin_amdgcn_wave_barrier alone is not a memory barrier to the compiler).
__device__ __forceinline__ void wave_lds_handoff() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// wave_sum4 in two halves, so columns 0/1 can be folded as soon as they exist
// (fewer live registers): pair32(c0, c1) leaves lanes 0-31 with column 0 and
// lanes 32-63 with column 1 (each over lane l and l ^ 32); fin16(pair32(c0, c1),
// pair32(c2, c3)) returns in every lane the 64-lane total of column
// kPair16Col[lane >> 4] = {0, 2, 1, 3}.
__device__ __forceinline__ float pair32(float a, float b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float fin16(float h01, float h23) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(h01), __float_as_uint(h23), false, false);
    float t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    t = dpp_step<0xb1, 0xf, 0xf>(t);   // quad_perm [1,0,3,2]
    t = dpp_step<0x4e, 0xf, 0xf>(t);   // quad_perm [2,3,0,1]
    t = dpp_step<0x141, 0xf, 0xf>(t);  // row_half_mirror
    t = dpp_step<0x140, 0xf, 0xf>(t);  // row_mirror
    return t;
}
__device__ __forceinline__ int fin16_column(int lane) { return (((lane >> 4) & 1) << 1) | (lane >> 5); }
// Distance-16 transposed step: lanes with bit 4 clear return a summed over lanes l and l ^ 16, lanes with
// bit 4 set return b summed the same way.
__device__ __forceinline__ float pair16(float a, float b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Distance-4 step after sum8 (row_ror:4): lanes with bits 2-3 clear return the sum over lanes l, l ^ 4,
// l ^ 8, l ^ 12 of the input to sum8.
__device__ __forceinline__ float sum4(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, true));
}
// Lane (l & ~3) + i's value in every lane of the quad (DPP quad_perm [i, i, i, i]).
template <int I>
__device__ __forceinline__ float quad_bcast(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), I * 0x55, 0xf, 0xf, false));
}
// Distance-8 step (row_ror:8 == lane ^ 8 inside a 16-lane row): every lane returns v(l) + v(l ^ 8).
__device__ __forceinline__ float sum8(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, true));
}

// Transposed butterfly: c[k] is this lane's value for column k (k = 0..7).
// Returns, in every lane l, the 64-lane total of column (l >> 3).  Six
// exchange levels serve all eight columns at once (v_permlane32_swap for lane
// distance 32, v_permlane16_swap for 16, DPP row_ror:8 for 8, then quad /
// half-row DPP), ~18 VALU ops for 8 sums instead of 8 x 6 DPP adds +
// readlanes of eight separate wave_sum()s.
__device__ __forceinline__ float wave_sum8(const float (&c)[8]) {
    float s[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // distance 32: low half keeps column k, high half column k+4
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(c[k]), __float_as_uint(c[k + 4]), false,
                                                        false);
        s[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    float u[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // distance 16: even rows keep s[k], odd rows s[k+2]
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s[k]), __float_as_uint(s[k + 2]), false,
                                                        false);
        u[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    // distance 8 (row_ror:8 == lane ^ 8 inside a 16-lane row): lanes 0-7 keep u[0], lanes 8-15 keep u[1]
    const bool hi8 = (threadIdx.x & 8) != 0;
    const float send = hi8 ? u[0] : u[1];
    const float keep = hi8 ? u[1] : u[0];
    float t = keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x128, 0xf, 0xf, false));
    // distances 1, 2, 4 inside each 8-lane group
    t = dpp_step<0xb1, 0xf, 0xf>(t);
    t = dpp_step<0x4e, 0xf, 0xf>(t);
    t = dpp_step<0x141, 0xf, 0xf>(t);  // row_half_mirror: quad sums are uniform, so this adds the other quad
    return t;
}

// Capacity guard of a launch queued before num_rendered reached the host (gsd_rasterize_forward): true
// when the count the tile scan wrote exceeds what the binning buffer holds -- the launch then does nothing
// and the host re-runs it with a buffer of the right size.  One uniform (scalar) load per workgroup.
__device__ __forceinline__ bool over_capacity(const uint32_t* k_guard, uint32_t k_cap) {
    return k_guard != nullptr && *k_guard > k_cap;
}

// XCD-aware remap of a 1-D block index: blocks b and b+8 are dealt to the same
// XCD (MI355X_MICROARCH.md "Workgroup dispatch"), so give each XCD a
// contiguous run of tiles -- neighbouring tiles gather the same Gaussians and
// then share that XCD's L2.  Speed only; any placement is correct.
__device__ __forceinline__ int xcd_swizzle(int b, int n) {
    const int full = n & ~7;
    if (b >= full) return b;
    const int per = full >> 3;
    return (b & 7) * per + (b >> 3);
}

}  // namespace gsd
