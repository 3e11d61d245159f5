// Calibration (round 6): wave64 VALU throughput cost per instruction FORM on gfx950, at 4 / 5 / 8 waves per SIMD --
// the forms the render kernels' inner loops are made of (scripts/calib/valu_rate.hip covered the kinds; the
// encodings differ: VOP2 e32 vs VOP3 e64, literal vs inline constant, DPP row_newbcast, SGPR-mask selects).
// 8 independent chains per lane, inline asm so the compiler cannot repack them; cycles at the clock the kernel
// itself measured (s_memtime / s_memrealtime).
// hipcc --offload-arch=gfx950 -O3 valu_cost.hip -o valu_cost && ./valu_cost
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_MODES 22
static const char* kNames[N_MODES] = {
    "v_fma_f32 v,v,0.5",          "v_fma_f32 v,v,v",           "v_fmac_f32_e32 v,v",       "v_mul_f32_e32 v,v",
    "v_mul_f32_e64 v,v",          "v_add_f32_e32 v,v",         "v_sub_f32_e32 1.0,v",      "v_min_f32_e32 lit,v",
    "v_fmamk_f32 lit",            "v_mul_f32_dpp newbcast",    "v_sub_f32_dpp newbcast",   "v_mov_b32_dpp newbcast",
    "v_fmac_f32_dpp newbcast",    "v_cndmask_b32_e64 0,v,s",   "v_cmp_gt_i32_e64 s,v,v",   "v_cmp_ngt_f32_e64 s,0,v",
    "v_exp_f32",                  "v_rcp_f32",                 "v_add_f32_dpp row_ror:8",  "v_pk_mul_f32",
    "v_pk_fma_f32",               "v_mul_f32 + v_fma_f32 alt"};

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, int iters, float a, unsigned long long* clk) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float x[8];
    f2 y[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int i = 0; i < 8; ++i) y[i] = f2{x[i], x[(i + 1) & 7]};
    const float b = a * 0.5f;
    const f2 m = {a, a}, c = {0.5f, 0.5f};
    unsigned long long sc = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
    unsigned long long sv[4] = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (MODE == 0) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(x[i]) : "v"(a));
            if (MODE == 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
            if (MODE == 2) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
            if (MODE == 3) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
            if (MODE == 4) asm volatile("v_mul_f32_e64 %0, %1, %0" : "+v"(x[i]) : "v"(a));
            if (MODE == 5) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
            if (MODE == 6) asm volatile("v_sub_f32_e32 %0, 1.0, %0" : "+v"(x[i]));
            if (MODE == 7) asm volatile("v_min_f32_e32 %0, 0x3f7d70a4, %0" : "+v"(x[i]));
            if (MODE == 8) asm volatile("v_fmamk_f32 %0, %0, 0x3fb8aa3b, %1" : "+v"(x[i]) : "v"(a));
            if (MODE == 9)
                asm volatile("v_mul_f32_dpp %0, %1, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                             : "+v"(x[i]) : "v"(a));
            if (MODE == 10)
                asm volatile("v_sub_f32_dpp %0, %1, %0 row_newbcast:5 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                             : "+v"(x[i]) : "v"(a));
            if (MODE == 11)
                asm volatile("v_mov_b32_dpp %0, %1 row_newbcast:5 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                             : "=v"(x[i]) : "v"(x[(i + 1) & 7]));
            if (MODE == 12)
                asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                             : "+v"(x[i]) : "v"(a), "v"(b));
            if (MODE == 13) asm volatile("v_cndmask_b32_e64 %0, 0, %0, %1" : "+v"(x[i]) : "s"(sc));
            if (MODE == 14) asm volatile("v_cmp_gt_i32_e64 %0, %1, %2" : "=s"(sv[i & 3]) : "v"(x[i]), "v"(a));
            if (MODE == 15) asm volatile("v_cmp_ngt_f32_e64 %0, 0, %1" : "=s"(sv[i & 3]) : "v"(x[i]));
            if (MODE == 16) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
            if (MODE == 17) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i]));
            if (MODE == 18)
                asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x[i]));
            if (MODE == 19) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(y[i]) : "v"(m));
            if (MODE == 20) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(y[i]) : "v"(m), "v"(c));
            if (MODE == 21) {
                if (i & 1)
                    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
                else
                    asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i] + y[i].x + y[i].y;
    for (int i = 0; i < 4; ++i) s += (float)(sv[i] & 1);
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - c0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

static unsigned long long* g_clk;
template <int MODE>
double run(float* out, int blocks, int iters, double* ghz) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, iters, 0.999f, g_clk);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    unsigned long long c[2];
    (void)hipMemcpy(c, g_clk, sizeof(c), hipMemcpyDeviceToHost);
    *ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 2.4;
    return ms;
}

template <int MODE>
void sweep(float* out) {
    const int iters = 2048;
    for (int wps : {4, 5, 8}) {
        const int blocks = 256 * 4 * wps;  // 1024 SIMDs x waves per SIMD (one wave per block)
        double ghz = 2.4;
        const double ms = run<MODE>(out, blocks, iters, &ghz);
        const double n_instr = (double)wps * iters * 8;
        printf("%-28s waves/SIMD %d: %.2f cycles/instr (%.2f GHz, %.3f ms)\n", kNames[MODE], wps,
               ms * 1e-3 * ghz * 1e9 / n_instr, ghz, ms);
    }
    if constexpr (MODE + 1 < N_MODES) sweep<MODE + 1>(out);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 1 << 26);
    (void)hipMalloc(&g_clk, 16);
    sweep<0>(out);
    return 0;
}
