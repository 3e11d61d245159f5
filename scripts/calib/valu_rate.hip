// Calibration: wave64 VALU issue cost on one SIMD at 1-8 waves/SIMD, per instruction kind
// (8 independent chains per lane, inline asm so the compiler cannot repack them).
// hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, int iters, float a, unsigned long long* clk) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float x[8];
    f2 y[4];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int i = 0; i < 4; ++i) y[i] = f2{x[2 * i], x[2 * i + 1]};
    const f2 m = {a, a}, c = {0.5f, 0.5f};
    unsigned long long sc = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
    unsigned long long sv[4] = {0, 0, 0, 0};
    asm volatile("v_cmp_gt_f32 vcc, %0, %1" :: "v"(x[0]), "v"(a) : "vcc");
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (MODE == 0) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(x[i]) : "v"(a));
            if (MODE == 1) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
            if (MODE == 2)
                asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
            if (MODE == 4 && (i & 1)) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x[i - 1]), "+v"(x[i]));
            if (MODE == 5) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i]));
            if (MODE == 6) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
            if (MODE == 7) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(a));
            if (MODE == 8) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "s"(sc));
            if (MODE == 9) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
            if (MODE == 10) asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 1) & 7]));
            if (MODE == 11) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x[i]));
            if (MODE == 12) asm volatile("v_cmp_gt_f32 vcc, %0, %1" :: "v"(x[i]), "v"(a) : "vcc");
            if (MODE == 13) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(sv[i & 3]) : "v"(x[i]), "v"(a));
        }
        if (MODE == 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(y[i]) : "v"(m), "v"(c));
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    for (int i = 0; i < 4; ++i) s += y[i].x + y[i].y + (float)(sv[i] & 1);
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // shader clock: s_memtime ticks per 100-MHz s_memrealtime tick
        clk[0] = __builtin_amdgcn_s_memtime() - c0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

static unsigned long long* g_clk;
static double g_ghz = 2.4;
template <int MODE>
float run(float* out, int blocks, int iters) {
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
    g_ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 2.4;
    return ms;
}

int main() {
    float* out;
    (void)hipMalloc(&out, 1 << 26);
    (void)hipMalloc(&g_clk, 16);
    const int iters = 4096;
    const char* names[14] = {"v_fma_f32", "v_exp_f32", "v_add_f32_dpp", "v_pk_fma_f32", "v_permlane32_swap",
                             "v_rcp_f32", "v_mul_f32", "v_cndmask_b32 vcc", "v_cndmask_b32 sgpr", "v_max_f32",
                             "v_mov_b32", "v_lshlrev_b32", "v_cmp vcc", "v_cmp_e64 sgpr"};
    for (int mode = 0; mode < 14; ++mode) {
        for (int wps : {4, 8}) {
            const int blocks = 256 * 4 * wps;  // 1024 SIMDs x waves per SIMD (one wave per block)
            float ms = 0;
            switch (mode) {
                case 0: ms = run<0>(out, blocks, iters); break;
                case 1: ms = run<1>(out, blocks, iters); break;
                case 2: ms = run<2>(out, blocks, iters); break;
                case 3: ms = run<3>(out, blocks, iters); break;
                case 4: ms = run<4>(out, blocks, iters); break;
                case 5: ms = run<5>(out, blocks, iters); break;
                case 6: ms = run<6>(out, blocks, iters); break;
                case 7: ms = run<7>(out, blocks, iters); break;
                case 8: ms = run<8>(out, blocks, iters); break;
                case 9: ms = run<9>(out, blocks, iters); break;
                case 10: ms = run<10>(out, blocks, iters); break;
                case 11: ms = run<11>(out, blocks, iters); break;
                case 12: ms = run<12>(out, blocks, iters); break;
                default: ms = run<13>(out, blocks, iters); break;
            }
            const double n_instr = (double)wps * iters * (mode == 3 || mode == 4 ? 4 : 8);
            printf("%-20s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD at the measured %.2f GHz "
                   "(%.2f at 2.4 GHz; %.3f ms)\n", names[mode], wps, ms * 1e-3 * g_ghz * 1e9 / n_instr, g_ghz,
                   ms * 1e-3 * 2.4e9 / n_instr, ms);
        }
    }
    return 0;
}
