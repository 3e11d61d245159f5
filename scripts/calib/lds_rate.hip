// Calibration: LDS throughput of float atomics against plain stores, per CU, for the access shapes the render
// backward uses (one workgroup of four waves per SIMD quad; every CU busy).  Cycles per wave-instruction per CU
// at the shader clock the kernel itself measures (s_memtime against the 100-MHz s_memrealtime).
// hipcc --offload-arch=gfx950 -O3 lds_rate.hip -o lds_rate && ./lds_rate
#include <hip/hip_runtime.h>
#include <cstdio>

// MODE: 0 ds_add_f32, 64 lanes, distinct consecutive dwords   1 ds_write_b32, same addresses
//       2 ds_add_f32, 16 lanes active (lanes 0-15)            3 ds_add_f32, 64 lanes, 4 lanes per address
//       4 ds_add_u32, 64 lanes, distinct                       5 ds_add_f32, 64 lanes, stride-9 pitch (9 s + q)
//       7 ds_add_f32, 64 lanes, all waves of the CU on the same 64 dwords (cross-wave same-address)
//       8 float add by compare-and-swap (ds_read_b32 + ds_cmpst_rtn_b32, retried on a lost race), 64 lanes distinct
//       9 the same, every wave of the workgroup on the same 64 dwords (races between waves)
//      10 three independent CAS adds per lane in flight together (the kernel's three quantities per hand-off)
//      11 ds_add_f64, 64 lanes distinct 8-B words          12 ds_add_u64, 64 lanes distinct
//      13 ds_add_rtn_f32, 64 lanes distinct                14 ds_write_b64, 64 lanes distinct
template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters, unsigned long long* clk) {
    __shared__ float s[8192];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 8192; i += 256) s[i] = 0.f;
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned addr;
    if (MODE == 3) addr = 4u * (wave * 64 + (lane >> 2));
    else if (MODE == 5) addr = 4u * (wave * 1024 + 9 * (lane >> 2) + (lane & 3));
    else if (MODE == 7 || MODE == 9) addr = 4u * lane;
    else addr = 4u * (wave * 64 + lane);
    const float one = 1.0f;
    const unsigned ione = 1u;
    float sink = 0.f;
    if (MODE != 2 || lane < 16) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (MODE == 0 || MODE == 2 || MODE == 3 || MODE == 5 || MODE == 7)
                    asm volatile("ds_add_f32 %0, %1" ::"v"(addr), "v"(one) : "memory");
                if (MODE == 1) asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(one) : "memory");
                if (MODE == 4) asm volatile("ds_add_u32 %0, %1" ::"v"(addr), "v"(ione) : "memory");
                if (MODE == 11) asm volatile("ds_add_f64 %0, %1" ::"v"(addr * 2), "v"(1.0) : "memory");
                if (MODE == 12) asm volatile("ds_add_u64 %0, %1" ::"v"(addr * 2), "v"(1ull) : "memory");
                if (MODE == 13) {
                    float r;
                    asm volatile("ds_add_rtn_f32 %0, %1, %2" : "=v"(r) : "v"(addr), "v"(one) : "memory");
                    sink += r;
                }
                if (MODE == 14) asm volatile("ds_write_b64 %0, %1" ::"v"(addr * 2), "v"(1ull) : "memory");
                if (MODE == 8 || MODE == 9) {
                    unsigned* p = reinterpret_cast<unsigned*>(s) + addr / 4;
                    unsigned old = *reinterpret_cast<volatile unsigned*>(p);
                    while (true) {
                        const unsigned prev = atomicCAS(p, old, __float_as_uint(__uint_as_float(old) + one));
                        if (prev == old) break;
                        old = prev;
                    }
                }
                if (MODE == 10 && u < 3) {
                    unsigned* p0 = reinterpret_cast<unsigned*>(s) + addr / 4;
                    unsigned* p1 = p0 + 1024;
                    unsigned* p2 = p0 + 2048;
                    unsigned o0 = *reinterpret_cast<volatile unsigned*>(p0), o1 = *reinterpret_cast<volatile unsigned*>(p1),
                             o2 = *reinterpret_cast<volatile unsigned*>(p2);
                    bool d0 = false, d1 = false, d2 = false;
                    while (!(d0 && d1 && d2)) {
                        if (!d0) { const unsigned q = atomicCAS(p0, o0, __float_as_uint(__uint_as_float(o0) + one)); d0 = q == o0; o0 = q; }
                        if (!d1) { const unsigned q = atomicCAS(p1, o1, __float_as_uint(__uint_as_float(o1) + one)); d1 = q == o1; o1 = q; }
                        if (!d2) { const unsigned q = atomicCAS(p2, o2, __float_as_uint(__uint_as_float(o2) + one)); d2 = q == o2; o2 = q; }
                    }
                }
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - c0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    out[blockIdx.x * 256 + threadIdx.x] = s[threadIdx.x] + sink;
}

static unsigned long long* g_clk;
template <int MODE>
void run(const char* name, float* out, int wg_per_cu, int iters) {
    const int blocks = 256 * wg_per_cu;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, g_clk);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    unsigned long long c[2];
    (void)hipMemcpy(c, g_clk, sizeof(c), hipMemcpyDeviceToHost);
    const double ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 2.4;
    const double instr_per_cu = (double)wg_per_cu * 4 * iters * (MODE == 10 ? 9 : 8);  // updates
    printf("%-44s WG/CU %d: %6.2f cycles per wave-instruction (update) per CU (%.2f GHz, %.3f ms)\n", name, wg_per_cu,
           ms * 1e-3 * ghz * 1e9 / instr_per_cu, ghz, ms);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
    (void)hipMalloc(&g_clk, 16);
    const int iters = 2048;
    for (int w : {1, 4}) {
        run<0>("ds_add_f32 64 lanes distinct", out, w, iters);
        run<1>("ds_write_b32 64 lanes distinct", out, w, iters);
        run<2>("ds_add_f32 16 lanes distinct", out, w, iters);
        run<3>("ds_add_f32 64 lanes, 4 per address", out, w, iters);
        run<4>("ds_add_u32 64 lanes distinct", out, w, iters);
        run<5>("ds_add_f32 64 lanes, 9 s + q pattern", out, w, iters);
        run<7>("ds_add_f32 64 lanes, every wave same 64", out, w, iters);
        run<8>("CAS float add 64 lanes distinct", out, w, iters);
        run<9>("CAS float add, every wave same 64", out, w, iters);
        run<10>("3 CAS float adds in flight, distinct", out, w, iters);
        run<11>("ds_add_f64 64 lanes distinct", out, w, iters);
        run<12>("ds_add_u64 64 lanes distinct", out, w, iters);
        run<13>("ds_add_rtn_f32 64 lanes distinct", out, w, iters);
        run<14>("ds_write_b64 64 lanes distinct", out, w, iters);
    }
    return 0;
}
