// VALU issue-rate calibration on gfx950: waves of independent chains of one instruction kind,
// timed with HIP events; prints wave64 instructions per SIMD per cycle at the measured clock
// (cycles from s_memtime over the kernel).  hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITER 4096
template <int KIND>
__global__ void __launch_bounds__(256) k_rate(float* out, unsigned long long* clk, float a, float b)
{
    unsigned long long t0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 y[4];
    for (int i = 0; i < 4; ++i) y[i] = f2{x[2 * i], x[2 * i + 1]};
    uint32_t u[8];
    for (int i = 0; i < 8; ++i) u[i] = threadIdx.x + i;
    double dd[8];
    for (int i = 0; i < 8; ++i) dd[i] = x[i];
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "s"(a), "v"(x[(i + 1) & 7]));
            if (KIND == 1 && i < 4) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(y[i]) : "v"(y[(i + 1) & 3]));
            if (KIND == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "s"(a));
            if (KIND == 3) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(dd[i]) : "v"(dd[(i + 1) & 7]));
            if (KIND == 4) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(u[i]));
        }
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i] + (float)u[i] + (float)dd[i];
    for (int i = 0; i < 4; ++i) s += y[i].x + y[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, int per_kind_instrs)
{
    const int blocks = 1024 * 8 / 4;          // 8 waves per SIMD (4-wave blocks over 1024 SIMDs)
    float* out; unsigned long long* clk;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    hipMalloc(&clk, sizeof(unsigned long long) * blocks);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k_rate<KIND>, dim3(blocks), dim3(256), 0, 0, out, clk, 1.0001f, 0.5f);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate<KIND>, dim3(blocks), dim3(256), 0, 0, out, clk, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[16]; hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    const double waves = blocks * 4.0, instr = (double)ITER * per_kind_instrs;
    const double per_simd = waves * instr / 1024.0;          // wave64 instructions per SIMD
    const double ghz_guess = 2.4;
    printf("%-14s %8.3f ms  %6.2f wave-instr/SIMD/ns  -> %.2f cycles per wave64 instr at %.1f GHz  (s_memtime per wave %llu)\n",
           name, ms, per_simd / (ms * 1e6), ms * 1e6 * ghz_guess / per_simd, ghz_guess, h[0]);
    hipFree(out); hipFree(clk);
}

int main()
{
    run<0>("v_fma_f32", 8);
    run<1>("v_pk_fma_f32", 4);
    run<2>("v_add_u32", 8);
    run<3>("v_fma_f64", 8);
    run<4>("v_mov_b32_dpp", 8);
    return 0;
}
