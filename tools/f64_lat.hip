// Dependent-chain latency of the RANSAC kernel's building blocks on one wave (s_memtime cycles per
// link): v_add_f64, v_mul_f64, v_fma_f64, an f64 division (the compiler's div_scale / rcp / fma /
// div_fmas / div_fixup sequence), ds_bpermute_b32 round trips, v_pk_add_f32, a v_cmp_f64 +
// v_cndmask select step.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/f64_lat tools/f64_lat.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 256

__device__ __forceinline__ unsigned long long clk()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ void k_lat(const double* in, double* out, unsigned long long* cyc)
{
    double a = in[threadIdx.x], b = in[64 + threadIdx.x];
    float2 p = make_float2((float)a, (float)b);
    int idx = threadIdx.x;
    unsigned long long t0, t1;
    // add chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; ++i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(b));
    t1 = clk();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    // mul chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; ++i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b));
    t1 = clk();
    if (threadIdx.x == 0) cyc[1] = t1 - t0;
    // fma chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; ++i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    t1 = clk();
    if (threadIdx.x == 0) cyc[2] = t1 - t0;
    // division chain (compiler sequence)
    double q = a;
    t0 = clk();
#pragma unroll 4
    for (int i = 0; i < N / 8; ++i) {
        q = b / q;
        asm volatile("" : "+v"(q));
    }
    t1 = clk();
    if (threadIdx.x == 0) cyc[3] = (t1 - t0) * 8;    // per 8 links, reported per N
    // ds_bpermute chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; ++i) idx = __builtin_amdgcn_ds_bpermute(idx << 2, idx) ^ 1;
    t1 = clk();
    if (threadIdx.x == 0) cyc[4] = t1 - t0;
    // pk_add_f32 chain
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; ++i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p) : "v"(p));
    t1 = clk();
    if (threadIdx.x == 0) cyc[5] = t1 - t0;
    // two independent add chains interleaved (throughput of two links)
    double c = b;
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; ++i) {
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(b));
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(c) : "v"(b));
    }
    t1 = clk();
    if (threadIdx.x == 0) cyc[6] = t1 - t0;
    // compare + select step on f64 (tournament link)
    double m = a;
    t0 = clk();
#pragma unroll 16
    for (int i = 0; i < N; ++i) {
        m = b > m ? b : m;
        asm volatile("" : "+v"(m), "+v"(b));
    }
    t1 = clk();
    if (threadIdx.x == 0) cyc[7] = t1 - t0;
    out[threadIdx.x] = a + c + q + (double)idx + p.x + p.y + m;
}

int main()
{
    double h[128];
    for (int i = 0; i < 128; ++i) h[i] = 1.0 + i * 1e-3;
    double *din, *dout;
    unsigned long long* dc;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, 64 * sizeof(double));
    hipMalloc(&dc, 8 * sizeof(unsigned long long));
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[8] = {"v_add_f64", "v_mul_f64", "v_fma_f64", "f64 division", "ds_bpermute_b32",
                            "v_pk_add_f32", "2 interleaved v_add_f64 chains (per pair)", "f64 compare+select"};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, din, dout, dc);
        unsigned long long c[8];
        if (hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
        if (rep < 2) continue;
        for (int i = 0; i < 8; ++i) printf("%-44s %6.1f cycles per link\n", names[i], (double)c[i] / N);
    }
    return 0;
}
