// Negative controls for tests/isa_hazards.py (compiled and disassembled by tests/test_isa_hazards.py on
// the CPU; never launched).  k_bad holds one deliberate wait-state violation per rule, each inside an
// inline-asm statement (hipcc pads none of them); k_good holds the same sequences with the wait states
// the rules ask for.  The checker must flag every rule in k_bad and nothing in k_good.
#include <hip/hip_runtime.h>
typedef float f2 __attribute__((ext_vector_type(2)));

extern "C" __global__ void k_bad(float* o, const float* a, int s)
{
    float x = a[threadIdx.x], y = a[threadIdx.x + 64], r0, r1, r2, r3, r4, r5, r6;
    int q;
    unsigned long long m;
    asm volatile("v_mul_f32 %0, %1, %1\n\tv_mov_b32_dpp %2, %0 wave_shr:1 row_mask:0xf bank_mask:0xf"
                 : "=&v"(r0), "+v"(x), "=&v"(r1));                                        // VALU -> DPP src0
    asm volatile("v_cmp_lt_f32_e64 %0, %2, %3\n\tv_cndmask_b32_e64 %1, %2, %3, %0"
                 : "=&s"(m), "=&v"(r2) : "v"(x), "v"(y));                                 // VALU SGPR -> VALU
    f2 p2 = {x, y}, p3, p4;
    asm volatile("v_pk_mul_f32 %0, %2, %2\n\tv_pk_add_f32 %1, %0, %2" : "=&v"(p3), "=&v"(p4) : "v"(p2));   // v_pk_*_f32 -> VALU
    r3 = p3.x; r4 = p4.y;
    asm volatile("v_sqrt_f32 %0, %1\n\tv_add_f32 %0, %0, %1" : "=&v"(r5) : "v"(y));       // trans -> VALU
    asm volatile("v_mul_f32 %1, %2, %2\n\tv_readfirstlane_b32 %0, %1" : "=&s"(q), "=&v"(r6) : "v"(x));   // VALU -> readfirstlane
    o[threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + (float)q + (float)(m & 1);
}

extern "C" __global__ void k_good(float* o, const float* a, int s)
{
    float x = a[threadIdx.x], y = a[threadIdx.x + 64], r0, r1, r2, r3, r4, r5, r6;
    int q;
    unsigned long long m;
    asm volatile("v_mul_f32 %0, %1, %1\n\ts_nop 1\n\tv_mov_b32_dpp %2, %0 wave_shr:1 row_mask:0xf bank_mask:0xf"
                 : "=&v"(r0), "+v"(x), "=&v"(r1));
    asm volatile("v_cmp_lt_f32_e64 %0, %2, %3\n\ts_nop 1\n\tv_cndmask_b32_e64 %1, %2, %3, %0"
                 : "=&s"(m), "=&v"(r2) : "v"(x), "v"(y));
    f2 p2 = {x, y}, p3, p4;
    asm volatile("v_pk_mul_f32 %0, %2, %2\n\ts_nop 0\n\tv_pk_add_f32 %1, %0, %2" : "=&v"(p3), "=&v"(p4) : "v"(p2));
    r3 = p3.x; r4 = p4.y;
    asm volatile("v_sqrt_f32 %0, %1\n\ts_nop 0\n\tv_add_f32 %0, %0, %1" : "=&v"(r5) : "v"(y));
    asm volatile("v_mul_f32 %1, %2, %2\n\ts_nop 0\n\tv_readfirstlane_b32 %0, %1\n\ts_nop 1" : "=&s"(q), "=&v"(r6) : "v"(x));
    asm volatile("s_nop 4" ::: "memory");
    o[threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + (float)q + (float)(m & 1);
}
