// Probe: which offsets of a raw buffer access (stride 0) take part in gfx950's range check?
//
// k_stencil (acs_visual_odometry_amd/csrc/vo_kernels.hip) drops stores with an out-of-range
// buffer offset instead of a branch: halo lanes by their voffset, and (round 3) the rows past a
// segment by an out-of-range *soffset*.  Whether soffset takes part in the check or is only added
// to the address (then such a store would land 1 GiB past the plane) was unverified.  Measured on
// MI355X: the check covers voffset + soffset -- stores and loads past num_records are dropped
// (loads return 0) whichever operand carries the offset, and a straddling access is cut at
// num_records.  tests/test_buffer_range.py asserts exactly that.
//
// One 1 GiB + 1 MiB allocation filled with 0xAB; the descriptor covers its first 4096 bytes.
//   case 0: store, voffset = 2 lane,              soffset = 0x40000000
//   case 1: store, voffset = 0x40000000 + 2 lane, soffset = 0
//   case 2: store, voffset = 4000 + 2 lane,       soffset = 0      (straddles num_records)
//   case 3: store, voffset = 2 lane,              soffset = 4000   (straddles with soffset)
//   case 4: load,  voffset = 2 lane,              soffset = 0x40000000 (of a 0x5A5A pattern)
//   case 5: atomic add of 1 (u32), voffset = 0x40000000 + 4 lane (out of range)
//   case 6: atomic add of 1 (u32), voffset = 4 lane (in range)
// Output: one JSON object per case on stdout.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define DW3 0x00020000
static constexpr size_t GIB = 1ull << 30;
static constexpr size_t TOTAL = GIB + (1u << 20);

__global__ void k_probe(uint8_t* base, int mode, uint16_t* loaded)
{
    const int lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 4096, DW3);
    const unsigned short v = (unsigned short)(0x1200 + lane);
    switch (mode) {
    case 0: __builtin_amdgcn_raw_buffer_store_b16(v, r, 2 * lane, 0x40000000, 0); break;
    case 1: __builtin_amdgcn_raw_buffer_store_b16(v, r, 0x40000000 + 2 * lane, 0, 0); break;
    case 2: __builtin_amdgcn_raw_buffer_store_b16(v, r, 4000 + 2 * lane, 0, 0); break;
    case 3: __builtin_amdgcn_raw_buffer_store_b16(v, r, 2 * lane, 4000, 0); break;
    case 4: loaded[lane] = __builtin_amdgcn_raw_buffer_load_b16(r, 2 * lane, 0x40000000, 0); break;
    case 5: (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, r, 0x40000000 + 4 * lane, 0, 0); break;
    case 6: (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, r, 4 * lane, 0, 0); break;
    }
}

static int check(hipError_t e, const char* what)
{
    if (e != hipSuccess) {
        fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
        return 1;
    }
    return 0;
}

int main()
{
    uint8_t* d = nullptr;
    uint16_t* dl = nullptr;
    if (check(hipMalloc(&d, TOTAL), "hipMalloc") || check(hipMalloc(&dl, 128), "hipMalloc")) return 1;
    std::vector<uint16_t> lo(2048), hi(64), ld(64);
    for (int mode = 0; mode < 7; ++mode) {
        if (check(hipMemset(d, 0xAB, TOTAL), "memset")) return 1;
        if (mode == 4 && check(hipMemset(d + GIB, 0x5A, 128), "memset")) return 1;
        if (check(hipMemset(dl, 0, 128), "memset")) return 1;
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d, mode, dl);
        if (check(hipDeviceSynchronize(), "kernel")) return 1;
        if (check(hipMemcpy(lo.data(), d, 4096, hipMemcpyDeviceToHost), "d2h")) return 1;
        if (check(hipMemcpy(hi.data(), d + GIB, 128, hipMemcpyDeviceToHost), "d2h")) return 1;
        if (check(hipMemcpy(ld.data(), dl, 128, hipMemcpyDeviceToHost), "d2h")) return 1;
        // lanes whose value landed: in the descriptor's range (by byte offset) and at +1 GiB
        int in_range = 0, at_gib = 0, first_lo = -1, last_lo = -1;
        for (int i = 0; i < 2048; ++i)
            if (lo[i] != 0xABAB) {
                ++in_range;
                if (first_lo < 0) first_lo = 2 * i;
                last_lo = 2 * i;
            }
        const uint16_t fill_hi = mode == 4 ? 0x5A5A : 0xABAB;
        for (int i = 0; i < 64; ++i) at_gib += hi[i] != fill_hi;
        int loaded_pattern = 0;
        int loaded_zero = 0;
        for (int i = 0; i < 64; ++i) {
            loaded_pattern += ld[i] == 0x5A5A;
            loaded_zero += mode == 4 && ld[i] == 0;
        }
        int atomics_in_range = 0;
        if (mode >= 5) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(lo.data());
            for (int i = 0; i < 64; ++i) atomics_in_range += w[i] == 0xABABABABu + 1u;
        }
        printf("{\"atomics_in_range\": %d, \"case\": %d, \"stores_in_range\": %d, \"first_byte\": %d, \"last_byte\": %d, "
               "\"stores_at_1gib\": %d, \"loads_of_1gib_pattern\": %d, \"loads_zero\": %d}\n",
               atomics_in_range, mode, in_range, first_lo, last_lo, at_gib, loaded_pattern, loaded_zero);
    }
    (void)hipFree(d);
    (void)hipFree(dl);
    return 0;
}
