// fetch_calib -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths
// the VO kernels use (MI355X_MICROARCH.md 'HBM': FETCH_SIZE reads 1/2 of the bytes of 16-B/lane
// streaming reads; other widths are uncalibrated).  Each kernel touches a 512 MiB buffer (twice
// the Infinity Cache) exactly once with one access width; compare the counters per dispatch with
// the byte count printed here:
//   rocprofv3 --pmc FETCH_SIZE -d <dir> -o fetch -- ./fetch_calib
//   rocprofv3 --pmc WRITE_SIZE -d <dir> -o write -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

// reads: every lane reads `T` elements at consecutive addresses across the wave (grid-stride)
template <typename T>
__global__ void rd(const T* __restrict__ a, size_t n, unsigned* out)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if constexpr (sizeof(T) == 16) {
            const uint4 v = reinterpret_cast<const uint4*>(a)[i];
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else {
            acc += (unsigned)a[i];
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;      // keeps the loads (a sum can reach it; the fill makes it unlikely)
}

// describe-like gathers: each lane reads single bytes at pseudo-random offsets of a 466 KB plane
// (one plane per workgroup row of the grid), `per` bytes per lane
__global__ void gather(const unsigned char* __restrict__ a, size_t planes, size_t plane, int per, unsigned* out)
{
    const size_t p = blockIdx.x % planes;
    const unsigned char* b = a + p * plane;
    unsigned acc = 0, x = blockIdx.x * 256u + threadIdx.x + 1u;
    for (int k = 0; k < per; ++k) {
        x = x * 1664525u + 1013904223u;
        acc += b[(x >> 8) % plane];
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

template <typename T>
__global__ void wr(T* __restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if constexpr (sizeof(T) == 16) reinterpret_cast<uint4*>(a)[i] = make_uint4(1u, 2u, 3u, (unsigned)i);
        else a[i] = (T)i;
    }
}

int main()
{
    const size_t bytes = (size_t)512 << 20;
    uint8_t* buf;
    unsigned* out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 1, bytes));
    const dim3 g(256 * 8 * 4), b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(rd<uint4>, g, b, 0, 0, (const uint4*)buf, bytes / 16, out);
        hipLaunchKernelGGL(rd<unsigned>, g, b, 0, 0, (const unsigned*)buf, bytes / 4, out);
        hipLaunchKernelGGL(rd<unsigned char>, g, b, 0, 0, (const unsigned char*)buf, bytes, out);
        // every byte of 1024 planes of 466,616 B (KITTI frames) is touched about 4 times
        hipLaunchKernelGGL(gather, dim3(1024 * 32), b, 0, 0, (const unsigned char*)buf, (size_t)1024, (size_t)466616,
                           228, out);
        hipLaunchKernelGGL(wr<uint4>, g, b, 0, 0, (uint4*)buf, bytes / 16);
        hipLaunchKernelGGL(wr<unsigned>, g, b, 0, 0, (unsigned*)buf, bytes / 4);
        hipLaunchKernelGGL(wr<unsigned char>, g, b, 0, 0, (unsigned char*)buf, bytes);
    }
    CHECK(hipDeviceSynchronize());
    std::printf("{\"bytes_per_dispatch\": %zu, \"gather_planes_bytes\": %zu}\n", bytes, (size_t)1024 * 466616);
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
