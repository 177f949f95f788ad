// Cross-queue ordering cost on one device: what a dependency between two HIP streams costs
// in queue time (events vs. stream wait-value packets vs. same-stream order).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/evtest tools/evtest.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_spin(unsigned long long cycles, unsigned* flag, unsigned v)
{
    unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) {}
    if (flag && threadIdx.x == 0 && blockIdx.x == 0)
        __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double run(const char* name, int mode, hipStream_t a, hipStream_t b, hipEvent_t* ev, unsigned* flag, int iters,
                  unsigned long long cyc)
{
    CK(hipDeviceSynchronize());
    CK(hipMemset(flag, 0, 64));
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 1; i <= iters; ++i) {
        switch (mode) {
        case 0:   // same stream, two kernels
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, cyc, nullptr, 0);
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, cyc, nullptr, 0);
            break;
        case 1:   // same stream + an event record between
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, cyc, nullptr, 0);
            CK(hipEventRecord(ev[i & 1], a));
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, cyc, nullptr, 0);
            break;
        case 2:   // ping-pong across streams with events
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, cyc, nullptr, 0);
            CK(hipEventRecord(ev[i & 1], a));
            CK(hipStreamWaitEvent(b, ev[i & 1], 0));
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, b, cyc, nullptr, 0);
            CK(hipEventRecord(ev[2 + (i & 1)], b));
            CK(hipStreamWaitEvent(a, ev[2 + (i & 1)], 0));
            break;
        case 3:   // ping-pong across streams with kernel-written flags + wait-value packets
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, cyc, flag, (unsigned)i);
            CK(hipStreamWaitValue32(b, flag, (unsigned)i, hipStreamWaitValueGte, 0xFFFFFFFFu));
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, b, cyc, flag + 16, (unsigned)i);
            CK(hipStreamWaitValue32(a, flag + 16, (unsigned)i, hipStreamWaitValueGte, 0xFFFFFFFFu));
            break;
        case 4:   // one stream alternating (the serial baseline of mode 2/3)
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, cyc, flag, (unsigned)i);
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, cyc, flag + 16, (unsigned)i);
            break;
        }
    }
    CK(hipDeviceSynchronize());
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    printf("%-44s %8.2f us per iteration (2 kernels of %llu cycles)\n", name, us, cyc);
    return us;
}

int main()
{
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    unsigned* flag;
    CK(hipMalloc(&flag, 256));
    int canwait = 0;
    CK(hipDeviceGetAttribute(&canwait, hipDeviceAttributeCanUseStreamWaitValue, 0));
    printf("stream wait value supported: %d\n", canwait);
    const unsigned flagsets[3] = {hipEventDisableTiming, hipEventDisableTiming | hipEventReleaseToDevice,
                                  hipEventDisableTiming | hipEventDisableSystemFence};
    const char* fsn[3] = {"DisableTiming", "DisableTiming|ReleaseToDevice", "DisableTiming|DisableSystemFence"};
    const int iters = 2000;
    for (unsigned long long cyc : {100ull, 2000ull}) {
        hipEvent_t ev[4];
        for (int i = 0; i < 4; ++i) CK(hipEventCreateWithFlags(&ev[i], flagsets[0]));
        run("same stream", 0, a, b, ev, flag, iters, cyc);
        run("same stream, kernel writes flag", 4, a, b, ev, flag, iters, cyc);
        for (int f = 0; f < 3; ++f) {
            for (int i = 0; i < 4; ++i) { CK(hipEventDestroy(ev[i])); CK(hipEventCreateWithFlags(&ev[i], flagsets[f])); }
            char nm[128];
            snprintf(nm, sizeof nm, "record between [%s]", fsn[f]);
            run(nm, 1, a, b, ev, flag, iters, cyc);
            snprintf(nm, sizeof nm, "ping-pong events [%s]", fsn[f]);
            run(nm, 2, a, b, ev, flag, iters, cyc);
        }
        if (canwait) run("ping-pong wait-value", 3, a, b, ev, flag, iters, cyc);
        for (int i = 0; i < 4; ++i) CK(hipEventDestroy(ev[i]));
    }
    return 0;
}
