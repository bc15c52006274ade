// Host <-> GPU doorbell latency probe (A/B for the VT loop kernel's mailbox; never used by the
// product). One block spins on a mailbox word until the host posts step k, then answers k in a
// host-memory word; the host times the round trip. Mailbox in (A) coherent host memory (the GPU
// polls across PCIe) or (B) fine-grained device memory written by the host through its mapping
// (the GPU polls its own HBM), if the runtime gives the host one.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/probe_lib/pingpong tools/pingpong.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void pong(const unsigned* mail, unsigned* answer, int iters, unsigned long long timeout)
{
    if (threadIdx.x != 0) return;
    for (unsigned k = 1; k <= (unsigned)iters; k++) {
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(mail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != k) {
            if ((unsigned long long)wall_clock64() - t0 > timeout) return;
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(answer, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double run(unsigned* mail_dev, unsigned* mail_host, unsigned* answer, int iters)
{
    *mail_host = 0;
    __atomic_store_n(answer, 0u, __ATOMIC_RELAXED);
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, 0, mail_dev, answer, iters, (unsigned long long)khz * 1000ull * 5);
    auto t0 = std::chrono::steady_clock::now();
    for (unsigned k = 1; k <= (unsigned)iters; k++) {
        __atomic_store_n(mail_host, k, __ATOMIC_RELEASE);
        const auto ts = std::chrono::steady_clock::now();
        while (__atomic_load_n(answer, __ATOMIC_ACQUIRE) != k) {
            if (std::chrono::steady_clock::now() - ts > std::chrono::seconds(5)) {
                printf("timeout at %u\n", k);
                hipDeviceSynchronize();
                return -1;
            }
        }
        if (k == 100) t0 = std::chrono::steady_clock::now();
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    hipDeviceSynchronize();
    return us / (iters - 100);
}

int main()
{
    const int iters = 20000;
    unsigned *hmail = nullptr, *answer = nullptr;
    if (hipHostMalloc(&hmail, 4096, hipHostMallocCoherent) != hipSuccess) return 1;
    if (hipHostMalloc(&answer, 4096, hipHostMallocCoherent) != hipSuccess) return 1;
    printf("A host-memory mailbox: %.2f us round trip\n", run(hmail, hmail, answer, iters));
    unsigned* dmail = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&dmail, 4096, hipDeviceMallocFinegrained);
    printf("fine-grained device alloc: %s\n", hipGetErrorString(e));
    if (e != hipSuccess) return 0;
    hipPointerAttribute_t attr{};
    e = hipPointerGetAttributes(&attr, dmail);
    printf("attributes: %s type %d host %p device %p\n", hipGetErrorString(e), (int)attr.type, attr.hostPointer,
           attr.devicePointer);
    if (e != hipSuccess || !attr.hostPointer) {
        printf("B: no host mapping of device memory\n");
        return 0;
    }
    printf("B device-memory mailbox: %.2f us round trip\n",
           run(dmail, static_cast<unsigned*>(attr.hostPointer), answer, iters));
    return 0;
}
