// Placement probe: which physical CU (XCC_ID + HW_ID) each block of a persistent-shaped
// grid lands on. 256-thread blocks with ~53 KB of LDS (3 blocks per CU, like the
// persistent tracking loop); every block spins ~200 us so the whole grid is resident.
// Output: one line per block: block xcc hwid start_ns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void place_kernel(unsigned* out, int lds_kb)
{
    __shared__ double s[53000 / 8];
    const unsigned xcc = __builtin_amdgcn_s_getreg(0xF814);   // HW_REG_XCC_ID, 32 bits
    const unsigned hw = __builtin_amdgcn_s_getreg(0xF804);    // HW_REG_HW_ID, 32 bits
    const unsigned long long t0 = wall_clock64();
    s[threadIdx.x] = (double)t0;
    __syncthreads();
    while (wall_clock64() - t0 < 20000) {}  // 200 us at 100 MHz
    if (threadIdx.x == 0) {
        out[4 * blockIdx.x + 0] = xcc;
        out[4 * blockIdx.x + 1] = hw;
        out[4 * blockIdx.x + 2] = (unsigned)(t0 & 0xffffffffu);
        out[4 * blockIdx.x + 3] = (unsigned)s[threadIdx.x + 1];
    }
}

int main(int argc, char** argv)
{
    for (int grid : {768, 512, 256}) {
        unsigned* d;
        hipMalloc(&d, grid * 16);
        for (int it = 0; it < 2; it++) {
            hipLaunchKernelGGL(place_kernel, dim3(grid), dim3(256), 0, 0, d, 53);
            hipDeviceSynchronize();
        }
        std::vector<unsigned> h(grid * 4);
        hipMemcpy(h.data(), d, grid * 16, hipMemcpyDeviceToHost);
        unsigned tmin = 0xffffffffu;
        for (int b = 0; b < grid; b++) tmin = h[4 * b + 2] < tmin ? h[4 * b + 2] : tmin;
        for (int b = 0; b < grid; b++)
            printf("%d %d %u 0x%08x %u\n", grid, b, h[4 * b], h[4 * b + 1], (h[4 * b + 2] - tmin) * 10);
        hipFree(d);
    }
    return 0;
}
