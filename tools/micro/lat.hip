// Latency probe: dependent chains of fp64 ops in one wave (wall clock 100 MHz and
// shader clock), to price the tracking tail's scalar arithmetic on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

__global__ void lat_kernel(double* out, unsigned long long* t, double x0, double y0, int reps)
{
    double x = x0 + threadIdx.x * 1e-9;
    const double y = y0;
    unsigned long long w0, c0;
    // 0: fma chain
    w0 = wall_clock64(); c0 = clock64();
    for (int i = 0; i < reps; i++) x = __builtin_fma(x, y, 1e-3);
    t[0] = wall_clock64() - w0; t[1] = clock64() - c0;
    // 1: division chain
    w0 = wall_clock64(); c0 = clock64();
    for (int i = 0; i < reps; i++) x = y / (x + 1.0);
    t[2] = wall_clock64() - w0; t[3] = clock64() - c0;
    // 2: sqrt chain
    w0 = wall_clock64(); c0 = clock64();
    for (int i = 0; i < reps; i++) x = sqrt(x + 1.0);
    t[4] = wall_clock64() - w0; t[5] = clock64() - c0;
    // 3: sincos chain
    w0 = wall_clock64(); c0 = clock64();
    for (int i = 0; i < reps; i++) { double s, c; sincos(x, &s, &c); x = s + c; }
    t[6] = wall_clock64() - w0; t[7] = clock64() - c0;
    // 4: round + cvt chain
    w0 = wall_clock64(); c0 = clock64();
    for (int i = 0; i < reps; i++) { long long n = (long long)rint(x * 1e3); x = (double)n * 1e-3 + 0.25; }
    t[8] = wall_clock64() - w0; t[9] = clock64() - c0;
    // 5: ds_read/write chain through LDS
    __shared__ double sh[64];
    w0 = wall_clock64(); c0 = clock64();
    for (int i = 0; i < reps; i++) { sh[(i + threadIdx.x) & 63] = x; __builtin_amdgcn_s_waitcnt(0xc07f); x = sh[(i + threadIdx.x + 1) & 63] + 1.0; }
    t[10] = wall_clock64() - w0; t[11] = clock64() - c0;
    out[threadIdx.x] = x;
}

int main()
{
    double* d_out; unsigned long long* d_t;
    hipMalloc(&d_out, 64 * sizeof(double)); hipMalloc(&d_t, 16 * sizeof(unsigned long long));
    const int reps = 1000;
    for (int it = 0; it < 3; it++) {
        hipLaunchKernelGGL(lat_kernel, dim3(1), dim3(64), 0, 0, d_out, d_t, 0.5, 0.999, reps);
        hipDeviceSynchronize();
    }
    unsigned long long t[16]; hipMemcpy(t, d_t, sizeof t, hipMemcpyDeviceToHost);
    const char* nm[] = {"fma", "div", "sqrt", "sincos", "rint+cvt", "lds rw"};
    for (int k = 0; k < 6; k++)
        printf("%-9s %8.2f ns/op  %8.1f clk/op  (clk %.2f GHz)\n", nm[k], t[2 * k] * 10.0 / reps,
               (double)t[2 * k + 1] / reps, (double)t[2 * k + 1] / (t[2 * k] * 10.0));
    return 0;
}
