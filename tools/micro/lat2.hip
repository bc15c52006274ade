// Latency of dependent fp64 / fp32 chains on gfx950, unrolled (no loop overhead in the
// chain): prices the tracking tail's scalar arithmetic. One wave per SIMD (grid 1 x 64) and
// four waves on one SIMD's CU (block of 256 = 4 waves, one per SIMD) give the same number
// if it is latency, not issue. Build: hipcc --offload-arch=gfx950 -O3 lat2.hip -o lat2
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))

__global__ void lat2_kernel(double* out, long long* t, double x0, double y0, float xf0)
{
    double x = x0 + threadIdx.x * 1e-9, y = y0;
    float xf = xf0 + threadIdx.x * 1e-6f;
    __shared__ double sh[256];
    long long c0;
    int k = 0;
// the chain may neither start before the first stamp nor end after the second: its input
// is "written" right after the first, and its result read into an SGPR before the second
#define TIME(body)                                                                          \
    __builtin_amdgcn_s_waitcnt(0);                                                          \
    c0 = clock64();                                                                         \
    asm volatile("" : "+v"(x), "+v"(xf));                                                   \
    body;                                                                                   \
    {                                                                                       \
        int dep = __builtin_amdgcn_readfirstlane((int)__double_as_longlong(x) ^ __float_as_int(xf)); \
        asm volatile("s_and_b32 %0, %0, %0" : "+s"(dep));                                    \
    }                                                                                       \
    if (threadIdx.x == 0) t[k] = clock64() - c0;                                            \
    k++;
    TIME(R64(x = __builtin_fma(x, y, 1e-3);))                       // 0 fma f64
    TIME(R64(x = x + y;))                                           // 1 add f64
    TIME(R64(x = x * y;))                                           // 2 mul f64
    TIME(R64(xf = __builtin_fmaf(xf, 0.999f, 1e-3f);))             // 3 fma f32
    TIME(R8(x = y / (x + 1.0);))                                    // 4 div f64 (x8)
    TIME(R8(x = __builtin_sqrt(x + 1.0);))                          // 5 sqrt f64 (x8)
    TIME(R8(x = __builtin_amdgcn_rcp(x + 1.0);))                    // 6 v_rcp_f64 + add (x8)
    TIME(R8(sh[threadIdx.x] = x; __builtin_amdgcn_s_waitcnt(0xc07f); x = sh[threadIdx.x ^ 1] + 1.0;))  // 7 lds w->r + add (x8)
    TIME(R8(x = __longlong_as_double((long long)__builtin_amdgcn_mov_dpp((int)__double_as_longlong(x), 0xB1, 0xF, 0xF, false) | ((long long)__builtin_amdgcn_mov_dpp((int)(__double_as_longlong(x) >> 32), 0xB1, 0xF, 0xF, false) << 32)) + y;))  // 8 dpp f64 + add (x8)
    TIME(R8(x = (double)__builtin_amdgcn_readfirstlane((int)x) + y;))  // 9 readfirstlane + cvt + add (x8)
    TIME(R8(__syncthreads(); x = x + y;))                           // 10 barrier + add (x8)
    TIME(R8(x = floor(x * y + 0.5);))                               // 11 mul + add + floor (x8)
    out[threadIdx.x] = x + xf;
}

int main()
{
    double* d_out;
    long long* d_t;
    hipMalloc(&d_out, 1024 * sizeof(double));
    hipMalloc(&d_t, 64 * sizeof(long long));
    const char* nm[] = {"fma f64", "add f64", "mul f64", "fma f32", "div f64", "sqrt f64", "rcp f64 + add",
                        "lds w->r + add", "dpp f64 + add", "readfirstlane+cvt+add", "barrier + add", "mul+add+floor"};
    const int per[] = {64, 64, 64, 64, 8, 8, 8, 8, 8, 8, 8, 8};
    for (int threads : {64, 256, 1024}) {
        long long t[16] = {};
        for (int it = 0; it < 3; it++) {
            hipLaunchKernelGGL(lat2_kernel, dim3(1), dim3(threads), 0, 0, d_out, d_t, 0.5, 0.999, 0.5f);
            hipDeviceSynchronize();
        }
        hipMemcpy(t, d_t, sizeof t, hipMemcpyDeviceToHost);
        printf("block of %d threads (%d waves per SIMD):\n", threads, threads / 256 > 0 ? threads / 256 : 1);
        for (int i = 0; i < 12; i++) printf("  %-24s %7.1f clk per op\n", nm[i], (double)t[i] / per[i]);
    }
    return 0;
}
