// ifmt.hip — IF record formats other than int8 I/Q (initParameters.m:35-38): the
// reference's sample forming (acquisition.m:28-37, :90-99; trackingCT.m:84-93) on the
// device, so the correlators keep one input convention each:
//   * acquisition: the block of one fread as fp64 complex samples (int8 real -> (x, 0);
//     int16 -> I - mean(I), Q - mean(Q) over the block, means from exact integer sums);
//   * tracking: int8 real staged as int8 I/Q pairs with Q = 0 (exact: the correlator
//     then computes x*sin(W), x*cos(W)); int16 I/Q staged as is, plus per-8-sample-group
//     prefix sums of I and Q so a step's mean over any [A, A+n) is two lookups.
#include <hipcub/hipcub.hpp>

#include "gnss_internal.h"

namespace gnss {
namespace {

constexpr int kT = 256;

// Exact integer sums of the n int16 I and Q values (order-free: int64 atomics).
__global__ __launch_bounds__(kT) void sum16_kernel(const short* __restrict__ v, int64_t n,
                                                   unsigned long long* __restrict__ sums)
{
    long long si = 0, sq = 0;
    for (int64_t k = (int64_t)blockIdx.x * kT + threadIdx.x; k < n; k += (int64_t)gridDim.x * kT) {
        const short2 x = reinterpret_cast<const short2*>(v)[k];
        si += x.x;
        sq += x.y;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        si += __shfl_xor(si, o, 64);
        sq += __shfl_xor(sq, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&sums[0], (unsigned long long)si);
        atomicAdd(&sums[1], (unsigned long long)sq);
    }
}

// out[k] = (I - mean(I), Q - mean(Q)); mean = sum / n rounded once (MATLAB mean of
// integer-valued doubles), the difference rounded once, as the reference forms it.
__global__ __launch_bounds__(kT) void center16_kernel(const short* __restrict__ v, int64_t n,
                                                      const unsigned long long* __restrict__ sums,
                                                      double2* __restrict__ out)
{
    const double mi = (double)(long long)sums[0] / (double)n;
    const double mq = (double)(long long)sums[1] / (double)n;
    for (int64_t k = (int64_t)blockIdx.x * kT + threadIdx.x; k < n; k += (int64_t)gridDim.x * kT) {
        const short2 x = reinterpret_cast<const short2*>(v)[k];
        out[k] = make_double2((double)x.x - mi, (double)x.y - mq);
    }
}

__global__ __launch_bounds__(kT) void real8_cpx_kernel(const int8_t* __restrict__ v, int64_t n,
                                                       double2* __restrict__ out)
{
    for (int64_t k = (int64_t)blockIdx.x * kT + threadIdx.x; k < n; k += (int64_t)gridDim.x * kT)
        out[k] = make_double2((double)v[k], 0.0);
}

__global__ __launch_bounds__(kT) void real8_iq8_kernel(const int8_t* __restrict__ v, int64_t n,
                                                       char2* __restrict__ out)
{
    for (int64_t k = (int64_t)blockIdx.x * kT + threadIdx.x; k < n; k += (int64_t)gridDim.x * kT)
        out[k] = make_char2(v[k], 0);
}

// Group g of 8 int16 I/Q samples (32 B): sum of I, sum of Q (g < ng); entry ng = 0 so
// the exclusive scan of ng + 1 entries ends with the total.
__global__ __launch_bounds__(kT) void group16_kernel(const short* __restrict__ v, int64_t ng,
                                                     long long* __restrict__ gi, long long* __restrict__ gq)
{
    for (int64_t g = (int64_t)blockIdx.x * kT + threadIdx.x; g <= ng; g += (int64_t)gridDim.x * kT) {
        long long si = 0, sq = 0;
        if (g < ng) {
            const int4* p = reinterpret_cast<const int4*>(v + 16 * g);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int4 w = p[h];
                const int ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    si += (short)(ws[q] & 0xFFFF);
                    sq += (short)((unsigned)ws[q] >> 16);
                }
            }
        }
        gi[g] = si;
        gq[g] = sq;
    }
}

int grid_for(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>((n + kT - 1) / kT, 1), 8192); }

}  // namespace

hipError_t launch_stage_cpx(const int8_t* src, int prec, int type, int64_t nsamp, double2* out,
                            unsigned long long* sums, hipStream_t s)
{
    if (prec == 2 && type == 2) {
        hipError_t e = hipMemsetAsync(sums, 0, 16, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(sum16_kernel, dim3(grid_for(nsamp)), dim3(kT), 0, s,
                           reinterpret_cast<const short*>(src), nsamp, sums);
        hipLaunchKernelGGL(center16_kernel, dim3(grid_for(nsamp)), dim3(kT), 0, s,
                           reinterpret_cast<const short*>(src), nsamp, (const unsigned long long*)sums, out);
    } else if (prec == 1 && type == 1) {
        hipLaunchKernelGGL(real8_cpx_kernel, dim3(grid_for(nsamp)), dim3(kT), 0, s, src, nsamp, out);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_real8_to_iq8(const int8_t* src, int64_t n, int8_t* dst, hipStream_t s)
{
    hipLaunchKernelGGL(real8_iq8_kernel, dim3(grid_for(n)), dim3(kT), 0, s, src, n,
                       reinterpret_cast<char2*>(dst));
    return hipGetLastError();
}

size_t prefix16_scratch_bytes(int64_t ngroups)
{
    size_t tb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const long long*)nullptr, (long long*)nullptr,
                                           (int)(ngroups + 1));
    return tb + 2 * sizeof(long long) * (size_t)(ngroups + 1) + 256;
}

hipError_t launch_prefix16(const short* src, int64_t ngroups, long long* pref_i, long long* pref_q,
                           void* scratch, size_t scratch_bytes, hipStream_t s)
{
    if (ngroups + 1 > INT32_MAX) return hipErrorInvalidValue;
    long long* gi = reinterpret_cast<long long*>(scratch);
    long long* gq = gi + (ngroups + 1);
    void* tmp = gq + (ngroups + 1);
    size_t tb = scratch_bytes - 2 * sizeof(long long) * (size_t)(ngroups + 1);
    hipLaunchKernelGGL(group16_kernel, dim3(grid_for(ngroups + 1)), dim3(kT), 0, s, src, ngroups, gi, gq);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, gi, pref_i, (int)(ngroups + 1), s);
    if (e != hipSuccess) return e;
    return hipcub::DeviceScan::ExclusiveSum(tmp, tb, gq, pref_q, (int)(ngroups + 1), s);
}

}  // namespace gnss
