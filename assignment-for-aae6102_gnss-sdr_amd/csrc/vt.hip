// vt.hip — the carrier wipe and sums of a vector-tracking step for gfx950
// (trackingVT_POS_updated.m:262-272): sum(imag(rawsignal .* carrsig)) and
// sum(real(rawsignal .* carrsig)) over each channel's numSample samples, with the
// reference's own Wave(k) = (2*pi*(carrFreq .* ((0:numSample)/Fs))) + remCarrPhase rounding
// per sample (exact IEEE division k/Fs) and an fp64 sincos of the 2*pi-reduced phase. The
// reference's replica quirk multiplies these two sums by one chip value per tap (vt.cpp),
// so no code replica is generated here. Each block reduces its lanes in a fixed order and
// stores one partial; the host adds the partials in block order (bit-reproducible).
#include "gnss_internal.h"

namespace gnss {

namespace {

constexpr int kVtThreads = 256;

__global__ __launch_bounds__(kVtThreads) void vt_sum_kernel(const int8_t* __restrict__ iq, int iq_pairs,
                                                            const VtDesc* __restrict__ desc, double Fs,
                                                            int nblk, double* __restrict__ part)
{
    const int ch = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
    const VtDesc d = desc[ch];
    double sI = 0.0, sQ = 0.0;
    for (int64_t k = (int64_t)blk * kVtThreads + tid; k < d.n; k += (int64_t)nblk * kVtThreads) {
        // Wave(k+1) in MATLAB's 1-based terms = 2*pi*(f*(k/Fs)) + phi0 (0-based k)
        const double W = kTwoPi * (d.f * ((double)k / Fs)) + d.phi0;
        const double q = rint(W * (1.0 / kTwoPi));
        double r = __builtin_fma(-q, kTwoPi, W);  // exact: both multiples of 2^-50 below 8
        r = __builtin_fma(-q, kTwoPiLo, r);
        double sn, cs;
        sincos(r, &sn, &cs);
        double xr, xi;
        if (iq_pairs) {
            xr = (double)iq[d.A + 2 * k];
            xi = (double)iq[d.A + 2 * k + 1];
        } else {  // int8 real record: rawsignal is real (:172-175)
            xr = (double)iq[d.A + k];
            xi = 0.0;
        }
        sI += xr * sn + xi * cs;  // imag(raw .* carrsig)
        sQ += xr * cs - xi * sn;  // real(raw .* carrsig)
    }
    __shared__ double s_i[kVtThreads], s_q[kVtThreads];
    s_i[tid] = sI;
    s_q[tid] = sQ;
    __syncthreads();
    for (int h = kVtThreads / 2; h > 0; h >>= 1) {  // fixed pairing
        if (tid < h) {
            s_i[tid] += s_i[tid + h];
            s_q[tid] += s_q[tid + h];
        }
        __syncthreads();
    }
    if (tid == 0) {
        part[((int64_t)ch * nblk + blk) * 2] = s_i[0];
        part[((int64_t)ch * nblk + blk) * 2 + 1] = s_q[0];
    }
}

}  // namespace

int vt_blocks(int64_t nmax) { return (int)std::min<int64_t>(64, (nmax + 32 * kVtThreads - 1) / (32 * kVtThreads)); }

hipError_t launch_vt_sums(const int8_t* iq, int iq_pairs, const VtDesc* desc, int nch, double Fs, int nblk,
                          double* part, hipStream_t s)
{
    hipLaunchKernelGGL(vt_sum_kernel, dim3(nblk, nch), dim3(kVtThreads), 0, s, iq, iq_pairs, desc, Fs, nblk, part);
    return hipGetLastError();
}

}  // namespace gnss
