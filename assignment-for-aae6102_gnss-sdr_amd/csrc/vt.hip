// vt.hip — vector-tracking steps for gfx950 (trackingVT_POS_updated.m:157-349, the tracking
// half): one workgroup per channel runs nsteps steps in one launch. Per step, lane 0 sizes
// the read and finds the replica chips (vt_prepare), every lane sums its strided share of
// the carrier-wiped samples -- sum(imag(rawsignal .* carrsig)), sum(real(rawsignal .*
// carrsig)) with the reference's own Wave(k) = (2*pi*(carrFreq .* ((0:numSample)/Fs))) +
// remCarrPhase rounding per sample (IEEE division k/Fs) and an fp64 sincos of the 2*pi-reduced
// phase -- the workgroup reduces them in a fixed pairing (bit-reproducible), and lane 0 runs
// the scalar end (vt_finish: remChip, remCarrPhase, C/N0, PLL, DLL discriminator, the record),
// the same source as the host half (vt.cpp). The reference's replica quirk multiplies the two
// sums by one chip value per tap, so no code replica is generated. Formats (:163-176): int8
// I/Q, int8 real, int16 I/Q with each read's means removed. A step is latency-bound (one
// channel's ~58 000 samples per ms on one CU); the entry point is the drop-in for the
// reference's loop, which runs one step of one channel at a time.
#include "gnss_internal.h"

#ifndef GNSS_VT_PROBE
#define GNSS_VT_PROBE 0  // (A/B probe builds only, tools/build_variant.sh)
#endif

namespace gnss {

namespace {

constexpr int kVtRun = 1024;

__device__ __forceinline__ int16_t ld_i16(const uint8_t* p)
{
    return (int16_t)((unsigned)p[0] | ((unsigned)p[1] << 8));
}

// Fixed-pairing tree over the workgroup: v[0] = the sum, the same bits for the same inputs
__device__ __forceinline__ void tree2(double* r0, double* r1, int tid)
{
    for (int h = kVtRun / 2; h > 0; h >>= 1) {
        __syncthreads();
        if (tid < h) {
            r0[tid] += r0[tid + h];
            r1[tid] += r1[tid + h];
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(kVtRun) void vt_run_kernel(VtRunArgs a)
{
    const int ch = blockIdx.x, tid = threadIdx.x;
    __shared__ gnss_vt_chan s_c;
    __shared__ VtPrep s_p;
    __shared__ int s_bad;
    __shared__ double s_r0[kVtRun], s_r1[kVtRun];
    if (tid == 0) s_c = a.chans[ch];
    const int bps = a.prec * a.dtype;  // bytes per sample (ftell advance, :344)
    const bool iq16 = a.prec == 2, real8 = a.prec == 1 && a.dtype == 1;
    const unsigned* cab = a.ca_bits + 32 * ch;
    for (int s = 0; s < a.nsteps; s++) {
        gnss_vt_out* o = a.out + (int64_t)s * a.n + ch;
        const double cf = a.codeFreq[(int64_t)s * a.n + ch];
        // every wave has read the last step's s_bad / s_p before lane 0 rewrites them
        __syncthreads();
        if (tid == 0) {
            VtPrep p = vt_prepare(a.Fs, a.codelength, a.pdi, s_c.remChip, s_c.codeFreq, cf);
            int bad = !(cf > 0) ? GNSS_EARG : p.bad;
            if (!bad) {
                const int64_t A = s_c.file_ptr, need = p.n * bps;
                // a short fread makes `rawsignal .* carrsig` fail in MATLAB (:172, :279)
                if (A + need > a.file_len) bad = GNSS_EIO;
                else if (A < a.base || A + need > a.base + a.len) bad = GNSS_EIO;  // (outside the window)
            }
            s_p = p;
            s_bad = bad;
            if (bad) o->status = bad;
        }
        __syncthreads();
        if (s_bad) break;
        const int64_t n = s_p.n;
        const uint8_t* r = a.rec + (s_c.file_ptr - a.base);
        const double f = s_c.carrFreq, phi0 = s_c.remCarrPhase;
        // int16: rawsignal = (I - mean(I)) + 1i*(Q - mean(Q)) over this read (:166-170); the
        // integer sums are exact in fp64, the mean one division as MATLAB's mean
        double mu_i = 0.0, mu_q = 0.0;
        if (iq16) {
            double si = 0.0, sq = 0.0;
            for (int64_t k = tid; k < n; k += kVtRun) {
                si += (double)ld_i16(r + 4 * k);
                sq += (double)ld_i16(r + 4 * k + 2);
            }
            s_r0[tid] = si;
            s_r1[tid] = sq;
            tree2(s_r0, s_r1, tid);
            mu_i = s_r0[0] / (double)n;
            mu_q = s_r1[0] / (double)n;
            __syncthreads();
        }
        double sI = 0.0, sQ = 0.0;
        for (int64_t k = tid; k < n; k += kVtRun) {
            // Wave(k+1) in MATLAB's 1-based terms = 2*pi*(f*(k/Fs)) + phi0 (0-based k)
            const double W = kTwoPi * (f * ((double)k / a.Fs)) + phi0;
            const double q = rint(W * (1.0 / kTwoPi));
            double rr = __builtin_fma(-q, kTwoPi, W);  // exact: both multiples of 2^-50 below 8
            rr = __builtin_fma(-q, kTwoPiLo, rr);
            double sn, cs;
            sincos(rr, &sn, &cs);
            double xr, xi;
            if (iq16) {
                xr = (double)ld_i16(r + 4 * k) - mu_i;
                xi = (double)ld_i16(r + 4 * k + 2) - mu_q;
            } else if (real8) {  // int8 real record: rawsignal is real (:172-175)
                xr = (double)(int8_t)r[k];
                xi = 0.0;
            } else {
                xr = (double)(int8_t)r[2 * k];
                xi = (double)(int8_t)r[2 * k + 1];
            }
            sI += xr * sn + xi * cs;  // imag(raw .* carrsig) (:279)
            sQ += xr * cs - xi * sn;  // real(raw .* carrsig) (:280)
        }
        s_r0[tid] = sI;
        s_r1[tid] = sQ;
        tree2(s_r0, s_r1, tid);
        if (tid == 0) {
            int code[3];
            for (int t = 0; t < 3; t++)
                code[t] = vt_code_at(s_p.j[t], a.pdi, [&](int i) { return ((cab[i >> 5] >> (i & 31)) & 1u) ? -1 : 1; });
            const int st = vt_finish(a.Fs, a.ms, a.pdi, bps, a.tau1carr, a.tau2carr, &s_c, s_p, code, cf,
                                     s_r0[0], s_r1[0], o);
            s_bad = st;
            if (st) o->status = st;
        }
        __syncthreads();
        if (s_bad) break;
    }
    __syncthreads();
    if (tid == 0) a.chans[ch] = s_c;
}


// Fixed-pairing tree over a kVtStepThreads block
__device__ __forceinline__ void tree2s(double* r0, double* r1, int tid)
{
    for (int h = kVtStepThreads / 2; h > 0; h >>= 1) {
        __syncthreads();
        if (tid < h) {
            r0[tid] += r0[tid + h];
            r1[tid] += r1[tid + h];
        }
    }
    __syncthreads();
}

// One step of every channel over nb blocks per channel (grid nb x n). The VT loop of
// trackingVT_POS_updated.m is a host-driven chain (the EKF predicts every step's code
// frequency from the last step's correlations), so a step's latency is the loop's rate:
// spreading a channel's ~58 000 samples over nb blocks turns vt_run_kernel's one-CU step
// into a chip-wide one, and the kernel is nothing but that spread: the host has sized the
// read and holds the channel state (gnss_tracking_vt), so each block sums the carrier-wiped
// samples of its contiguous slice exactly as vt_run_kernel does per sample and reduces its 256
// lanes in a fixed tree; the grid's last block to finish adds each channel's nb partials in
// block order and writes the channel's two sums through to the caller's coherent host memory
// with the step's number beside them. No block waits for another; the host runs the scalar
// end (vt_finish) of each channel.
__global__ __launch_bounds__(kVtStepThreads) void vt_step_kernel(VtStepArgs a)
{
    const int b = blockIdx.x, ch = blockIdx.y, nb = gridDim.x, tid = threadIdx.x;
    __shared__ double s_r0[kVtStepThreads], s_r1[kVtStepThreads];
    const int64_t n = a.ns[ch];  // (0: the channel sits the step out)
    const int64_t chunk = (n + nb - 1) / nb;
    const int64_t k0 = (int64_t)b * chunk, k1 = k0 + chunk < n ? k0 + chunk : n;
    const uint8_t* r = a.rec + a.off[ch];
    const double f = a.f[ch], phi0 = a.phi0[ch], Fs = a.Fs;
    const bool real8 = a.real8;
    // the lane's samples k0 + tid + 256 i, four at a time (independent divisions and sincos in
    // flight together), added in increasing k as the one-at-a-time loop would
    auto term = [&](int64_t k, double& tI, double& tQ) {
        const double W = kTwoPi * (f * ((double)k / Fs)) + phi0;  // Wave(k+1) (:275-276)
        const double q = rint(W * (1.0 / kTwoPi));
        double rr = __builtin_fma(-q, kTwoPi, W);
        rr = __builtin_fma(-q, kTwoPiLo, rr);
        double sn, cs;
        if constexpr ((GNSS_VT_PROBE & 1) != 0) {  // (A/B probe: no sincos)
            sn = rr;
            cs = 1.0;
        } else {
            sincos(rr, &sn, &cs);
        }
        double xr, xi;
        if (real8) {
            xr = (double)(int8_t)r[k];
            xi = 0.0;
        } else {
            xr = (double)(int8_t)r[2 * k];
            xi = (double)(int8_t)r[2 * k + 1];
        }
        tI = xr * sn + xi * cs;  // imag(raw .* carrsig) (:279)
        tQ = xr * cs - xi * sn;  // real(raw .* carrsig) (:280)
    };
    double sI = 0.0, sQ = 0.0;
    constexpr int U = 4, TS = kVtStepThreads;
    int64_t k = k0 + tid;
    for (; k + (U - 1) * TS < k1; k += U * TS) {
        double tI[U], tQ[U];
#pragma unroll
        for (int u = 0; u < U; u++) term(k + u * TS, tI[u], tQ[u]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            sI += tI[u];
            sQ += tQ[u];
        }
    }
    for (; k < k1; k += TS) {
        double tI, tQ;
        term(k, tI, tQ);
        sI += tI;
        sQ += tQ;
    }
    s_r0[tid] = sI;
    s_r1[tid] = sQ;
    tree2s(s_r0, s_r1, tid);
    __shared__ int s_last;
    if (tid == 0) {
        // device-coherent stores (past this XCD's L2), drained before the block's ticket: the
        // grid's last block reads them with device-coherent loads. (No agent-scope release /
        // acquire fences: on gfx950 those write back and invalidate the whole L2.)
        double* pp = a.part + ((int64_t)ch * nb + b) * 2;
        __hip_atomic_store(pp, s_r0[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pp + 1, s_r1[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned total = (unsigned)nb * gridDim.y;
        s_last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
    }
    __syncthreads();
    if (!s_last) return;
    // the grid's last block: lane c adds channel c's nb partials in block order (the same
    // sequential sum for every nb), writes the two sums through to the caller's host memory,
    // and once every lane's are drained, lane 0 re-arms the ticket and posts the step's number
    const int nch = gridDim.y;
    if (tid < nch) {
        const double* pp = a.part + (int64_t)tid * nb * 2;
        double I = 0.0, Q = 0.0;
        constexpr int kB = 8;  // (loads in flight per batch)
        for (int b0 = 0; b0 < nb; b0 += kB) {
            double v[2 * kB];
            const int m = nb - b0 < kB ? nb - b0 : kB;
#pragma unroll
            for (int j = 0; j < 2 * kB; j++)
                v[j] = j < 2 * m ? __hip_atomic_load(pp + 2 * b0 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
            for (int j = 0; j < m; j++) {
                I += v[2 * j];
                Q += v[2 * j + 1];
            }
        }
        __hip_atomic_store(a.sums + 2 * tid, I, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.sums + 2 * tid + 1, Q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

hipError_t launch_vt_run(const VtRunArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(vt_run_kernel, dim3(a.n), dim3(kVtRun), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_vt_step(const VtStepArgs& a, int n, int nb, hipStream_t s)
{
    if (n < 1 || n > GNSS_VT_MAX_CH || nb < 1 || nb > GNSS_VT_MAX_BLOCKS || !a.rec || !a.part || !a.sums || !a.done || !a.ticket)
        return hipErrorInvalidValue;
    for (int i = 0; i < n; i++)
        if (a.ns[i] < 0 || a.off[i] < 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(vt_step_kernel, dim3(nb, n), dim3(kVtStepThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace gnss
