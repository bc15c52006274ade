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
constexpr bool kVtStamps = (GNSS_VT_PROBE & 4) != 0;

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
// A channel's nb block partials add up in kVtGroups runs of consecutive blocks (run g: blocks
// [g*len, (g+1)*len), len = ceil(nb / kVtGroups), each added in block order from 0) and then the
// runs in order: lane 8c + g of the adding block holds run g of channel c, so a channel's sum takes
// ~nb / 8 dependent adds rather than nb. vt_step_kernel's last block and vt_loop_kernel's lead
// form the same association: the same bits.
constexpr int kVtGroups = 8;
static_assert(GNSS_VT_MAX_CH * kVtGroups <= kVtStepThreads && 64 % kVtGroups == 0, "a channel's runs in one wave");
__device__ __forceinline__ void vt_run_range(int nb, int g, int* k0, int* k1)
{
    const int len = (nb + kVtGroups - 1) / kVtGroups;
    *k0 = g * len < nb ? g * len : nb;
    *k1 = *k0 + len < nb ? *k0 + len : nb;
}
// the runs of lane 8c + g's channel added in order (every lane of the wave calls it)
__device__ __forceinline__ double vt_runs_total(double run, int tid)
{
    double t = 0.0;
#pragma unroll
    for (int g = 0; g < kVtGroups; g++) t += __shfl(run, (tid & ~(kVtGroups - 1)) + g);
    return t;
}

// The sums of block (b, ch) over its slice of channel ch's read (ns samples at byte `off` of
// the window, carrier frequency f and phase phi0; ns 0: the channel sits the step out), left
// in s_r0[0] / s_r1[0] (LDS arrays of at least kVtStepThreads / 64 entries; ends with a barrier).
__device__ __forceinline__ void vt_block_sums(const uint8_t* rec, double Fs, bool real8, const VtBlockStep& st,
                                              int b, int nb, int tid, double* s_r0, double* s_r1,
                                              unsigned long long* mark6 = nullptr, unsigned long long* mark7 = nullptr)
{
    auto mark = [&](unsigned long long* m) {  // (probe builds: this block's marks 6 / 7, by its lane 0)
        if constexpr (kVtStamps)
            if (m && tid == 0)
                __hip_atomic_store(m, (unsigned long long)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    const int64_t n = st.ns;
    const int64_t chunk = (n + nb - 1) / nb;
    const int64_t k0 = (int64_t)b * chunk, k1 = k0 + chunk < n ? k0 + chunk : n;
    const uint8_t* r = rec + st.off;
    const double f = st.f, phi0 = st.phi0, rfs = st.rfs;
    // the lane's samples k0 + tid + 256 i, four at a time (independent divisions and sincos in
    // flight together), added in increasing k as the one-at-a-time loop would. k/Fs: Markstein's
    // correction of k * RN(1/Fs), the IEEE quotient for every k of the read (host-verified), or
    // the division; sin / cos of the 2*pi-reduced phase: sincos_small (< 1 ulp, as the CT
    // correlator's)
    auto term = [&](int64_t k, double& tI, double& tQ) {
        const double t = rfs != 0.0 ? div_markstein((double)k, Fs, rfs) : (double)k / Fs;
        const double W = kTwoPi * (f * t) + phi0;  // Wave(k+1) (:275-276)
        const double q = rint(W * (1.0 / kTwoPi));
        double rr = __builtin_fma(-q, kTwoPi, W);
        rr = __builtin_fma(-q, kTwoPiLo, rr);
        double sn, cs;
        if constexpr ((GNSS_VT_PROBE & 1) != 0) {  // (A/B probe: no sincos)
            sn = rr;
            cs = 1.0;
        } else {
            sincos_small(rr, &sn, &cs);
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
    // (a slice's last few samples per lane in flight together too -- loop mode's slices are 3
    // samples a lane: the terms past the slice are computed at the lane's first sample of the
    // batch and not added, so every lane adds the same terms in the same order)
    for (int64_t k = k0 + tid; k < k1; k += U * TS) {
        double tI[U], tQ[U];
#pragma unroll
        for (int u = 0; u < U; u++) term(k + u * TS < k1 ? k + u * TS : k, tI[u], tQ[u]);
#pragma unroll
        for (int u = 0; u < U; u++)
            if (k + u * TS < k1) {
                sI += tI[u];
                sQ += tQ[u];
            }
    }
    mark(mark6);
    // the block's sum: a fixed butterfly within each wave (xor 32, 16, ..., 1), then the four
    // wave sums in order -- the same bits for the same terms
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        sI += __shfl_xor(sI, m);
        sQ += __shfl_xor(sQ, m);
    }
    mark(mark7);
    if ((tid & 63) == 0) {
        s_r0[tid >> 6] = sI;
        s_r1[tid >> 6] = sQ;
    }
    __syncthreads();
    if (tid == 0) {
        double I = s_r0[0], Q = s_r1[0];
#pragma unroll
        for (int w = 1; w < kVtStepThreads / 64; w++) {
            I += s_r0[w];
            Q += s_r1[w];
        }
        s_r0[0] = I;
        s_r1[0] = Q;
    }
    __syncthreads();
}

// The step of block (b, ch) in a one-step launch (vt_step_kernel): its sums, then the hand-off
// through device memory and a ticket; the grid's last block posts `seq`.
__device__ __forceinline__ void vt_step_block(const uint8_t* rec, double Fs, bool real8, const VtBlockStep& st,
                                              double* part, double* sums, unsigned* done, unsigned* ticket,
                                              unsigned seq, int b, int ch, int nb, int nch, int tid, double* s_r0,
                                              double* s_r1, int* s_last)
{
    vt_block_sums(rec, Fs, real8, st, b, nb, tid, s_r0, s_r1);
    if (tid == 0) {
        // device-coherent stores (past this XCD's L2), drained before the block's ticket: the
        // grid's last block reads them with device-coherent loads. (No agent-scope release /
        // acquire fences: on gfx950 those write back and invalidate the whole L2.)
        double* pp = part + ((int64_t)ch * nb + b) * 2;
        __hip_atomic_store(pp, s_r0[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pp + 1, s_r1[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned total = (unsigned)nb * nch;
        *s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
    }
    __syncthreads();
    if (!*s_last) return;
    // the grid's last block: the partials come into LDS a block's worth at a time (lane k loads
    // partial k, all in flight together), lane c adds channel c's in block order (the same
    // sequential sum for every nb), writes the two sums through to the caller's host memory,
    // and once every lane's are drained, lane 0 re-arms the ticket (drained too: a later step's
    // first ticket must see it) and posts the step's number
    // (lane 8c + g: run g of channel c, accumulated over the chunks in block order)
    const int tot = nch * nb, c = tid / kVtGroups;
    int r0 = 0, r1 = 0;
    vt_run_range(nb, tid % kVtGroups, &r0, &r1);
    double I = 0.0, Q = 0.0;
    for (int base = 0; base < tot; base += kVtStepThreads) {
        const int m = tot - base < kVtStepThreads ? tot - base : kVtStepThreads;
        __syncthreads();  // (the last chunk's adds are done before its slots are reused)
        if (tid < m) {
            const double* pp = part + 2 * (int64_t)(base + tid);
            s_r0[tid] = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_r1[tid] = __hip_atomic_load(pp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (c < nch) {
            const int lo = c * nb + r0 > base ? c * nb + r0 : base;
            const int hi = c * nb + r1 < base + m ? c * nb + r1 : base + m;
            for (int k = lo; k < hi; k++) {
                I += s_r0[k - base];
                Q += s_r1[k - base];
            }
        }
    }
    I = vt_runs_total(I, tid);
    Q = vt_runs_total(Q, tid);
    if (c < nch && tid % kVtGroups == 0) {
        __hip_atomic_store(sums + 2 * c, I, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(sums + 2 * c + 1, Q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(kVtStepThreads) void vt_step_kernel(VtStepArgs a)
{
    __shared__ double s_r0[kVtStepThreads], s_r1[kVtStepThreads];
    __shared__ int s_last;
    const int ch = blockIdx.y;
    const VtBlockStep st{a.off[ch], a.ns[ch], a.f[ch], a.phi0[ch], a.rfs[ch]};
    vt_step_block(a.rec, a.Fs, a.real8, st, a.part, a.sums, a.done, a.ticket, a.seq, blockIdx.x, ch, gridDim.x,
                  gridDim.y, threadIdx.x, s_r0, s_r1, &s_last);
}

// The same steps from ONE launch (gnss_tracking_vt's loop mode). Block (0, 0), the lead, polls
// the host's mailbox granules (coherent host memory: each channel's read as kVtStepWords 16-B
// granules tagged with the step's number) and relays them as granules of the same tag in device
// memory; every other block polls its channel's, so one block, not the grid, polls across PCIe.
// Each block publishes its two sums as granules of the step's tag, and the lead, its own slice
// done, gathers every block's into LDS, adds each channel's in block order (the sums of
// vt_step_kernel, bit for bit) and writes them to the host as tagged granules. Mailbox granules
// tagged kVtLoopStop, or no new step within a.timeout, end the launch (the lead relays the stop
// tag). A step's blocks need no other block of the grid to be running but the lead, so the
// launch only has to fit on the chip (launch_vt_loop bounds the grid).
// word w of a relayed step (VtBlockStep's order; the integers travel as their bits)
__device__ __forceinline__ void step_word(VtBlockStep& st, int w, double v)
{
    if (w == 0) st.off = __double_as_longlong(v);
    else if (w == 1) st.ns = __double_as_longlong(v);
    else if (w == 2) st.f = v;
    else if (w == 3) st.phi0 = v;
    else st.rfs = v;
}

static_assert(GNSS_VT_MAX_CH * kVtStepWords <= kVtStepThreads, "the lead relays one mailbox granule per lane");
static_assert(2 * kVtLoopMaxBlocks <= 8 * kVtStepThreads, "the lead's gather: at most 8 granules per lane");

// (probe builds, GNSS_VT_PROBE & 4: wall-clock marks of a step: 0 the lead has the mailbox, 1 it
// has relayed it, 2 the last block has it, 3 the last block's sums, 4 the lead has gathered them,
// 5 the lead has written the channel sums; 6 / 7 the last block's terms / its lanes' butterfly)
// (lead marks 0, 1, 4, 5 at stamps[step][k]; per-block marks 2, 3, 6, 7 at
// stamps[kVtStampSteps * 8 + (step * 4 + slot) * kVtLoopMaxBlocks + block]: no two blocks share a
// word, so the marks do not serialise the step they time)
__device__ __forceinline__ unsigned long long* vt_mark_slot(const VtLoopArgs& a, unsigned seq, int k, int blk)
{
    if (!a.stamps || seq < 1 || seq > (unsigned)kVtStampSteps) return nullptr;
    if (blk < 0) return a.stamps + (size_t)(seq - 1) * 8 + k;
    const int slot = k == 2 ? 0 : k == 3 ? 1 : k == 6 ? 2 : 3;
    return a.stamps + (size_t)kVtStampSteps * 8 + ((size_t)(seq - 1) * 4 + slot) * kVtLoopMaxBlocks + blk;
}
__device__ __forceinline__ void vt_mark(const VtLoopArgs& a, unsigned seq, int k, int blk = -1)
{
    if constexpr (kVtStamps) {
        if (unsigned long long* m = vt_mark_slot(a, seq, k, blk))
            __hip_atomic_store(m, (unsigned long long)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// (at least 4 waves per SIMD: the 1 024-block bound resident on 256 CUs at 4 blocks per CU)
__global__ __launch_bounds__(kVtStepThreads, 4) void vt_loop_kernel(VtLoopArgs a)
{
    __shared__ double s_r0[kVtStepThreads], s_r1[kVtStepThreads];
    __shared__ double s_part[2 * kVtLoopMaxBlocks];
    __shared__ int s_go;
    __shared__ VtBlockStep s_st;
    const int b = blockIdx.x, ch = blockIdx.y, tid = threadIdx.x, nb = gridDim.x, nch = gridDim.y;
    const bool lead = b == 0 && ch == 0;
    const __amdgpu_buffer_rsrc_t gs = __builtin_amdgcn_make_buffer_rsrc(a.gstep, (short)0,
                                                                        nch * kVtStepWords * 16, kBufRsrcWord3);
    const __amdgpu_buffer_rsrc_t gp = __builtin_amdgcn_make_buffer_rsrc(a.gpart, (short)0, nch * nb * 2 * 16,
                                                                        kBufRsrcWord3);
    const __amdgpu_buffer_rsrc_t hm = __builtin_amdgcn_make_buffer_rsrc((void*)a.mail, (short)0,
                                                                        2 * nch * kVtStepWords * 16, kBufRsrcWord3);
    const __amdgpu_buffer_rsrc_t hs = __builtin_amdgcn_make_buffer_rsrc(a.sums, (short)0, nch * 2 * 16, kBufRsrcWord3);
    for (unsigned seq = a.seq0;; seq++) {
        if (lead) {
            // lane c * kVtStepWords + w polls word w of channel c's read across PCIe (system
            // coherence: past every cache) until it carries this step's number, then relays it
            // as a granule of the same tag -- a stop tag (or the wait's bound) relays the stop
            const int nw = nch * kVtStepWords;
            int stop = 0;
            u32x4 g = {0u, 0u, 0u, 0u};
            if (tid < nw) {
                const uint64_t t0 = (uint64_t)wall_clock64();
                for (;;) {
                    g = load16_sys(hm, (int)(seq & 1) * nw + tid);  // (step seq's half of the mailbox)
                    if (g.y == seq && g.w == seq) break;
                    if ((g.y == kVtLoopStop && g.w == kVtLoopStop) || (uint64_t)wall_clock64() - t0 > a.timeout) {
                        stop = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                const int c = tid / kVtStepWords, w = tid - c * kVtStepWords;
                if (c == 0) step_word(s_st, w, value16(g));  // (the lead's own channel)
            }
            stop = __syncthreads_or(stop);
            if (tid == 0) vt_mark(a, seq, 0);
            if (tid < nw) publish16(gs, tid, stop ? 0.0 : value16(g), stop ? kVtLoopStop : seq);
            if (tid == 0) s_go = !stop;
            if (tid == 0) vt_mark(a, seq, 1);
        } else if (tid < 64) {
            // wave 0: lanes 0..kVtStepWords-1 poll the channel's granules until every one
            // carries this step's tag (or the stop tag)
            const bool mine = tid < kVtStepWords;
            const uint64_t t0 = (uint64_t)wall_clock64();
            int go = 0;
            for (;;) {
                const u32x4 g = mine ? load16(gs, ch * kVtStepWords + tid) : u32x4{0u, 0u, 0u, 0u};
                const unsigned long long ok = __ballot(mine && g.y == seq && g.w == seq);
                const unsigned long long stop = __ballot(mine && g.y == kVtLoopStop && g.w == kVtLoopStop);
                if (stop) break;
                if ((ok & ((1ull << kVtStepWords) - 1)) == (1ull << kVtStepWords) - 1) {
                    if (mine) step_word(s_st, tid, value16(g));
                    go = 1;
                    if (tid == 0) vt_mark(a, seq, 2, ch * nb + b);
                    break;
                }
                if ((uint64_t)wall_clock64() - t0 > a.timeout) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (tid == 0) s_go = go;
        }
        __syncthreads();
        if (!s_go) return;
        const VtBlockStep st = s_st;
        vt_block_sums(a.rec, a.Fs, a.real8, st, b, nb, tid, s_r0, s_r1,
                      kVtStamps ? vt_mark_slot(a, seq, 6, ch * nb + b) : nullptr,
                      kVtStamps ? vt_mark_slot(a, seq, 7, ch * nb + b) : nullptr);
        if (tid == 0) vt_mark(a, seq, 3, ch * nb + b);
        if (tid < 2) publish16(gp, 2 * (ch * nb + b) + tid, tid ? s_r1[0] : s_r0[0], seq);
        // the channel's next read continues this one (:161-176) with about as many samples: the
        // block touches its slice of it (one word per 64-B line, inside the window) while the
        // next step is on its way, so the step's loads find it in this XCD's L2
        {
            const int bps = a.real8 ? 1 : 2;
            const int64_t n = st.ns, chunk = (n + nb - 1) / nb;
            const int64_t lo = st.off + n * bps + (int64_t)b * chunk * bps, hi = lo + chunk * bps;
            if (n > 0 && hi <= a.rec_len) {
                const int64_t l0 = lo & ~(int64_t)63;
                const int64_t at = l0 + (int64_t)tid * 64;
                if (at < hi) (void)*reinterpret_cast<const volatile unsigned*>(a.rec + at);
            }
        }
        if (lead) {
            // every block's two sums, lane-strided (a granule seen once is not read again), into LDS
            const int ng = 2 * nch * nb;
            unsigned long long todo = 0;  // bit k: granule tid + k * kVtStepThreads still missing
            for (int k = 0, e = tid; e < ng; k++, e += kVtStepThreads) todo |= 1ull << k;
            const uint64_t t0 = (uint64_t)wall_clock64();
            constexpr int kG = 2 * kVtLoopMaxBlocks / kVtStepThreads;  // granules per lane at most
            while (todo) {
                u32x4 g[kG];  // (every missing granule's load in flight together, then the checks)
#pragma unroll
                for (int k = 0; k < kG; k++)
                    if ((todo >> k) & 1ull) g[k] = load16(gp, tid + k * kVtStepThreads);
#pragma unroll
                for (int k = 0; k < kG; k++)
                    if (((todo >> k) & 1ull) && g[k].y == seq && g[k].w == seq) {
                        s_part[tid + k * kVtStepThreads] = value16(g[k]);
                        todo &= ~(1ull << k);
                    }
                if (todo && (uint64_t)wall_clock64() - t0 > a.timeout) break;
            }
            if (__syncthreads_or(todo != 0)) return;  // (timed out: the host sees the launch end)
            if (tid == 0) vt_mark(a, seq, 4);
            // lane 8c + g adds run g of channel c's partials, the runs add up in order (the
            // association vt_step_block's last block forms), and the channel's two sums go to the
            // host as granules of the step's tag
            const int c = tid / kVtGroups;
            double I = 0.0, Q = 0.0;
            if (c < nch) {
                int k0 = 0, k1 = 0;
                vt_run_range(nb, tid % kVtGroups, &k0, &k1);
                for (int k = k0; k < k1; k++) {
                    I += s_part[2 * (c * nb + k)];
                    Q += s_part[2 * (c * nb + k) + 1];
                }
            }
            I = vt_runs_total(I, tid);
            Q = vt_runs_total(Q, tid);
            if (c < nch && tid % kVtGroups == 0) {
                publish16_sys(hs, 2 * c, I, seq);
                publish16_sys(hs, 2 * c + 1, Q, seq);
                if (tid == 0) vt_mark(a, seq, 5);
            }
        }
        __syncthreads();  // (every lane is past the step before the next one's LDS writes)
    }
}

}  // namespace

hipError_t launch_vt_run(const VtRunArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(vt_run_kernel, dim3(a.n), dim3(kVtRun), 0, s, a);
    return hipGetLastError();
}

int vt_loop_resident_blocks(int device)
{
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, vt_loop_kernel, kVtStepThreads, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        return 0;
    return std::min(per_cu * cus, kVtLoopMaxBlocks);
}

hipError_t launch_vt_loop(const VtLoopArgs& a, int n, int nb, hipStream_t s)
{
    if (n < 1 || n > GNSS_VT_MAX_CH || nb < 1 || (int64_t)n * nb > kVtLoopMaxBlocks || !a.rec || !a.mail || !a.sums ||
        !a.gstep || !a.gpart)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(vt_loop_kernel, dim3(nb, n), dim3(kVtStepThreads), 0, s, a);
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
