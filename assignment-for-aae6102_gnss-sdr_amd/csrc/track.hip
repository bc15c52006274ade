// track.hip — trackingCT.m correlator + DLL/PLL loop for gfx950 (MI355X).
//
// One launch = one tracking step (1 ms or 10 ms of IF) for every channel of the
// call. The loop is sequential per channel (step n+1's NCO depends on step n's
// discriminators, trackingCT.m:136-150 -> :79-107), so the design is:
//   * every block re-derives the step plan (numSample, colon ranges) from the
//     channel state in HBM — identical fp64 arithmetic in every block;
//   * blocks stream a contiguous slice of the channel's IF window (int8 I/Q,
//     16 B = 8 samples per lane per load), generate carrier and E/P/L (or ACF)
//     replicas on chip and accumulate fp32 partial correlations;
//   * the last block to arrive (agent-scope release/acquire ticket) reduces the
//     partials in a fixed order (bit-reproducible), runs C/N0 + DLL/PLL in fp64
//     and writes the next state and the step record.
// Reference: SDR_MATLAB-main/acqtckpos/trackingCT.m (citations inline).
#include "gnss_internal.h"

namespace gnss {

namespace {

struct StepPlan {
    int64_t n;          // numSample
    int64_t delayValue;
    double remSample;
    double d;           // codeFreq/Fs
    int64_t A;          // first absolute sample of the window
};

// trackingCT.m:79-82 (1 ms) and :411-415 (10 ms).
__device__ __forceinline__ StepPlan plan_step(const TrkParams& p, const TrkChan& c, int pdi,
                                              int phaseC)
{
    StepPlan s;
    const double cps = c.codeFreq / p.Fs;
    if (phaseC) {
        s.delayValue = c.numSample - (int64_t)(p.S * pdi);
        s.remSample = (p.codelength * pdi - c.remChip) / cps;
        s.n = (int64_t)round((p.codelength * pdi - c.remChip) / cps);
    } else {
        s.remSample = (p.codelength - c.remChip) / cps;
        s.n = (int64_t)round((p.codelength * pdi - c.remChip) / cps);
        s.delayValue = s.n - (int64_t)(p.S * pdi);
    }
    s.d = cps;
    s.A = c.pos / 2;
    return s;
}


__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double ld_agent(const double* ptr)
{
    return __hip_atomic_load(ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The scalar end of a step (last-arriving block, one thread): trackingCT.m:102-170
// (1 ms) / :435-524 (10 ms), fp64, same operation order as the reference.
__device__ void finalize_step(const TrkParams& p, const TrkBuffers& b, int ch, int pdi,
                              int phaseC, const StepPlan& sp, const double* sums)
{
    TrkChan& c = b.chan[ch];
    const int64_t n = sp.n;
    const int nt = p.ntaps;
    double s[2 * GNSS_MAX_TAPS];
    for (int v = 0; v < 2 * nt; v++) s[v] = phaseC ? -sums[v] : sums[v];  // :447-449

    // remChip = (t_CodePrompt(numSample) + codeFreq/Fs) - codeFreqBasis*ms*pdi (:102)
    {
        const double a = (0 + p.taps[p.iP]) + c.remChip;
        const double bb = ((double)(n - 1) * sp.d + p.taps[p.iP]) + c.remChip;
        Colon col = colon_make(a, sp.d, bb);
        c.remChip = (colon_elem(col, n - 1) + c.codeFreq / p.Fs) - p.codeFreqBasis * p.ms * pdi;
    }
    // remPhase = rem(Wave(numSample+1), 2*pi) (:104-106)
    c.remPhase = fmod(kTwoPi * (c.carrierFreq * ((double)n / p.Fs)) + c.remPhase, kTwoPi);

    const double E_i = s[2 * p.iE], E_q = s[2 * p.iE + 1];
    const double P_i = s[2 * p.iP], P_q = s[2 * p.iP + 1];
    const double L_i = s[2 * p.iL], L_q = s[2 * p.iL + 1];

    // C/N0 (:120-134)
    c.index_int += 1;
    c.Zk[c.index_int - 1] = P_i * P_i + P_q * P_q;
    if (c.index_int % 20 == 0) {
        double mean = 0;
        for (int k = 0; k < 20; k++) mean += c.Zk[k];
        mean = mean / 20;
        double var = 0;
        for (int k = 0; k < 20; k++) var += (c.Zk[k] - mean) * (c.Zk[k] - mean);
        var = var / 19;
        const double m2v = mean * mean - var;
        const double scale = 1 / (1 * p.ms * pdi);
        double cn;
        if (m2v >= 0) {
            const double NA2 = sqrt(m2v);
            const double varIQ = 0.5 * (mean - NA2);
            cn = fabs(10 * log10(scale * NA2 / (2 * varIQ)));
        } else {  // complex sqrt branch of MATLAB (quirk A.16)
            const double y = sqrt(-m2v);
            const double nr = 0, ni = scale * y;
            const double dr = 2 * (0.5 * mean), di = 2 * (0.5 * -y);
            const double den = dr * dr + di * di;
            const double zr = (nr * dr + ni * di) / den, zi = (ni * dr - nr * di) / den;
            const double lr = 10 * (log(hypot(zr, zi)) / log(10.0));
            const double li = 10 * (atan2(zi, zr) / log(10.0));
            cn = hypot(lr, li);
        }
        double* cn0 = phaseC ? b.cn0_10 : b.cn0_1;
        if (c.snrIndex <= p.cn0_cap) cn0[(int64_t)ch * p.cn0_cap + c.snrIndex - 1] = cn;
        c.index_int = 0;
        c.snrIndex += 1;
    }

    // DLL (:136-143), PLL (:145-150); phase C keeps T = 0.001 (:473,480)
    const double E = sqrt(E_i * E_i + E_q * E_q);
    const double L = sqrt(L_i * L_i + L_q * L_q);
    const double DLLdiscri = 0.5 * (E - L) / (E + L);
    const double T = phaseC ? 0.001 : (0.001 * pdi);
    const double code_output = c.code_outputLast + (p.tau2code / p.tau1code) * (DLLdiscri - c.DLLdiscriLast) +
                               DLLdiscri * (T / p.tau1code);
    c.DLLdiscriLast = DLLdiscri;
    c.code_outputLast = code_output;
    c.codeFreq = p.codeFreqBasis - code_output;
    const double PLLdiscri = atan(P_q / P_i) / kTwoPi;
    const double carrier_output = c.carrier_outputLast +
                                  (p.tau2carr / p.tau1carr) * (PLLdiscri - c.PLLdiscriLast) +
                                  PLLdiscri * (T / p.tau1carr);
    c.carrier_outputLast = carrier_output;
    c.PLLdiscriLast = PLLdiscri;
    c.carrierFreq = c.carrierFreqBasis + carrier_output;

    // bookkeeping + record (:153-170 / :507-524)
    c.numSample = n;
    c.remSample = sp.remSample;
    c.pos += 2 * n;  // ftell after fread
    c.Index += phaseC ? 10 : 1;
    const int64_t col = c.nstep;  // 0-based IndexSmall - 1
    int64_t* dvpre = b.dvpre + (int64_t)ch * (p.rec_cap + 1);
    dvpre[col + 1] = dvpre[col] + sp.delayValue;
    c.nstep = col + 1;
    // sum(delayValue(1:Index)) over an nsv x N matrix (column-major, quirk A.11)
    int64_t cols = 0;
    if (c.Index >= c.sv1) cols = (c.Index - c.sv1) / p.nsv + 1;
    if (cols > c.nstep) cols = c.nstep;
    const double codedelay = (double)c.codedelay0 + (double)dvpre[cols];
    const double absS = (double)c.pos;
    double m = fmod(absS / p.dataBytesPerSample, p.Fs * p.ms);  // mod() of positives
    const int64_t slot = c.slot;
    if (slot < p.rec_cap) {
        double* r = b.rec + ((int64_t)ch * p.rec_cap + slot) * GNSS_NFIELDS;
        r[GNSS_F_P_i] = P_i;             r[GNSS_F_P_q] = P_q;
        r[GNSS_F_E_i] = E_i;             r[GNSS_F_E_q] = E_q;
        r[GNSS_F_L_i] = L_i;             r[GNSS_F_L_q] = L_q;
        r[GNSS_F_PLLdiscri] = PLLdiscri; r[GNSS_F_DLLdiscri] = DLLdiscri;
        r[GNSS_F_codedelay] = codedelay; r[GNSS_F_remChip] = c.remChip;
        r[GNSS_F_codeFreq] = c.codeFreq; r[GNSS_F_carrierFreq] = c.carrierFreq;
        r[GNSS_F_remPhase] = c.remPhase; r[GNSS_F_remSample] = sp.remSample;
        r[GNSS_F_numSample] = (double)n; r[GNSS_F_delayValue] = (double)sp.delayValue;
        r[GNSS_F_absoluteSample] = absS; r[GNSS_F_codedelay2] = m;
        if (b.taps_rec) {
            double* tr = b.taps_rec + ((int64_t)ch * p.rec_cap + slot) * (2 * nt);
            for (int v = 0; v < 2 * nt; v++) tr[v] = s[v];
        }
    }
    if (!phaseC && slot < b.n1) b.p_i_1ms[(int64_t)ch * b.n1 + slot] = P_i;
    c.slot = slot + 1;
}

}  // namespace

// ---------------------------------------------------------------------------
// The correlator step kernel. NT = taps (3: E/P/L, 11: ACF), compile-time so the
// accumulators stay in VGPRs.
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(kTrkThreads) void track_step_kernel(TrkParams p, TrkBuffers b,
                                                                  int pdi, int phaseC, int bpc,
                                                                  int U)
{
    const int ch = blockIdx.x / bpc;
    const int blk = blockIdx.x - ch * bpc;
    const int tid = threadIdx.x;

    __shared__ float s_ca[1024];
    __shared__ double s_tap_a[NT], s_tap_c[NT];
    __shared__ double s_red[kTrkThreads / 64][2 * NT];
    __shared__ int s_last;
    __shared__ double s_fin[2 * NT];
    __shared__ double s_part[kMaxBpc * 2 * NT];

    const TrkChan* cp = b.chan + ch;
    if (cp->status != GNSS_OK) return;
    if (!phaseC && cp->Index + 1 > cp->n1_target) return;  // this channel's 1-ms run is done
    const TrkChan c = *cp;
    const StepPlan sp = plan_step(p, c, pdi, phaseC);
    const int64_t n = sp.n;
    const int64_t A = sp.A;

    // window checks (identical in every block -> every block returns together)
    const int64_t byte0 = 2 * A, byte1 = 2 * (A + n);
    const int64_t g_first = A >> 3, g_last = (A + n - 1) >> 3;
    const int64_t G = (int64_t)kTrkThreads * U;
    int bad = GNSS_OK;
    if (n <= 0) bad = GNSS_EINDEX;
    else if (byte1 > p.file_len) bad = phaseC ? GNSS_EIO : GNSS_ENODATA;  // :108-112 / :442
    else if (byte0 < p.buf_base || byte1 > p.buf_base + p.buf_len) bad = GNSS_EIO;
    else if ((g_last - g_first + 1) > G * bpc) bad = GNSS_EINDEX;  // grid too small
    if (bad != GNSS_OK) {
        if (blk == 0 && tid == 0) b.chan[ch].status = bad;
        return;
    }

    for (int i = tid; i < 1023; i += kTrkThreads) s_ca[i] = b.ca[(int64_t)ch * 1023 + i];
    if (tid < NT) {
        const double a = (0 + p.taps[tid]) + c.remChip;
        const double bb = ((double)(n - 1) * sp.d + p.taps[tid]) + c.remChip;
        Colon col = colon_make(a, sp.d, bb);
        s_tap_a[tid] = col.a;
        s_tap_c[tid] = col.c;
        if (col.n != n - 1 && blk == 0) b.chan[ch].status = GNSS_EINDEX;
    }
    __syncthreads();

    const double inv_d = 1.0 / sp.d;
    const int64_t nint = n - 1;

    // ---- carrier: Wave(k) = (2*pi*(carrierFreq*(k/Fs))) + remPhase, fp64, with the
    // reference's roundings reproduced exactly (trackingCT.m:104-107). Per 8-sample
    // group: one sincos at the first sample; the others are rotated by the exact
    // per-sample increment delta = 2*pi*f/Fs (double-double) and corrected by
    // eta = (Wave(k) - Wave(k0)) - m*delta, the rounding residue of Wave.
    const double f = c.carrierFreq, phi0 = c.remPhase, Fs = p.Fs, rFs = p.inv_Fs;
    const bool exact_div = p.exact_div != 0;
    auto wave = [&](double kd) -> double {
        double t;
        if (exact_div) {
            t = kd / Fs;
        } else {  // RN(k/Fs) via one FMA-corrected reciprocal (host-verified exact)
            const double q = kd * rFs;
            const double e = __builtin_fma(-q, Fs, kd);
            t = __builtin_fma(e, rFs, q);
        }
        const double x = f * t;
        const double y = kTwoPi * x;
        return y + phi0;
    };
    double dhi, dlo;
    {
        const double p0 = kTwoPi * f;
        double pe = __builtin_fma(kTwoPi, f, -p0);
        pe = pe + kTwoPiLo * f;
        const double q = p0 / Fs;
        const double r = __builtin_fma(-q, Fs, p0);
        const double ql = (r + pe) / Fs;
        dhi = __longlong_as_double(__double_as_longlong(q) & ~0x1FLL);  // 48-bit: m*dhi exact
        dlo = (q - dhi) + ql;
    }
    __shared__ double s_rc[8], s_rs[8];
    if (tid < 8) {
        double sn, cs;
        sincos((double)tid * dhi + (double)tid * dlo, &sn, &cs);
        s_rc[tid] = cs;
        s_rs[tid] = sn;
    }
    __syncthreads();
    double rc[8], rs[8];
#pragma unroll
    for (int m = 0; m < 8; m++) { rc[m] = s_rc[m]; rs[m] = s_rs[m]; }

    double accI[NT], accQ[NT];
#pragma unroll
    for (int s = 0; s < NT; s++) { accI[s] = 0.0; accQ[s] = 0.0; }

    const int8_t* iq = b.iq - p.buf_base;  // absolute-byte addressing
    for (int u = 0; u < U; u++) {
        const int64_t g = g_first + (int64_t)blk * G + (int64_t)u * kTrkThreads + tid;
        if (g > g_last) break;
        const int64_t k0 = 8 * g - A;  // relative index of sample m = 0 of this group
        const int4 raw = *reinterpret_cast<const int4*>(iq + 16 * g);
        const int mlo = k0 < 0 ? (int)(-k0) : 0;
        const int mhi = (n - k0) < 8 ? (int)(n - k0) : 8;  // valid m in [mlo, mhi)
        const int64_t kf = k0 + mlo;

        // ---- code replica: per tap the chip at the first valid sample and the
        // in-group position of the (at most one) chip boundary. Exact fp64 colon
        // values; an ambiguous boundary (|r - round r| < 1e-6) takes the per-sample
        // exact path. sel bit m -> chip c0 + 1.
        float v0[NT], v1[NT];
        unsigned sel[NT];
#pragma unroll
        for (int s = 0; s < NT; s++) {
            Colon col{s_tap_a[s], sp.d, s_tap_c[s], nint};
            const double t0 = colon_elem(col, kf);
            const double c0 = ceil(t0);
            const double r = (c0 - t0) * inv_d;
            const double rr = rint(r);
            const int64_t ic0 = (int64_t)c0;
            v0[s] = s_ca[ca_index(ic0)];
            v1[s] = s_ca[ca_index(ic0 + 1)];
            unsigned m = 0;
            if (fabs(r - rr) < 1e-6 && rr < 8.0) {
                for (int j = mlo + 1; j < mhi; j++) {
                    const double t = colon_elem(col, k0 + j);
                    if ((int64_t)ceil(t) != ic0) m |= 1u << j;
                }
            } else {
                const int pb = mlo + (int)floor(r) + 1;
                m = pb >= 8 ? 0u : (0xFFu << pb) & 0xFFu;
            }
            sel[s] = m;
        }

        // ---- carrier phasor of sample m = 0
        const double kd0 = (double)k0;
        const double W0 = wave(kd0);
        double s0, c0;
        sincos(W0, &s0, &c0);

        const int w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int m = 0; m < 8; m++) {
            const int word = w[m >> 1];
            const int sh = (m & 1) * 16;
            double xr = (double)(int8_t)((word >> sh) & 0xFF);
            double xi = (double)(int8_t)((word >> (sh + 8)) & 0xFF);
            if (m < mlo || m >= mhi) { xr = 0.0; xi = 0.0; }
            double cw = c0, sw = s0;
            if (m > 0) {
                const double dm = wave(kd0 + (double)m) - W0;
                const double eta = (dm - (double)m * dhi) - (double)m * dlo;
                const double cm = __builtin_fma(c0, rc[m], -(s0 * rs[m]));
                const double sm = __builtin_fma(s0, rc[m], c0 * rs[m]);
                cw = __builtin_fma(-eta, sm, cm);
                sw = __builtin_fma(eta, cm, sm);
            }
            const double I = __builtin_fma(xr, sw, xi * cw);    // imag(raw.*carrsig)
            const double Q = __builtin_fma(xr, cw, -(xi * sw)); // real(raw.*carrsig)
#pragma unroll
            for (int s = 0; s < NT; s++) {
                const double code = ((sel[s] >> m) & 1u) ? v1[s] : v0[s];
                accI[s] = __builtin_fma(code, I, accI[s]);
                accQ[s] = __builtin_fma(code, Q, accQ[s]);
            }
        }
    }

    // ---- block reduction (fp64), fixed order
    const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int s = 0; s < NT; s++) {
        const double si = wave_sum(accI[s]);
        const double sq = wave_sum(accQ[s]);
        if (lane == 0) { s_red[wv][2 * s] = si; s_red[wv][2 * s + 1] = sq; }
    }
    __syncthreads();
    double* part = b.partial + ((int64_t)ch * bpc + blk) * (2 * NT);
    if (tid < 64) {
        if (tid < 2 * NT) {
            double v = 0;
#pragma unroll
            for (int k = 0; k < kTrkThreads / 64; k++) v += s_red[k][tid];
            part[tid] = v;
        }
        // publish (guide G16 R1): storing wave drains, lane 0 releases + tickets
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned old = __hip_atomic_fetch_add(b.arrive + ch, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            const int last = (old == (unsigned)(bpc - 1));
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            s_last = last;
        }
    }
    __syncthreads();
    if (!s_last) return;

    // ---- last arriver: deterministic reduction of all block partials
    const double* allp = b.partial + (int64_t)ch * bpc * (2 * NT);
    for (int i = tid; i < bpc * 2 * NT; i += kTrkThreads) s_part[i] = ld_agent(allp + i);
    __syncthreads();
    if (tid < 2 * NT) {
        double v = 0;
        for (int k = 0; k < bpc; k++) v += s_part[k * (2 * NT) + tid];
        s_fin[tid] = v;
    }
    __syncthreads();
    if (tid == 0) {
        b.arrive[ch] = 0;
        if (b.dbg_sums) {
            for (int v = 0; v < 2 * NT; v++) b.dbg_sums[ch * 2 * NT + v] = s_fin[v];
        } else {
            finalize_step(p, b, ch, pdi, phaseC, sp, s_fin);
        }
    }
}

__global__ void track_snapshot_kernel(TrkBuffers b, int nch)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nch) b.snap[i] = b.chan[i];
}

// trackingCT.m:178-213 on the phase-A P_i (length msToProcessCT_1ms).
__global__ void track_bitedge_kernel(TrkBuffers b, int nch)
{
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch >= nch) return;
    TrkChan& c = b.chan[ch];
    if (c.status != GNSS_OK) return;
    const double* P = b.p_i_1ms + (int64_t)ch * b.n1;
    const int64_t len = b.n1;
    int cx = 0;
    for (int64_t i = 7; i <= len - 1; i++) {
        const double pi = P[i - 1];
        const int si = (pi > 0) - (pi < 0);
        bool ok = true;
        for (int j = 6; j >= 1 && ok; j--) {
            const double q = P[i - j - 1];
            ok = ((q > 0) - (q < 0)) != si;
        }
        for (int j = 1; j <= 17 && ok; j++) {
            if (i + j > len) { c.status = GNSS_EINDEX; return; }
            const double q = P[i + j - 1];
            ok = ((q > 0) - (q < 0)) == si;
        }
        if (ok && i >= 600) { cx = (int)(i % 20) - 1; break; }
    }
    c.countinx = cx;
    c.n1_target = b.n1 + cx;
}

// Entry to phase C (trackingCT.m:379-406): countinx = -1 resumes from the state
// after step msToProcessCT_1ms - 1 (quirk A.9); fresh C/N0 counters; seek to the
// nominal (skip + 1000 + countinx) ms position (quirk A.12).
__global__ void track_phase_c_init_kernel(TrkParams p, TrkBuffers b, int64_t skip, int nch)
{
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch >= nch) return;
    TrkChan c = b.chan[ch];
    if (c.status != GNSS_OK) return;
    const int cx = c.countinx;
    if (cx < 0) {
        c = b.snap[ch];
        c.countinx = cx;
        c.n1_target = b.n1 + cx;
    }
    const int64_t S = (int64_t)p.S;
    c.pos = (int64_t)((S - c.codedelay0 + 1 + (skip + b.n1 + cx) * S) * (int64_t)p.dataBytesPerSample);
    c.index_int = 0;
    c.snrIndex = 1;
    c.nstep = 0;
    c.Index = b.n1 + cx;
    c.slot = b.n1 + cx;
    b.dvpre[(int64_t)ch * (p.rec_cap + 1)] = 0;
    b.chan[ch] = c;
}

hipError_t launch_track_step(const TrkParams& p, const TrkBuffers& b, int pdi, int phaseC,
                             int bpc, int U, hipStream_t s)
{
    dim3 grid(p.nch * bpc), block(kTrkThreads);
    switch (p.ntaps) {
    case 3:
        hipLaunchKernelGGL(track_step_kernel<3>, grid, block, 0, s, p, b, pdi, phaseC, bpc, U);
        break;
    case 11:
        hipLaunchKernelGGL(track_step_kernel<11>, grid, block, 0, s, p, b, pdi, phaseC, bpc, U);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_track_snapshot(const TrkParams& p, const TrkBuffers& b, hipStream_t s)
{
    hipLaunchKernelGGL(track_snapshot_kernel, dim3((p.nch + 63) / 64), dim3(64), 0, s, b, p.nch);
    return hipGetLastError();
}

hipError_t launch_track_bitedge(const TrkParams& p, const TrkBuffers& b, hipStream_t s)
{
    hipLaunchKernelGGL(track_bitedge_kernel, dim3((p.nch + 63) / 64), dim3(64), 0, s, b, p.nch);
    return hipGetLastError();
}

hipError_t launch_track_phase_c_init(const TrkParams& p, const TrkBuffers& b, int64_t skip,
                                     hipStream_t s)
{
    hipLaunchKernelGGL(track_phase_c_init_kernel, dim3((p.nch + 63) / 64), dim3(64), 0, s, p, b,
                       skip, p.nch);
    return hipGetLastError();
}

}  // namespace gnss
