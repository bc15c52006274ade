// track.hip — trackingCT.m correlator + DLL/PLL loop for gfx950 (MI355X).
//
// One launch = one tracking step (1 ms or 10 ms of IF) for every channel of the
// call. The loop is sequential per channel (step n+1's NCO depends on step n's
// discriminators, trackingCT.m:136-150 -> :79-107), so a step is a latency
// chain and the design minimises it:
//   * the previous step's last block prepares a StepDesc (numSample, colon
//     ranges per tap, carrier constants, end-of-step NCO values) so a block's
//     prologue is a handful of scalar loads;
//   * every lane owns 8 consecutive samples (one 16-B load of int8 I/Q issued
//     first thing), generates the E/P/L (or ACF) replica from exact fp64 colon
//     arithmetic and the carrier from the reference's own fp64 Wave rounding,
//     and accumulates fp64 partial correlations;
//   * blocks hand partials to the last arriver with write-through (sc1) stores
//     and one agent-scope ticket add (guide G16, table row 1: no fences); the
//     last block reduces them in a fixed order (bit-reproducible), runs C/N0 +
//     DLL/PLL in fp64 and prepares the next StepDesc with its first wave.
// Reference: SDR_MATLAB-main/acqtckpos/trackingCT.m (citations inline).
#include "gnss_internal.h"

namespace gnss {

namespace {

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double ld_sc1(const double* ptr)
{
    return __hip_atomic_load(ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_sc1(double* ptr, double v)
{
    __hip_atomic_store(ptr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// CarrTime = k/Fs (trackingCT.m:104) as the IEEE quotient: one FMA-corrected
// reciprocal (host-verified exact for this Fs and k range) or a true division.
__device__ __forceinline__ double carr_time(double kd, double Fs, double rFs, bool exact_div)
{
    if (exact_div) return kd / Fs;
    const double q = kd * rFs;
    const double e = __builtin_fma(-q, Fs, kd);
    return __builtin_fma(e, rFs, q);
}

// Wave(k) = (2*pi*(carrierFreq .* CarrTime)) + remPhase with the reference's roundings
__device__ __forceinline__ double wave_at(double kd, double f, double phi0, double Fs, double rFs,
                                          bool exact_div)
{
    const double t = carr_time(kd, Fs, rFs, exact_div);
    const double x = f * t;
    const double y = kTwoPi * x;
    return y + phi0;
}

// Prepare the descriptor of the step that follows state `c` (trackingCT.m:79-107 /
// :411-441), executed by the 64 lanes of one wave: lanes < ntaps build the colon of
// their tap, lanes < 8 the carrier rotations e^{i m delta}, lane 0 the scalars.
__device__ void prepare_desc(const TrkParams& p, const TrkChan& c, int pdi, int phaseC, int lane,
                             StepDesc* d)
{
    const double cps = c.codeFreq / p.Fs;
    int64_t n, dv;
    double remSample;
    if (phaseC) {
        dv = c.numSample - (int64_t)(p.S * pdi);                      // :411
        remSample = (p.codelength * pdi - c.remChip) / cps;            // :414
        n = (int64_t)round((p.codelength * pdi - c.remChip) / cps);    // :415
    } else {
        remSample = (p.codelength - c.remChip) / cps;                  // :79
        n = (int64_t)round((p.codelength * pdi - c.remChip) / cps);    // :80
        dv = n - (int64_t)(p.S * pdi);                                 // :82
    }
    const int64_t A = c.pos / 2;
    int bad = GNSS_OK;
    if (n <= 0 || n > (int64_t)(p.S * pdi * 1.01) + 64) bad = GNSS_EINDEX;
    else if (2 * (A + n) > p.file_len) bad = phaseC ? GNSS_EIO : GNSS_ENODATA;  // :108-112 / :442
    else if (2 * A < p.buf_base || 2 * (A + n) > p.buf_base + p.buf_len) bad = GNSS_EIO;

    // carrier increment delta = 2*pi*f/Fs as a double-double; dhi has 48 bits so
    // m*dhi (m < 8) is exact
    const double f = c.carrierFreq;
    double dhi, dlo;
    {
        const double p0 = kTwoPi * f;
        double pe = __builtin_fma(kTwoPi, f, -p0);
        pe = pe + kTwoPiLo * f;
        const double q = p0 / p.Fs;
        const double r = __builtin_fma(-q, p.Fs, p0);
        const double ql = (r + pe) / p.Fs;
        dhi = __longlong_as_double(__double_as_longlong(q) & ~0x1FLL);
        dlo = (q - dhi) + ql;
    }
    if (lane < p.ntaps) {
        // t = (0 + Spacing + remChip) : cps : ((numSample-1)*cps + Spacing + remChip) (:96-98)
        const double a = (0 + p.taps[lane]) + c.remChip;
        const double bb = ((double)(n - 1) * cps + p.taps[lane]) + c.remChip;
        const Colon col = colon_make(a, cps, bb);
        d->tap_a[lane] = col.a;
        d->tap_c[lane] = col.c;
        const int64_t c0 = (int64_t)ceil(colon_elem(col, 0));
        const int64_t c1 = (int64_t)ceil(colon_elem(col, n - 1));
        int tb = (col.n != n - 1 || c0 < 0 || c1 > 1023LL * pdi + 1) ? GNSS_EINDEX : GNSS_OK;
        if (lane == p.iP) {
            // remChip = (t_CodePrompt(numSample) + codeFreq/Fs) - codeFreqBasis*ms*pdi (:102)
            d->remChip_next = (colon_elem(col, n - 1) + c.codeFreq / p.Fs) -
                              p.codeFreqBasis * p.ms * pdi;
        }
        if (tb != GNSS_OK && bad == GNSS_OK) bad = tb;
    }
    if (lane < 9) {
        double sn, cs;
        sincos((double)lane * dhi + (double)lane * dlo, &sn, &cs);
        d->rc[lane] = cs;
        d->rs[lane] = sn;
    }
    if (lane == 9) {
        // remPhase = rem(Wave(numSample+1), 2*pi) (:104-106)
        d->remPhase_next = fmod(kTwoPi * (f * ((double)n / p.Fs)) + c.remPhase, kTwoPi);
    }
    // any lane's failure wins (bitwise-or of the positive codes is enough to flag)
    int badw = bad;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) badw = max(badw, __shfl_xor(badw, o, 64));
    if (lane == 0) {
        d->n = n;
        d->delayValue = dv;
        d->A = A;
        d->g_first = A >> 3;
        d->g_last = (A + n - 1) >> 3;
        d->Index = c.Index;
        d->remSample = remSample;
        d->d = cps;
        d->inv_d = 1.0 / cps;
        d->f = f;
        d->phi0 = c.remPhase;
        d->dhi = dhi;
        d->dlo = dlo;
        d->pdi = pdi;
        d->phaseC = phaseC;
        d->bad = badw;
    }
}

// The scalar end of a step (trackingCT.m:102-170 / :435-524), fp64, same operation
// order as the reference. Returns the updated state in `c`.
__device__ void finalize_step(const TrkParams& p, const TrkBuffers& b, int ch, const StepDesc& d,
                              const double* sums, TrkChan& c)
{
    const int64_t n = d.n;
    const int pdi = d.pdi, phaseC = d.phaseC;
    const int nt = p.ntaps;
    const double* s = sums;  // already negated for phase C (:447-449)

    c.remChip = d.remChip_next;
    c.remPhase = d.remPhase_next;
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
    const double code_output = c.code_outputLast +
                               (p.tau2code / p.tau1code) * (DLLdiscri - c.DLLdiscriLast) +
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
    c.remSample = d.remSample;
    c.pos += 2 * n;  // ftell after fread
    c.Index += phaseC ? 10 : 1;
    const int64_t col = c.nstep;  // 0-based IndexSmall - 1
    int64_t* dvpre = b.dvpre + (int64_t)ch * (p.rec_cap + 1);
    const int64_t dvsum = dvpre[col] + d.delayValue;
    dvpre[col + 1] = dvsum;
    c.nstep = col + 1;
    // sum(delayValue(1:Index)) over an nsv x N matrix (column-major, quirk A.11)
    int64_t cols = 0;
    if (c.Index >= c.sv1) cols = (c.Index - c.sv1) / p.nsv + 1;
    if (cols > c.nstep) cols = c.nstep;
    const double codedelay = (double)c.codedelay0 + (double)(cols == c.nstep ? dvsum : dvpre[cols]);
    const double absS = (double)c.pos;
    const double m = fmod(absS / p.dataBytesPerSample, p.Fs * p.ms);  // mod() of positives
    const int64_t slot = c.slot;
    if (slot < p.rec_cap) {
        double* r = b.rec + ((int64_t)ch * p.rec_cap + slot) * GNSS_NFIELDS;
        r[GNSS_F_P_i] = P_i;             r[GNSS_F_P_q] = P_q;
        r[GNSS_F_E_i] = E_i;             r[GNSS_F_E_q] = E_q;
        r[GNSS_F_L_i] = L_i;             r[GNSS_F_L_q] = L_q;
        r[GNSS_F_PLLdiscri] = PLLdiscri; r[GNSS_F_DLLdiscri] = DLLdiscri;
        r[GNSS_F_codedelay] = codedelay; r[GNSS_F_remChip] = c.remChip;
        r[GNSS_F_codeFreq] = c.codeFreq; r[GNSS_F_carrierFreq] = c.carrierFreq;
        r[GNSS_F_remPhase] = c.remPhase; r[GNSS_F_remSample] = d.remSample;
        r[GNSS_F_numSample] = (double)n; r[GNSS_F_delayValue] = (double)d.delayValue;
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
// The correlator step kernel. NT = taps (3: E/P/L, 11: ACF), SUB = 8-sample
// sub-groups per lane (contiguous), both compile-time so the accumulators stay
// in VGPRs. Grid: nch x bpc blocks; block b of a channel owns the 256*SUB
// consecutive 8-sample groups starting at g_first + 256*SUB*b.
// ---------------------------------------------------------------------------
template <int NT, int SUB>
__global__ __launch_bounds__(kTrkThreads) void track_step_kernel(TrkParams p, TrkBuffers b, int bpc)
{
    const int ch = blockIdx.x / bpc;
    const int blk = blockIdx.x - ch * bpc;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int NV = 2 * NT;
    constexpr int J = kTrkThreads / NV;

    __shared__ double s_red[kTrkThreads / 64][NV];
    __shared__ double s_tmp[J * NV];
    __shared__ double s_fin[NV];
    __shared__ int s_last;

    const StepDesc* dp = b.desc + ch;
    const TrkChan* cp = b.chan + ch;
    const int64_t g_first = dp->g_first, g_last = dp->g_last;
    const int64_t g0 = g_first + ((int64_t)blk * kTrkThreads + tid) * SUB;  // first group of the lane
    // issue the IF loads first (clamped so every lane loads something valid)
    const int8_t* iq = b.iq - p.buf_base;  // absolute-byte addressing
    const int bad = dp->bad;
    int4 raw[SUB];
#pragma unroll
    for (int j = 0; j < SUB; j++) {
        const int64_t gj = g0 + j <= g_last ? g0 + j : g_last;
        raw[j] = bad ? make_int4(0, 0, 0, 0) : *reinterpret_cast<const int4*>(iq + 16 * gj);
    }
    const unsigned cabits = lane < 32 ? b.ca_bits[ch * 32 + lane] : 0u;

    if (cp->status != GNSS_OK) return;
    if (!dp->phaseC && dp->Index + 1 > cp->n1_target) return;  // 1-ms run of this channel done
    if (bad) {
        if (blk == 0 && tid == 0) b.chan[ch].status = bad;
        return;
    }

    const int64_t n = dp->n, A = dp->A;
    const double d = dp->d, inv_d = dp->inv_d;
    const double f = dp->f, phi0 = dp->phi0, dhi = dp->dhi, dlo = dp->dlo;
    const double Fs = p.Fs, rFs = p.inv_Fs;
    const bool exact_div = p.exact_div != 0;

    const int64_t ks = 8 * g0 - A;  // relative index of the lane's first sample
    const int mlo = ks < 0 ? (int)(-ks) : 0;  // only the window's first lane has ks < 0
    const int64_t kf = ks + mlo < n - 1 ? ks + mlo : n - 1;

    // ---- code replica per tap: chip ic at the sub-group's first sample and the
    // distance R (samples) from that sample to the next chip boundary; the boundary
    // falls at m = floor(R) + 1 (at most one per 8 samples since 8*cps < 1). Exact
    // fp64 colon values at the lane start, then R -= 8 / += 1/cps per sub-group; an
    // ambiguous boundary (|R - round R| < 1e-6) takes the per-sample exact path.
    int64_t ic[NT];
    double R[NT];
#pragma unroll
    for (int s = 0; s < NT; s++) {
        const Colon col{dp->tap_a[s], d, dp->tap_c[s], n - 1};
        const double t0 = colon_elem(col, kf);
        const double c0 = ceil(t0);
        ic[s] = (int64_t)c0;
        R[s] = (double)(kf - ks) + (c0 - t0) * inv_d;
    }

    // ---- carrier: Wave(k) exactly as the reference rounds it (trackingCT.m:104-107);
    // one sincos per lane, every other sample rotated by e^{i m delta} and corrected
    // by eta = (Wave(k) - Wave(kb)) - m*delta, the rounding residue of Wave.
    double kb = (double)ks;
    double Wb = wave_at(kb, f, phi0, Fs, rFs, exact_div);
    double sb, cb;
    sincos(Wb, &sb, &cb);

    double accI[NT], accQ[NT];
#pragma unroll
    for (int s = 0; s < NT; s++) { accI[s] = 0.0; accQ[s] = 0.0; }

#pragma unroll
    for (int j = 0; j < SUB; j++) {
        const int64_t kj = ks + 8 * j;
        const int lo = j == 0 ? mlo : 0;
        const int hi = (n - kj) < 8 ? (int)(n - kj) : 8;  // valid m in [lo, hi)
        double v0[NT], v1[NT];
        unsigned sel[NT];
#pragma unroll
        for (int s = 0; s < NT; s++) {
            const int i0 = ca_index(ic[s]), i1 = ca_index(ic[s] + 1);
            const unsigned w0 = __shfl(cabits, i0 >> 5, 64), w1 = __shfl(cabits, i1 >> 5, 64);
            v0[s] = ((w0 >> (i0 & 31)) & 1u) ? -1.0 : 1.0;
            v1[s] = ((w1 >> (i1 & 31)) & 1u) ? -1.0 : 1.0;
            const double rr = rint(R[s]);
            unsigned m = 0;
            if (fabs(R[s] - rr) < 1e-6 && rr < 8.0 && hi > 0) {
                // exact per-sample chips, then an exact restart at the next sub-group
                const Colon col{dp->tap_a[s], d, dp->tap_c[s], n - 1};
                // the lane's first valid sample has chip ic by construction; later
                // sub-groups may already start past the boundary (R <= 0)
                for (int q = j == 0 ? lo + 1 : 0; q < hi; q++)
                    if ((int64_t)ceil(colon_elem(col, kj + q)) != ic[s]) m |= 1u << q;
                const int64_t kn = kj + 8 < n - 1 ? kj + 8 : n - 1;
                const double tn = colon_elem(col, kn);
                const double cn = ceil(tn);
                ic[s] = (int64_t)cn;
                R[s] = (double)(kn - (kj + 8)) + (cn - tn) * inv_d;
            } else {
                const double fl = floor(R[s]);
                const int pb = (int)fl + 1;
                m = pb >= 8 ? 0u : (0xFFu << pb) & 0xFFu;
                if (pb < 8) { ic[s] += 1; R[s] += inv_d; }
                R[s] -= 8.0;
            }
            sel[s] = m;
        }

        const int w[4] = {raw[j].x, raw[j].y, raw[j].z, raw[j].w};
#pragma unroll
        for (int m = 0; m < 8; m++) {
            const int word = w[m >> 1];
            const int sh = (m & 1) * 16;
            double xr = (double)(int8_t)((word >> sh) & 0xFF);
            double xi = (double)(int8_t)((word >> (sh + 8)) & 0xFF);
            if (m < lo || m >= hi) { xr = 0.0; xi = 0.0; }
            double cw = cb, sw = sb;
            if (m > 0) {
                const double dm = wave_at(kb + (double)m, f, phi0, Fs, rFs, exact_div) - Wb;
                const double eta = (dm - (double)m * dhi) - (double)m * dlo;
                const double rcm = dp->rc[m], rsm = dp->rs[m];
                const double cm = __builtin_fma(cb, rcm, -(sb * rsm));
                const double sm = __builtin_fma(sb, rcm, cb * rsm);
                cw = __builtin_fma(-eta, sm, cm);
                sw = __builtin_fma(eta, cm, sm);
            }
            const double I = __builtin_fma(xr, sw, xi * cw);     // imag(raw.*carrsig)
            const double Q = __builtin_fma(xr, cw, -(xi * sw));  // real(raw.*carrsig)
#pragma unroll
            for (int s = 0; s < NT; s++) {
                const double code = ((sel[s] >> m) & 1u) ? v1[s] : v0[s];
                accI[s] = __builtin_fma(code, I, accI[s]);
                accQ[s] = __builtin_fma(code, Q, accQ[s]);
            }
        }
        if (j + 1 < SUB) {  // chain the base phasor to the next sub-group, exactly
            const double Wn = wave_at(kb + 8.0, f, phi0, Fs, rFs, exact_div);
            const double eta = ((Wn - Wb) - 8.0 * dhi) - 8.0 * dlo;
            const double rc8 = dp->rc[8], rs8 = dp->rs[8];
            const double cm = __builtin_fma(cb, rc8, -(sb * rs8));
            const double sm = __builtin_fma(sb, rc8, cb * rs8);
            cb = __builtin_fma(-eta, sm, cm);
            sb = __builtin_fma(eta, cm, sm);
            Wb = Wn;
            kb += 8.0;
        }
    }

    // ---- block reduction (fixed order), then hand the partial to the last arriver
#pragma unroll
    for (int s = 0; s < NT; s++) {
        const double si = wave_sum(accI[s]);
        const double sq = wave_sum(accQ[s]);
        if (lane == 0) { s_red[wv][2 * s] = si; s_red[wv][2 * s + 1] = sq; }
    }
    __syncthreads();
    double* allp = b.partial + (int64_t)ch * bpc * NV;
    if (wv == 0) {
        if (lane < NV) {
            double v = 0;
#pragma unroll
            for (int k = 0; k < kTrkThreads / 64; k++) v += s_red[k][lane];
            st_sc1(allp + (int64_t)blk * NV + lane, v);  // write-through
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains
        int last = 0;
        if (lane == 0) {
            const unsigned old = __hip_atomic_fetch_add(b.arrive + ch, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            last = (old == (unsigned)(bpc - 1));
            s_last = last;
        }
    }
    __syncthreads();
    if (!s_last) return;

    // ---- last arriver: deterministic reduction of all block partials (sc1 loads)
    if (tid < J * NV) {
        const int v = tid % NV, j = tid / NV;
        double a = 0;
        int k = j;
        for (; k + 3 * J < bpc; k += 4 * J) {
            const double x0 = ld_sc1(allp + (int64_t)k * NV + v);
            const double x1 = ld_sc1(allp + (int64_t)(k + J) * NV + v);
            const double x2 = ld_sc1(allp + (int64_t)(k + 2 * J) * NV + v);
            const double x3 = ld_sc1(allp + (int64_t)(k + 3 * J) * NV + v);
            a += x0; a += x1; a += x2; a += x3;
        }
        for (; k < bpc; k += J) a += ld_sc1(allp + (int64_t)k * NV + v);
        s_tmp[j * NV + v] = a;
    }
    __syncthreads();
    if (tid < NV) {
        double a = 0;
        for (int j = 0; j < J; j++) a += s_tmp[j * NV + tid];
        s_fin[tid] = a;
    }
    __syncthreads();
    if (wv != 0) return;
    const StepDesc dd = *dp;
    if (b.dbg_sums) {
        if (lane < NV) b.dbg_sums[ch * NV + lane] = s_fin[lane];
        if (lane == 0) b.arrive[ch] = 0;
        return;
    }
    __shared__ TrkChan s_c;
    if (dd.phaseC && lane < NV) s_fin[lane] = -s_fin[lane];  // :447-449
    if (lane == 0) {
        b.arrive[ch] = 0;
        s_c = *cp;
        finalize_step(p, b, ch, dd, s_fin, s_c);
        b.chan[ch] = s_c;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): lane 0's LDS store is visible
    __builtin_amdgcn_wave_barrier();
    const TrkChan cn = s_c;
    prepare_desc(p, cn, dd.pdi, dd.phaseC, lane, b.desc + ch);
}

// Prepare the StepDesc of every channel from its current state (start of a phase).
__global__ void track_prepare_kernel(TrkParams p, TrkBuffers b, int pdi, int phaseC)
{
    const int ch = blockIdx.x;
    const TrkChan c = b.chan[ch];
    prepare_desc(p, c, pdi, phaseC, threadIdx.x, b.desc + ch);
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
// nominal (skip + 1000 + countinx) ms position (quirk A.12); first 10-ms StepDesc.
__global__ void track_phase_c_init_kernel(TrkParams p, TrkBuffers b, int64_t skip)
{
    const int ch = blockIdx.x;
    __shared__ TrkChan s_c;
    if (threadIdx.x == 0) {
        TrkChan c = b.chan[ch];
        if (c.status == GNSS_OK) {
            const int cx = c.countinx;
            if (cx < 0) {
                c = b.snap[ch];
                c.countinx = cx;
                c.n1_target = b.n1 + cx;
            }
            const int64_t S = (int64_t)p.S;
            c.pos = (int64_t)((S - c.codedelay0 + 1 + (skip + b.n1 + cx) * S) *
                              (int64_t)p.dataBytesPerSample);
            c.index_int = 0;
            c.snrIndex = 1;
            c.nstep = 0;
            c.Index = b.n1 + cx;
            c.slot = b.n1 + cx;
            b.dvpre[(int64_t)ch * (p.rec_cap + 1)] = 0;
            b.chan[ch] = c;
        }
        s_c = c;
    }
    __syncthreads();
    const TrkChan c = s_c;
    if (c.status == GNSS_OK) prepare_desc(p, c, 10, 1, threadIdx.x, b.desc + ch);
}

hipError_t launch_track_step(const TrkParams& p, const TrkBuffers& b, int bpc, int sub,
                             hipStream_t s)
{
    dim3 grid(p.nch * bpc), block(kTrkThreads);
#define GNSS_STEP(NT_, SUB_)                                                                   \
    if (p.ntaps == NT_ && sub == SUB_) {                                                       \
        hipLaunchKernelGGL((track_step_kernel<NT_, SUB_>), grid, block, 0, s, p, b, bpc);      \
        return hipGetLastError();                                                              \
    }
    GNSS_STEP(3, 1) GNSS_STEP(3, 2) GNSS_STEP(3, 4)
    GNSS_STEP(11, 1) GNSS_STEP(11, 2) GNSS_STEP(11, 4)
#undef GNSS_STEP
    return hipErrorInvalidValue;
}

hipError_t launch_track_prepare(const TrkParams& p, const TrkBuffers& b, int pdi, int phaseC,
                                hipStream_t s)
{
    hipLaunchKernelGGL(track_prepare_kernel, dim3(p.nch), dim3(64), 0, s, p, b, pdi, phaseC);
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
    hipLaunchKernelGGL(track_phase_c_init_kernel, dim3(p.nch), dim3(64), 0, s, p, b, skip);
    return hipGetLastError();
}

}  // namespace gnss
