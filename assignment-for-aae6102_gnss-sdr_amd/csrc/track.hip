// track.hip — trackingCT.m correlator + DLL/PLL loop for gfx950 (MI355X).
//
// One launch = one tracking step (1 ms or 10 ms of IF) for every channel of the
// call. The loop is sequential per channel (step n+1's NCO depends on step n's
// discriminators, trackingCT.m:136-150 -> :79-107), so a step is a latency
// chain and the design minimises it:
//   * the previous step's last block prepares a StepDesc (numSample, colon
//     ranges per tap, carrier constants, end-of-step NCO values) so a block's
//     prologue is a handful of scalar loads;
//   * every lane owns 8*SUB consecutive samples (16-B loads of int8 I/Q issued
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

// Timing probe (GNSS_STAMPS): per-launch wall-clock stamps (100 MHz) of channel 0,
// row = [8 tail marks][kMaxBpc block starts][kMaxBpc computed][kMaxBpc tickets]; plain
// stores, one writer per word (atomics on shared words would queue behind each other).
constexpr int kStampRow = 8 + 3 * kMaxBpc;

__device__ __forceinline__ unsigned long long* stamp_row(const TrkBuffers& b)
{
    const unsigned long long cnt = __hip_atomic_load(b.stamps + (size_t)kStampSlots * kStampRow,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return b.stamps + (cnt % kStampSlots) * kStampRow;
}

__device__ __forceinline__ void stamp_max(unsigned long long* row, int k, unsigned long long v)
{
    row[k] = v;
}

// A wave-uniform value read from LDS into SGPRs (keeps it out of the VGPR budget).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni(int64_t v)
{
    const int lo = __builtin_amdgcn_readfirstlane((int)v);
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double uni(double v) { return __longlong_as_double(uni((int64_t)__double_as_longlong(v))); }

// Global-address-space views (pointers held in TrkBuffers would otherwise be flat:
// flat loads count on lgkmcnt too, so every LDS wait would also wait for them).
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const i32x4 g_i32x4;
typedef __attribute__((address_space(1))) double g_dbl;
typedef __attribute__((address_space(1))) long long g_i64;
typedef __attribute__((address_space(1))) unsigned g_u32;
typedef __attribute__((address_space(1))) unsigned long long g_u64;
typedef __attribute__((address_space(1))) const StepDesc g_desc;
typedef __attribute__((address_space(1))) const TrkChan g_chan;
typedef __attribute__((address_space(1))) const unsigned g_cu32;

__device__ __forceinline__ int4 ld_g16(const int8_t* p)
{
    const i32x4 v = *(g_i32x4*)p;
    return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ double ld_sc1(const double* ptr)
{
    return __hip_atomic_load((g_dbl*)ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_sc1(double* ptr, double v)
{
    __hip_atomic_store((g_dbl*)ptr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned atomic_add_agent(unsigned* p, unsigned v)
{
    return __hip_atomic_fetch_add((g_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void store_agent(unsigned* p, unsigned v)
{
    __hip_atomic_store((g_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void store_agent(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_store((g_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long load_agent(const unsigned long long* p)
{
    return __hip_atomic_load((g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The scalar tail's per-launch constants, held in registers for the whole step loop: built
// once from TrkParams at the launch's start and laundered through a volatile asm, so the
// compiler can neither re-load them from memory on every step (each reload was a scalar
// load and its wait on the tail's dependent chain) nor hoist anything across. The tail's
// functions take it in place of TrkParams (same field names; the int16 layout, fmt 1, never
// runs in the persistent loop).
struct TailK {
    double Fs, inv_Fs, codelength, S, codeFreqBasis, ms;
    double dll_r, dll_t1, dll_t10, pll_r, pll_t1, pll_t10, tau1code, tau1carr, qcap_dmax;
    int32_t exact_div, conv, given, chip_off, ntaps, iE, iP, iL, bps;
    int64_t file_len, buf_base, buf_len;
    const double* taps;
    const double* tap_post;
    static constexpr int fmt = 0;
    static constexpr const long long* pref_i = nullptr;
    static constexpr const long long* pref_q = nullptr;
    static constexpr const short* stage16 = nullptr;
};

template <class T>
__device__ __forceinline__ void launder_s(T& v)
{
    asm volatile("" : "+s"(v));
}

__device__ __forceinline__ TailK tail_k(const TrkParams& p)
{
    TailK k;
    k.Fs = p.Fs; k.inv_Fs = p.inv_Fs; k.codelength = p.codelength; k.S = p.S;
    k.codeFreqBasis = p.codeFreqBasis; k.ms = p.ms;
    k.dll_r = p.dll_r; k.dll_t1 = p.dll_t1; k.dll_t10 = p.dll_t10;
    k.pll_r = p.pll_r; k.pll_t1 = p.pll_t1; k.pll_t10 = p.pll_t10;
    k.tau1code = p.tau1code; k.tau1carr = p.tau1carr; k.qcap_dmax = p.qcap_dmax;
    k.exact_div = p.exact_div; k.conv = p.conv; k.given = p.given; k.chip_off = p.chip_off;
    k.ntaps = p.ntaps; k.iE = p.iE; k.iP = p.iP; k.iL = p.iL; k.bps = p.bps;
    k.file_len = p.file_len; k.buf_base = p.buf_base; k.buf_len = p.buf_len;
    k.taps = p.taps; k.tap_post = p.tap_post;
    launder_s(k.Fs); launder_s(k.inv_Fs); launder_s(k.codelength); launder_s(k.S);
    launder_s(k.codeFreqBasis); launder_s(k.ms);
    launder_s(k.dll_r); launder_s(k.dll_t1); launder_s(k.dll_t10);
    launder_s(k.pll_r); launder_s(k.pll_t1); launder_s(k.pll_t10);
    launder_s(k.tau1code); launder_s(k.tau1carr); launder_s(k.qcap_dmax);
    launder_s(k.exact_div); launder_s(k.conv); launder_s(k.given); launder_s(k.chip_off);
    launder_s(k.ntaps); launder_s(k.iE); launder_s(k.iP); launder_s(k.iL); launder_s(k.bps);
    launder_s(k.file_len); launder_s(k.buf_base); launder_s(k.buf_len);
    return k;
}

// CarrTime = k/Fs (trackingCT.m:104) as the IEEE quotient: one FMA-corrected
// reciprocal (host-verified exact for this Fs and k range, fast_div_exact) or a true division.
template <bool DIVIDE>
__device__ __forceinline__ double carr_time(double kd, double Fs, double rFs)
{
    if constexpr (DIVIDE) return kd / Fs;
    return div_markstein(kd, Fs, rFs);
}

// Wave(k) = (2*pi*(carrierFreq .* CarrTime)) + remPhase with the reference's roundings
template <bool DIVIDE>
__device__ __forceinline__ double wave_at(double kd, double f, double phi0, double Fs, double rFs)
{
    const double t = carr_time<DIVIDE>(kd, Fs, rFs);
    const double x = f * t;
    const double y = kTwoPi * x;
    return y + phi0;
}

// (sincos_small: gnss_internal.h, shared with the VT kernels)
#ifndef GNSS_FAST_SINCOS
#define GNSS_FAST_SINCOS 1
#endif
__device__ __forceinline__ void sincos_table(double x, double* sn, double* cs)
{
    if constexpr (GNSS_FAST_SINCOS) sincos_small(x, sn, cs);
    else sincos(x, sn, cs);
}

// sin/cos of a carrier phase Wave (up to ~3e5 rad): reduced by 2*pi as a double-double
// first (W - k*kTwoPi is exact: both are multiples of 2^-50 below 8 in magnitude), so the
// library's small-argument path runs instead of its Payne-Hanek reduction.
__device__ __forceinline__ void sincos_wave(double W, double* sn, double* cs)
{
    const double k = rint(W * (1.0 / kTwoPi));
    double r = __builtin_fma(-k, kTwoPi, W);
    r = __builtin_fma(-k, kTwoPiLo, r);
    sincos_table(r, sn, cs);
}

// The NCO state a step is prepared from.
struct NcoState {
    double remChip, remPhase, codeFreq, carrierFreq;
    int64_t numSample, pos, Index;
};

__device__ __forceinline__ NcoState nco_of(const TrkChan& c)
{
    return NcoState{c.remChip, c.remPhase, c.codeFreq, c.carrierFreq, c.numSample, c.pos, c.Index};
}

// rem(x, 2*pi) (trackingCT.m:106), exact like C fmod: |x| < 2^52 * 2*pi, the quotient
// is exact or one too large, and x - q*2*pi is then representable (a multiple of 2^-50
// below 8 in magnitude), so the FMA and the correction are exact.
__device__ __forceinline__ double rem_2pi(double x)
{
    const double q = trunc(div_const(x, kTwoPi, kInvTwoPi));
    double r = __builtin_fma(-q, kTwoPi, x);
    if (x >= 0) {
        if (r < 0) r += kTwoPi;
    } else {
        if (r > 0) r -= kTwoPi;
    }
    return r;
}

// numSample / delayValue of the step that follows state `c` (trackingCT.m:79-82 /
// :411-415; trackingCT_POS_updated.m:188-191 with ceil). The quotient q =
// fl(num / cps) is only rounded, so it is taken from num * (1/cps) (a refined reciprocal,
// within a few ulp of q) unless that lands within 1e-7 of a rounding boundary (.5 for
// round, an integer for ceil), where the IEEE division decides: the same n, without a
// division on the critical path. remSample (a record field only) is step_rem_sample().
struct StepSize {
    double cps, inv_cps, nd;  // nd = (double)n, exact
    int64_t n, dv;
};

// codeFreq / Fs, (r + pe) / Fs, k / Fs: the IEEE quotient (div_const, correctly rounded for
// every numerator)
template <class P>
__device__ __forceinline__ double over_fs(const P& p, double x)
{
    return div_const(x, p.Fs, p.inv_Fs);
}

// 1/x to about 1 ulp: hardware reciprocal and two Newton steps (the lanes' boundary search
// only needs 1e-9 relative; exactness never depends on it)
__device__ __forceinline__ double fast_rcp(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
}

template <class P>
__device__ __forceinline__ StepSize step_size(const P& p, const NcoState& c, int pdi, int phaseC)
{
    StepSize z;
    z.cps = over_fs(p, c.codeFreq);
    // 1/cps = Fs/codeFreq from the reciprocal of codeFreq (beside the quotient, not after it)
    z.inv_cps = p.Fs * fast_rcp(c.codeFreq);
    const double num = p.codelength * pdi - c.remChip;
    const double qa = num * z.inv_cps;
    if (p.conv || p.given) {  // ceil
        z.nd = fabs(qa - rint(qa)) > 1e-7 ? ceil(qa) : ceil(num / z.cps);
        z.n = (int64_t)z.nd;
        z.dv = z.n - (int64_t)(p.S * pdi);
        return z;
    }
    // round (half away from zero; q > 0)
    const double fr = qa - floor(qa);
    z.nd = fabs(fr - 0.5) > 1e-7 ? floor(qa + 0.5) : round(num / z.cps);
    z.n = (int64_t)z.nd;
    z.dv = phaseC ? c.numSample - (int64_t)(p.S * pdi)  // :411 (the previous step's numSample)
                  : z.n - (int64_t)(p.S * pdi);         // :82
    return z;
}

// remSample of the step (trackingCT.m:79 / :414), for the record
template <class P>
__device__ __forceinline__ double step_rem_sample(const P& p, const NcoState& c, int pdi, int phaseC)
{
    if (p.conv) return 0.0;  // (trackingCT_POS_updated.m has none)
    const double cps = over_fs(p, c.codeFreq);
    return phaseC ? (p.codelength * pdi - c.remChip) / cps : (p.codelength - c.remChip) / cps;
}

// Prepare the descriptor of the step that follows state `c` (trackingCT.m:79-107 /
// :411-441). Three waves work on it side by side (divergent lanes of one wave would run
// one after the other):
//   role 0 (code): lanes < ntaps build the colon of their tap, lane 0 the scalars;
//   role 1 (carrier): lanes < 32 the rotation table e^{i phi_m} (depends on f only);
//   role 2: lane 63 the next remPhase (needs numSample).
// `taps` = the tap spacings (a copy in LDS where the caller has one).
// An LDS double through a generic pointer known to point into LDS (a flat load would also
// wait on vmcnt, i.e. on this wave's outstanding global traffic).
__device__ __forceinline__ double lds_at(const double* q, int i)
{
    return ((__attribute__((address_space(3))) const double*)q)[i];
}

// The step's scalar fields and its numSample / file / staging checks (trackingCT.m:79-82,
// 108-112, 442): lane 0 writes them; GNSS_* or GNSS_OK returned in every lane.
template <class P>
__device__ __forceinline__ int desc_scalars(const P& p, const NcoState& c, const StepSize& z, int pdi,
                                            int phaseC, int lane, StepDesc* d)
{
    const int64_t n = z.n;
    // first sample of the fread (ftell / bytes per sample; bps = 1, 2 or 4 divides pos)
    const int64_t A = c.pos >> (p.bps == 4 ? 2 : p.bps == 2 ? 1 : 0);
    const int64_t sb = p.fmt ? 4 : 2;  // staged bytes per sample
    int bad = GNSS_OK;
    if (!(z.nd > 0) || z.nd > floor(p.S * pdi * 1.01) + 64) bad = GNSS_EINDEX;
    else if (p.bps * (A + n) > p.file_len) bad = (phaseC || p.conv || p.given) ? GNSS_EIO : GNSS_ENODATA;  // :108-112 / :442
    else if (sb * A < p.buf_base || sb * (A + n) > p.buf_base + p.buf_len) bad = GNSS_EIO;
    if (lane == 0) {
        double mr = 0.0, mi = 0.0;
        if (p.fmt == 1 && bad == GNSS_OK) {
            // rawsignal0DC = I - mean(I) + 1i*(Q - mean(Q)) over the n samples read
            // (trackingCT.m:84-88 / :417-421): integer sums, exact, from the group prefix
            // sums plus the samples of the partial group; mean = sum / n rounded once
            const int64_t gb = p.buf_base / 32;  // first staged 8-sample group
            auto pre = [&](int64_t k, long long& si, long long& sq) {
                const int64_t g = k >> 3;
                si = p.pref_i[g - gb];
                sq = p.pref_q[g - gb];
                for (int64_t j = 8 * g; j < k; j++) {
                    si += p.stage16[2 * j];
                    sq += p.stage16[2 * j + 1];
                }
            };
            long long i0, q0, i1, q1;
            pre(A, i0, q0);
            pre(A + n, i1, q1);
            mr = (double)(i1 - i0) / (double)n;
            mi = (double)(q1 - q0) / (double)n;
        }
        d->mu_r = mr;
        d->mu_i = mi;
        d->n = n;
        d->delayValue = z.dv;
        d->A = A;
        d->g_first = A >> 3;
        d->g_last = (A + n - 1) >> 3;
        d->Index = c.Index;
        d->d = z.cps;
        d->inv_d = z.inv_cps;
        d->rc0 = c.remChip;
        d->pdi = pdi;
        d->phaseC = phaseC;
        d->bad = bad;
    }
    return bad;
}

// The replica colons of the taps (trackingCT.m:96-102): lane s < ntaps stores tap s's colon
// start / end (all the correlator lanes need), then checks its replica index range and, for
// the prompt, the next remChip. Returns GNSS_EINDEX in a lane whose index range fails.
template <class P>
__device__ __forceinline__ int desc_taps(const P& p, const NcoState& c, const StepSize& z, int pdi,
                                         int lane, StepDesc* d, const double* taps, const double* posts)
{
    if (lane >= p.ntaps) return GNSS_OK;
    // t = (0 + Spacing + remChip) : cps : ((numSample-1)*cps + Spacing + remChip) (:96-98);
    // n - 1 as the exact double z.nd - 1 (no integer round trip on the critical path)
    const double cps = z.cps;
    const double tap = taps ? lds_at(taps, lane) : p.taps[lane];
    const double post = posts ? lds_at(posts, lane) : p.tap_post[lane];
    const double a = (0 + tap) + c.remChip;
    const double bb = ((z.nd - 1) * cps + tap) + c.remChip;
    const Colon col = colon_make_hint2(a, cps, bb, z.n - 1, z.nd - 1);
    d->tap_a[lane] = col.a;
    d->tap_c[lane] = col.c;
    // (after the stores: the lanes need only a, c) elements 0 and n-1 of a colon of n - 1
    // intervals are a and c
    const bool whole = col.n == z.n - 1;
    const double c0 = ceil(col.a + post);
    const double c1 = ceil(col.c + post);
    if (lane == p.iP) {
        // remChip = (t_CodePrompt(numSample) + codeFreq/Fs) - codeFreqBasis*ms*pdi (:102);
        // trackingCT_POS_updated.m:220: ... - signal.codelength*pdi (codeFreq/Fs = cps)
        d->remChip_next = ((whole ? col.c : colon_elem(col, z.n - 1)) + cps) -
                          (p.conv ? p.codelength * pdi : p.codeFreqBasis * p.ms * pdi);
    }
    // Code index ceil(t) + 1 + chip_off within [1, 1023*pdi + 2 + chip_off]
    return (!whole || c0 + p.chip_off < 0 || c1 > 1023.0 * pdi + 1) ? GNSS_EINDEX : GNSS_OK;
}

// remPhase after the step (trackingCT.m:104-106) and remSample (:79 / :414, a record field),
// from the descriptor alone
template <class P>
__device__ __forceinline__ void desc_rem(const P& p, StepDesc* d)
{
    const double nd = (double)d->n;
    d->remPhase_next = rem_2pi(kTwoPi * (d->f * over_fs(p, nd)) + d->phi0);
    d->remSample = p.conv ? 0.0  // (trackingCT_POS_updated.m has none)
                 : d->phaseC ? (p.codelength * d->pdi - d->rc0) / d->d : (p.codelength - d->rc0) / d->d;
}

// Prepare the descriptor of the step that follows state `c` (trackingCT.m:79-107 /
// :411-441). Waves work on it side by side (divergent lanes of one wave would run one
// after the other):
//   role 0 (code): lanes < ntaps build the colon of their tap; without `split` lane 0 also
//     the scalars and the checks, and the result folds into `bad`;
//   role 1 (carrier): lanes < 32 the rotation table e^{i phi_m} (depends on f only);
//   role 2: lane 63 the next remPhase and remSample (needs numSample and the table's f);
//   role 3 (split only): the scalars and their checks.
// split (the persistent loop): roles 0 / 1 / 3 on three waves in the tail, role 2 by the
// flush wave during the next step (desc_rem): the tail's code chain is the colon alone.
// `taps` / `posts` = the tap spacings / prompt offsets (copies in LDS where the caller has).
template <class P>
__device__ __forceinline__ void prepare_desc_i(const P& p, const NcoState& c, int pdi, int phaseC, int role,
                             int lane, StepDesc* d, const double* taps = nullptr,
                             unsigned long long* dbg = nullptr, const double* posts = nullptr,
                             bool split = false)
{
    if (role == 1) {
        // carrier increment delta = 2*pi*f/Fs as a double-double; dhi has 48 bits so
        // m*dhi (m < 32) is exact. phi[m] is the rotation basis of lane_correlate, not a
        // quantity of the reference (the per-sample Wave is formed exactly and eta takes up
        // the difference), so its quotients need no correct rounding: Markstein's step alone
        const double f = c.carrierFreq;
        double dhi, dlo;
        {
            const double p0 = kTwoPi * f;
            double pe = __builtin_fma(kTwoPi, f, -p0);
            pe = pe + kTwoPiLo * f;
            const double q = div_markstein(p0, p.Fs, p.inv_Fs);
            const double r = __builtin_fma(-q, p.Fs, p0);
            const double ql = div_markstein(r + pe, p.Fs, p.inv_Fs);
            dhi = __longlong_as_double(__double_as_longlong(q) & ~0x1FLL);
            dlo = (q - dhi) + ql;
        }
        if (lane < kLaneMax) {
            // phi[m] rounds once (m*dhi is exact)
            const double ph = (double)lane * dhi + (double)lane * dlo;
            double sn, cs;
            sincos_table(ph, &sn, &cs);
            d->phi[lane] = ph;
            d->rcs[lane] = make_double2(cs, sn);
            if (lane == 0) {
                d->f = f;
                d->phi0 = c.remPhase;
                d->dhi = dhi;
                d->dlo = dlo;
            }
        }
        return;
    }
    const StepSize z = step_size(p, c, pdi, phaseC);
    if (role == 2) {
        if (lane == 63) {
            // remPhase = rem(Wave(numSample+1), 2*pi) (:104-106)
            d->remPhase_next = rem_2pi(kTwoPi * (c.carrierFreq * over_fs(p, z.nd)) + c.remPhase);
        } else if (lane == 62) {
            d->remSample = step_rem_sample(p, c, pdi, phaseC);  // (off the code role's path)
        }
        return;
    }
    if (role == 3) {
        (void)desc_scalars(p, c, z, pdi, phaseC, lane, d);
        return;
    }
    if (dbg && lane == 0) dbg[0] = wall_clock64();
    const int tb = desc_taps(p, c, z, pdi, lane, d, taps, posts);
    if (dbg && lane == 0) dbg[1] = wall_clock64();
    // the first failing lane's code wins (every failing tap lane has GNSS_EINDEX)
    const int btap = __ballot(tb != GNSS_OK) ? GNSS_EINDEX : GNSS_OK;
    if (split) {
        if (lane == 0) d->bad_tap = btap;
        return;
    }
    const int bs = desc_scalars(p, c, z, pdi, phaseC, lane, d);
    if (lane == 0) {
        d->bad = bs != GNSS_OK ? bs : btap;
        d->bad_tap = GNSS_OK;
    }
}
// out-of-line copy for the persistent kernel (keeps its register budget)
__device__ __noinline__ void prepare_desc(const TrkParams& p, const NcoState& c, int pdi, int phaseC, int role, int lane, StepDesc* d)
{
    prepare_desc_i(p, c, pdi, phaseC, role, lane, d);
}

// All three roles of prepare_desc by a 192-thread block (wave = role).
__device__ __forceinline__ void prepare_desc_block(const TrkParams& p, const NcoState& c, int pdi, int phaseC,
                                                   StepDesc* d)
{
    prepare_desc(p, c, pdi, phaseC, threadIdx.x >> 6, threadIdx.x & 63, d);
}


// atan for the PLL discriminator. The classic four-interval reduction with an
// 11-term odd polynomial (error < 1 ulp). Its constants are literals materialised into
// scalar registers at their use (kc(): a volatile asm the compiler can neither hoist out of
// the step loop -- the library atan cost +40 VGPRs over the correlator -- nor turn into a
// memory load: a table read here was a flat load of global memory on the PLL's critical
// path, several hundred cycles).
__device__ __forceinline__ double kc(double v)
{
    asm volatile("" : "+s"(v));
    return v;
}

__device__ __forceinline__ double atan_tab(double x)
{
    const double ax = fabs(x);
    if (!(ax < 0x1p66)) return x != x ? x : copysign(kc(1.57079632679489655800e+00) + kc(6.12323399573676603587e-17), x);
    int id;
    double y;
    if (ax < 0.4375) {
        if (ax < 0x1p-27) return x;
        id = -1;
        y = x;
    } else if (ax < 1.1875) {
        if (ax < 0.6875) { id = 0; y = (2.0 * ax - 1.0) / (2.0 + ax); }
        else { id = 1; y = (ax - 1.0) / (ax + 1.0); }
    } else if (ax < 2.4375) {
        id = 2; y = (ax - 1.5) / (1.0 + 1.5 * ax);
    } else {
        id = 3; y = -1.0 / ax;
    }
    const double z = y * y, w = z * z;
    const double s1 = z * (kc(3.33333333333329318027e-01) + w * (kc(1.42857142725034663711e-01) +
                      w * (kc(9.09088713343650656196e-02) + w * (kc(6.66107313738753120669e-02) +
                      w * (kc(4.97687799461593236017e-02) + w * kc(1.62858201153657823623e-02))))));
    const double s2 = w * (kc(-1.99999999998764832476e-01) + w * (kc(-1.11111104054623557880e-01) +
                      w * (kc(-7.69187620504482999495e-02) + w * (kc(-5.83357013379057348645e-02) +
                      w * kc(-3.65315727442169155270e-02)))));
    if (id < 0) return y - y * (s1 + s2);
    const double hi = id == 0 ? kc(4.63647609000806093515e-01) : id == 1 ? kc(7.85398163397448278999e-01)
                    : id == 2 ? kc(9.82793723247329054082e-01) : kc(1.57079632679489655800e+00);
    const double lo = id == 0 ? kc(2.26987774529616870924e-17) : id == 1 ? kc(3.06161699786838301793e-17)
                    : id == 2 ? kc(1.39033110312309984516e-17) : kc(6.12323399573676603587e-17);
    const double r = hi - ((y * (s1 + s2) - lo) - y);
    return x < 0 ? -r : r;
}

// The DLL / PLL update of one step (trackingCT.m:136-150 / :469-483), fp64, same
// operation order as the reference; phase C keeps T = 0.001 (:473,480). Every lane
// that calls it computes the same values.
struct LoopUpd {
    double DLLdiscri, code_output, codeFreq, PLLdiscri, carrier_output, carrierFreq;
};

template <class P>
__device__ __forceinline__ LoopUpd loop_update_i(const P& p, const TrkChan& c, double E_i,
                                               double E_q, double P_i, double P_q, double L_i,
                                               double L_q, int pdi, int phaseC, int which = 3)
{
    // which: 1 = the DLL half only, 2 = the PLL half only, 3 = both (wave-uniform)
    LoopUpd u{0, 0, 0, 0, 0, 0};
    // trackingCT_POS_updated.m:257-258,266-267 use t = signal.ms at every pdi
    const double T = p.conv ? p.ms : phaseC ? 0.001 : (0.001 * pdi);
    if (which & 1) {
        const double E = sqrt(E_i * E_i + E_q * E_q);
        const double L = sqrt(L_i * L_i + L_q * L_q);
        u.DLLdiscri = 0.5 * (E - L) / (E + L);
        // (tau2/tau1 and T/tau1 are the host's IEEE quotients, TrkParams.dll_*)
        const double tq = pdi == 1 ? p.dll_t1 : (phaseC || p.conv) ? p.dll_t10 : T / p.tau1code;
        u.code_output = c.code_outputLast + p.dll_r * (u.DLLdiscri - c.DLLdiscriLast) + u.DLLdiscri * tq;
        // trackingCT_POS_updated.m:262: codeFreq = codeFreqBasis + codeNco
        u.codeFreq = p.conv ? p.codeFreqBasis + u.code_output : p.codeFreqBasis - u.code_output;
    }
    if (which & 2) {
        u.PLLdiscri = div_const(atan_tab(P_q / P_i), kTwoPi, kInvTwoPi);
        u.carrier_output = c.carrier_outputLast +
                           p.pll_r * (u.PLLdiscri - c.PLLdiscriLast) +
                           u.PLLdiscri * (pdi == 1 ? p.pll_t1 : (phaseC || p.conv) ? p.pll_t10 : T / p.tau1carr);
        u.carrierFreq = c.carrierFreqBasis + u.carrier_output;
    }
    return u;
}
// out-of-line copy for the persistent kernel (keeps its register budget)
__device__ __noinline__ LoopUpd loop_update(const TrkParams& p, const TrkChan& c, double E_i, double E_q, double P_i, double P_q, double L_i, double L_q, int pdi, int phaseC)
{
    return loop_update_i(p, c, E_i, E_q, P_i, P_q, L_i, L_q, pdi, phaseC);
}


// Per-step values of the finished step the side writers need (read before the
// next descriptor overwrites the current one).
struct StepOut {
    int64_t n, delayValue;
    double remSample, remChip, remPhase;
    int pdi, phaseC;
};

// TckResultCT fields of the step (trackingCT.m:153-170 / :507-524) and the phase-A
// P_i kept for the bit-edge search. `s` = the step's (negated in phase C) sums.
// The prefix of delayValue sums the step's codedelay reads (quirk A.11): cumulative
// column `cols` of an nsv x N matrix read column-major, capped at the step count.
__device__ __forceinline__ int64_t record_cols(const TrkParams& p, const TrkChan& c, int phaseC)
{
    const int64_t Index = c.Index + (phaseC ? 10 : 1);
    const int64_t nstep = c.nstep + 1;
    if (p.conv) return nstep;  // sum(delayValue(svIndex,(1:Index))), trackingCT_POS_updated.m:290
    int64_t cols = 0;  // (32-bit quotient: Index < 2^31; a 64-bit one is ~150 scalar ops)
    if (Index >= c.sv1) cols = (int64_t)((uint32_t)(Index - c.sv1) / (uint32_t)p.nsv) + 1;
    return cols > nstep ? nstep : cols;
}

// `pre`, when given, holds dvpre[nstep] and dvpre[cols] loaded ahead by the caller.
// part (the persistent loop splits a step's record over two blocks, each writing its half
// while the exchange is in flight, so neither becomes the step's last block; every block holds
// the same state): 1 = the sums and the codedelay bookkeeping (delayValue prefix sums, `pre`),
// 2 = the loop / NCO fields, the mod() fields and the 1-ms P_i series; 3 = all.
__device__ __forceinline__ void write_record_i(const TrkParams& p, const TrkBuffers& b, int ch, const TrkChan& c,
                             const StepOut& o, const LoopUpd& u, const double* s,
                             const int64_t* pre = nullptr, int part = 3)
{
    const double P_i = s[2 * p.iP], P_q = s[2 * p.iP + 1];
    const int64_t slot = c.slot;
    // global-address-space views: flat stores count on lgkmcnt too, so every LDS wait after
    // one (s_fin, the state) would wait for the store's completion
    g_dbl* r = (g_dbl*)(b.rec + ((int64_t)ch * p.rec_cap + slot) * GNSS_NFIELDS);
    if (part & 1) {
        const int64_t col = c.nstep;          // 0-based IndexSmall - 1
        g_i64* dvpre = (g_i64*)(b.dvpre + (int64_t)ch * (p.rec_cap + 1));
        const int64_t dvsum = (pre ? pre[0] : dvpre[col]) + o.delayValue;
        dvpre[col + 1] = dvsum;
        const int64_t nstep = col + 1;
        // sum(delayValue(1:Index)) over an nsv x N matrix (column-major, quirk A.11)
        const int64_t cols = record_cols(p, c, o.phaseC);
        const double codedelay =
            (double)c.codedelay0 + (double)(cols == nstep ? dvsum : (pre ? pre[1] : dvpre[cols]));
        if (slot < p.rec_cap) {
            r[GNSS_F_P_i] = P_i;                     r[GNSS_F_P_q] = P_q;
            r[GNSS_F_E_i] = s[2 * p.iE];             r[GNSS_F_E_q] = s[2 * p.iE + 1];
            r[GNSS_F_L_i] = s[2 * p.iL];             r[GNSS_F_L_q] = s[2 * p.iL + 1];
            r[GNSS_F_codedelay] = codedelay;
        }
    }
    if (part & 2) {
        const int64_t pos = c.pos + p.bps * o.n;  // ftell after fread
        const double absS = (double)pos;
        const double m = fmod_pos(absS / p.dataBytesPerSample, p.Fs * p.ms);  // mod() of positives
        if (slot < p.rec_cap) {
            r[GNSS_F_PLLdiscri] = u.PLLdiscri;       r[GNSS_F_DLLdiscri] = u.DLLdiscri;
            r[GNSS_F_remChip] = o.remChip;
            r[GNSS_F_codeFreq] = u.codeFreq;         r[GNSS_F_carrierFreq] = u.carrierFreq;
            // (trackingCT_POS_updated.m:289 has no remSample: the slot holds absoluteSampleCodedelay)
            r[GNSS_F_remPhase] = o.remPhase;         r[GNSS_F_remSample] = p.conv ? m : o.remSample;
            r[GNSS_F_numSample] = (double)o.n;       r[GNSS_F_delayValue] = (double)o.delayValue;
            r[GNSS_F_absoluteSample] = absS;         r[GNSS_F_codedelay2] = m;
        }
        if (!o.phaseC && slot < b.n1) ((g_dbl*)b.p_i_1ms)[(int64_t)ch * b.n1 + slot] = P_i;
    }
}
// out-of-line copy for the persistent kernel (keeps its register budget)
__device__ __noinline__ void write_record(const TrkParams& p, const TrkBuffers& b, int ch, const TrkChan& c, const StepOut& o, const LoopUpd& u, const double* s)
{
    write_record_i(p, b, ch, c, o, u, s);
}


// C/N0 of one 20-sample window of |P|^2 (trackingCT.m:124-131; moment method), out of
// line: it runs once every 20 steps and its log/hypot/atan2 would otherwise sit in the
// registers of the persistent step loop.
// (out of line: keeps the persistent step loop's register budget; the arithmetic is
// cn0_moment's, shared with the vector-tracking steps)
__device__ __noinline__ double cn0_estimate(const double (&Z)[20], double T)
{
    return cn0_moment(Z, T);
}

// The channel state after the step, with the C/N0 estimator (trackingCT.m:120-134).
__device__ __forceinline__ void write_state_i(const TrkParams& p, const TrkBuffers& b, int ch, TrkChan* g,
                            const TrkChan& c, const StepOut& o, const LoopUpd& u, const double* s,
                            bool io = true)
{
    const double P_i = s[2 * p.iP], P_q = s[2 * p.iP + 1];
    int index_int = c.index_int + 1;
    int snrIndex = c.snrIndex;
    const double zk = P_i * P_i + P_q * P_q;
    for (int k = 0; k < 20; k++) g->Zk[k] = k == index_int - 1 ? zk : c.Zk[k];
    if (index_int % 20 == 0 && io) {
        double Z[20];
#pragma unroll
        for (int k = 0; k < 20; k++) Z[k] = k == index_int - 1 ? zk : c.Zk[k];
        const double cn = cn0_estimate(Z, 1 * p.ms * o.pdi);
        double* cn0 = o.phaseC ? b.cn0_10 : b.cn0_1;
        if (snrIndex <= p.cn0_cap) cn0[(int64_t)ch * p.cn0_cap + snrIndex - 1] = cn;
        index_int = 0;
        snrIndex += 1;
    } else if (index_int % 20 == 0) {  // (a replica of the state: counters only)
        index_int = 0;
        snrIndex += 1;
    }
    g->remChip = o.remChip;
    g->remPhase = o.remPhase;
    g->remSample = o.remSample;
    g->carrier_outputLast = u.carrier_output;
    g->PLLdiscriLast = u.PLLdiscri;
    g->code_outputLast = u.code_output;
    g->DLLdiscriLast = u.DLLdiscri;
    g->codeFreq = u.codeFreq;
    g->carrierFreq = u.carrierFreq;
    g->numSample = o.n;
    g->pos = c.pos + p.bps * o.n;
    g->Index = c.Index + (o.phaseC ? 10 : 1);
    g->nstep = c.nstep + 1;
    g->slot = c.slot + 1;
    g->index_int = index_int;
    g->snrIndex = snrIndex;
}
// out-of-line copy for the persistent kernel (keeps its register budget)
__device__ __noinline__ void write_state(const TrkParams& p, const TrkBuffers& b, int ch, TrkChan* g, const TrkChan& c, const StepOut& o, const LoopUpd& u, const double* s, bool io)
{
    write_state_i(p, b, ch, g, c, o, u, s, io);
}

// The same update in place (the persistent loop's single LDS copy of the state): one Zk
// element changes per step, nothing is copied. C/N0 only where `io`.
__device__ __forceinline__ void update_state_inplace(const TrkParams& p, const TrkBuffers& b, int ch,
                                                     TrkChan& c, const StepOut& o, const LoopUpd& u,
                                                     const double* s, bool io)
{
    const double P_i = s[2 * p.iP], P_q = s[2 * p.iP + 1];
    int index_int = c.index_int + 1;  // 1..20
    int snrIndex = c.snrIndex;
    c.Zk[index_int - 1] = P_i * P_i + P_q * P_q;
    if (index_int % 20 == 0) {
        if (io) {
            double Z[20];
#pragma unroll
            for (int k = 0; k < 20; k++) Z[k] = c.Zk[k];
            const double cn = cn0_estimate(Z, 1 * p.ms * o.pdi);
            g_dbl* cn0 = (g_dbl*)(o.phaseC ? b.cn0_10 : b.cn0_1);
            if (snrIndex <= p.cn0_cap) cn0[(int64_t)ch * p.cn0_cap + snrIndex - 1] = cn;
        }
        index_int = 0;
        snrIndex += 1;
    }
    const int64_t pos = c.pos, Index = c.Index, nstep = c.nstep, slot = c.slot;
    c.remChip = o.remChip;
    c.remPhase = o.remPhase;
    c.remSample = o.remSample;
    c.carrier_outputLast = u.carrier_output;
    c.PLLdiscriLast = u.PLLdiscri;
    c.code_outputLast = u.code_output;
    c.DLLdiscriLast = u.DLLdiscri;
    c.codeFreq = u.codeFreq;
    c.carrierFreq = u.carrierFreq;
    c.numSample = o.n;
    c.pos = pos + p.bps * o.n;
    c.Index = Index + (o.phaseC ? 10 : 1);
    c.nstep = nstep + 1;
    c.slot = slot + 1;
    c.index_int = index_int;
    c.snrIndex = snrIndex;
}


}  // namespace

// One lane's 8*SUB samples starting at window-relative sample ks of the step described
// by `dp` (trackingCT.m:96-118): the lane's NT tap sums, I = imag(raw .* carrsig) in oI,
// Q = real(raw .* carrsig) in oQ. `raw` = the lane's 16-B IF groups, `myslot` = this
// lane's column of the LDS running-sum slots (slot m at myslot[m * kTrkThreads]),
// `zero` = an LDS double2 holding 0 (read when a tap's boundary is outside the subgroup).
// RELOAD (descriptor in LDS): read the rotation table where it is used rather than
// letting the compiler hoist all 96 values into VGPRs.
//   * carrier: w_m = x_m * e^{i(Wave(k_m) - Wave(k_0))} in the frame of the lane's
//     first sample, Wave(k) rounded exactly as the reference rounds it; the rotation
//     is the table e^{i phi_m} plus the first-order residue eta = (Wave(k_m) - Wave(k_0))
//     - phi_m (|eta| ~ 1e-10). One sincos per lane rotates the lane's sums back;
//   * code: M * codeFreq/Fs < 1, so every tap's replica Code(ceil(t)+1) changes at most
//     once in the lane, at sample p (exact colon arithmetic at the lane start, exact
//     re-evaluation within 1e-6 sample of a boundary). With the running sum of w in
//     LDS, the tap sum is v1*Sum + (v0 - v1)*Prefix(p).
// The lane's 16-B IF groups: in registers (step kernel) or staged in LDS (persistent loop)
__device__ __forceinline__ double2 ld_rcs(const StepDesc* d, int m) { return d->rcs[m]; }
__device__ __forceinline__ double2 ld_rcs(g_desc* d, int m)
{
    typedef __attribute__((address_space(1))) const double g_cdbl;
    g_cdbl* q = (g_cdbl*)&d->rcs[m];
    return make_double2(q[0], q[1]);
}

template <int SUB> struct RegRaw {
    const int4 (&r)[SUB];
    __device__ __forceinline__ int4 get(int j) const { return r[j]; }
};
struct LdsRaw {
    const int4* p;  // this lane's group j at p[j * kTrkThreads]
    __device__ __forceinline__ int4 get(int j) const { return p[j * kTrkThreads]; }
};

// Timing-probe builds only (tools/build_probe.sh, never the product library): bit 1 drops
// the lane's sincos, bit 2 the per-tap boundary search, bit 4 the per-sample Wave / eta
// (the rotation table alone), bit 8 the whole lane correlate. Their sums are wrong; they time
// (and count the instructions of) the correlator's parts. Bit 16 repeats the scalar tail
// (right sums, the same descriptor) four extra times per step between stamps 18 and 19.
#ifndef GNSS_CORR_PROBE
#define GNSS_CORR_PROBE 0
#endif
#ifndef GNSS_IO_DR_WAVE
#define GNSS_IO_DR_WAVE 2  // (A/B: the wave of block 0 that runs the remPhase role)
#endif
#ifndef GNSS_SWEEP_IO_ALL
#define GNSS_SWEEP_IO_ALL 0  // (A/B: block 0's wave 1 polls after its flush, as the other blocks' do)
#endif
#ifndef GNSS_FLUSH_PROBE
#define GNSS_FLUSH_PROBE 0  // (A/B probe: 1 = block 0 writes no record)
#endif

// (GNSS_QCAP: gnss_internal.h)
// The C/A code bits as the lanes hold them (lane w < 32: word w, bit i of word w = chip
// 32 w + i of the 1023, bit set = -1) extended circularly for the tap window below: bit 31 of
// word 31 (index 1023) = chip 0, word 32 (lane 32) = chips 1..32, word 33 = chips 33..64, so
// any 64-bit run starting at an index <= 1022 reads the code without a wrap. Call with every
// lane of the wave active; lanes < 31 keep their word.
__device__ __forceinline__ unsigned ca_bits_ext(unsigned cabits, int lane)
{
    const unsigned w0 = __shfl(cabits, 0, 64), w1 = __shfl(cabits, 1, 64), w2 = __shfl(cabits, 2, 64);
    if (lane == 31) return cabits | ((w0 & 1u) << 31);
    if (lane == 32) return (w0 >> 1) | (w1 << 31);
    if (lane == 33) return (w1 >> 1) | (w2 << 31);
    return cabits;
}

#ifndef GNSS_SWP
#define GNSS_SWP 0  // (lane_correlate: 1 / 2 = the next sample's Wave formed one sample ahead)
#endif
#ifndef GNSS_REGCAP
#define GNSS_REGCAP 0  // (lane_correlate: 1 = tap prefixes captured in registers at 3 taps)
#endif
#ifndef GNSS_PHI_REG
#define GNSS_PHI_REG 0  // (lane_correlate: 1 = the rotation basis phi[m] formed in registers)
#endif
#ifndef GNSS_TAPWIN
#define GNSS_TAPWIN 1  // (A/B: 0 = per-tap colon element, scalar tap loads and two code shuffles)
#endif
template <int NT, int SUB, bool DIVIDE, bool RELOAD, int FMT, class Desc, class Raw>
__device__ __forceinline__ void lane_correlate(const TrkParams& p, const Desc* dp, const Raw& raw,
                                               int64_t ks, unsigned cabits, double2* myslot,
                                               const double2* zero, double (&oI)[NT], double (&oQ)[NT],
                                               const double* posts = nullptr)
{
    constexpr int M = 8 * SUB;
    constexpr int T = kTrkThreads;
    // Capture queue (the persistent loop above 3 taps, where the host has checked that a lane
    // holds at most kQcapMax distinct interior boundaries, TrkParams.qcap): a tap's prefix is
    // the lane's running sum at its last sample before the boundary, cap. Instead of reading
    // every tap's slot after every 8-sample subgroup (NT x SUB LDS reads and 2 NT x SUB adds),
    // the running sum is stored at the distinct interior capture samples only (queue entry =
    // the sample's rank among them), and each tap reads its one entry in the epilogue. The
    // value is the same running sum, so the same bits (pre = v + 0.0 either way).
    constexpr bool QC = RELOAD && (GNSS_QCAP == 2 || (GNSS_QCAP && NT > 3));
    if constexpr ((GNSS_CORR_PROBE & 8) != 0) {  // (probe: no correlate at all)
#pragma unroll
        for (int s = 0; s < NT; s++) { oI[s] = 0.0; oQ[s] = 0.0; }
        return;
    }
    const int64_t n = uni(dp->n);
    const double d = uni(dp->d), inv_d = uni(dp->inv_d);
    const double f = uni(dp->f), phi0 = uni(dp->phi0);
    const double Fs = p.Fs, rFs = p.inv_Fs;

    // ---- valid samples of the lane: [lo, hi) (only the window's two end lanes are partial);
    // window-relative sample indices are below 2^31 (a step reads <= kMaxBpc * 256 * 32 samples),
    // so the index arithmetic is 32-bit
    const int ksi = (int)ks, ni = (int)n;
    const int lo = ksi < 0 ? (-ksi < M ? -ksi : M) : 0;
    const int hi = ni - ksi < M ? (ni - ksi > 0 ? ni - ksi : 0) : M;

    // ---- code replica per tap: chip c0 at the first valid sample, the sample p of the
    // lane's (single) chip boundary, and the two code values around it
    const int kfi0 = ksi + lo;
    const int kfi = kfi0 < 0 ? 0 : (kfi0 > ni - 1 ? ni - 1 : kfi0);
    const int64_t kf = kfi;
    int cap[NT];
    // code values around each tap's boundary as sign bits (bit s set: -1): a0 before it,
    // a1 after; v1 = a1 and dv = a0 - a1 are rebuilt in the epilogue (2 VGPRs, not 4*NT)
    unsigned neg0 = 0u, neg1 = 0u;
    // Tap window (GNSS_TAPWIN, the persistent loop: descriptor and tap offsets in LDS): the
    // parts of colon_elem(col_s, kf) that no tap changes (which end of the colon kf is counted
    // from, (double)kf * d, (double)(n - 1 - kf) * d) once per lane; every tap's colon ends read
    // from LDS into vector registers (broadcast reads, no scalar round trip per tap); and the
    // code bits of all taps from ONE 64-bit window of the circularly extended code table
    // (ca_bits_ext) instead of two shuffles per tap: the taps' chips at the lane start lie within
    // kTapSpan chips of each other (the host checks the tap offsets). The same values as
    // colon_elem and ca_index32, so the same bits.
    // Round 6: every tap's common case straight-line and branch-free (the colon end by selects,
    // 32-bit indices), and ONE rare branch for the lanes where any tap's boundary is too close to
    // call in floating point or that hold the colon's middle element: they redo that tap's search
    // exactly as before (the fast path's R is fused, the exact path's is not; both give the same
    // cap wherever the fast path is used: its R lies more than 1e-6 from an integer).
    constexpr bool TW = GNSS_TAPWIN && RELOAD && (GNSS_CORR_PROBE & 66) == 0;
    if constexpr (TW) {
        const int nn = ni - 1;
        const bool mid = 2 * kfi == nn, lower = kfi <= nn / 2;
        const double KD = (double)kfi * d, NKD = (double)(nn - kfi) * d;
        const double kend = lower ? KD : -NKD;  // a + KD (lower half), c - NKD = c + (-NKD) (upper)
        const double dk = (double)(kfi - ksi);
        int c0i[NT];
        int cmin = 0x7fffffff;
        bool exact = mid;
#pragma unroll
        for (int s = 0; s < NT; s++) {
            const double a = lds_at(dp->tap_a, s), c = lds_at(dp->tap_c, s);
            const double t0 = ((lower ? a : c) + kend) + lds_at(posts, s);
            const double c0 = ceil(t0);
            const double R = __builtin_fma(c0 - t0, inv_d, dk);  // samples to the boundary
            exact = exact || fabs(R - rint(R)) < 1e-6;
            const int pb = (int)floor(R) + 1;
            cap[s] = (pb < M ? pb : M) - 1;  // Prefix(p) = running sum through sample p-1
            c0i[s] = (int)c0;
        }
        if (exact) {  // (rare) this lane's search as the general form does it, tap by tap
#pragma unroll
            for (int s = 0; s < NT; s++) {
                const double a = lds_at(dp->tap_a, s), c = lds_at(dp->tap_c, s);
                const double post = lds_at(posts, s);
                const double t0 = (mid ? (a + c) / 2 : lower ? a + KD : c - NKD) + post;
                const double c0 = ceil(t0);
                const double R = dk + (c0 - t0) * inv_d;
                const double rr = rint(R);
                int pb = (int)floor(R) + 1;
                if (fabs(R - rr) < 1e-6) {  // too close to call in floating point: exact colon value
                    const int ms = (int)rr;
                    pb = ms;
                    const int64_t kx = ks + ms;
                    if (ms >= 0 && ms < M && kx >= 0 && kx <= n - 1)
                        pb = ceil(colon_elem(Colon{a, d, c, (int64_t)nn}, kx) + post) > c0 ? ms : ms + 1;
                }
                cap[s] = (pb < M ? pb : M) - 1;
                c0i[s] = (int)c0;
            }
        }
#pragma unroll
        for (int s = 0; s < NT; s++) {
            if constexpr ((GNSS_CORR_PROBE & 32) != 0) cap[s] = M - 1 - s;
            cmin = c0i[s] < cmin ? c0i[s] : cmin;
        }
        const unsigned ib = ca_index32(cmin + p.chip_off);
        const unsigned wlo = __shfl(cabits, (int)(ib >> 5), 64), whi = __shfl(cabits, (int)(ib >> 5) + 1, 64);
        const unsigned long long W = (((unsigned long long)whi << 32) | wlo) >> (ib & 31);
#pragma unroll
        for (int s = 0; s < NT; s++) {
            const int o = c0i[s] - cmin;
            neg0 |= (unsigned)((W >> o) & 1ull) << s;
            neg1 |= (unsigned)((W >> (o + 1)) & 1ull) << s;
        }
    }
#pragma unroll
    for (int s = 0; s < (TW ? 0 : NT); s++) {
        if constexpr ((GNSS_CORR_PROBE & 2) != 0) {
            cap[s] = M - 1 - s;
            neg0 |= (cabits & 1u) << s;
            continue;
        }
        if constexpr ((GNSS_CORR_PROBE & 64) != 0) {  // (probe: no search; a runtime cap, the captures as usual)
            cap[s] = (int)((ks + 5 * s) & 31) - 4;
            neg0 |= (cabits & 1u) << s;
            continue;
        }
        const Colon col{uni(dp->tap_a[s]), d, uni(dp->tap_c[s]), n - 1};
        // the replica index is ceil(t + post): post = 0, or the prompt's +0.05 of
        // trackingCT_POS_updated.m:216 (t + 0.0 is t exactly)
        const double post = p.tap_post[s];
        const double t0 = colon_elem(col, kf) + post;
        const double c0 = ceil(t0);
        const double R = (double)(int)(kf - ks) + (c0 - t0) * inv_d;  // samples to the boundary
        const double rr = rint(R);
        int pb = (int)floor(R) + 1;
        if (fabs(R - rr) < 1e-6) {  // too close to call in floating point: exact colon value
            const int ms = (int)rr;
            pb = ms;
            const int64_t kx = ks + ms;
            if (ms >= 0 && ms < M && kx >= 0 && kx <= n - 1)
                pb = ceil(colon_elem(col, kx) + post) > c0 ? ms : ms + 1;
        }
        cap[s] = (pb < M ? pb : M) - 1;  // Prefix(p) = running sum through sample p-1
        if constexpr ((GNSS_CORR_PROBE & 32) != 0) cap[s] = M - 1 - s;  // (probe: the search runs, its cap is ignored)
        const unsigned i0 = ca_index32((int)c0 + p.chip_off);
        const unsigned i1 = i0 == 1022u ? 0u : i0 + 1u;
        const unsigned w0 = __shfl(cabits, (int)(i0 >> 5), 64);
        const unsigned w1 = __shfl(cabits, (int)(i1 >> 5), 64);
        neg0 |= ((w0 >> (i0 & 31)) & 1u) << s;
        neg1 |= ((w1 >> (i1 & 31)) & 1u) << s;
    }

    // ---- carrier base of the lane
    const double kb = (double)(int)ks;
    const double Wb = wave_at<DIVIDE>(kb, f, phi0, Fs, rFs);
    double sb, cb;
    if constexpr ((GNSS_CORR_PROBE & 1) != 0) {
        sb = Wb * 1e-9;
        cb = 1.0;
    } else {
        sincos_wave(Wb, &sb, &cb);
    }

    double run_r = 0.0, run_i = 0.0;
    double pre_r[QC ? 1 : NT], pre_i[QC ? 1 : NT];
    if constexpr (!QC) {
#pragma unroll
        for (int s = 0; s < NT; s++) { pre_r[s] = 0.0; pre_i[s] = 0.0; }
    }
    unsigned cmask = 0u;  // QC: the lane's interior capture samples (0 <= cap < M - 1)
    if constexpr (QC) {
#pragma unroll
        for (int s = 0; s < NT; s++)
            if (cap[s] >= 0 && cap[s] < M - 1) cmask |= 1u << cap[s];
    }

    // fmt 1: I - mean(I), Q - mean(Q) per sample, as the reference forms rawsignal0DC
    double mu_r = 0.0, mu_i = 0.0;
    if constexpr (FMT == 1) {
        mu_r = uni(dp->mu_r);
        mu_i = uni(dp->mu_i);
    }

    // GNSS_REGCAP (3 taps, no capture queue): each tap's prefix is taken from the running sum in
    // registers at its capture sample by a select, instead of through the LDS slots (a 16-B store
    // per sample and a read per tap per subgroup): the correlate's only LDS traffic is then the
    // rotation table's reads, which no store ahead of them delays. Same values, same bits.
    constexpr bool RC = GNSS_REGCAP && !QC && NT <= 3;
    // GNSS_PHI_REG: the rotation basis phi[m] = m*dhi + m*dlo formed in registers (as
    // prepare_desc forms the table entry: the same operations, the same bits) instead of read
    double dhi_l = 0.0, dlo_l = 0.0;
    if constexpr (GNSS_PHI_REG) {
        dhi_l = uni(dp->dhi);
        dlo_l = uni(dp->dlo);
    }
    // GNSS_SWP (A/B knob): the next sample's exact Wave formed one sample ahead (before this
    // sample's rotation and accumulation), so two independent dependency chains are in flight;
    // 2 also fences each sample's instructions from the next one's (sched_barrier), so the
    // scheduler interleaves exactly those two chains. Same operations, same bits.
    double Wpipe = 0.0;
    if constexpr (GNSS_SWP) Wpipe = wave_at<DIVIDE>(kb + 1.0, f, phi0, Fs, rFs);
    // one 8-sample subgroup: running sums into the LDS slots, tap prefixes captured
    auto subgroup = [&](const int j) {
        // fmt 0: 8 int8 I/Q pairs in one 16-B group; fmt 1: 8 int16 I/Q pairs in two
        constexpr int NW = FMT == 1 ? 8 : 4;
        unsigned wd[NW];
        bool part = lo > 8 * j || hi < 8 * j + 8;
        if constexpr (FMT == 1) {
            const int4 ra = raw.get(2 * j), rb = raw.get(2 * j + 1);
            wd[0] = (unsigned)ra.x; wd[1] = (unsigned)ra.y; wd[2] = (unsigned)ra.z; wd[3] = (unsigned)ra.w;
            wd[4] = (unsigned)rb.x; wd[5] = (unsigned)rb.y; wd[6] = (unsigned)rb.z; wd[7] = (unsigned)rb.w;
        } else {
            const int4 rj = raw.get(j);
            wd[0] = (unsigned)rj.x; wd[1] = (unsigned)rj.y; wd[2] = (unsigned)rj.z; wd[3] = (unsigned)rj.w;
            if (part) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int m0 = 8 * j + 2 * q;
                    const unsigned k0 = (m0 >= lo && m0 < hi) ? 0x0000FFFFu : 0u;
                    const unsigned k1 = (m0 + 1 >= lo && m0 + 1 < hi) ? 0xFFFF0000u : 0u;
                    wd[q] &= k0 | k1;
                }
            }
        }
        const double kbj = kb + (double)(8 * j);
#pragma unroll
        for (int mm = 0; mm < 8; mm++) {
            const int m = 8 * j + mm;
            double xr, xi;
            if constexpr (FMT == 1) {
                const unsigned word = wd[mm];
                xr = (double)(short)(word & 0xFFFFu) - mu_r;
                xi = (double)(short)(word >> 16) - mu_i;
                if (part && !(m >= lo && m < hi)) { xr = 0.0; xi = 0.0; }
            } else {
                const unsigned word = wd[mm >> 1];
                const int sh = (mm & 1) * 16;
                xr = (double)(int8_t)((word >> sh) & 0xFF);
                xi = (double)(int8_t)((word >> (sh + 8)) & 0xFF);
            }
            // m = 0: W = Wb, phi[0] = 0, rcs[0] = (1, 0) (prepare_desc: 0*dhi + 0*dlo, sincos(0))
            // -> w = x exactly, no rotation
            if constexpr ((GNSS_CORR_PROBE & 4) != 0) {
                const double2 rcs = ld_rcs(dp, m);
                run_r = __builtin_fma(xr, rcs.x, run_r);
                run_r = __builtin_fma(-xi, rcs.y, run_r);
                run_i = __builtin_fma(xr, rcs.y, run_i);
                run_i = __builtin_fma(xi, rcs.x, run_i);
            } else if (m > 0) {
                // w = x * (rc + i rs) * (1 + i eta): the first-order residue folded into the
                // rotation, the products accumulated by FMA into the running sums
                double W;
                if constexpr (GNSS_SWP) {
                    W = Wpipe;
                    if (m + 1 < M) Wpipe = wave_at<DIVIDE>(kbj + (double)(mm + 1), f, phi0, Fs, rFs);
                } else {
                    W = wave_at<DIVIDE>(kbj + (double)mm, f, phi0, Fs, rFs);
                }
                double phm;
                if constexpr (GNSS_PHI_REG) phm = (double)m * dhi_l + (double)m * dlo_l;
                else phm = dp->phi[m];
                const double eta = (W - Wb) - phm;
                const double2 rcs = ld_rcs(dp, m);
                const double rc = __builtin_fma(-eta, rcs.y, rcs.x);
                const double rs = __builtin_fma(eta, rcs.x, rcs.y);
                run_r = __builtin_fma(xr, rc, run_r);
                run_r = __builtin_fma(-xi, rs, run_r);
                run_i = __builtin_fma(xr, rs, run_i);
                run_i = __builtin_fma(xi, rc, run_i);
            } else {
                run_r += xr;
                run_i += xi;
            }
            if constexpr (QC) {
                if ((cmask >> m) & 1u)
                    myslot[__builtin_popcount(cmask & ((1u << m) - 1u)) * T] = make_double2(run_r, run_i);
            } else if constexpr (RC) {
#pragma unroll
                for (int s = 0; s < NT; s++) {
                    const bool at = cap[s] == m;
                    pre_r[s] = at ? run_r : pre_r[s];
                    pre_i[s] = at ? run_i : pre_i[s];
                }
            } else {
                myslot[mm * T] = make_double2(run_r, run_i);
            }
            if constexpr (GNSS_SWP == 2) __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (!QC && !RC) {
#pragma unroll
            for (int s = 0; s < NT; s++) {
                const unsigned idx = (unsigned)(cap[s] - 8 * j);
                const double2 v = *(idx < 8u ? myslot + idx * T : zero);
                pre_r[s] += v.x;
                pre_i[s] += v.y;
            }
        }
    };
#ifndef GNSS_UNROLL_TAPS
#define GNSS_UNROLL_TAPS 0  // (A/B: 1 = the > 3-tap subgroup loop unrolled like the 3-tap one)
#endif
    if constexpr (RELOAD && ((NT > 3 && !GNSS_UNROLL_TAPS) || (RC && GNSS_REGCAP == 2))) {
        // descriptor in LDS: one subgroup at a time (unrolled, the compiler would keep
        // every subgroup's table values live)
#pragma unroll 1
        for (int j = 0; j < SUB; j++) subgroup(j);
    } else if constexpr (RELOAD) {
#pragma unroll
        for (int j = 0; j < SUB; j++) subgroup(j);
    } else {
#pragma unroll
        for (int j = 0; j < SUB; j++) subgroup(j);
    }

    // ---- tap sums of the lane, rotated back by e^{i Wave(k_0)}:
    // I = imag(raw .* carrsig), Q = real(raw .* carrsig) (trackingCT.m:107-118)
#pragma unroll
    for (int s = 0; s < NT; s++) {
        const double a0 = ((neg0 >> s) & 1u) ? -1.0 : 1.0;
        const double v1 = ((neg1 >> s) & 1u) ? -1.0 : 1.0;
        const double dv = a0 - v1;
        double pr, pi;
        if constexpr (QC) {
            const int cs = cap[s];
            const int q = __builtin_popcount(cmask & ((1u << (cs > 0 ? cs : 0)) - 1u));
            const double2 v = myslot[(q < 8 ? q : 7) * T];  // (read even where unused: no divergence)
            pr = (cs < 0 ? 0.0 : cs == M - 1 ? run_r : v.x) + 0.0;
            pi = (cs < 0 ? 0.0 : cs == M - 1 ? run_i : v.y) + 0.0;
        } else {
            pr = pre_r[s];
            pi = pre_i[s];
        }
        const double ur = __builtin_fma(dv, pr, v1 * run_r);
        const double ui = __builtin_fma(dv, pi, v1 * run_i);
        oI[s] = __builtin_fma(cb, ui, sb * ur);
        oQ[s] = __builtin_fma(cb, ur, -(sb * ui));
    }
}

// Block-level sum of the lanes' tap sums in a fixed order (bit-reproducible). On return
// thread v < 2*NT holds block sum v (I of tap v/2 for even v, Q for odd); s_mem is
// free again for the caller. s_mem: [2NT][T] + [2NT][32] doubles.
// A double moved across lanes by a DPP control (both halves; every lane active).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// LDS barrier that leaves global loads (the next step's IF prefetch) in flight:
// __syncthreads() would wait vmcnt(0) first.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
}

// The two fixed-order reductions both step loops share (their results are bit-identical
// for a given lane geometry, whichever kernel, grid or channel set runs the step).
//
// Block: the NV tap sums of the block's 256 lanes: 8-lane runs, then four runs per lane,
// then a DPP quad butterfly. Slots are free on entry (caller's barrier); the value is in
// lanes tid = 4v (v < NV); LDS barriers only (global loads in flight stay so).
// Taps per pass of the block reduction (each pass: three barriers): all of them at 3 taps;
// above, in the per-step kernel, two passes of half the taps each, so the reduction's LDS
// (2 * taps * (T + 32) doubles) stays small and the one-pass form's extra registers (98 -> 129
// VGPRs at 11 taps) do not cut that kernel's occupancy. The persistent kernel reduces up to
// GNSS_RED_ONEPASS taps in one pass: its 11-tap forms run two blocks per CU (their VGPRs),
// where the one-pass slots still fit (59-71 KB of LDS a block). Every value is reduced by the
// same lanes in the same order whichever pass it is in (same bits).
#ifndef GNSS_RED_ONEPASS
#define GNSS_RED_ONEPASS 11
#endif
template <int NT> constexpr int red_taps() { return NT > 3 ? (NT + 1) / 2 : NT; }
template <int NT> constexpr int run_red_taps() { return NT <= GNSS_RED_ONEPASS ? NT : red_taps<NT>(); }
template <int HT> constexpr int red_words() { return 2 * HT * (kTrkThreads + 32); }

// GNSS_RED 1 (round 5, A/B knob, off): each value summed over a wave without LDS -- the DPP
// butterfly over quads, half rows and rows (every lane of a row ends with the row's sum, the
// same bits in each: IEEE addition commutes), the four rows' sums read from lanes 0 / 16 / 32 /
// 48 and added as (r0 + r1) + (r2 + r3) -- then the four waves' sums through LDS as
// (w0 + w1) + (w2 + w3). One barrier instead of three, but 8 lane reads per value: measured
// slower (block partial 0.48 -> 0.68 us; 10-ms launch 36.8-37.0 -> 37.8-38.0 ms at 3 taps,
// 203 -> 217 ms at 32 channels x 11 taps; profiles/r05_ab_block_tree.txt). A different order
// also moves the last bits, so the full-length goldens' tie flips move (config 3 channel 5
// parts at step 3 944 with it). GNSS_RED 2 combines the rows by DPP broadcasts instead of
// lane reads (same bits as 1): +1 % at 3 taps, equal at 11.
#ifndef GNSS_RED
#define GNSS_RED 0
#endif
// a double read from one lane (the result is uniform)
__device__ __forceinline__ double readlane_f64(double v, int l)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// a double moved across lanes by a DPP control with a row mask; lanes of disabled rows get 0
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64_rows(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// one value's sum over the wave's 64 lanes in the fixed order above (every lane active)
__device__ __forceinline__ double wave_sum(double a)
{
    if constexpr (GNSS_RED == 2) {
        // (GNSS_RED 2: the rows combined by DPP broadcasts instead of lane reads -- row 1 +=
        // row 0 and row 3 += row 2 (row_bcast:15), then rows 2, 3 += row 1 (row_bcast:31): lane
        // 63 ends with (r3 + r2) + (r1 + r0); the other lanes' values are not used)
        a += dpp_f64<0xB1>(a);
        a += dpp_f64<0x4E>(a);
        a += dpp_f64<0x141>(a);
        a += dpp_f64<0x140>(a);
        a += dpp_f64_rows<0x142, 0xA>(a);
        a += dpp_f64_rows<0x143, 0xC>(a);
        return a;
    }
    a += dpp_f64<0xB1>(a);   // quad_perm [1,0,3,2]
    a += dpp_f64<0x4E>(a);   // quad_perm [2,3,0,1]
    a += dpp_f64<0x141>(a);  // row_half_mirror: the other quad of the 8
    a += dpp_f64<0x140>(a);  // row_mirror: the other 8 of the 16
    return (readlane_f64(a, 0) + readlane_f64(a, 16)) + (readlane_f64(a, 32) + readlane_f64(a, 48));
}

// the waves' sums of the values of mask `sel` (pass value w = the w-th selected I / Q), combined:
// value w in lanes 4w .. 4w + 3 on return; s_mem free on entry and on return
template <int NT>
__device__ __forceinline__ double block_tree(double* s_mem, const double (&oI)[NT], const double (&oQ)[NT],
                                             int tid, unsigned sel)
{
    constexpr int NV = 2 * NT;
    const int wv = tid >> 6, lane = tid & 63;
    double* ws = s_mem;  // [4][NV]
    int w = 0;
#pragma unroll
    for (int s = 0; s < NT; s++) {
        if ((sel >> s) & 1u) {  // (sel uniform)
            const double si = wave_sum(oI[s]), sq = wave_sum(oQ[s]);
            if (lane == (GNSS_RED == 2 ? 63 : 0)) {
                ws[wv * NV + 2 * w] = si;
                ws[wv * NV + 2 * w + 1] = sq;
            }
            w++;
        }
    }
    lds_barrier();
    double a = 0.0;
    if (tid < 2 * w * 4) {
        const int v = tid >> 2;
        a = (ws[v] + ws[NV + v]) + (ws[2 * NV + v] + ws[3 * NV + v]);
    }
    lds_barrier();  // ws read before the caller reuses s_mem
    return a;
}

template <int NT, int HT = red_taps<NT>()>
__device__ __forceinline__ double block_partial(double* s_mem, const double (&oI)[NT],
                                                const double (&oQ)[NT], int tid)
{
    if constexpr (GNSS_RED) return block_tree<NT>(s_mem, oI, oQ, tid, (1u << NT) - 1u);
    constexpr int T = kTrkThreads;
    double* red = s_mem;                 // [2 HT][T]
    double* red2 = s_mem + 2 * HT * T;   // [2 HT][32]
    double a = 0.0;
#pragma unroll
    for (int q0 = 0; q0 < NT; q0 += HT) {  // taps q0 .. q0 + HT - 1 (values 2 q0 ..)
        const int nv = (NT - q0 < HT ? NT - q0 : HT) * 2;
#pragma unroll
        for (int q = 0; q < HT; q++) {
            if (q0 + q < NT) {
                red[(2 * q) * T + tid] = oI[q0 + q];
                red[(2 * q + 1) * T + tid] = oQ[q0 + q];
            }
        }
        lds_barrier();
        for (int e = tid; e < nv * 32; e += T) {
            const double* r = red + (e >> 5) * T + (e & 31) * 8;
            double x = r[0];
#pragma unroll
            for (int k = 1; k < 8; k++) x += r[k];
            red2[e] = x;
        }
        lds_barrier();
        // 4 lanes per value: value v = 2 q0 + (tid - 8 q0) / 4 in lanes 4v .. 4v + 3
        const int t = tid - 8 * q0;
        if (t >= 0 && t < nv * 4) {
            const double* r = red2 + (t >> 2) * 32 + (t & 3) * 8;
            a = r[0];
#pragma unroll
            for (int k = 1; k < 8; k++) a += r[k];
        }
        // (the butterfly on every lane: DPP reads its quad, whose lanes are all this pass's or none)
        if (t >= 0 && t < nv * 4) {
            a += dpp_f64<0xB1>(a);  // quad_perm [1,0,3,2]
            a += dpp_f64<0x4E>(a);  // quad_perm [2,3,0,1] (IEEE addition commutes: lanes agree)
        }
        lds_barrier();  // red / red2 read before the next pass or the caller reuses the slots
    }
    return a;
}

// One pass of block_partial over a chosen set of taps (the persistent loop's split of the
// > 3-tap reduction: the loop's E/P/L first, the other taps after their publication). The
// taps of bit mask `sel` (at most HT of them) take part in tap order: the q-th
// one's I / Q are the pass's values 2q / 2q + 1, reduced by exactly block_partial's lanes and
// order (8-lane runs, four runs per lane, the DPP quad butterfly), so every value has the bits
// block_partial gives it. Value w of the pass ends in lanes 4w .. 4w + 3.
template <int NT, int HT>
__device__ __forceinline__ double block_pass(double* s_mem, const double (&oI)[NT], const double (&oQ)[NT],
                                             int tid, unsigned sel)
{
    if constexpr (GNSS_RED) return block_tree<NT>(s_mem, oI, oQ, tid, sel);
    constexpr int T = kTrkThreads;
    double* red = s_mem;                 // [2 HT][T]
    double* red2 = s_mem + 2 * HT * T;   // [2 HT][32]
#pragma unroll
    for (int s = 0; s < NT; s++) {
        if ((sel >> s) & 1u) {  // (sel wave-uniform: scalar branches)
            const int q = __builtin_popcount(sel & ((1u << s) - 1u));
            red[(2 * q) * T + tid] = oI[s];
            red[(2 * q + 1) * T + tid] = oQ[s];
        }
    }
    lds_barrier();
    const int nv = 2 * __builtin_popcount(sel);
    for (int e = tid; e < nv * 32; e += T) {
        const double* r = red + (e >> 5) * T + (e & 31) * 8;
        double x = r[0];
#pragma unroll
        for (int k = 1; k < 8; k++) x += r[k];
        red2[e] = x;
    }
    lds_barrier();
    double a = 0.0;
    if (tid < nv * 4) {
        const double* r = red2 + (tid >> 2) * 32 + (tid & 3) * 8;
        a = r[0];
#pragma unroll
        for (int k = 1; k < 8; k++) a += r[k];
        a += dpp_f64<0xB1>(a);  // quad_perm [1,0,3,2]
        a += dpp_f64<0x4E>(a);  // quad_perm [2,3,0,1]
    }
    lds_barrier();  // red / red2 read before the next pass or the caller reuses the slots
    return a;
}

// Channel: the sum over the bpc block partials of value v = tid / L (tid < L*NV, L = 16
// lanes per value where 16*NV fits the block, else 8): lane q = tid % L adds blocks q,
// q+L, ... in order, then a DPP butterfly over the L lanes. Every lane of the L returns the
// sum. load(k, v) = block k's partial of value v.
template <int NV> constexpr int chan_lanes()
{
    return 16 * NV <= kTrkThreads ? 16 : 8 * NV <= kTrkThreads ? 8 : 4;  // (25 taps: 4)
}

// The same sum with the lane count L given (the persistent loop's deferred taps keep the L
// of the whole tap set, chan_lanes<2 NT>(), whatever subset of values it sums at once).
template <int L, class Load>
__device__ __forceinline__ double channel_sum_l(int bpc, int tid, Load load)
{
    const int v = tid / L, q = tid % L;
    double a = 0.0;
#pragma unroll 4
    for (int k = q; k < bpc; k += L) a += load(k, v);
    a += dpp_f64<0xB1>(a);   // quad_perm [1,0,3,2]
    a += dpp_f64<0x4E>(a);   // quad_perm [2,3,0,1]
    if constexpr (L >= 8) a += dpp_f64<0x141>(a);   // row_half_mirror: the other quad of the 8
    if constexpr (L == 16) a += dpp_f64<0x140>(a);  // row_mirror: the other 8 of the 16
    return a;
}

template <int NV, class Load>
__device__ __forceinline__ double channel_sum(int bpc, int tid, Load load)
{
    constexpr int L = chan_lanes<NV>();
    const int v = tid / L, q = tid % L;
    double a = 0.0;
#pragma unroll 4
    for (int k = q; k < bpc; k += L) a += load(k, v);
    a += dpp_f64<0xB1>(a);   // quad_perm [1,0,3,2]
    a += dpp_f64<0x4E>(a);   // quad_perm [2,3,0,1]
    if constexpr (L >= 8) a += dpp_f64<0x141>(a);   // row_half_mirror: the other quad of the 8
    if constexpr (L == 16) a += dpp_f64<0x140>(a);  // row_mirror: the other 8 of the 16
    return a;
}

// ---------------------------------------------------------------------------
// The correlator step kernel: one launch per tracking step of every channel (the
// fallback when the persistent loop below cannot keep its grid resident, and the
// per-step parity hook). NT = taps (3: E/P/L, 11: ACF), SUB = 8-sample groups per
// lane (M = 8*SUB contiguous samples), both compile-time so the accumulators stay in
// VGPRs. Grid: nch x bpc blocks; block b of a channel owns the 256*SUB consecutive
// 8-sample groups starting at g_first + 256*SUB*b.
// ---------------------------------------------------------------------------
template <int NT, int SUB, bool DIVIDE, int FMT = 0>
__global__ __launch_bounds__(kTrkThreads) void track_step_kernel(const TrkParams* __restrict__ pp,
                                                                const TrkBuffers* __restrict__ bp, int bpc)
{
    const TrkParams& p = *pp;  // (in device memory: the tail's calls take them by reference)
    const TrkBuffers& b = *bp;
    constexpr int M = 8 * SUB;
    constexpr int NV = 2 * NT;
    constexpr int T = kTrkThreads;
    static_assert(M <= kLaneMax, "lane span exceeds the rotation table");
    const int ch = blockIdx.x / bpc;
    const int blk = blockIdx.x - ch * bpc;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

    // LDS: running sums slot[8][T], then the block reduction
    constexpr int kSlot = 8 * T * 2;
    constexpr int kRed = red_words<red_taps<NT>()>();
    __shared__ __attribute__((aligned(16))) double s_mem[kSlot > kRed ? kSlot : kRed];
    __shared__ double s_fin[NV];
    __shared__ int s_last;
    __shared__ TrkChan s_c;
    __shared__ double2 s_zero;

    g_desc* dp = (g_desc*)(b.desc + ch);  // global views: scalar loads, no flat waits
    g_chan* cp = (g_chan*)(b.chan + ch);
    unsigned long long* srow = kProbe && b.stamps && ch == 0 ? stamp_row(b) : nullptr;
    if (srow && tid == 0) stamp_max(srow, 8 + blk, wall_clock64());  // block start
    const int64_t g_first = dp->g_first, g_last = dp->g_last;
    const int64_t g0 = g_first + ((int64_t)blk * T + tid) * SUB;  // first group of the lane
    // issue the IF loads first (clamped so every lane loads something valid)
    const int8_t* iq = b.iq - p.buf_base;  // absolute-byte addressing
    const int bad = dp->bad ? dp->bad : dp->bad_tap;
    constexpr int GB = FMT == 1 ? 2 : 1;  // 16-B loads per 8-sample group
    int4 raw[SUB * GB];
#pragma unroll
    for (int j = 0; j < SUB; j++) {
        const int64_t gj = g0 + j <= g_last ? g0 + j : g_last;
#pragma unroll
        for (int h = 0; h < GB; h++)
            raw[GB * j + h] = bad ? make_int4(0, 0, 0, 0) : ld_g16(iq + 16 * GB * gj + 16 * h);
    }
    const unsigned cabits = lane < 32 ? ((g_cu32*)b.ca_bits)[ch * 32 + lane] : 0u;
    // the channel state, for whichever block arrives last
    constexpr int kChanWords = (int)(sizeof(TrkChan) / 8);
    if (tid < kChanWords)
        reinterpret_cast<uint64_t*>(&s_c)[tid] = ((const g_u64*)cp)[tid];

    if (cp->status != GNSS_OK) return;
    if (!dp->phaseC && dp->Index + 1 > cp->n1_target) return;  // 1-ms run of this channel done
    if (bad || dp->d * M >= 1.0) {  // (a code rate beyond Fs/M breaks the one-boundary lane)
        if (blk == 0 && tid == 0) b.chan[ch].status = bad ? bad : GNSS_EINDEX;
        return;
    }
    double oI[NT], oQ[NT];
    if (kProbe && (p.probe & 2)) {  // timing probe: no correlation (loads, reduction and hand-off only)
#pragma unroll
        for (int s = 0; s < NT; s++) { oI[s] = (double)raw[0].x; oQ[s] = 0.0; }
    } else {
        if (tid == 0) s_zero = make_double2(0.0, 0.0);
        __syncthreads();
        lane_correlate<NT, SUB, DIVIDE, false, FMT>(p, dp, RegRaw<SUB * GB>{raw}, 8 * g0 - dp->A, cabits,
                                        reinterpret_cast<double2*>(s_mem) + tid, &s_zero, oI, oQ);
    }

    // ---- block reduction (fixed order), then hand the partial to the last arriver
    __syncthreads();  // every wave is done with the slots
    const double bsum = block_partial<NT>(s_mem, oI, oQ, tid);
    if (srow && tid == 0) stamp_max(srow, 8 + kMaxBpc + blk, wall_clock64());  // block computed
    double* allp = b.partial + (int64_t)ch * bpc * NV;
    if (tid < NV * 4 && (tid & 3) == 0) st_sc1(allp + (int64_t)blk * NV + (tid >> 2), bsum);  // write-through
    if constexpr (NV * 4 > 64) {  // (11 taps: waves 0 and 1 store) every storing wave drains
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
    }
    if (wv == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains
        if (lane == 0) {
            // two-level ticket: the blocks of the channel in this XCD group, then the
            // last of each group on the channel's counter (every counter on its own line)
            const int g = blockIdx.x & 7;
            const int first = ((g - (ch * bpc) % 8) % 8 + 8) % 8;  // first blk of group g
            const unsigned cnt = first < bpc ? (unsigned)((bpc - 1 - first) / 8 + 1) : 0u;
            unsigned* sub = b.arrive + (ch * kArrivePerChan + g) * kArriveStride;
            unsigned* top = b.arrive + (ch * kArrivePerChan + 8) * kArriveStride;
            if (srow) stamp_max(srow, 8 + 2 * kMaxBpc + blk, wall_clock64());  // last ticket issued
            int last = 0;
            if (bpc <= 32) {  // few arrivals: one level
                if (atomic_add_agent(top, 1u) ==
                    (unsigned)bpc - 1) {
                    store_agent(top, 0u);
                    last = 1;
                }
            } else if (atomic_add_agent(sub, 1u) ==
                       cnt - 1) {
                store_agent(sub, 0u);
                const unsigned ngroups = bpc < 8 ? (unsigned)bpc : 8u;
                if (atomic_add_agent(top, 1u) ==
                    ngroups - 1) {
                    store_agent(top, 0u);
                    last = 1;
                }
            }
            s_last = last;
        }
    }
    __syncthreads();
    if (!s_last) return;

    // ---- last arriver: deterministic reduction of all block partials (sc1 loads)
    if (srow && tid == 0) stamp_max(srow, 3, wall_clock64());
    double csum = 0.0;
    constexpr int CL = chan_lanes<NV>();
    if (tid < CL * NV)
        csum = channel_sum<NV>(bpc, tid, [&](int k, int v) { return ld_sc1(allp + (int64_t)k * NV + v); });
    // the step's values the writers need, read before the next descriptor replaces them
    StepOut o;
    o.n = dp->n;
    o.delayValue = dp->delayValue;
    o.remSample = dp->remSample;
    o.remChip = dp->remChip_next;
    o.remPhase = dp->remPhase_next;
    o.pdi = dp->pdi;
    o.phaseC = dp->phaseC;
    const bool dbg = b.dbg_sums || (kProbe && (p.probe & 1));
    if (tid < CL * NV && tid % CL == 0) {
        const int v = tid / CL;
        if (dbg) {
            if (b.dbg_sums) b.dbg_sums[ch * NV + v] = csum;
        } else {
            s_fin[v] = o.phaseC ? -csum : csum;  // :447-449
        }
    }
    if (dbg) return;
    __syncthreads();
    if (srow && tid == 0) stamp_max(srow, 4, wall_clock64());  // sums final
    // every wave computes the loop update (same values in every lane); then waves 0, 3
    // and 2 prepare the next step (code half, carrier table, remPhase) while wave 1
    // writes the record and wave 2 the state
    const LoopUpd u = loop_update_i(p, s_c, s_fin[2 * p.iE], s_fin[2 * p.iE + 1], s_fin[2 * p.iP],
                                  s_fin[2 * p.iP + 1], s_fin[2 * p.iL], s_fin[2 * p.iL + 1], o.pdi,
                                  o.phaseC);
    NcoState nx;
    nx.remChip = o.remChip;
    nx.remPhase = o.remPhase;
    nx.codeFreq = u.codeFreq;
    nx.carrierFreq = u.carrierFreq;
    nx.numSample = o.n;
    nx.pos = s_c.pos + p.bps * o.n;
    nx.Index = s_c.Index + (o.phaseC ? 10 : 1);
    if (wv == 0 || wv == 3) {
        if (kProbe && (p.probe & 8)) return;
        if (srow && wv == 0 && lane == 0) stamp_max(srow, 5, wall_clock64());  // loop updated
        prepare_desc_i(p, nx, o.pdi, o.phaseC, wv == 0 ? 0 : 1, lane, b.desc + ch);
        if (srow && wv == 0 && lane == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stamp_max(srow, 6, wall_clock64());  // next descriptor stored
        }
        if (srow && wv == 0 && (p.probe & 32)) {  // the same again with a warm instruction cache
            if (lane == 0) stamp_max(srow, 0, wall_clock64());
            const LoopUpd u2 = loop_update_i(p, s_c, s_fin[2 * p.iE], s_fin[2 * p.iE + 1],
                                           s_fin[2 * p.iP], s_fin[2 * p.iP + 1], s_fin[2 * p.iL],
                                           s_fin[2 * p.iL + 1], o.pdi, o.phaseC);
            nx.codeFreq = u2.codeFreq;
            nx.carrierFreq = u2.carrierFreq;
            if (lane == 0) stamp_max(srow, 1, wall_clock64());
            prepare_desc_i(p, nx, o.pdi, o.phaseC, 0, lane, b.desc + ch);
            if (lane == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                stamp_max(srow, 2, wall_clock64());
            }
        }
    } else if (kProbe && (p.probe & 4)) {
        return;
    } else if (wv == 1) {
        if (lane == 0) write_record_i(p, b, ch, s_c, o, u, s_fin);
        if (b.taps_rec && lane < NV && s_c.slot < p.rec_cap)
            b.taps_rec[((int64_t)ch * p.rec_cap + s_c.slot) * NV + lane] = s_fin[lane];
    } else {
        prepare_desc_i(p, nx, o.pdi, o.phaseC, 2, lane, b.desc + ch);  // lane 63: remPhase
        if (lane != 0) return;
        write_state_i(p, b, ch, b.chan + ch, s_c, o, u, s_fin);
        if (srow) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stamp_max(srow, 7, wall_clock64());  // state stored
            __hip_atomic_fetch_add(b.stamps + (size_t)kStampSlots * kStampRow, 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---------------------------------------------------------------------------
// The persistent step loop: one launch runs `nsteps` tracking steps of every channel.
// The blocks of a channel stay resident and loop over the steps; block 0 of the channel
// also reduces the block partials, runs the loop update in the step kernel's wave roles
// and publishes the next descriptor, with the channel state kept in its LDS for the
// whole launch. Hand-offs inside the launch are R2 granules (guide G16): 8-byte
// {tag, 32-bit word} relaxed agent-scope stores, polled until every tag matches
// (block partials -> block 0; descriptor -> every block). The next step's IF bytes
// are prefetched while the descriptor is in flight (its start, A + n, is known).
// Every wait is bounded (~2 s): on timeout run_err is set and the blocks leave.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void publish_words(unsigned long long* g, const unsigned* src, int n,
                                              unsigned tag, int tid)
{
    for (int e = tid; e < n; e += kTrkThreads)
        store_agent(g + e, ((unsigned long long)tag << 32) | src[e]);
}

// Poll n granules until every tag equals `tag`; their words land in dst (LDS). Called by
// every thread of the block; the np pollers (pid 0..np-1, pid < 0: not polling) each poll
// granules pid + k*np with no block barrier per round, a granule seen once is not read
// again (its producer may already have moved on); one barrier at the end. false (and
// run_err set) on timeout (~2 s). n <= 64*np.
__device__ bool sweep_words(const unsigned long long* g, int n, unsigned tag, unsigned* dst,
                            int pid, int np, unsigned* err)
{
    unsigned long long todo = 0;  // bit k: granule pid + k*np still missing
    if (pid >= 0)
        for (int k = 0, e = pid; e < n; k++, e += np) todo |= 1ull << k;
    unsigned long long t0 = 0;
    int late = 0;
    while (todo) {
        for (int k = 0; (todo >> k) != 0; k++) {
            if (!((todo >> k) & 1ull)) continue;
            const int e = pid + k * np;
            const unsigned long long v = load_agent(g + e);
            if ((unsigned)(v >> 32) == tag) {
                dst[e] = (unsigned)v;
                todo &= ~(1ull << k);
            }
        }
        if (!todo) break;
        // 100 MHz wall clock, read only once the wait is long
        if (++late >= 64) {
            const unsigned long long t = wall_clock64();
            if (!t0) t0 = t;
            else if (t - t0 > 200000000ull) { atomicExch(err, 1u); break; }
            late = 0;
        }
    }
    return !__syncthreads_or(todo != 0);
}

// (16-B granules {lo, tag, hi, tag}, publish16: gnss_internal.h, shared with the VT loop)
// granule loads a poller keeps in flight per batch: one at a time for E / P / L (2-3 granules a
// poller, where batching measured 1 % slower), GNSS_SWEEP_BATCH above 3 taps (8-11 a poller: the
// 11-tap 4-channel launch 49.5 -> 45.9 ms at 4, profiles/r06_ab_sweep_batch.txt)
#ifndef GNSS_SWEEP_BATCH
#define GNSS_SWEEP_BATCH 4
#endif

// Poll n 16-B granules until both tags of each equal `tag`; granule e's words land in
// dst[2e], dst[2e+1]. Same protocol as sweep_words (pollers pid 0..np-1, n <= 64*np).
template <int SB>
__device__ bool sweep16(__amdgpu_buffer_rsrc_t r, int n, unsigned tag, unsigned* dst, int pid, int np,
                        unsigned* err, int base)
{
    unsigned long long todo = 0;
    if (pid >= 0)
        for (int k = 0, e = pid; e < n; k++, e += np) todo |= 1ull << k;
    unsigned long long t0 = 0;
    int late = 0;
    while (todo) {
        // a pass over the missing granules, SB loads in flight at a time (each checked only once
        // all of its batch are issued: one round trip per batch, not per granule; the words land
        // where they did, so the sums keep their bits)
        for (unsigned long long rem = todo; rem;) {
            int ks[SB];
            u32x4 v[SB];
#pragma unroll
            for (int j = 0; j < SB; j++) {
                ks[j] = rem ? __builtin_ctzll(rem) : -1;
                if (rem) {
                    rem &= rem - 1;
                    v[j] = __builtin_amdgcn_raw_buffer_load_b128(r, (base + pid + ks[j] * np) * 16, 0, kPolSc1);
                }
            }
#pragma unroll
            for (int j = 0; j < SB; j++)
                if (ks[j] >= 0 && v[j].y == tag && v[j].w == tag) {
                    const int e = pid + ks[j] * np;
                    dst[2 * e] = v[j].x;
                    dst[2 * e + 1] = v[j].z;
                    todo &= ~(1ull << ks[j]);
                }
        }
        if (!todo) break;
        if constexpr (GNSS_XCHG_SLEEP > 0) __builtin_amdgcn_s_sleep(GNSS_XCHG_SLEEP);  // (A/B knob)
        if (++late >= 64) {
            const unsigned long long t = wall_clock64();
            if (!t0) t0 = t;
            else if (t - t0 > 200000000ull) { atomicExch(err, 1u); break; }
            late = 0;
        }
    }
    // The closing barrier must not wait for this block's outstanding global STORES (block 0's
    // wave 1 has just written the previous step's record there: __syncthreads' fence would
    // hold the whole block for their completion, ~1.9 us, and block 0 would start every step
    // last). The polls' own loads have completed (their tags were compared), the gathered
    // words are in LDS: a wave vote through LDS and an LDS-only barrier suffice.
    __shared__ unsigned s_vote[kTrkThreads / 64];
    const unsigned any_left = __ballot(todo != 0) != 0ull ? 1u : 0u;
    if ((threadIdx.x & 63) == 0) s_vote[threadIdx.x >> 6] = any_left;
    lds_barrier();
    unsigned v = 0;
#pragma unroll
    for (int w = 0; w < kTrkThreads / 64; w++) v |= s_vote[w];
    return v == 0;
}

// sweep16 over two granule ranges at once (the persistent loop's > 3-tap form: this step's
// E/P/L partials, plus in the blocks that own deferred taps the previous step's partials of
// those taps). Logical granule e < n1 is base1 + e (tag1, words to dst1[2e]); e >= n1 is
// base2 + e - n1 (tag2, dst2). Same pollers, bound and closing vote as sweep16.
__device__ bool sweep16x2(__amdgpu_buffer_rsrc_t r, int n1, int base1, unsigned tag1, unsigned* dst1, int n2,
                          int base2, unsigned tag2, unsigned* dst2, int pid, int np, unsigned* err)
{
    const int n = n1 + n2;
    unsigned long long todo = 0;
    if (pid >= 0)
        for (int k = 0, e = pid; e < n; k++, e += np) todo |= 1ull << k;
    unsigned long long t0 = 0;
    int late = 0;
    while (todo) {
        for (int k = 0; (todo >> k) != 0; k++) {
            if (!((todo >> k) & 1ull)) continue;
            const int e = pid + k * np;
            const bool first = e < n1;
            const int e2 = first ? e : e - n1;
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, ((first ? base1 : base2) + e2) * 16, 0, kPolSc1);
            const unsigned tg = first ? tag1 : tag2;
            if (v.y == tg && v.w == tg) {
                unsigned* d = first ? dst1 : dst2;
                d[2 * e2] = v.x;
                d[2 * e2 + 1] = v.z;
                todo &= ~(1ull << k);
            }
        }
        if (!todo) break;
        if (++late >= 64) {
            const unsigned long long t = wall_clock64();
            if (!t0) t0 = t;
            else if (t - t0 > 200000000ull) { atomicExch(err, 1u); break; }
            late = 0;
        }
    }
    __shared__ unsigned s_vote2[kTrkThreads / 64];
    const unsigned any_left = __ballot(todo != 0) != 0ull ? 1u : 0u;
    if ((threadIdx.x & 63) == 0) s_vote2[threadIdx.x >> 6] = any_left;
    lds_barrier();
    unsigned v = 0;
#pragma unroll
    for (int w = 0; w < kTrkThreads / 64; w++) v |= s_vote2[w];
    return v == 0;
}

// Grid census (guide G16: residency is a precondition, not a given): every block
// arrives on one counter; the last arrival starts the launch, a block that waits ~20 ms
// aborts it instead (one CAS decides). On abort every block leaves before touching any
// state, run_err[0] = 2, and the host re-runs the steps with the step kernel.
__device__ bool census(unsigned* w, int tid)
{
    __shared__ int s_go;
    if (tid == 0) {
        unsigned* arrive = w + 1;
        unsigned* state = w + 2;  // 0 pending, 1 go, 2 abort
        if (atomic_add_agent(arrive, 1u) == gridDim.x - 1)
            atomicCAS(state, 0u, 1u);
        const unsigned long long t0 = wall_clock64();
        unsigned st;
        while ((st = __hip_atomic_load((g_u32*)state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0) {
            if (wall_clock64() - t0 > 2000000ull) atomicCAS(state, 0u, 2u);
            __builtin_amdgcn_s_sleep(2);
        }
        if (st == 2) atomicCAS(w, 0u, 2u);
        s_go = st == 1;
    }
    __syncthreads();
    return s_go != 0;
}

// The next step's 16-B IF groups of this lane straight into LDS (global_load_lds, no
// VGPRs): group j of lane tid at s_raw[j*256 + tid]; each wave-instruction writes its
// 64 lanes' 1 KiB contiguously from the wave's base.
template <int SUB>
__device__ __forceinline__ void prefetch_raw(const int8_t* iq, int64_t g0, int64_t gmax, int4* s_raw,
                                             int tid)
{
    const int wbase = tid & ~63;
#pragma unroll
    for (int j = 0; j < SUB; j++) {
        int64_t gj = g0 + j;
        gj = gj < gmax ? gj : gmax;
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(iq + 16 * gj),
                                         (__attribute__((address_space(3))) void*)(s_raw + j * kTrkThreads + wbase),
                                         16, 0, 0);
    }
}

// Persistent step loop, grid nch x bpc. Every block of a channel keeps its own copy of
// the channel's scalar state and descriptor and runs the scalar end of every step itself
// (the same fp64 code on the same sums: bit-identical copies), so a step needs one
// exchange only: each block publishes its partial sums and reads everyone's. Block 0
// of the channel writes the records, C/N0 and, at the end, the state.
#ifndef GNSS_DEFER
#define GNSS_DEFER 0  // (A/B: 0 = every tap through the step's exchange, the round-4 form)
#endif
#ifndef GNSS_WPE_TAPS
#define GNSS_WPE_TAPS 2  // (A/B: waves per EU of the > 3-tap persistent forms; 3 = three blocks per CU)
#endif
template <int NT, int SUB, bool DIVIDE, bool VB = false>
__global__ __launch_bounds__(kTrkThreads) __attribute__((amdgpu_waves_per_eu(NT > 3 ? GNSS_WPE_TAPS : 3, NT > 3 ? GNSS_WPE_TAPS : 3))) void track_run_kernel(const TrkParams* __restrict__ pp,
                                                               const TrkBuffers* __restrict__ bp, int bpc,
                                                               int vpb, int nsteps, unsigned tag0)
{
    const TrkParams& p = *pp;
    const TailK tk = tail_k(p);  // (the scalar tail's constants, in registers)
    const TrkBuffers& b = *bp;
    constexpr int M = 8 * SUB;
    constexpr int NV = 2 * NT;
    constexpr int T = kTrkThreads;
    static_assert(M <= kLaneMax, "lane span exceeds the rotation table");
    // vpb virtual blocks per resident block (config 5: 32 channels x 11 taps on one GPU):
    // block pblk correlates the channel's blocks blk .. blk + nvb - 1 of the step's lane
    // geometry one after the other, each with the same lanes, reduction and granule as a
    // block of its own, so the sums are the same bits whatever vpb is. (VB = false: the
    // one-block-per-block form, the loop compiled away -- the headline's 8 channels.)
    const int vpb_ = VB ? vpb : 1;
    const int pbpc = (bpc + vpb_ - 1) / vpb_;
    // (A/B knob GNSS_XCD_LOCAL: with 8 channels, channel = the block's XCD (blocks are dealt
    // round-robin over the 8 XCDs), so a channel's exchange stays in one L2)
    // (GNSS_XCD_LOCAL 2, the control experiment: with 8 channels x 96 blocks, a CU's three
    // blocks b, b + 256, b + 512 (profiles/r03_channel_lockstep.txt) are one channel's, as
    // XCD-local placement makes them, but each channel's 32 CUs span all 8 XCDs)
    const bool xl = GNSS_XCD_LOCAL == 1 && !VB && p.nch == 8;
    const bool cul = GNSS_XCD_LOCAL == 2 && !VB && p.nch == 8 && pbpc == 96;
    const int ch = xl ? (int)(blockIdx.x & 7) : cul ? (int)((blockIdx.x & 255) >> 5) : (int)(blockIdx.x / pbpc);
    const int pblk = xl ? (int)(blockIdx.x >> 3)
                    : cul ? (int)((blockIdx.x & 31) * 3 + (blockIdx.x >> 8)) : (int)(blockIdx.x - ch * pbpc);
    const int blk = pblk * vpb_;
    const int nvb = VB ? (bpc - blk < vpb_ ? bpc - blk : vpb_) : 1;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool io = pblk == 0;

    constexpr int kSlot = 8 * T * 2;                  // running sums [8][T] double2
    constexpr int kRed = red_words<run_red_taps<NT>()>();  // block reduction
    constexpr int kPart = run_bpc_cap(NT) * NV;       // everyone's partials (as words)
    // Above 3 taps only E / P / L cross the step's exchange (kDefer, below); GNSS_DEFER 2 (one
    // block of the step per resident block) has one wave reduce the other taps' block partials
    // while the rest poll: their lane values staged at s_mem + kPwD, [value][T], and that wave's
    // run sums after them. The exchange's words then need bpc * (E/P/L values + owned values).
    constexpr bool kDefer = GNSS_DEFER && NT > 3;
    constexpr bool kWave1 = GNSS_DEFER == 2 && kDefer && !VB;
    // (defer_reduce restates the round-4 block order for its one wave)
    static_assert(!kWave1 || GNSS_RED == 0, "GNSS_DEFER 2 needs GNSS_RED 0");
    constexpr int kPwD = run_bpc_cap(NT) * 8 + 2 * NT;  // (pbpc = bpc: own_n <= nBv / bpc + 1)
    constexpr int kStage = 2 * (NT - 1) * T;
    constexpr int kMemW = kWave1 ? kPwD + kStage + 2 * NT * 32 : 0;
    constexpr int kMem1 = kSlot > kRed ? kSlot : kRed;
    constexpr int kMem0 = kMem1 > kMemW ? kMem1 : kMemW;
    constexpr int kMem = kMem0 > kPart + 16 * NV ? kMem0 : kPart + 16 * NV;
    __shared__ __attribute__((aligned(16))) double s_mem[kMem];
    __shared__ __attribute__((aligned(16))) int4 s_raw[SUB * T];   // this step's IF
    __shared__ __attribute__((aligned(16))) StepDesc s_d[2];       // this step / the next
    __shared__ __attribute__((aligned(16))) TrkChan s_c;           // the channel state
    __shared__ StepOut s_o;                                        // the step whose state and
    __shared__ LoopUpd s_u;                                        //   record are pending
    __shared__ double s_fin[NV];
    __shared__ double s_taps[GNSS_MAX_TAPS], s_post[GNSS_MAX_TAPS];
    __shared__ double2 s_zero;

    if (!census(b.run_err, tid)) return;
    g_chan* cp = (g_chan*)(b.chan + ch);
    if (cp->status != GNSS_OK) return;  // set before this launch: channel-uniform
    const int64_t n1_target = cp->n1_target;
    const int8_t* iq = b.iq - p.buf_base;  // absolute-byte addressing
    const int64_t gmax = (p.buf_base + p.buf_len) / 16 - 1;  // last resident 16-B group
    // (circularly extended for lane_correlate's tap window, ca_bits_ext)
    const unsigned cabits = ca_bits_ext(lane < 32 ? ((g_cu32*)b.ca_bits)[ch * 32 + lane] : 0u, lane);
    // this channel's granules (gran_per_chan): 3 taps [parity][block][value] x 16 B; above,
    // region A [parity][block][E/P/L value] and region B [step mod 4][value][block]
    const __amdgpu_buffer_rsrc_t pg = __builtin_amdgcn_make_buffer_rsrc(
        b.pgran + (int64_t)ch * 2 * gran_per_chan(NT), (short)0, gran_per_chan(NT) * 16, kBufRsrcWord3);
    constexpr int kChanWords = (int)(sizeof(TrkChan) / 8);

    // Above 3 taps (config 5's 11-tap ACF) only E / P / L feed the loop (trackingCT.m:470-483):
    // they are reduced, published and swept first (region A); the other taps' values (B,
    // only when the caller asked for the taps) are reduced after that publication, overlapping
    // the exchange, and the previous step's are swept beside this step's E/P/L by the blocks
    // that own them (a run of B values per block, blocks 4, 5, ...), whose idle tail wave
    // sums them and writes the taps one step late. Every value keeps its reduction lanes and
    // order (block_pass, channel_sum_l with the whole tap set's lane count), so the records
    // and taps are the bits of the one-exchange form and of the per-step kernel.
    constexpr int CL = chan_lanes<NV>();
    constexpr int HT = run_red_taps<NT>();
    // The configuration lives in LDS and is read where it is used (volatile LDS loads, never
    // hoisted into registers that would live across the step loop: this kernel is at its
    // register budget). selA / selB: the loop's taps / the others; NA: E/P/L values; nBv: B
    // values; hb: B taps per reduction pass; [own_lo, own_lo + own_n): this block's B values;
    // bslot / bneg (wave 1): the slot and phase-C sign of the step whose B values are due.
    struct DeferCfg {
        unsigned selA, selB;
        int NA, nBv, hb, own_lo, own_n, bneg;
        int64_t bslot;
        int vmap[kDefer ? NV : 1];  // A values, then B values -> value index 2 tap + I/Q
    };
    __shared__ DeferCfg s_df;
    typedef __attribute__((address_space(3))) volatile const int lds_vint;
    typedef __attribute__((address_space(3))) volatile const long long lds_vi64;
    auto dfi = [&](const int& f) { return uni((int)*(lds_vint*)&f); };
    auto NA_ = [&]() { return kDefer ? dfi(s_df.NA) : NV; };
    auto own_n_ = [&]() { return kDefer ? dfi(s_df.own_n) : 0; };
    const bool dob = kDefer && b.taps_rec != nullptr;
    if constexpr (kDefer) {
        if (tid == 0) {
            unsigned selA = 0, selB = 0;
            for (int s = 0; s < NT; s++) {
                if (s == tk.iE || s == tk.iP || s == tk.iL) selA |= 1u << s;
                else selB |= 1u << s;
            }
            const int nA = __builtin_popcount(selA), nB = __builtin_popcount(selB);
            const int nBv = 2 * nB, npass = (nB + HT - 1) / HT;
            int own_lo = 0, own_n = 0;
            if (dob && nBv > 0) {  // this block's run of B values
                const int c = (nBv + pbpc - 1) / pbpc;
                const int nown = (nBv + c - 1) / c;
                const int r = ((pblk - 4) % pbpc + pbpc) % pbpc;
                if (r < nown) {
                    own_lo = r * c;
                    own_n = nBv - own_lo < c ? nBv - own_lo : c;
                }
            }
            s_df.selA = selA;
            s_df.selB = selB;
            s_df.NA = 2 * nA;
            s_df.nBv = nBv;
            s_df.hb = npass > 0 ? (nB + npass - 1) / npass : 1;
            s_df.own_lo = own_lo;
            s_df.own_n = own_n;
            s_df.bneg = 0;
            s_df.bslot = 0;
            for (int s = 0; s < NT; s++) {
                const unsigned below = (1u << s) - 1u;
                const int v = ((selA >> s) & 1u) ? 2 * __builtin_popcount(selA & below)
                                                 : 2 * nA + 2 * __builtin_popcount(selB & below);
                s_df.vmap[v] = 2 * s;
                s_df.vmap[v + 1] = 2 * s + 1;
            }
        }
    }
    // B taps of pass ps (1-based): ranks (ps - 1) * hb .. ps * hb - 1 among the B taps
    auto sel_pass = [&](int ps) {
        const unsigned selB = (unsigned)dfi(*(const int*)&s_df.selB);
        const int hb = dfi(s_df.hb);
        unsigned m = 0u;
        int r = 0;
        for (int s = 0; s < NT; s++)
            if ((selB >> s) & 1u) {
                if (r >= (ps - 1) * hb && r < ps * hb) m |= 1u << s;
                r++;
            }
        return m;
    };

    // step 0's descriptor and the state, as the previous launch left them
    for (int e = tid; e < kDescWords; e += T)
        reinterpret_cast<unsigned*>(&s_d[0])[e] = ((const g_u32*)(b.desc + ch))[e];
    if (tid < kChanWords) reinterpret_cast<uint64_t*>(&s_c)[tid] = ((const g_u64*)cp)[tid];
    if (tid == 0) s_zero = make_double2(0.0, 0.0);
    if (tid < NT) {
        s_taps[tid] = p.taps[tid];
        s_post[tid] = p.tap_post[tid];
    }
    __syncthreads();
    // The record's parts, the taps and the C/N0 value go to different blocks (one when the channel
    // has one), so that no block's flush outlasts the exchange it overlaps: one block doing all of
    // it measured ~1.7 us, and that block then started every step last
    // (profiles/r04_block0_lateness.txt). Part 1 (the sums and the codedelay bookkeeping) is not
    // on block 0 either (round 5): block 0 then polls with all four waves like
    // the others, and in the 1-ms phase it was still the last to finish its correlate.
    const int duty_a = pbpc > 3 ? 3 : 0, duty_b = pbpc > 1 ? 1 : 0, duty_c = pbpc > 2 ? 2 : duty_b;
    const bool dio = pblk == duty_a;  // the block holding the record's part 1
    // blocks whose wave 1 flush is long (record part 1; part 2 and the tap record, ~1 us against
    // ~0.5 elsewhere, profiles/r05_stamps_1ms.txt) poll with waves 0, 2, 3 only
#ifndef GNSS_DSW_B
#define GNSS_DSW_B 1  // (A/B: 0 = only the part-1 block polls without wave 1)
#endif
    const bool dsw = dio || (GNSS_DSW_B && pblk == duty_b);
    // (that block's wave 1, lane 0: dvpre[s_c.nstep], the running delayValue prefix its flushes
    // extend -- no read-back of its own stores)
    int64_t dvrun = 0;
    if (dio && wv == 1 && lane == 0) dvrun = ((const g_i64*)(b.dvpre + (int64_t)ch * (p.rec_cap + 1)))[s_c.nstep];
    if (!s_d[0].bad && !s_d[0].bad_tap)
        prefetch_raw<SUB>(iq, s_d[0].g_first + ((int64_t)blk * T + tid) * SUB, gmax, s_raw, tid);

    int cur = 0;   // s_d[cur]: this step
    bool pend = false;  // a finished step's state / record still to write (s_o, s_u, s_fin)
    int64_t pre[2] = {0, 0};  // the part-1 block: its record's delayValue prefix reads, issued early
    bool pre_ok = false;      //   (for the pending step)
    // The pending step's side effects, by wave 1 while the next step's partials are in
    // flight (off the critical path): the state replica (every block, in place) and, in the
    // duty blocks above, the record, C/N0 and taps.
    int s_now = 0;  // (probe stamps of the flush)
    // the owned B values of a finished step, swept into pb: summed (8 lanes per value, the
    // order of channel_sum<NV>) and written to the taps, by one wave
    auto defer_write = [&](const unsigned* pb) {
        constexpr int VPW = 64 / CL;  // values per wave pass
        const int own_n = own_n_(), own_lo = dfi(s_df.own_lo), NA = NA_(), bneg = dfi(s_df.bneg);
        const int64_t bslot = uni((int64_t)*(lds_vi64*)&s_df.bslot);
        for (int c0 = 0; c0 < own_n; c0 += VPW) {
            const double a = channel_sum_l<CL>(bpc, lane, [&](int k, int vl) {
                const int vv = c0 + vl;
                if (vv >= own_n) return 0.0;
                const unsigned lo = pb[(vv * bpc + k) * 2], hi = pb[(vv * bpc + k) * 2 + 1];
                return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
            });
            const int vv = c0 + lane / CL;
            if (lane % CL == 0 && vv < own_n && bslot < p.rec_cap)
                ((g_dbl*)b.taps_rec)[((int64_t)ch * p.rec_cap + bslot) * NV + s_df.vmap[NA + own_lo + vv]] =
                    bneg ? -a : a;  // (phase C: negated like every tap, :447-449)
        }
    };
    // after a launch's last flush: the owned B values of finished step sf, swept and written
    auto defer_final = [&](int sf) {
        if (!kDefer || sf < 0) return;
        const int own_n = own_n_();  // (block-uniform)
        if (own_n <= 0) return;
        unsigned* pb = reinterpret_cast<unsigned*>(s_mem);
        if (!sweep16x2(pg, 0, 0, 0u, pb, own_n * bpc,
                       gran_region_b(NT) + (sf & 3) * gran_slot_b(NT) + dfi(s_df.own_lo) * bpc, tag0 + sf + 1, pb,
                       tid, T, b.run_err))
            return;
        if (wv == 1) defer_write(pb);
    };
    // GNSS_DEFER 2: one wave's reduction of the staged other-tap lane values of step `step`,
    // exactly block_partial's order per value (8-lane runs in order, four runs per lane, the
    // DPP quad butterfly), published to region B
    auto defer_reduce = [&](int step) {
        const double* stg = s_mem + kPwD;
        double* r2 = s_mem + kPwD + kStage;  // [value][32] run sums
        const int nbv = dfi(s_df.nBv);
        for (int e = lane; e < nbv * 32; e += 64) {
            const double* r = stg + (e >> 5) * T + (e & 31) * 8;
            double x = r[0];
#pragma unroll
            for (int k = 1; k < 8; k++) x += r[k];
            r2[e] = x;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the run sums are in LDS (this wave's)
        double a = 0.0;
        if (lane < nbv * 4) {
            const double* r = r2 + (lane >> 2) * 32 + (lane & 3) * 8;
            a = r[0];
#pragma unroll
            for (int k = 1; k < 8; k++) a += r[k];
            a += dpp_f64<0xB1>(a);  // quad_perm [1,0,3,2]
            a += dpp_f64<0x4E>(a);  // quad_perm [2,3,0,1]
            if ((lane & 3) == 0)
                publish16(pg, gran_region_b(NT) + (step & 3) * gran_slot_b(NT) + (lane >> 2) * bpc + blk, a,
                          tag0 + step + 1);
        }
    };
    auto flush = [&]() {
        if (wv == 1) {
            // (probe GNSS_FLUSH_PROBE & 2: block 0's record part twice, stamped at [2000..2002]
            // of the step's row: cold, then warm)
            unsigned long long* fr = kProbe && (GNSS_FLUSH_PROBE & 2) && b.stamps && ch == 0 && io && lane == 0
                                         ? b.stamps + (size_t)(s_now % kStampSlots) * kStampRow : nullptr;
            if (fr) fr[2000] = wall_clock64();
            if (lane == 0 && !(GNSS_FLUSH_PROBE & 1)) {
                if (dio) {
                    if (!pre_ok) {  // (a launch's last flush: the column's prefix read here)
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        const g_i64* dvp = (const g_i64*)(b.dvpre + (int64_t)ch * (p.rec_cap + 1));
                        const int64_t cols = record_cols(p, s_c, s_o.phaseC);
                        pre[1] = cols < s_c.nstep + 1 ? dvp[cols] : 0;
                    }
                    pre[0] = dvrun;
                    write_record_i(p, b, ch, s_c, s_o, s_u, s_fin, pre, duty_b == duty_a ? 3 : 1);
                    dvrun += s_o.delayValue;  // = dvpre[nstep + 1], the value just stored
                }
                else if (pblk == duty_b) write_record_i(p, b, ch, s_c, s_o, s_u, s_fin, nullptr, 2);
            }
            if (fr) {
                fr[2001] = wall_clock64();
                write_record_i(p, b, ch, s_c, s_o, s_u, s_fin, pre, 3);
                fr[2002] = wall_clock64();
            }
            if (pblk == duty_b && b.taps_rec && lane < NA_() && s_c.slot < p.rec_cap) {
                // (above 3 taps the loop's values only: the others follow a step later, defer_write)
                const int v = kDefer ? s_df.vmap[lane] : lane;
                ((g_dbl*)b.taps_rec)[((int64_t)ch * p.rec_cap + s_c.slot) * NV + v] = s_fin[v];
            }
            if (kDefer && lane == 0) {  // the pending step's slot and sign, for its deferred taps
                s_df.bslot = s_c.slot;
                s_df.bneg = s_o.phaseC;
            }
            if (lane == 0) update_state_inplace(p, b, ch, s_c, s_o, s_u, s_fin, pblk == duty_c);
        }
        pend = false;
        pre_ok = false;
    };
    // timing probe: per-channel launch span in row 0, words 20 + 3 ch .. (block 0)
    const unsigned long long t_start = kProbe ? wall_clock64() : 0ull;
    for (int s = 0; s < nsteps; s++) {
        s_now = s;
        const StepDesc& D = s_d[cur];
        const int bad = D.bad ? D.bad : D.bad_tap;
        const bool stop = !D.phaseC && D.Index + 1 > n1_target;  // 1-ms run of this channel done
        // (a code rate beyond Fs/M breaks the one-boundary lane; above 3 taps one beyond the
        // capture queue's checked rate would overflow the queue)
        if (bad || stop || D.d * M >= 1.0 || (GNSS_QCAP && NT > kQcapMax && D.d > tk.qcap_dmax)) {
            const bool had = pend;
            if (pend) flush();
            if (had) defer_final(s - 1);
            if (io && tid == 64) desc_rem(tk, &s_d[cur]);  // (complete for a step-kernel follow-up)
            __syncthreads();
            if (io) {  // leave the state and this (unused) descriptor for the host / next launch
                if (tid == 0 && !stop) s_c.status = bad ? bad : GNSS_EINDEX;
                __syncthreads();
                if (tid < kChanWords)
                    reinterpret_cast<uint64_t*>(b.chan + ch)[tid] = reinterpret_cast<const uint64_t*>(&s_c)[tid];
                for (int e = tid; e < kDescWords; e += T)
                    reinterpret_cast<unsigned*>(b.desc + ch)[e] = reinterpret_cast<const unsigned*>(&D)[e];
            }
            return;
        }
        const int64_t A = uni(D.A), n = uni(D.n);
        // timing probe (GNSS_STAMPS), channel 0, row s: [0] step start, [1] computed,
        // [2] partial out, [3] all partials in, [4] next descriptor ready (block 0);
        // [5..9] the same for the channel's last block
        unsigned long long* srow = kProbe && b.stamps && ch == 0 && (io || pblk == pbpc - 1)
                                       ? b.stamps + (size_t)(s % kStampSlots) * kStampRow + (io ? 0 : 5) : nullptr;
        if (srow && tid == 0) srow[0] = wall_clock64();
        // (probe: every block of channel 0, its step start at [40 + blk] and its correlate's end
        // at [40 + 256 + blk] of the step's row)
        unsigned long long* brow = kProbe && b.stamps && ch == 0 ? b.stamps + (size_t)(s % kStampSlots) * kStampRow : nullptr;
        if (brow && tid == 0) brow[40 + blk] = wall_clock64();

        // ---- correlate this block's lanes (IF prefetched into s_raw). The CU's other
        // blocks (other channels) may be in their latency-bound scalar end meanwhile: the
        // correlator runs at a low wave priority, everything after it at the highest. The
        // low level rotates with the step (0..2) so the channels sharing a CU take turns
        // (by age alone the first-dispatched channel would always win and the last one set
        // the launch's length).
        for (int jv = 0; jv < nvb; jv++) {
            const int vb = blk + jv;
            switch ((kProbe && (p.probe & 64)) ? ch % 3 : (kProbe && (p.probe & 128)) ? 0 : (s + ch) % 3) {
            case 0: __builtin_amdgcn_s_setprio(0); break;
            case 1: __builtin_amdgcn_s_setprio(1); break;
            default: __builtin_amdgcn_s_setprio(2); break;
            }
            {
                const int64_t g0 = uni(D.g_first) + ((int64_t)vb * T + tid) * SUB;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's global_load_lds landed
                double oI[NT], oQ[NT];
                lane_correlate<NT, SUB, DIVIDE, true, 0>(p, &D, LdsRaw{s_raw + tid}, 8 * g0 - A, cabits,
                                                      reinterpret_cast<double2*>(s_mem) + tid, &s_zero, oI, oQ,
                                                      s_post);
                __syncthreads();  // slots and s_raw free
                if (pend && dio && wv == 1 && lane == 0 && jv == 0) {
                    // the pending record's older delayValue prefix (quirk A.11's column), loaded
                    // here and not at the step's start: an outstanding load there held this
                    // wave at the correlate's vmcnt(0) wait (its IF landed long before)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the last flush's stores)
                    const g_i64* dvp = (const g_i64*)(b.dvpre + (int64_t)ch * (p.rec_cap + 1));
                    const int64_t cols = record_cols(p, s_c, s_o.phaseC);
                    pre[1] = cols < s_c.nstep + 1 ? dvp[cols] : 0;
                    pre_ok = true;
                }
                // the next virtual block's IF, every lane its own groups (waited for at the
                // top of its iteration), in flight during this block's reduction
                if (VB && jv + 1 < nvb)
                    prefetch_raw<SUB>(iq, uni(D.g_first) + ((int64_t)(vb + 1) * T + tid) * SUB, gmax, s_raw, tid);
                __builtin_amdgcn_s_setprio(3);
                if (srow && tid == 0) srow[1] = wall_clock64();
                if (brow && tid == 0) brow[40 + 256 + vb] = wall_clock64();
                // block sum in a fixed order, published as granules
                if constexpr (!kDefer) {
                    const double bsum = block_partial<NT, HT>(s_mem, oI, oQ, tid);
                    if (tid < NV * 4 && (tid & 3) == 0)
                        publish16(pg, ((s & 1) * kMaxBpcRun + vb) * NV + (tid >> 2), bsum, tag0 + s + 1);
                } else {
                    // E / P / L first (region A), then the other taps (region B, slot s mod 4),
                    // reduced while the exchange is in flight
                    const double ba = block_pass<NT, HT>(s_mem, oI, oQ, tid, (unsigned)dfi(*(const int*)&s_df.selA));
                    const int NA = NA_();
                    if (tid < NA * 4 && (tid & 3) == 0)
                        publish16(pg, ((s & 1) * kMaxBpcRun + vb) * NA + (tid >> 2), ba, tag0 + s + 1);
                    if (kWave1 && dob) {
                        // the other taps' lane values to LDS ([value][T], value = 2 rank + I/Q);
                        // one wave reduces them during the sweep (defer_reduce)
                        double* stg = s_mem + kPwD;
                        const unsigned sb = (unsigned)dfi(*(const int*)&s_df.selB);
#pragma unroll
                        for (int s2 = 0; s2 < NT; s2++)
                            if ((sb >> s2) & 1u) {
                                const int r = __builtin_popcount(sb & ((1u << s2) - 1u));
                                stg[(2 * r) * T + tid] = oI[s2];
                                stg[(2 * r + 1) * T + tid] = oQ[s2];
                            }
                        lds_barrier();
                    } else if (dob) {
                        const int hb = dfi(s_df.hb), nB = dfi(s_df.nBv) / 2;
                        for (int ps = 1; (ps - 1) * hb < nB; ps++) {
                            const unsigned sel = sel_pass(ps);
                            const double bb = block_pass<NT, HT>(s_mem, oI, oQ, tid, sel);
                            if (tid < 2 * __builtin_popcount(sel) * 4 && (tid & 3) == 0)
                                publish16(pg, gran_region_b(NT) + (s & 3) * gran_slot_b(NT) +
                                                  (2 * (ps - 1) * hb + (tid >> 2)) * bpc + vb,
                                          bb, tag0 + s + 1);
                        }
                    }
                }
                if (srow && tid == 0) srow[2] = wall_clock64();
                if (kProbe && b.stamps && ch == 0 && tid == 0) {  // latest partial of the channel (all blocks)
                    unsigned long long* r = b.stamps + (size_t)(s % kStampSlots) * kStampRow;
                    atomicMax(r + 23, wall_clock64());
                    atomicMax(r + 24, ~wall_clock64());  // (earliest, complemented)
                }
            }
        }

        // the step's remPhase / remSample (role 2 of the descriptor, off the tail: the
        // next tail reads them after the sweep's closing barrier)
        // (by wave 2, a poller, so that wave 1's flush of the previous step starts at once)
        if (wv == (io ? GNSS_IO_DR_WAVE : 2) && lane == 0) desc_rem(tk, &s_d[cur]);
        const bool bsw = kDefer && pend && own_n_() > 0;  // the previous step's owned B values are due
        if (pend) {
            if (srow && tid == 64) srow[16] = wall_clock64();
            if (brow && tid == 64) brow[40 + 1024 + blk] = wall_clock64();  // (probe: every block's flush)
            flush();  // (the sweep's closing barrier publishes it)
            if (srow && tid == 64) srow[17] = wall_clock64();
            if (brow && tid == 64) brow[40 + 1280 + blk] = wall_clock64();
        }

        // ---- every block's partial, summed in a fixed order (bit-identical in all blocks)
        unsigned* pw = reinterpret_cast<unsigned*>(s_mem);
        {
            // (the part-1 and part-2 blocks: waves 0, 2, 3 poll while wave 1 writes the record;
            // the other blocks' wave 1 flush is short and it joins the polling after it)
            int pid = GNSS_SWEEP_IO_ALL || !dsw ? tid : (wv == 1 ? -1 : tid - (wv > 1 ? 64 : 0));
            int np = GNSS_SWEEP_IO_ALL || !dsw ? 4 * 64 : 3 * 64;
            if (kWave1 && dob) {
                // the B wave (wave 1, or wave 3 in the part-1 block, whose wave 1 writes the
                // record) reduces the other taps and publishes them; the rest poll
                const int bw = dsw ? 3 : 1;
                if (wv == bw) defer_reduce(s);
                // pollers: waves 0, 2, 3 (ranks 0, 1, 2); in the part-1 block waves 0, 2
                const int rank = wv == 0 ? 0 : wv - 1;
                pid = (wv == bw || wv == 1) ? -1 : rank * 64 + lane;
                np = dsw ? 2 * 64 : 3 * 64;
            }
            if constexpr (!kDefer) {
                if (!sweep16<(NT > 3 ? GNSS_SWEEP_BATCH : 1)>(pg, bpc * NV, tag0 + s + 1, pw, pid, np, b.run_err,
                                                               (s & 1) * kMaxBpcRun * NV))
                    return;
            } else {
                // this step's E / P / L, and the owned B values of the previous step (long published)
                const int NA = NA_();
                if (!sweep16x2(pg, bpc * NA, (s & 1) * kMaxBpcRun * NA, tag0 + s + 1, pw, bsw ? own_n_() * bpc : 0,
                               gran_region_b(NT) + ((s - 1) & 3) * gran_slot_b(NT) + dfi(s_df.own_lo) * bpc, tag0 + s,
                               pw + 2 * bpc * NA, pid, np, b.run_err))
                    return;
            }
        }
        if (srow && tid == 0) srow[3] = wall_clock64();
        if (brow && tid == 0) brow[40 + 512 + blk] = wall_clock64();  // (probe: this block's all-in)
        // wave 2 issues the whole block's next IF (it starts at A + n, ftell after this
        // read; the polls above would have queued behind it) and waits for it at the end
        // of the tail: the correlator waves never stall on it
        if (wv == 2 && s + 1 < nsteps) {
#pragma unroll
            for (int h = 0; h < 4; h++)
                prefetch_raw<SUB>(iq, ((A + n) >> 3) + ((int64_t)blk * T + h * 64 + lane) * SUB, gmax, s_raw,
                                  h * 64 + lane);
        }
        if (tid < CL * NA_()) {  // (above 3 taps: the E / P / L values, at their value index)
            const int NA = NA_();
            const double a = channel_sum_l<CL>(bpc, tid, [&](int k, int v) {
                const unsigned lo = pw[(k * NA + v) * 2], hi = pw[(k * NA + v) * 2 + 1];
                return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
            });
            const int vi = kDefer ? s_df.vmap[tid / CL] : tid / CL;
            if constexpr (GNSS_CORR_PROBE != 0)  // (probe builds: E = P = L = 1, a steady loop)
                if (tid % CL == 0) s_fin[vi] = (vi & 1) ? 0.0 * a : 1.0 + 0.0 * a;
            if constexpr (GNSS_CORR_PROBE == 0)
                if (tid % CL == 0) s_fin[vi] = D.phaseC ? -a : a;  // :447-449
        }
        const int phaseC = D.phaseC;
        lds_barrier();
        if (srow && io && tid == 0) srow[10] = wall_clock64();

        // ---- the loop update and the next descriptor: wave 0 its code half (DLL half of
        // the update), wave 3 its carrier table (PLL half), wave 2 the next remPhase; wave 1
        // keeps the full update for this step's side effects (written next step)
        const TrkChan& c = s_c;
        StepOut o;
        o.n = n;
        o.delayValue = D.delayValue;
        o.remSample = D.remSample;
        o.remChip = D.remChip_next;
        o.remPhase = D.remPhase_next;
        o.pdi = D.pdi;
        o.phaseC = phaseC;
        if constexpr ((GNSS_CORR_PROBE & 16) != 0) {
            // (probe: the tail's loop update and descriptor four extra times -- the same values
            // into the same descriptor -- between stamps 18 and 19: its cost in place, warm)
            if (srow && io && tid == 0) srow[18] = wall_clock64();
            for (int rep = 0; rep < 4; rep++) {
                const LoopUpd ur = loop_update_i(tk, c, s_fin[2 * tk.iE], s_fin[2 * tk.iE + 1], s_fin[2 * tk.iP],
                                                 s_fin[2 * tk.iP + 1], s_fin[2 * tk.iL], s_fin[2 * tk.iL + 1], o.pdi,
                                                 o.phaseC, wv == 0 || wv == 2 ? 1 : wv == 3 ? 2 : 3);
                NcoState nr{o.remChip, o.remPhase, ur.codeFreq, ur.carrierFreq, o.n, c.pos + tk.bps * o.n,
                            c.Index + (o.phaseC ? 10 : 1)};
                if (srow && io && rep == 0 && lane == 0) srow[29 + wv] = wall_clock64();  // (loop update done)
                if (wv == 0 || wv == 3)
                    prepare_desc_i(tk, nr, o.pdi, o.phaseC, wv == 0 ? 0 : 1, lane, &s_d[cur ^ 1], s_taps, nullptr,
                                   s_post, true);
                else if (wv == 2)
                    prepare_desc_i(tk, nr, o.pdi, o.phaseC, 3, lane, &s_d[cur ^ 1], s_taps, nullptr, s_post, true);
                if (srow && io && rep == 0 && lane == 0) srow[25 + wv] = wall_clock64();  // (role done)
                lds_barrier();
            }
            if (srow && io && tid == 0) srow[19] = wall_clock64();
        }
        const LoopUpd u = loop_update_i(tk, c, s_fin[2 * tk.iE], s_fin[2 * tk.iE + 1], s_fin[2 * tk.iP],
                                      s_fin[2 * tk.iP + 1], s_fin[2 * tk.iL], s_fin[2 * tk.iL + 1], o.pdi,
                                      o.phaseC, wv == 0 || wv == 2 ? 1 : wv == 3 ? 2 : 3);  // (each role's half)
        if (srow && io && tid == 0) srow[11] = wall_clock64();
        NcoState nx;
        nx.remChip = o.remChip;
        nx.remPhase = o.remPhase;
        nx.codeFreq = u.codeFreq;
        nx.carrierFreq = u.carrierFreq;
        nx.numSample = o.n;
        nx.pos = c.pos + tk.bps * o.n;
        nx.Index = c.Index + (o.phaseC ? 10 : 1);
        if (wv == 0 || wv == 3) {  // the tap colons / the carrier table of the next descriptor
            prepare_desc_i(tk, nx, o.pdi, o.phaseC, wv == 0 ? 0 : 1, lane, &s_d[cur ^ 1], s_taps,
                           srow && io ? srow + 14 : nullptr, s_post, true);
            if (srow && io && lane == 0) srow[wv == 0 ? 12 : 13] = wall_clock64();
        } else if (wv == 1) {
            if (lane == 0) {
                s_o = o;
                s_u = u;
            }
            // (idle otherwise: the previous step's owned B values, swept beside this step's
            // E / P / L, summed and written)
            if (bsw) defer_write(pw + 2 * bpc * NA_());
        } else {  // wave 2: the next step's scalars and checks, then its IF has landed
            prepare_desc_i(tk, nx, o.pdi, o.phaseC, 3, lane, &s_d[cur ^ 1], s_taps, nullptr, s_post, true);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        pend = true;
        lds_barrier();
        if (srow && tid == 0) srow[4] = wall_clock64();
        if (brow && tid == 0) brow[40 + 768 + blk] = wall_clock64();  // (probe: this block's next step ready)
        cur ^= 1;
    }
    if (kProbe && b.stamps && io && tid == 0 && ch < 64) {
        b.stamps[20 + 3 * ch] = t_start;
        b.stamps[21 + 3 * ch] = wall_clock64();
        b.stamps[22 + 3 * ch] = (unsigned long long)nsteps;
    }
    const bool had = pend;
    if (pend) flush();
    if (had) defer_final(nsteps - 1);
    if (io && tid == 64) desc_rem(tk, &s_d[cur]);  // (complete for a step-kernel follow-up)
    __syncthreads();
    if (io) {  // the state and the next step's descriptor for the next launch
        if (tid < kChanWords)
            reinterpret_cast<uint64_t*>(b.chan + ch)[tid] = reinterpret_cast<const uint64_t*>(&s_c)[tid];
        for (int e = tid; e < kDescWords; e += T)
            reinterpret_cast<unsigned*>(b.desc + ch)[e] = reinterpret_cast<const unsigned*>(&s_d[cur])[e];
    }
}

// Prepare the StepDesc of every channel from its current state (start of a phase).
__global__ void track_prepare_kernel(const TrkParams* __restrict__ pp, const TrkBuffers* __restrict__ bp,
                                     int pdi, int phaseC)
{
    const TrkParams& p = *pp;
    const TrkBuffers& b = *bp;
    const int ch = blockIdx.x;
    const TrkChan c = b.chan[ch];
    prepare_desc_block(p, nco_of(c), pdi, phaseC, b.desc + ch);
}

__global__ void track_snapshot_kernel(const TrkBuffers* __restrict__ bp, int nch)
{
    const TrkBuffers& b = *bp;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nch) b.snap[i] = b.chan[i];
}

// trackingCT.m:178-213 on the phase-A P_i (length msToProcessCT_1ms): the scan over i
// stops at the first i whose 6-before / 17-after sign test passes with i >= 600, or at
// the first i whose test runs past the end (MATLAB's index error). Every i's outcome
// depends on P alone, so one block per channel tests all i at once and keeps the first
// stopping one (the serial scan's answer).
__global__ void track_bitedge_kernel(const TrkBuffers* __restrict__ bp, int nch)
{
    const TrkBuffers& b = *bp;
    const int ch = blockIdx.x;
    __shared__ int s_first;
    if (threadIdx.x == 0) s_first = 0x7fffffff;
    __syncthreads();
    TrkChan& c = b.chan[ch];
    if (c.status != GNSS_OK) return;  // (block-uniform)
    const double* P = b.p_i_1ms + (int64_t)ch * b.n1;
    const int64_t len = b.n1;
    auto sgn = [](double x) { return (x > 0) - (x < 0); };
    int mine = 0x7fffffff;
    for (int64_t i = 7 + (int64_t)threadIdx.x; i <= len - 1; i += (int64_t)blockDim.x) {
        const int si = sgn(P[i - 1]);
        int before = 1;  // the 6 samples before differ in sign
        for (int j = 6; j >= 1; j--) before &= sgn(P[i - j - 1]) != si ? 1 : 0;
        int stop = 0;
        if (before) {
            int k = 1;  // the 17 after agree; reaching past the end first is MATLAB's error
            for (; k <= 17; k++) {
                if (i + k > len) { stop = 1; break; }
                if (sgn(P[i + k - 1]) != si) break;
            }
            if (k > 17 && i >= 600) stop = 1;
        }
        if (stop && (int)i < mine) mine = (int)i;
    }
    if (mine != 0x7fffffff) atomicMin(&s_first, mine);
    __syncthreads();
    if (threadIdx.x != 0) return;
    const int64_t i = s_first;
    int cx = 0;
    if (i != 0x7fffffff) {
        // re-run the stopping i's test serially to tell the error from the hit
        const int si = sgn(P[i - 1]);
        bool ok = true;
        for (int j = 6; j >= 1 && ok; j--) ok = sgn(P[i - j - 1]) != si;
        for (int j = 1; j <= 17 && ok; j++) {
            if (i + j > len) { c.status = GNSS_EINDEX; return; }
            ok = sgn(P[i + j - 1]) == si;
        }
        cx = (int)(i % 20) - 1;
    }
    c.countinx = cx;
    c.n1_target = b.n1 + cx;
}

// Entry to phase C (trackingCT.m:379-406): countinx = -1 resumes from the state
// after step msToProcessCT_1ms - 1 (quirk A.9); fresh C/N0 counters; seek to the
// nominal (skip + 1000 + countinx) ms position (quirk A.12); first 10-ms StepDesc.
__global__ void track_phase_c_init_kernel(const TrkParams* __restrict__ pp, const TrkBuffers* __restrict__ bp,
                                          int64_t skip)
{
    const TrkParams& p = *pp;
    const TrkBuffers& b = *bp;
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
    if (c.status == GNSS_OK) prepare_desc_block(p, nco_of(c), 10, 1, b.desc + ch);
}

hipError_t launch_track_step(const TrkParams& p, const TrkBuffers& b, const TrkDev& d, int bpc, int sub,
                             hipStream_t s)
{
    dim3 grid(p.nch * bpc), block(kTrkThreads);
#define GNSS_STEP(NT_, SUB_, DIV_, FMT_)                                                       \
    if (p.ntaps == NT_ && sub == SUB_ && (p.exact_div != 0) == DIV_ && p.fmt == FMT_) {        \
        hipLaunchKernelGGL((track_step_kernel<NT_, SUB_, DIV_, FMT_>), grid, block, 0, s, d.p, d.b, bpc); \
        return hipGetLastError();                                                              \
    }
    GNSS_STEP(3, 1, false, 0) GNSS_STEP(3, 2, false, 0) GNSS_STEP(3, 3, false, 0) GNSS_STEP(3, 4, false, 0)
    GNSS_STEP(11, 1, false, 0) GNSS_STEP(11, 2, false, 0) GNSS_STEP(11, 3, false, 0) GNSS_STEP(11, 4, false, 0)
    GNSS_STEP(3, 1, true, 0) GNSS_STEP(11, 1, true, 0)
    // the 25 taps of trackingCT_POS_updated_multicorrelator.m (int8; 8- and 24-sample lanes)
    GNSS_STEP(25, 1, false, 0) GNSS_STEP(25, 3, false, 0) GNSS_STEP(25, 1, true, 0)
    // int16 I/Q records (per-read mean removal): the per-step path only
    GNSS_STEP(3, 1, false, 1) GNSS_STEP(3, 3, false, 1) GNSS_STEP(11, 1, false, 1) GNSS_STEP(11, 3, false, 1)
    GNSS_STEP(3, 1, true, 1) GNSS_STEP(11, 1, true, 1)
#undef GNSS_STEP
    return hipErrorInvalidValue;
}

hipError_t launch_track_run(const TrkParams& p, const TrkBuffers& b, const TrkDev& d, int bpc, int vpb, int sub,
                            int nsteps, unsigned tag0, hipStream_t s)
{
    if (vpb < 1 || bpc < 1) return hipErrorInvalidValue;
    dim3 grid(p.nch * ((bpc + vpb - 1) / vpb)), block(kTrkThreads);
#define GNSS_RUN(NT_, SUB_, DIV_)                                                              \
    if (p.ntaps == NT_ && sub == SUB_ && (p.exact_div != 0) == DIV_ && vpb == 1) {            \
        hipLaunchKernelGGL((track_run_kernel<NT_, SUB_, DIV_, false>), grid, block, 0, s, d.p, d.b, bpc, vpb, \
                           nsteps, tag0);                                                      \
        return hipGetLastError();                                                              \
    }
#define GNSS_RUNV(NT_, SUB_, DIV_)                                                             \
    if (p.ntaps == NT_ && sub == SUB_ && (p.exact_div != 0) == DIV_ && vpb > 1) {             \
        hipLaunchKernelGGL((track_run_kernel<NT_, SUB_, DIV_, true>), grid, block, 0, s, d.p, d.b, bpc, vpb, \
                           nsteps, tag0);                                                      \
        return hipGetLastError();                                                              \
    }
    GNSS_RUN(3, 1, false) GNSS_RUN(3, 2, false) GNSS_RUN(3, 3, false) GNSS_RUN(3, 4, false)
    GNSS_RUN(11, 1, false) GNSS_RUN(11, 2, false) GNSS_RUN(11, 3, false) GNSS_RUN(11, 4, false)
    GNSS_RUN(3, 1, true) GNSS_RUN(11, 1, true)
    GNSS_RUNV(3, 1, false) GNSS_RUNV(3, 3, false) GNSS_RUNV(11, 1, false) GNSS_RUNV(11, 3, false)
#undef GNSS_RUN
#undef GNSS_RUNV
    return hipErrorInvalidValue;
}

int track_run_blocks_per_cu(const TrkParams& p, int sub, bool vb)
{
    int nb = 0;
#define GNSS_OCC(NT_, SUB_, DIV_, VB_)                                                         \
    if (p.ntaps == NT_ && sub == SUB_ && (p.exact_div != 0) == DIV_ && vb == VB_) {            \
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(                                      \
                &nb, reinterpret_cast<const void*>(track_run_kernel<NT_, SUB_, DIV_, VB_>),     \
                kTrkThreads, 0) != hipSuccess)                                                 \
            nb = 0;                                                                            \
        return nb;                                                                             \
    }
    GNSS_OCC(3, 1, false, false) GNSS_OCC(3, 2, false, false) GNSS_OCC(3, 3, false, false)
    GNSS_OCC(3, 4, false, false) GNSS_OCC(11, 1, false, false) GNSS_OCC(11, 2, false, false)
    GNSS_OCC(11, 3, false, false) GNSS_OCC(11, 4, false, false) GNSS_OCC(3, 1, true, false)
    GNSS_OCC(11, 1, true, false)
    // virtual-block forms (several of the step's blocks per resident block)
    GNSS_OCC(3, 1, false, true) GNSS_OCC(3, 3, false, true) GNSS_OCC(11, 1, false, true)
    GNSS_OCC(11, 3, false, true)
#undef GNSS_OCC
    return 0;
}

// Device-resident outputs (gnss_track_out.flags & GNSS_OUT_DEVICE): the MATLAB layout of
// the compact per-step records, expanded on the GPU — one row per millisecond with each
// 10-ms step's value on its ten rows (trackingCT.m:507-524), a zeroed tail. Channel i's
// field f: src[(slot * stride) + f] -> dst[(chan * nf + f) * ML + k]. grid: (x: row chunks,
// y: nch * nf).
// ntaps > 0: the taps array, compact field f = 2 * tap + (I 0 / Q 1) -> [chan][I/Q][tap].
__global__ void track_expand_kernel(const double* __restrict__ src, int64_t rec_cap, int stride, int nf,
                                    const int64_t* __restrict__ job, double* __restrict__ dst, int64_t ML,
                                    int64_t n10, int ntaps)
{
    const int i = blockIdx.y / nf, f = blockIdx.y - i * nf;
    const int64_t n1 = job[2 * i], c = job[2 * i + 1];
    const double* s = src + (int64_t)i * rec_cap * stride + f;
    const int fo = ntaps ? (f & 1) * ntaps + (f >> 1) : f;
    double* o = dst + (c * nf + fo) * ML;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < ML; k += (int64_t)gridDim.x * blockDim.x) {
        double v = 0.0;
        if (k < n1) v = s[k * stride];
        else if (k < n1 + 10 * n10) v = s[(n1 + (k - n1) / 10) * stride];
        o[k] = v;
    }
}

hipError_t launch_track_expand(const double* src, int64_t rec_cap, int stride, int nf, int nch,
                               const int64_t* job, double* dst, int64_t ML, int64_t n10, int ntaps,
                               hipStream_t s)
{
    const int64_t chunks = (ML + 255) / 256;
    hipLaunchKernelGGL(track_expand_kernel, dim3((unsigned)(chunks < 64 ? chunks : 64), (unsigned)(nch * nf)),
                       dim3(256), 0, s, src, rec_cap, stride, nf, job, dst, ML, n10, ntaps);
    return hipGetLastError();
}

hipError_t launch_track_prepare(const TrkParams& p, const TrkBuffers& b, const TrkDev& d, int pdi,
                                int phaseC, hipStream_t s)
{
    hipLaunchKernelGGL(track_prepare_kernel, dim3(p.nch), dim3(192), 0, s, d.p, d.b, pdi, phaseC);
    return hipGetLastError();
}

hipError_t launch_track_snapshot(const TrkParams& p, const TrkBuffers& b, const TrkDev& d, hipStream_t s)
{
    hipLaunchKernelGGL(track_snapshot_kernel, dim3((p.nch + 63) / 64), dim3(64), 0, s, d.b, p.nch);
    return hipGetLastError();
}

hipError_t launch_track_bitedge(const TrkParams& p, const TrkBuffers& b, const TrkDev& d, hipStream_t s)
{
    hipLaunchKernelGGL(track_bitedge_kernel, dim3(p.nch), dim3(256), 0, s, d.b, p.nch);
    return hipGetLastError();
}

hipError_t launch_track_phase_c_init(const TrkParams& p, const TrkBuffers& b, const TrkDev& d,
                                     int64_t skip, hipStream_t s)
{
    hipLaunchKernelGGL(track_phase_c_init_kernel, dim3(p.nch), dim3(192), 0, s, d.p, d.b, skip);
    return hipGetLastError();
}

}  // namespace gnss
