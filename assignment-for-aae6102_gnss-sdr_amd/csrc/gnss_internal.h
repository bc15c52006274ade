// gnss_internal.h — internal declarations shared by the C-ABI host code
// (gnss_api.cpp) and the gfx950 kernels (track.hip, acq.hip, synth.hip).
// Not part of the public boundary (that is include/gnss_mi355x.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gnss_mi355x.h"

#define GNSS_HD __host__ __device__ __forceinline__

namespace gnss {

// MATLAB colon a:d:b, MathWorks' published colonop construction (both ends toward
// the midpoint). Evaluated in fp64 with contraction disabled (-ffp-contract=off for
// every translation unit) so host, device and the CPU oracle agree bit for bit.
struct Colon {
    double a, d, c;
    int64_t n;  // intervals; elements = n + 1
};

GNSS_HD Colon colon_make(double a, double d, double b)
{
    Colon r{a, d, b, -1};
    if (!(a - a == 0) || !(d - d == 0) || !(b - b == 0)) return r;  // non-finite
    if (d == 0 || (a < b && d < 0) || (b < a && d > 0)) return r;
    double tol = 2.0 * 2.220446049250313e-16 * fmax(fabs(a), fabs(b));
    double sig = d > 0 ? 1.0 : -1.0;
    double n;
    if (a == floor(a) && d == 1) {
        n = floor(b) - a;
    } else if (a == floor(a) && d == floor(d)) {
        double q = floor(a / d);
        double rr = a - q * d;
        n = floor((b - rr) / d) - q;
    } else {
        n = round((b - a) / d);
        if (sig * (a + n * d - b) > tol) n = n - 1;
    }
    double c = a + n * d;
    if (sig * (c - b) > -tol) c = b;
    r.c = c;
    r.n = (int64_t)n;
    return r;
}

// colon_make when the caller knows the interval count to expect (b = a + hint*d up to
// rounding): if fl(b - a) is within 0.4*d of hint*d, round(fl(b - a)/d) == hint
// and the division is skipped; otherwise the general construction runs.
GNSS_HD Colon colon_make_hint(double a, double d, double b, int64_t hint)
{
    const double X = b - a;
    const double r = fma(-(double)hint, d, X);
    if (!(d > 0) || !(fabs(r) < 0.4 * d) || a == floor(a)) return colon_make(a, d, b);
    Colon o{a, d, b, hint};
    const double tol = 2.0 * 2.220446049250313e-16 * fmax(fabs(a), fabs(b));
    double n = (double)hint;
    if (a + n * d - b > tol) n = n - 1;
    double c = a + n * d;
    if (c - b > -tol) c = b;
    o.c = c;
    o.n = (int64_t)n;
    return o;
}

// colon_make_hint with the hint also as an exact double hd (== hint): no integer
// conversion on the tracking tail's critical path, the interval count by a select.
GNSS_HD Colon colon_make_hint2(double a, double d, double b, int64_t hint, double hd)
{
    const double X = b - a;
    const double r = fma(-hd, d, X);
    if (!(d > 0) || !(fabs(r) < 0.4 * d) || a == floor(a)) return colon_make(a, d, b);
    const double tol = 2.0 * 2.220446049250313e-16 * fmax(fabs(a), fabs(b));
    const bool dec = a + hd * d - b > tol;
    const double nd = dec ? hd - 1 : hd;
    double c = a + nd * d;
    if (c - b > -tol) c = b;
    return Colon{a, d, c, dec ? hint - 1 : hint};
}

GNSS_HD double colon_elem(const Colon& r, int64_t k)
{
    if (2 * k == r.n) return (r.a + r.c) / 2;
    if (k <= r.n / 2) return r.a + (double)k * r.d;
    return r.c - (double)(r.n - k) * r.d;
}

// Code = [CA(1023) repmat(CA,1,pdi) CA(1)]; Code(ceil(t)+1) = CA0[(ceil(t)+1022) % 1023]
GNSS_HD int ca_index(int64_t chip)
{
    int64_t r = (chip + 1022) % 1023;
    return (int)(r < 0 ? r + 1023 : r);
}

// The same for chip >= -1022 (every chip a step can address, ceil(t) in [-1, 1023*pdi+1]):
// one 32-bit unsigned division by a constant.
GNSS_HD unsigned ca_index32(int chip)
{
    return (unsigned)(chip + 1022) % 1023u;
}

// fmod of non-negative x by positive y with a quotient below 2^53, exact like C fmod:
// trunc(RN(x/y)) is the true quotient or one more, and x - q*y is representable in both
// cases, so the FMA is exact and one correction finishes it (the library fmod loops
// over the exponent difference).
GNSS_HD double fmod_pos(double x, double y)
{
    const double q = trunc(x / y);
    double r = __builtin_fma(-q, y, x);
    if (r < 0) r += y;
    return r;
}

constexpr double kTwoPi = 2.0 * 3.14159265358979323846;  // MATLAB 2*pi
constexpr double kTwoPiLo = 2.4492935982947064e-16;      // 2*pi - kTwoPi
constexpr double kInvTwoPi = 1.0 / kTwoPi;               // RN(1/kTwoPi)

// x / b correctly rounded, for a divisor known ahead (Fs, 2*pi: b > 0) with rb = RN(1/b),
// for every numerator whose quotient is a normal number above 2^-969 (all the tracking
// tail's: codeFreq, 2*pi*f, phases, atan outputs, sample counts). q = RN(x*rb) is within
// 2 ulps of x/b and q1 = RN(q + r*rb), r = x - q*b (by FMA), within half an ulp plus
// ~2^-52 ulp of it (the exact q + r*rb differs from x/b by (x - q*b)(rb - 1/b)); q1 is
// therefore RN(x/b) or its neighbour on x/b's side. The remainder r1 = x - q1*b is exact
// (q1 within an ulp) and x/b - q1 = r1/b, so q1 is RN(x/b) iff |r1| < b*h, h half the
// spacing from q1 to that neighbour (a quarter ulp below a power of two); b*h is exact and a
// quotient of two doubles is never a midpoint, so the test decides, and a failed test means
// the neighbour. (Markstein's correction alone is proven only for q within one ulp; this
// needs no divisor-specific proof.) Checked against IEEE division: tests/native/markstein.cpp.
// q1 within an ulp of x/b -> RN(x/b) (the rounding test above)
GNSS_HD double div_round_fix(double x, double b, double q1)
{
    const double r1 = __builtin_fma(-q1, b, x);
    int64_t bits = __builtin_bit_cast(int64_t, q1);
    const int64_t mag = bits & 0x7fffffffffffffffLL;
    const bool away = (r1 > 0) == (q1 > 0);  // |x/b| > |q1|
    const double ulp = __builtin_bit_cast(double, (mag & 0x7ff0000000000000LL) - (52LL << 52));
    const double h = ((mag & 0x000fffffffffffffLL) != 0 || away) ? 0.5 * ulp : 0.25 * ulp;
    if (r1 != 0 && __builtin_fabs(r1) > h * b) bits += away ? 1 : -1;
    return __builtin_bit_cast(double, bits);
}

GNSS_HD double div_const(double x, double b, double rb)
{
    const double q = x * rb;
    const double r = __builtin_fma(-q, b, x);
    return div_round_fix(x, b, __builtin_fma(r, rb, q));
}

// Markstein's correction alone (the first three steps above): the IEEE quotient k/Fs for the
// integer sample counts k of CarrTime (trackingCT.m:104), verified exhaustively over the
// step's k range for the run's Fs on the host (fast_div_exact); the per-sample path
GNSS_HD double div_markstein(double x, double b, double rb)
{
    const double q = x * rb;
    const double r = __builtin_fma(-q, b, x);
    return __builtin_fma(r, rb, q);
}

// sin and cos of a small argument (|x| <= ~40 rad: the lane's reduced carrier phase, the rotation
// table's phi[m], a VT sample's 2*pi-reduced phase) with a short dependent chain, for the
// correlators' lane rotation and the rotation table (track.hip GNSS_FAST_SINCOS; 0 = the device
// library's sincos) and the VT step's samples (vt.hip). Reduction by pi/2 in two
// parts (q * PIO2_HI exact for |q| < 2^20: PIO2_HI has 33 significant bits), then the classic
// fdlibm minimax kernels on [-pi/4, pi/4] (__kernel_sin / __kernel_cos, error < 1 ulp), the two
// polynomials evaluated side by side, and the quadrant's swap / negation by selects. Accuracy is
// the library's (< 1 ulp); the bits differ from it in the last place for some arguments, which
// moves the tracking sums by rounding only (the parity tests judge them against the oracle).
__device__ __forceinline__ void sincos_small(double x, double* sn, double* cs)
{
    constexpr double kTwoOverPi = 6.36619772367581382433e-01;
    constexpr double kPio2Hi = 1.57079632673412561417e+00;  // first 33 bits of pi/2
    constexpr double kPio2Lo = 6.07710050650619224932e-11;  // RN(pi/2 - kPio2Hi)
    const double q = rint(x * kTwoOverPi);
    double y = __builtin_fma(-q, kPio2Hi, x);  // exact (q * kPio2Hi exact, |x - q*kPio2Hi| small)
    const double t = q * kPio2Lo;              // (fdlibm __ieee754_rem_pio2's first round)
    const double yh = y - t;
    const double yl = (y - yh) - t;            // the tail of the reduced argument
    y = yh;
    const double z = y * y;
    // __kernel_sin(y, yl, 1) and __kernel_cos(y, yl) (fdlibm, public domain)
    const double rs = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
        1.58969099521155010221e-10, -2.50507602534068634195e-08), 2.75573137070700676789e-06),
        -1.98412698298579493134e-04), 8.33333333332248946124e-03);
    const double rc = z * __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
        __builtin_fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
        -2.75573143513906633035e-07), 2.48015872894767294178e-05), -1.38888888888741095749e-03),
        4.16666666666666019037e-02);
    const double v = z * y;
    const double s = y - ((z * (0.5 * yl - v * rs) - yl) - v * -1.66666666666666324348e-01);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + (z * rc - y * yl));
    const int n = (int)q & 3;
    const double a = (n & 1) ? c : s, b = (n & 1) ? s : c;
    *sn = (n & 2) ? -a : a;
    *cs = ((n + 1) & 2) ? -b : b;
}


// 16-B granules {lo, tag, hi, tag}: one fp64 value per granule, written by one
// buffer_store_dwordx4 sc1 and read by one buffer_load_dwordx4 sc1 (MI355X_MICROARCH.md
// hand-off table: 16-B sc1 stores and loads; each half carries the tag, so a torn read
// is simply not accepted). Half the polls of two 8-B granules per value. The tracking
// loop's hand-offs (track.hip) and the VT loop's (vt.hip).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBufRsrcWord3 = 0x00020000;  // raw buffer, gfx9 family
constexpr int kPolSc1 = 16;                // cache policy: sc1 (device coherence)

__device__ __forceinline__ void publish16(__amdgpu_buffer_rsrc_t r, int unit, double v, unsigned tag)
{
    const unsigned long long w = (unsigned long long)__double_as_longlong(v);
    const u32x4 g = {(unsigned)w, tag, (unsigned)(w >> 32), tag};
    __builtin_amdgcn_raw_buffer_store_b128(g, r, unit * 16, 0, kPolSc1);
}
__device__ __forceinline__ u32x4 load16(__amdgpu_buffer_rsrc_t r, int unit)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, unit * 16, 0, kPolSc1);
}
// the same across PCIe to coherent host memory: system coherence (sc0 sc1), past every cache
constexpr int kPolSys = 17;
__device__ __forceinline__ void publish16_sys(__amdgpu_buffer_rsrc_t r, int unit, double v, unsigned tag)
{
    const unsigned long long w = (unsigned long long)__double_as_longlong(v);
    const u32x4 g = {(unsigned)w, tag, (unsigned)(w >> 32), tag};
    __builtin_amdgcn_raw_buffer_store_b128(g, r, unit * 16, 0, kPolSys);
}
__device__ __forceinline__ u32x4 load16_sys(__amdgpu_buffer_rsrc_t r, int unit)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, unit * 16, 0, kPolSys);
}
__device__ __forceinline__ double value16(u32x4 g)
{
    return __longlong_as_double((long long)(((unsigned long long)g.z << 32) | g.x));
}

// ----------------------------------------------------------------------------
// Tracking state (one per channel, fp64), lives in HBM across step launches.
// ----------------------------------------------------------------------------
struct TrkChan {
    // NCO / loop-filter state (trackingCT.m:42-58)
    double remChip, remPhase, remSample;
    double carrier_outputLast, PLLdiscriLast, code_outputLast, DLLdiscriLast;
    double codeFreq, carrierFreqBasis, carrierFreq;
    double Zk[20];
    int64_t numSample;  // numSample of the last executed step
    int64_t pos;        // file position indicator (bytes) for the next read
    int64_t Index;      // MATLAB Index after the last step
    int64_t nstep;      // steps executed in the current phase (IndexSmall)
    int64_t slot;       // compact record slot of the next step
    int64_t n1_target;  // last 1-ms step to run (1000 + countinx)
    int64_t codedelay0;
    int32_t index_int, snrIndex;
    int32_t sv1;        // global 1-based svindex (quirk A.11)
    int32_t prn;
    int32_t status;     // GNSS_* of this channel
    int32_t countinx;
};

// Per-step compact record: the 18 TckResultCT fields of one step.
struct TrkParams {
    double Fs, codeFreqBasis, ms, codelength;
    double S;                 // signal.Sample
    double tau1code, tau2code, tau1carr, tau2carr;
    double dataBytesPerSample;  // dataPrecision*dataType
    double inv_Fs;            // RN(1/Fs)
    int32_t exact_div;        // 1: FMA-corrected k/Fs not verified for this Fs -> divide
    int64_t buf_base;         // staged byte held at iq[0] (staged byte of sample k = sbps*k)
    int64_t buf_len;          // staged bytes resident
    int64_t file_len;         // bytes in the record (EOF)
    int32_t ntaps, iE, iP, iL;
    int32_t nsv;              // GLOBAL number of channels (quirk A.11)
    int32_t nch;              // channels in this launch set
    int32_t rec_cap;          // compact record slots per channel
    int32_t cn0_cap;          // rows per channel per phase array
    int32_t probe;            // timing probe (GNSS_PROBE): 1 = skip the scalar loop update
    // IF record format (initParameters.m:36-37): bps = file bytes per sample
    // (dataPrecision*dataType); fmt = the staged layout the correlator reads:
    // 0 = int8 I/Q pairs (int8 real records are staged with Q = 0), 1 = int16 I/Q pairs
    // with the per-read mean removed (trackingCT.m:84-88) from prefix sums
    int32_t bps, fmt;
    const long long* pref_i;  // fmt 1: sum of I over the staged samples before group g
    const long long* pref_q;  //   (8-sample groups from buf_base), Q likewise
    const short* stage16;     // fmt 1: the staged int16 I/Q (absolute: stage16[2k] = I of k)
    double taps[GNSS_MAX_TAPS];
    // the persistent loop above 3 taps (lane_correlate's capture queue, at most kQcapMax
    // interior boundaries per lane): the host checked that bound for code rates up to this many
    // chips per sample; a step beyond it stops the channel with GNSS_EINDEX, as d*M >= 1 does
    double qcap_dmax;
    // Loop conventions: 0 = trackingCT.m; 1 = trackingCT_POS_updated.m:179-408 (numSample
    // by ceil, prompt replica Code(ceil(t + 0.05) + 1), codeFreq = f0 + codeNco, loop T =
    // signal.ms for every pdi, Index + 1 per step, no phase-C negation or re-seek,
    // codedelay from the channel's own delayValue row)
    // loop-filter quotients of trackingCT.m:140,147 (T_POS_updated.m:257,266), IEEE on the
    // host: tau2/tau1, and T/tau1 for pdi 1 and for the 10-ms steps (T = 1 ms in both)
    double dll_r, dll_t1, dll_t10, pll_r, pll_t1, pll_t10;
    int32_t conv;
    // replica index offset: 0 = Code(ceil(t) + 1) with Code = [CA(end) CA.. CA(1)]; 1 =
    // Code(ceil(t) + 2) with Code = [CA(end) CA.. CA(1) CA(2)]
    // (trackingCT_POS_updated_multicorrelator.m:94,233-258)
    int32_t chip_off;
    // trackingCT_multiCorr-GIVEN.m's loop (trackingCT conventions otherwise): numSample by
    // ceil (:60) and a short read raises (no "Not enough raw data" branch) -> GNSS_EIO
    int32_t given;
    // added to a tap's colon element before ceil (the +0.05 of trackingCT_POS_updated.m:216)
    double tap_post[GNSS_MAX_TAPS];
};

// Samples per lane of the step kernel: 8 * SUB, SUB <= 4.
constexpr int kLaneMax = 32;

// Everything the blocks of one step need, prepared by the previous step's last
// block (or a prepare kernel at a phase start) so a block prologue is scalar loads.
struct StepDesc {
    int64_t n, delayValue, A, g_first, g_last, Index;
    double remSample, d, inv_d, f, phi0, dhi, dlo, remChip_next, remPhase_next;
    double mu_r, mu_i;  // fmt 1: mean of I / Q over the step's samples (else 0)
    // carrier rotation of lane sample m against the lane's first sample:
    // phi[m] = RN(m*dhi + m*dlo) ~ m * 2*pi*f/Fs, rcs[m] = (cos, sin)(phi[m])
    double phi[kLaneMax];
    double2 rcs[kLaneMax];
    double tap_a[GNSS_MAX_TAPS], tap_c[GNSS_MAX_TAPS];  // colon start / end per tap
    double rc0;          // remChip at the step's start (for remSample)
    int32_t pdi, phaseC;
    int32_t bad;         // GNSS_* of the step (file / staging / numSample checks)
    int32_t bad_tap;     // GNSS_EINDEX: a replica index out of range (checked after bad)
};

struct TrkBuffers {
    const int8_t* iq;         // IF bytes (dev)
    TrkChan* chan;            // [nch]
    TrkChan* snap;            // [nch] state after step msToProcessCT_1ms - 1
    StepDesc* desc;           // [nch] next step of each channel
    const unsigned* ca_bits;  // [nch][32] C/A chips, bit set = -1
    double* partial;          // [nch][max_blocks][2*ntaps]
    unsigned int* arrive;     // [nch][kArrivePerChan][kArriveStride] arrival counters
    double* rec;              // [nch][rec_cap][GNSS_NFIELDS]
    double* taps_rec;         // [nch][rec_cap][2*ntaps] or null
    double* cn0_1;            // [nch][cn0_cap]
    double* cn0_10;           // [nch][cn0_cap]
    int64_t* dvpre;           // [nch][rec_cap+1] delayValue prefix sums of the current phase
    double* p_i_1ms;          // [nch][n1] phase-A P_i for the bit-edge search
    double* dbg_sums;         // if set: last arriver stores the raw sums [nch][2*ntaps], no finalize
    unsigned long long* stamps;  // timing probe (GNSS_STAMPS): [kStampSlots][8] wall clock + counter
    // persistent step loop (track_run_kernel): R2 hand-off granules {tag:32 | word:32}
    unsigned long long* pgran;   // [nch][gran_per_chan(ntaps)][2] block partials (16-B granules)
    unsigned* run_err;           // set when a hand-off wait times out
    int32_t n1;               // msToProcessCT_1ms
};

// Device copies of one call's TrkParams / TrkBuffers: the kernels take pointers (a
// by-value aggregate whose address reaches a non-inlined function is copied to scratch
// by every lane).
struct TrkDev {
    const TrkParams* p;
    const TrkBuffers* b;
};

// Launch wrappers (track.hip); p / b are the host copies (grid sizes, dispatch)
hipError_t launch_track_step(const TrkParams& p, const TrkBuffers& b, const TrkDev& d,
                             int blocks_per_chan, int sub, hipStream_t s);
// Persistent form: `nsteps` steps of every channel in one launch (all nch*bpc blocks
// resident); tags of this launch's hand-offs are tag0 + 1 .. tag0 + nsteps.
hipError_t launch_track_run(const TrkParams& p, const TrkBuffers& b, const TrkDev& d,
                            int blocks_per_chan, int vblocks_per_block, int sub, int nsteps, unsigned tag0,
                            hipStream_t s);
// blocks of the persistent kernel one CU can hold (occupancy query), for the host's
// residency check
int track_run_blocks_per_cu(const TrkParams& p, int sub, bool vblocks = false);
hipError_t launch_track_prepare(const TrkParams& p, const TrkBuffers& b, const TrkDev& d, int pdi,
                                int phaseC, hipStream_t s);
hipError_t launch_track_snapshot(const TrkParams& p, const TrkBuffers& b, const TrkDev& d, hipStream_t s);
hipError_t launch_track_bitedge(const TrkParams& p, const TrkBuffers& b, const TrkDev& d, hipStream_t s);
hipError_t launch_track_phase_c_init(const TrkParams& p, const TrkBuffers& b, const TrkDev& d,
                                     int64_t skip, hipStream_t s);
// GNSS_OUT_DEVICE: expand the compact records [i][rec_cap][stride] (field f of nf) into the
// caller's device array [chan][nf][ML]; job[2i] = rows before the 10-ms values, job[2i+1] =
// output channel index (device array).
hipError_t launch_track_expand(const double* src, int64_t rec_cap, int stride, int nf, int nch,
                               const int64_t* job, double* dst, int64_t ML, int64_t n10, int ntaps,
                               hipStream_t s);

// Timing probes (per-step wall-clock stamps, the GNSS_PROBE bits) exist only in the probe
// builds (tools/build_probe.sh, tools/build_commit_lib.sh: -DGNSS_PROBE_BUILD=1): in the
// product library every stamp / probe branch of the kernels folds away at compile time.
#ifndef GNSS_PROBE_BUILD
#define GNSS_PROBE_BUILD 0
#endif
constexpr bool kProbe = GNSS_PROBE_BUILD != 0;
// A/B knobs of the tracking exchange (tools/build_variant.sh; product: 0): s_sleep between
// the sweep's poll rounds, and a channel's blocks on one XCD (8 channels).
#ifndef GNSS_XCHG_SLEEP
#define GNSS_XCHG_SLEEP 0
#endif
#ifndef GNSS_XCD_LOCAL
#define GNSS_XCD_LOCAL 0
#endif

constexpr int kTrkThreads = 256;
constexpr int kArriveStride = 64;   // words: one 256-B line per counter
constexpr int kArrivePerChan = 9;   // 8 XCD-group counters + the channel counter
constexpr int kStampSlots = 2200;
constexpr int kMaxBpc = 1024; // blocks per channel per step (partial buffer)
constexpr int kMaxBpcRun = 256;  // blocks per channel of the persistent kernel
// ... as its LDS holds them: above 3 taps 192 (the partials' LDS then leaves room for three
// blocks per CU; 192 blocks of 24-sample lanes = 1.18 M samples per step)
constexpr int run_bpc_cap(int ntaps) { return ntaps > 3 ? 192 : kMaxBpcRun; }
constexpr int kMaxVpb = 16;      // virtual blocks per resident block of the persistent kernel
// lane_correlate's capture queue (A/B knob): 0 = every tap's prefix read after every 8-sample
// subgroup (the default: the queue measured 8-16 % slower at 11 taps and 8 % at 3,
// profiles/r05_ab_cfg5_variants.txt); 1 = the queue above 3 taps; 2 = at 3 taps too
#ifndef GNSS_QCAP
#define GNSS_QCAP 0
#endif
// the persistent loop's tap window (lane_correlate): tap offsets (+ prompt post) within this
// many chips of each other, so every tap's chip at a lane's start lies in one 32-chip run
constexpr double kTapSpan = 30.0;
constexpr int kQcapMax = 8;      // capture-queue entries per lane (lane_correlate, the LDS slots)

// The most taps whose replica boundary can fall inside one lane of M samples when the code
// advances at most dmax chips per sample: tap s's boundaries sit where frac(t + off_s) wraps,
// so a lane spanning (M - 1) dmax chips holds a boundary of every tap whose fractional offset
// lies in a window of that width (taps whose offsets differ by whole chips count once each).
inline int max_taps_in_lane(const double* taps, const double* post, int n, int M, double dmax)
{
    const double w = (M - 1) * dmax + 1e-9;
    int best = 0;
    for (int a = 0; a < n; a++) {
        const double x = taps[a] + (post ? post[a] : 0.0);
        int c = 0;
        for (int b = 0; b < n; b++) {
            double f = (taps[b] + (post ? post[b] : 0.0)) - x;
            f -= floor(f);
            if (f < w || f > 1.0 - 1e-9) c++;
        }
        best = c > best ? c : best;
    }
    return best;
}
// The persistent kernel's 16-B hand-off granules per channel. 3 taps: [2 (step parity)]
// [kMaxBpcRun][6]. Above 3 taps only the loop's E/P/L go through the step's exchange
// ([2][kMaxBpcRun][<= 6], region A); the other taps' partials (region B) are published after
// them and summed one step later by their owner blocks: [kDeferSlots (step mod 4)]
// [value < 2 ntaps][kMaxBpcRun]. Four slots: a block can run at most two steps ahead of the
// owner that still reads a slot.
constexpr int kDeferSlots = 4;
constexpr int gran_region_b(int ntaps) { return ntaps > 3 ? 2 * kMaxBpcRun * 6 : 0; }
constexpr int gran_slot_b(int ntaps) { return 2 * ntaps * kMaxBpcRun; }
constexpr int gran_per_chan(int ntaps)
{
    return ntaps > 3 ? gran_region_b(ntaps) + kDeferSlots * gran_slot_b(ntaps) : 2 * kMaxBpcRun * 2 * ntaps;
}
constexpr int kDescWords = (int)(sizeof(StepDesc) / 4);

// ----------------------------------------------------------------------------
// Acquisition (acq.hip)
// ----------------------------------------------------------------------------
struct AcqPeak {           // per-PRN detector result
    double peak;
    int32_t fbin;          // 0-based
    int32_t cp;            // 0-based code phase
    double snr;
    double peak2;
};

hipError_t launch_acq_wipe(const int8_t* iq, const double2* xs, int64_t S, int datalen, int nbins, double IF,
                           double freqMin, double freqStep, double Fs, float2* out, hipStream_t s);
hipError_t launch_acq_code(const float* ca, const int32_t* prn_slot, int nprn, int64_t S,
                           double codeFreqBasis, double Fs, float2* out, hipStream_t s);
hipError_t launch_acq_mul(const float2* code_spec, const float2* sig_spec, int nprn, int nsig,
                          int64_t S, float2* out, hipStream_t s);
hipError_t launch_acq_power(const float2* y, int nprn, int nbins, int datalen, int64_t S,
                            int first_ms, float* corr, hipStream_t s);
// the same at fp64 (the reference's precision)
hipError_t launch_acq_wipe(const int8_t* iq, const double2* xs, int64_t S, int datalen, int nbins, double IF,
                           double freqMin, double freqStep, double Fs, double2* out, hipStream_t s);
hipError_t launch_acq_code(const float* ca, const int32_t* prn_slot, int nprn, int64_t S,
                           double codeFreqBasis, double Fs, double2* out, hipStream_t s);
hipError_t launch_acq_mul(const double2* code_spec, const double2* sig_spec, int nprn, int nsig,
                          int64_t S, double2* out, hipStream_t s);
hipError_t launch_acq_power(const double2* y, int nprn, int nbins, int datalen, int64_t S,
                            int first_ms, double* corr, hipStream_t s);
hipError_t launch_acq_peak(const float* corr, int nprn, int nbins, int64_t S, int cshift,
                           int perm, AcqPeak* out, void* scratch, hipStream_t s);
hipError_t launch_acq_peak(const double* corr, int nprn, int nbins, int64_t S, int cshift,
                           int perm, AcqPeak* out, void* scratch, hipStream_t s);

// Two-pass FFT correlator for S = P * 2000 (acq_fft.hip)
bool acq_fft_supported(int64_t S);
// V = float2 (fp32 fast mode) or double2 (fp64, the reference's precision)
// (a subset: the code spectra when `codes`, and the signal spectra of bins [bin0, bin0 + nbc) of
// every ms; nbc < 0 = to the last bin. The defaults: the whole pass)
template <class V>
hipError_t launch_acq_fft_forward(const int8_t* iq, const double2* xs, int64_t S, int datalen, int nbins, double IF,
                                  double freqMin, double freqStep, double Fs, const float* ca,
                                  int nprn, double codeFreqBasis, const V* tw_row,
                                  const V* tw_col, V* B, V* X, hipStream_t s, int bin0 = 0, int nbc = -1,
                                  bool codes = true);
// parts: kAcqCols (the column pass into A), kAcqRows (the row pass out of A into corr), or both
constexpr int kAcqCols = 1, kAcqRows = 2;
hipError_t launch_acq_fft_correlate(const float2* C, const float2* X, int64_t S, int datalen,
                                    int nbins, int nprn, int first_pair, int npair,
                                    const float2* tw_row, const float2* tw_col, float2* A,
                                    float* corr, hipStream_t s, int parts = kAcqCols | kAcqRows);
hipError_t launch_acq_fft_correlate(const double2* C, const double2* X, int64_t S, int datalen,
                                    int nbins, int nprn, int first_pair, int npair,
                                    const double2* tw_row, const double2* tw_col, double2* A,
                                    double* corr, hipStream_t s, int parts = kAcqCols | kAcqRows);
// fp64, the column pass of one batch and the row pass of the previous one in one launch, their
// blocks interleaved (the row blocks within the grid's first `front` percent); see acq_fft.hip
hipError_t launch_acq_fft_pair(const double2* C, const double2* X, int64_t S, int datalen, int nbins, int nprn,
                               int cols_first, int cols_n, double2* Acols, int rows_first, int rows_n,
                               const double2* Arows, const double2* tw_row, const double2* tw_col, double* corr,
                               int front, hipStream_t s);
// fp64, every (bin, PRN) pair in one persistent launch with the column/row intermediate
// kept in each XCD's L2 (nslot ring slots per XCD, 2..4); see acq_fft.hip
size_t acq_fused_sync_bytes();
size_t acq_fused_err_offset();  // byte offset of the error word in the sync block
size_t acq_fused_ring_bytes(int64_t S);
hipError_t launch_acq_fft_correlate_fused(const double2* C, const double2* X, int64_t S, int datalen, int nbins,
                                          int nprn, int nslot, const double2* tw_row, const double2* tw_col,
                                          double2* ring, void* sync, double* corr, hipStream_t s);
bool fine_fft_supported(int64_t S, int L);
// (a batch of nsv SVs per launch: scratch for nsv, SV k's code delay cd[k] on the device, its
// code table ca + 1023 k, its 1-based arg-max kbest[k])
size_t fine_fft_scratch_bytes(int64_t S, int L, int datalen, int nsv);
hipError_t launch_fine_fft_tables(int64_t S, int L, int datalen, void* scratch, hipStream_t s);
hipError_t launch_fine_fft_argmax(const int8_t* iq, const double2* xs, int64_t S, int L, int datalen,
                                  const int32_t* cd, int nsv, const float* ca, double Fs, double codeFreqBasis,
                                  double codelength, int shifted, void* scratch, int64_t* kbest, hipStream_t s);
hipError_t launch_fine_build(const int8_t* iq, const double2* xs, int64_t S, int L, const int32_t* codedelay,
                             const float* ca, int nsv, double Fs, double codeFreqBasis,
                             double codelength, int64_t N, double2* out, hipStream_t s);
hipError_t launch_fine_argmax(const double2* F, int nsv, int64_t N, int shifted, void* scratch,
                              int64_t* kbest, hipStream_t s);

size_t acq_scratch_bytes(int nprn, int nsv);

// IF record formats (ifmt.hip)
// one fread's samples as fp64 complex (prec 1 / type 1: (x, 0); prec 2 / type 2: I, Q
// minus their means); sums = 2 words of device scratch
hipError_t launch_stage_cpx(const int8_t* src, int prec, int type, int64_t nsamp, double2* out,
                            unsigned long long* sums, hipStream_t s);
// int8 real samples -> int8 I/Q pairs with Q = 0
hipError_t launch_real8_to_iq8(const int8_t* src, int64_t n, int8_t* dst, hipStream_t s);
// int16 I/Q: exclusive prefix sums of I and Q over ngroups 8-sample groups (ngroups + 1
// entries each)
size_t prefix16_scratch_bytes(int64_t ngroups);
hipError_t launch_prefix16(const short* src, int64_t ngroups, long long* pref_i, long long* pref_q,
                           void* scratch, size_t scratch_bytes, hipStream_t s);

// The acquisition kernels' sample source: the record's int8 I/Q bytes, or an fp64
// complex staging of another format (launch_stage_cpx).
struct SrcIQ8 {
    const int8_t* p;
    __device__ __forceinline__ double2 at(int64_t n) const
    {
        const char2 r = *reinterpret_cast<const char2*>(p + 2 * n);
        return make_double2((double)r.x, (double)r.y);
    }
};
struct SrcC64 {
    const double2* p;
    __device__ __forceinline__ double2 at(int64_t n) const { return p[n]; }
};

// ---- Vector tracking (trackingVT_POS_updated.m:157-349): the scalar arithmetic of a step,
// one source for the host half (vt.cpp, gnss_vt_nco_step) and the kernel's scalar end
// (vt.hip), compiled with -ffp-contract=off on both sides so every operation rounds as
// MATLAB's does (libm calls aside: atan / log10 / atan2 / hypot within an ulp).

// C/N0 of one K = 20 block of Zk = P_i^2 + P_q^2 (trackingCT.m:120-134 and
// trackingVT_POS_updated.m:297-301, the same estimator): mean, var over N - 1,
// NA2 = sqrt(mean^2 - var) (complex where negative, quirk A.16), |10 log10(NA2 / (2 varIQ) / T)|
GNSS_HD double cn0_moment(const double* Z, double T)
{
    double mean = 0;
    for (int k = 0; k < 20; k++) mean += Z[k];
    mean = mean / 20;
    double var = 0;
    for (int k = 0; k < 20; k++) var += (Z[k] - mean) * (Z[k] - mean);
    var = var / 19;
    const double m2v = mean * mean - var;
    const double scale = 1 / T;
    if (m2v >= 0) {
        const double NA2 = sqrt(m2v);
        const double varIQ = 0.5 * (mean - NA2);
        return fabs(10 * log10(scale * NA2 / (2 * varIQ)));
    }
    const double y = sqrt(-m2v);  // NA2 = i*y
    const double nr = 0, ni = scale * y;
    const double dr = 2 * (0.5 * mean), di = 2 * (0.5 * -y);
    const double den = dr * dr + di * di;
    const double zr = (nr * dr + ni * di) / den, zi = (ni * dr - nr * di) / den;
    const double lr = 10 * (log(hypot(zr, zi)) / log(10.0));
    const double li = 10 * (atan2(zi, zr) / log(10.0));
    return hypot(lr, li);
}

// Spacing = 0.7:-0.05:-0.7 (:27) as MATLAB's colon builds it; element i1 (1-based)
GNSS_HD double vt_spacing(int i1)
{
    return colon_elem(colon_make(0.7, -0.05, -0.7), i1 - 1);
}

// The step's read size and replica chips (:161, :217-249): numSample with the LAST step's
// code frequency; the E / P / L colons (0 + Spacing + remChip) : cps : ((n-1)*cps + Spacing +
// remChip) with the new one must each have n elements (ceil_mx's concatenation and
// t_CodePrompt(numSample)); chip index j = ceil(t(1)) + 1, clamped to 1025 (:240-246
// inspects that one element), within Code = [CA(end) repmat(CA,1,pdi) CA(1)] (:110).
struct VtPrep {
    int64_t n;
    int64_t j[3];  // 1-based indices into Code for E / P / L
    int bad;
};
GNSS_HD VtPrep vt_prepare(double Fs, double codelength, int pdi, double remChip, double codeFreq_old,
                          double codeFreq_new)
{
    VtPrep p{0, {1, 1, 1}, GNSS_OK};
    const double ns = ceil((codelength * pdi - remChip) / (codeFreq_old / Fs));
    if (!(ns >= 1) || ns > 1e9) {
        p.bad = GNSS_EINDEX;
        return p;
    }
    p.n = (int64_t)ns;
    const double cps = codeFreq_new / Fs;  // :218
    const int sp[3] = {5, 15, 25};
    const int64_t len = 1023 * (int64_t)pdi + 2;
    for (int s = 0; s < 3; s++) {
        const double spc = vt_spacing(sp[s]);
        const double a = (0 + spc) + remChip;
        const Colon c = colon_make(a, cps, ((double)(p.n - 1) * cps + spc) + remChip);
        if (c.n != p.n - 1) p.bad = GNSS_EINDEX;
        double j = ceil(a) + 1;
        if (j > 1025) j = 1025;
        if (!(j >= 1) || j > (double)len) p.bad = GNSS_EINDEX;
        p.j[s] = p.bad ? 1 : (int64_t)j;
    }
    return p;
}

// Code(j) for Code = [CA(1023) CA ... CA CA(1)], from CA chip values ca(i) (i 0-based)
template <class CaAt>
GNSS_HD int vt_code_at(int64_t j, int pdi, CaAt ca)
{
    const int64_t len = 1023 * (int64_t)pdi + 2;
    return j == 1 ? ca(1022) : j == len ? ca(0) : ca((int)((j - 2) % 1023));
}

// remCarrPhase after a read of n samples: rem(Wave(numSample+1), 2*pi) (:275-276, :285) --
// vt_finish's, and gnss_tracking_vt's for the next step's read before the sums are in
GNSS_HD double vt_rem_carr_phase(double carrFreq, int64_t n, double Fs, double remCarrPhase)
{
    const double W = kTwoPi * (carrFreq * ((double)n / Fs)) + remCarrPhase;
    return fmod(W, kTwoPi);
}

// The PLL of a step (:305-311) from its prompt sums: carrError, carrNco and the next carrFreq --
// vt_finish's, and gnss_tracking_vt's to post the next step's frequency first
struct VtPll {
    double carrError, carrNco, carrFreq;
};
GNSS_HD VtPll vt_pll(const gnss_vt_chan& c, int pdi, double tau1carr, double tau2carr, double P_i, double P_q)
{
    VtPll r;
    r.carrError = atan(P_q / P_i) / (2.0 * 3.14159265358979323846);
    r.carrNco = c.oldCarrNco + (tau2carr / tau1carr) * (r.carrError - c.oldCarrError) +
                r.carrError * (pdi * 1e-3 / tau1carr);
    r.carrFreq = c.carrFreqBasis + r.carrNco;
    return r;
}

// The rest of the step from its sums (:247-249, :284-347): E / P / L, remChip, remCarrPhase,
// the C/N0 estimator, PLL, DLL discriminator, the record; advances `c`. bps = bytes per
// sample (dataPrecision * dataType), code[3] = the E / P / L chip values.
GNSS_HD int vt_finish(double Fs, double ms, int pdi, int bps, double tau1carr, double tau2carr,
                      gnss_vt_chan* c, const VtPrep& p, const int* code, double codeFreq_new, double sI,
                      double sQ, gnss_vt_out* o)
{
    const int64_t n = p.n;
    const double cps = codeFreq_new / Fs;
    const double sp = vt_spacing(15);
    const Colon col = colon_make((0 + sp) + c->remChip, cps, ((double)(n - 1) * cps + sp) + c->remChip);
    if (col.n != n - 1) return GNSS_EINDEX;
    const double remChip = (colon_elem(col, n - 1) + cps) - 1023 * pdi;  // :284
    // Wave(numSample+1) = 2*pi*(carrFreq * (numSample/Fs)) + remCarrPhase (:275-276, :285)
    const double remCarrPhase = vt_rem_carr_phase(c->carrFreq, n, Fs, c->remCarrPhase);
    o->E_i = code[0] * sI;
    o->E_q = code[0] * sQ;
    o->P_i = code[1] * sI;
    o->P_q = code[1] * sQ;
    o->L_i = code[2] * sI;
    o->L_q = code[2] * sQ;
    // C/N0 (:292-304; flag_snr is 1 throughout)
    o->CN0 = 0;
    o->cn0_row = 0;
    c->index_int += 1;
    c->Zk[c->index_int - 1] = o->P_i * o->P_i + o->P_q * o->P_q;
    if (c->index_int % 20 == 0) {
        o->CN0 = cn0_moment(c->Zk, 1 * ms * pdi);
        o->cn0_row = c->snrIndex;
        c->index_int = 0;
        c->snrIndex += 1;
    }
    // PLL (:305-311)
    const VtPll pll = vt_pll(*c, pdi, tau1carr, tau2carr, o->P_i, o->P_q);
    const double carrError = pll.carrError, carrNco = pll.carrNco, carrFreq = pll.carrFreq;
    // DLL discriminator (:314-316)
    const double E = sqrt(o->E_i * o->E_i + o->E_q * o->E_q);
    const double L = sqrt(o->L_i * o->L_i + o->L_q * o->L_q);
    o->codeError = -0.5 * (E - L) / (E + L);
    o->carrError = carrError;
    o->carrNco = carrNco;
    o->remChip = remChip;
    o->remCarrPhase = remCarrPhase;
    o->codeFreq = codeFreq_new;
    o->carrFreq = carrFreq;
    o->numSample = n;
    // ftell after reading numSample samples (:162-176, :344); codedelay =
    // mod(absoluteSample / (dataPrecision * dataType), Fs * ms) (:347)
    const int64_t absS = c->file_ptr + n * bps;
    o->absoluteSample = absS;
    o->codedelay = fmod_pos((double)absS / bps, Fs * ms);
    o->status = GNSS_OK;
    c->file_ptr = absS;
    c->remChip = remChip;
    c->remCarrPhase = remCarrPhase;
    c->codeFreq = codeFreq_new;
    c->carrFreq = carrFreq;
    c->oldCarrNco = carrNco;
    c->oldCarrError = carrError;
    return GNSS_OK;
}

// The vector half (vtnav.cpp) split around the VT kernel, so that gnss_tracking_vt can run
// the parts that need no correlation of the step while the kernel runs. Host only.
// A channel's orbit (svPosVel.m) at transmit time t: a pure function of the ephemeris and t,
// so one computed ahead for the t the prediction then forms is the one it would compute.
struct VtOrbit {
    double t;
    double sv[3], vel[3], clkm, clkv, grp;
    int st;
};
// transmitTimeVT + numSample / Fs (trackingVT_POS_updated.m:181), as the prediction forms it
double vt_transmit_next(const gnss_vt_nav& v, int i, int64_t numSample);
void vt_orbit(const gnss_vt_nav& v, int i, double t, VtOrbit* o);
// gnss_vt_nav_predict with an orbit computed ahead (used when its t is the step's; else computed)
int vt_nav_predict_at(gnss_vt_nav* v, int i, int64_t numSample, const VtOrbit* ahead, double* codeFreq,
                      double* deltaPr, double sv_vel[3]);
// The EKF update's geometry half (:357-398 without the measurements): H, the rate prediction
// of each channel, the gain and the updated covariance; needs the step's predictions only.
struct VtGain {
    int st;
    double H[2 * GNSS_VT_MAX_CH * 8], K[8 * 2 * GNSS_VT_MAX_CH], cov[64], T[64];
    double prr_pred[GNSS_VT_MAX_CH], clkv[GNSS_VT_MAX_CH], sv_unrot[GNSS_VT_MAX_CH][3];
    double svr_last[3], vel_last[3], localTime;
};
void vt_nav_gain(const gnss_vt_nav& v, VtGain* g);
// ... and its measurement half: gnss_vt_nav_update == vt_nav_gain then vt_nav_correct
int vt_nav_correct(gnss_vt_nav* v, const VtGain& g, const double* codeError, const double* codeFreq,
                   const double* carrFreq, gnss_vt_navsol* sol);
// remChip after a step of n samples at code frequency codeFreq_new (vt_finish, :284): the read
// sizes of a VT channel do not depend on its samples, so the next step's is known a step ahead
inline double vt_remchip_next(double Fs, int pdi, double remChip, double codeFreq_new, int64_t n)
{
    const double cps = codeFreq_new / Fs;
    const double sp = vt_spacing(15);
    const Colon col = colon_make((0 + sp) + remChip, cps, ((double)(n - 1) * cps + sp) + remChip);
    return (colon_elem(col, n - 1) + cps) - 1023 * pdi;
}

// calcLoopCoef.m:41-45
GNSS_HD void calc_loop_coef(double LBW, double zeta, double k, double& t1, double& t2)
{
    const double Wn = LBW * 8 * zeta / (4 * (zeta * zeta) + 1);
    t1 = k / (Wn * Wn);
    t2 = 2.0 * zeta / Wn;
}

// The multi-step kernel (vt.hip): one workgroup per channel loops over nsteps steps.
struct VtRunArgs {
    const uint8_t* rec;       // staged record window; byte b of the file at rec[b - base]
    int64_t base, len;        // window [base, base + len) in file bytes
    int64_t file_len;         // the file's length (bytes): EIO past it
    gnss_vt_chan* chans;      // [n], advanced in place
    const double* codeFreq;   // [nsteps][n]
    gnss_vt_out* out;         // [nsteps][n]
    const unsigned* ca_bits;  // [n][32] C/A chips as sign bits (bit set: -1)
    double Fs, ms, codelength, tau1carr, tau2carr;
    int n, nsteps, pdi, prec, dtype;
};
hipError_t launch_vt_run(const VtRunArgs& a, hipStream_t s);
// One step of n channels over n x nb blocks (int8 records), the EKF loop's step: the host
// sizes each read and keeps the channel states; block b of channel c sums the carrier-wiped
// samples [b*chunk, (b+1)*chunk) of the read (chunk = ceil(ns / nb)) into part[(c*nb + b)*2 ..];
// the grid's last block adds each channel's partials in block order into sums[2c ..] and then
// posts `seq` to *done (coherent host memory, system scope), so the host takes the sums
// without waiting for the grid to retire.
struct VtStepArgs {
    const uint8_t* rec;             // staged record window
    double Fs;
    int real8;                      // int8 real samples (else int8 I/Q)
    unsigned seq;                   // the step's number
    double* part;                   // [n][nb][2], device memory
    double* sums;                   // [n][2], coherent host memory
    unsigned* done;                 // [1], coherent host memory
    unsigned* ticket;               // [1], device memory, 0 between launches
    int64_t off[GNSS_VT_MAX_CH];    // the read's first byte in the window
    int64_t ns[GNSS_VT_MAX_CH];     // samples read (0: the channel sits the step out)
    double f[GNSS_VT_MAX_CH];       // carrFreq
    double phi0[GNSS_VT_MAX_CH];    // remCarrPhase
    double rfs[GNSS_VT_MAX_CH];     // RN(1/Fs) if k/Fs = div_markstein for k < ns (host-verified), else 0
};
hipError_t launch_vt_step(const VtStepArgs& a, int n, int nb, hipStream_t s);
// The EKF loop's steps from one launch (vt_loop_kernel). Both directions are 16-B granules
// {lo, tag, hi, tag} in coherent host memory, tagged with the step's number (seq0, seq0 + 1,
// ...): the host writes each channel's read as kVtStepWords granules (vt_gran_put), read by one
// block that relays them through device memory to the rest and gathers their sums; the step
// completes when the channel sums' 2n granules carry its number (vt_sums_get). Read granules
// tagged kVtLoopStop end the launch, and so does no new step within `timeout` (then the host
// sees the stream idle with the step not done). Each 8-B half is written and read whole, so a
// granule read while it is rewritten has one stale tag and is not accepted.
struct alignas(16) VtGran {
    uint64_t lo, hi;  // {value bits 0..31, tag}, {value bits 32..63, tag}
};
inline void vt_gran_put(VtGran* g, uint64_t bits, unsigned tag)
{
    __atomic_store_n(&g->lo, (bits & 0xffffffffull) | ((uint64_t)tag << 32), __ATOMIC_RELAXED);
    __atomic_store_n(&g->hi, (bits >> 32) | ((uint64_t)tag << 32), __ATOMIC_RELAXED);
}
// the value of a granule carrying `tag`, else false
inline bool vt_gran_get(const VtGran* g, unsigned tag, uint64_t* bits)
{
    const uint64_t lo = __atomic_load_n(&g->lo, __ATOMIC_ACQUIRE), hi = __atomic_load_n(&g->hi, __ATOMIC_ACQUIRE);
    if ((unsigned)(lo >> 32) != tag || (unsigned)(hi >> 32) != tag) return false;
    *bits = (lo & 0xffffffffull) | (hi << 32);
    return true;
}
struct VtBlockStep {  // one channel's read of a step
    int64_t off, ns;     // first byte in the window, samples (0: the channel sits the step out)
    double f, phi0;      // carrFreq, remCarrPhase
    double rfs;          // VtStepArgs::rfs
};
constexpr unsigned kVtLoopStop = 0xffffffffu;
constexpr int kVtStepWords = 5;  // VtBlockStep's words, relayed as 16-B granules
struct VtLoopArgs {
    const uint8_t* rec;
    int64_t rec_len;     // the window's bytes (the next read's prefetch stays inside)
    double Fs;
    int real8;
    unsigned seq0;
    const VtGran* mail;  // [2][n][kVtStepWords], coherent host memory: the steps' reads, step seq in
                         // half seq & 1 (the next step's early words never overwrite a step the
                         // lead may not have read yet)
    VtGran* sums;        // [n][2], coherent host memory: the channels' sums
    uint64_t timeout;    // wall-clock ticks (wall_clock64) a block waits for a step
    void* gstep;         // [n][kVtStepWords] 16-B granules, device memory: the relayed reads
    void* gpart;         // [n][nb][2] 16-B granules, device memory: the blocks' sums
    unsigned long long* stamps;  // probe builds (vt.hip GNSS_VT_PROBE & 4): [kVtStampSteps][8] marks
};
constexpr int kVtStampSteps = 2000;
constexpr int kVtLoopMaxBlocks = 1024;  // (co-resident on 256 CUs with room to spare)
constexpr double kVtLoopTimeoutS = 10;  // seconds a loop block waits for the next step
hipError_t launch_vt_loop(const VtLoopArgs& a, int n, int nb, hipStream_t s);
// blocks of vt_loop_kernel resident at once on `device` (occupancy x CUs, at most
// kVtLoopMaxBlocks): a loop grid must fit, since a step waits for every block's sums
int vt_loop_resident_blocks(int device);
constexpr int kVtStepThreads = 256;
constexpr int kVtStepSamples = 8 * kVtStepThreads;  // samples per block at the nominal read
constexpr int kVtLoopSamples = 3 * kVtStepThreads;  // ... in loop mode (vt_loop_kernel)
// generateCAcode.m's 1023 +-1 chips of `prn` (host)
void ca_chips(int prn, float* out);

// Synthetic IF (synth.hip)
hipError_t launch_synth_if(const gnss_synth& cfg, const float* ca, uint64_t sample0,
                           uint64_t nsamples, int8_t* dst, hipStream_t s);

}  // namespace gnss
