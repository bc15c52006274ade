// acq_fft.hip — acquisition.m's FFT work for gfx950 without rocFFT's Bluestein path:
//  (1) the parallel-code-phase search (acquisition.m:47-61) as a two-pass mixed-radix FFT
//      correlator in fp64 (the reference's precision) or fp32 (fast mode) for S = P * 2000
//      with P prime (Opensky 58000 = 29 * 2000,
//      Urban 26000 = 13 * 2000);
//  (2) the fine-frequency search (acquisition.m:103-116) in fp64: the zero-padded
//      N = L*S*datalen point FFT of the 10-ms code-wiped block, split into datalen
//      transforms of M = L*S points (X[datalen*q + r] = DFT_M(x .* w_N^(-n*r))[q]),
//      each a three-level FFT (P x L x 2000), reduced to the first fftshift-ed argmax
//      without storing the spectrum.
//
// A length-S transform does not fit one CU's LDS (464 KB of complex fp32), so every
// transform is a four-step FFT: P-point DFTs down the columns of a P x 2000 view (in
// registers, one column per lane) and 2000-point DFTs along the rows (Stockham in
// LDS, radices 5 5 5 16), with the four-step twiddle folded into the neighbouring pass.
// Correlator passes, loads and epilogues fused:
//   forward  F1: rows  x[P*n1 + n2] (carrier wipe / code replica built on the fly)
//                -> B[n2][k1] * w_S^(-n2*k1)
//            F2: cols  DFT_P over n2 -> X[k1 + 2000*k2] (natural order)
//   inverse  I1: cols  Z[k] = C_p[k] * conj(X_{ms,bin}[k]) (acquisition.m:57-59),
//                DFT_P over k2, * w_S^(+k1*tau2) -> A[tau2][k1]
//            I2: rows  DFT_2000 over k1 -> y[tau2 + P*tau1]; |y|^2 / S^2 summed over
//                the ms in order (acquisition.m:53-61) in registers -> corr[tau2][tau1]
// The correlation surface is stored tau2-major ("permuted"); the detector maps
// storage index s = tau2*2000 + tau1 to the code phase tau = tau2 + P*tau1.
#include "gnss_internal.h"

// FFT values need no bit-for-bit replay of the reference: let the compiler fuse a product
// into the sum it feeds. Where a sum has two products (a*b + c*d) the contraction could fuse
// either one, chosen by the schedule, so two kernels running the same source (the fused
// and the two-launch correlators, a refactored body) could round differently: those sums are
// written with the fused product fixed (fma2 below).
#pragma clang fp contract(fast)

namespace gnss {

namespace {

constexpr int kRow = 2000;      // row length, 5*5*5*16
constexpr int kRowPad = 2100;   // LDS row of the radix-20-first transforms (stage_batch SW)
constexpr int kRowThreads = 256;
constexpr int kColThreads = 256;

// cos/sin(2*pi*m/P) (tools/gen_dft_consts.py 13 29); the fp32 kernels round them
template <int P> struct PrimeTab;
template <> struct PrimeTab<13> {
    static constexpr double c[13] = {1.0, 0.8854560256532099, 0.5680647467311559, 0.120536680255323, -0.35460488704253545, -0.7485107481711012, -0.970941817426052, -0.9709418174260521, -0.7485107481711013, -0.3546048870425359, 0.1205366802553232, 0.5680647467311548, 0.88545602565321};
    static constexpr double s[13] = {0.0, 0.4647231720437685, 0.8229838658936564, 0.992708874098054, 0.9350162426854148, 0.6631226582407952, 0.23931566428755768, -0.23931566428755743, -0.663122658240795, -0.9350162426854147, -0.992708874098054, -0.822983865893657, -0.4647231720437684};
};
template <> struct PrimeTab<29> {
    static constexpr double c[29] = {1.0, 0.9766205557100867, 0.907575419670957, 0.7960930657056438, 0.6473862847818277, 0.46840844069979015, 0.26752833852922075, 0.05413890858541761, -0.16178199655276473, -0.37013815533991423, -0.5611870653623823, -0.7259954919231306, -0.8568571761675893, -0.9476531711828025, -0.9941379571543596, -0.9941379571543597, -0.9476531711828025, -0.8568571761675892, -0.7259954919231311, -0.5611870653623825, -0.37013815533991445, -0.16178199655276476, 0.0541389085854167, 0.2675283385292201, 0.4684084406997903, 0.6473862847818279, 0.796093065705644, 0.9075754196709569, 0.9766205557100867};
    static constexpr double s[29] = {0.0, 0.21497044021102407, 0.4198891015602646, 0.6051742151937652, 0.7621620551276365, 0.8835120444460229, 0.963549992519223, 0.9985334138511238, 0.9868265225415261, 0.9289767198167915, 0.8276889981568906, 0.6876994588534235, 0.5155538571770216, 0.3193015301359798, 0.10811901842394192, -0.10811901842394124, -0.31930153013597995, -0.5155538571770218, -0.6876994588534231, -0.8276889981568905, -0.9289767198167914, -0.9868265225415261, -0.9985334138511239, -0.9635499925192231, -0.8835120444460228, -0.7621620551276362, -0.6051742151937649, -0.41988910156026493, -0.21497044021102438};
};

template <class V> struct RealOf;
template <> struct RealOf<float2> { using T = float; };
template <> struct RealOf<double2> { using T = double; };
template <class V> using Re = typename RealOf<V>::T;

template <class V> __device__ __forceinline__ V mk(Re<V> x, Re<V> y)
{
    V r;
    r.x = x;
    r.y = y;
    return r;
}
// a*b + cd (cd = c*d rounded): the fused product fixed, whatever the schedule
__device__ __forceinline__ float fma2(float a, float b, float cd) { return __builtin_fmaf(a, b, cd); }
__device__ __forceinline__ double fma2(double a, double b, double cd) { return __builtin_fma(a, b, cd); }
template <class V> __device__ __forceinline__ V cadd(V a, V b) { return mk<V>(a.x + b.x, a.y + b.y); }
template <class V> __device__ __forceinline__ V csub(V a, V b) { return mk<V>(a.x - b.x, a.y - b.y); }
template <class V> __device__ __forceinline__ V cmul(V a, V b)
{
    return mk<V>(fma2(a.x, b.x, -(a.y * b.y)), fma2(a.x, b.y, a.y * b.x));
}
template <class V> __device__ __forceinline__ V cmulc(V a, V b)  // a * conj(b)
{
    return mk<V>(fma2(a.x, b.x, a.y * b.y), fma2(a.y, b.x, -(a.x * b.y)));
}
// multiply by -j (DIR = -1, forward) or +j (DIR = +1, inverse)
template <int DIR, class V> __device__ __forceinline__ V mul_dj(V a)
{
    return DIR < 0 ? mk<V>(a.y, -a.x) : mk<V>(-a.y, a.x);
}
// multiply by tw (forward) or conj(tw) (inverse); tables hold e^{-j...}
template <int DIR, class V> __device__ __forceinline__ V twid(V a, V tw)
{
    return DIR < 0 ? cmul(a, tw) : cmulc(a, tw);
}

// ---- small DFTs in registers; DIR = -1: X[k] = sum x[n] e^{-j2pi nk/N}, +1: e^{+j..}
template <int DIR, class V> __device__ __forceinline__ void dft4(V& a, V& b, V& c, V& d)
{
    const V t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = mul_dj<DIR>(csub(b, d));
    a = cadd(t0, t2);
    c = csub(t0, t2);
    b = cadd(t1, t3);
    d = csub(t1, t3);
}

template <int DIR, class V> __device__ __forceinline__ void dft5(V (&v)[5])
{
    using R = Re<V>;
    constexpr R c1 = (R)0.30901699437494745, c2 = (R)-0.8090169943749475;  // cos(2pi/5), cos(4pi/5)
    constexpr R s1 = (R)0.9510565162951535, s2 = (R)0.5877852522924731;    // sin(2pi/5), sin(4pi/5)
    const V t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]);
    const V t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
    const V b1 = mk<V>(v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y);
    const V b2 = mk<V>(v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y);
    const V e1 = mul_dj<DIR>(mk<V>(fma2(s1, t3.x, s2 * t4.x), fma2(s1, t3.y, s2 * t4.y)));
    const V e2 = mul_dj<DIR>(mk<V>(fma2(s2, t3.x, -(s1 * t4.x)), fma2(s2, t3.y, -(s1 * t4.y))));
    v[0] = mk<V>(v[0].x + t1.x + t2.x, v[0].y + t1.y + t2.y);
    v[1] = cadd(b1, e1);
    v[4] = csub(b1, e1);
    v[2] = cadd(b2, e2);
    v[3] = csub(b2, e2);
}

// 10 = 2 x 5: even/odd 5-point DFTs and one radix-2 combine
template <int DIR, class V> __device__ __forceinline__ void dft10(V (&v)[10])
{
    using R = Re<V>;
    constexpr R c[5] = {(R)1.0, (R)0.8090169943749475, (R)0.30901699437494745, (R)-0.30901699437494745,
                        (R)-0.8090169943749475};  // cos(2 pi k/10)
    constexpr R s[5] = {(R)0.0, (R)0.5877852522924731, (R)0.9510565162951535, (R)0.9510565162951535,
                        (R)0.5877852522924731};   // sin(2 pi k/10)
    V e[5] = {v[0], v[2], v[4], v[6], v[8]}, o[5] = {v[1], v[3], v[5], v[7], v[9]};
    dft5<DIR>(e);
    dft5<DIR>(o);
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const V t = cmul(o[k], mk<V>(c[k], DIR < 0 ? -s[k] : s[k]));
        v[k] = cadd(e[k], t);
        v[k + 5] = csub(e[k], t);
    }
}

constexpr double kC16 = 0.9238795325112867, kS16 = 0.3826834323650898, kR2 = 0.7071067811865476;
constexpr double kTc16[10] = {1., kC16, kR2, kS16, 0., -kS16, -kR2, -kC16, -1., -kC16};  // cos(2 pi m/16)
constexpr double kTs16[10] = {0., kS16, kR2, kC16, 1., kC16, kR2, kS16, 0., -kS16};    // sin(2 pi m/16)

// 16 = 4 x 4: x index n = 4*n1 + n2, output k = k1 + 4*k2, natural order in v
template <int DIR, class V> __device__ __forceinline__ void dft16(V (&v)[16])
{
    using R = Re<V>;
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) dft4<DIR>(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
    // y[n2][k1] sits in v[4*k1 + n2]; twiddle w16^(n2*k1)
#pragma unroll
    for (int k1 = 1; k1 < 4; k1++)
#pragma unroll
        for (int n2 = 1; n2 < 4; n2++) {
            const int m = n2 * k1;  // <= 9
            const V w = mk<V>((R)kTc16[m], DIR < 0 ? (R)-kTs16[m] : (R)kTs16[m]);
            v[4 * k1 + n2] = cmul(v[4 * k1 + n2], w);
        }
    V o[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) {
        V a = v[4 * k1], b = v[4 * k1 + 1], c = v[4 * k1 + 2], d = v[4 * k1 + 3];
        dft4<DIR>(a, b, c, d);
        o[k1] = a; o[k1 + 4] = b; o[k1 + 8] = c; o[k1 + 12] = d;
    }
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = o[i];
}

// P-point DFT (P odd prime) by conjugate-pair symmetry: 4*((P-1)/2)^2 FMAs. The pairs
// a_n = x_n + x_{P-n}, d_n = x_n - x_{P-n} overwrite v; outputs go through `put(k, X_k)`.
template <int P, int DIR, class V, class Put>
__device__ __forceinline__ void dft_prime(V (&v)[P], Put put)
{
    using R = Re<V>;
    constexpr int H = (P - 1) / 2;
    using T = PrimeTab<P>;
    const V x0 = v[0];
    V sum = x0;
#pragma unroll
    for (int n = 1; n <= H; n++) {
        const V a = cadd(v[n], v[P - n]), d = csub(v[n], v[P - n]);
        v[n] = a;
        v[P - n] = d;
        sum = cadd(sum, a);
    }
    put(0, sum);
#pragma unroll
    for (int k = 1; k <= H; k++) {
        R re = x0.x, im = x0.y, sr = 0, si = 0;
#pragma unroll
        for (int n = 1; n <= H; n++) {
            const int m = (n * k) % P;
            re += v[n].x * (R)T::c[m];
            im += v[n].y * (R)T::c[m];
            sr += v[P - n].y * (R)T::s[m];
            si += v[P - n].x * (R)T::s[m];
        }
        // sum_n d_n * (-+ j sin): forward (e^{-j}) adds (+sr, -si)
        if (DIR < 0) {
            put(k, mk<V>(re + sr, im - si));
            put(P - k, mk<V>(re - sr, im + si));
        } else {
            put(k, mk<V>(re - sr, im + si));
            put(P - k, mk<V>(re + sr, im - si));
        }
    }
}

// ---- 2000-point Stockham in LDS (one buffer: every stage reads to registers, syncs,
// writes): radices 5, 5, 5, 16 (Ns = 1, 5, 25, 125), natural order at the end.
// tw[m] = e^{-j 2 pi m / 2000}. Callers sync after filling `a`.
template <int DIR, int NS, class V, class TW>
__device__ __forceinline__ void stage5(V* a, const TW& tw, int tid)
{
    constexpr int NB = kRow / 5, PER = (NB + kRowThreads - 1) / kRowThreads;
    V v[PER][5];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int j0 = tid + q * kRowThreads, j = j0 < NB ? j0 : NB - 1;
        const int k = j % NS;
#pragma unroll
        for (int i = 0; i < 5; i++) v[q][i] = a[j + i * NB];
        if (NS > 1) {
#pragma unroll
            for (int i = 1; i < 5; i++) v[q][i] = twid<DIR>(v[q][i], tw[i * k * (kRow / (NS * 5))]);
        }
        dft5<DIR>(v[q]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int j = tid + q * kRowThreads;
        if (j < NB) {
            const int k = j % NS, d = (j / NS) * NS * 5 + k;
#pragma unroll
            for (int i = 0; i < 5; i++) a[d + i * NS] = v[q][i];
        }
    }
    __syncthreads();
}

template <int DIR, class V, class TW>
__device__ __forceinline__ void fft2000(V* a, const TW& tw, int tid)
{
    stage5<DIR, 1>(a, tw, tid);
    stage5<DIR, 5>(a, tw, tid);
    stage5<DIR, 25>(a, tw, tid);
    constexpr int NB = kRow / 16;  // radix 16, Ns = 125: k = j
    const int j = tid < NB ? tid : NB - 1;
    V v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = a[j + i * NB];
#pragma unroll
    for (int i = 1; i < 16; i++) v[i] = twid<DIR>(v[i], tw[i * j]);
    dft16<DIR>(v);
    __syncthreads();
    if (tid < NB) {
#pragma unroll
        for (int i = 0; i < 16; i++) a[tid + i * NB] = v[i];
    }
    __syncthreads();
}

// 20 = 5 x 4: x index n = 4*n1 + n2, output k = k1 + 5*k2 (natural order in v)
constexpr double kTc20[13] = {1., 0.9510565162951535, 0.8090169943749475, 0.5877852522924731,
                              0.30901699437494745, 0., -0.30901699437494745, -0.5877852522924731,
                              -0.8090169943749475, -0.9510565162951535, -1., -0.9510565162951535,
                              -0.8090169943749475};  // cos(2 pi m/20)
constexpr double kTs20[13] = {0., 0.30901699437494745, 0.5877852522924731, 0.8090169943749475,
                              0.9510565162951535, 1., 0.9510565162951535, 0.8090169943749475,
                              0.5877852522924731, 0.30901699437494745, 0., -0.30901699437494745,
                              -0.5877852522924731};  // sin(2 pi m/20)
template <int DIR, class V> __device__ __forceinline__ void dft20(V (&v)[20])
{
    using R = Re<V>;
    V y[4][5];  // y[n2][k1] = DFT_5 over n1 of x[4*n1 + n2]
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) {
#pragma unroll
        for (int n1 = 0; n1 < 5; n1++) y[n2][n1] = v[4 * n1 + n2];
        dft5<DIR>(y[n2]);
    }
#pragma unroll
    for (int n2 = 1; n2 < 4; n2++)
#pragma unroll
        for (int k1 = 1; k1 < 5; k1++) {
            const int m = n2 * k1;  // <= 12
            y[n2][k1] = cmul(y[n2][k1], mk<V>((R)kTc20[m], DIR < 0 ? (R)-kTs20[m] : (R)kTs20[m]));
        }
#pragma unroll
    for (int k1 = 0; k1 < 5; k1++) {
        V a = y[0][k1], b = y[1][k1], c = y[2][k1], d = y[3][k1];
        dft4<DIR>(a, b, c, d);
        v[k1] = a; v[k1 + 5] = b; v[k1 + 10] = c; v[k1 + 15] = d;
    }
}

template <int R, int DIR, class V> __device__ __forceinline__ void dft_r(V (&v)[R])
{
    if constexpr (R == 5) dft5<DIR>(v);
    else if constexpr (R == 10) dft10<DIR>(v);
    else if constexpr (R == 16) dft16<DIR>(v);
    else dft20<DIR>(v);
}

// Twiddles of the radix-20-first row transforms' two twiddled stages, laid out so a stage's
// lanes read consecutive entries (a lane j of the Ns = 20 stage reads w^(10*i*(j mod 20)),
// of the Ns = 200 stage w^(i*j): from the plain 2000-entry table that is a gather at a lane
// stride of 10*i or i entries, up to 16-way LDS bank conflicts): t2[(i-1)*20 + k] =
// w^(10*i*k), t3[(i-1)*200 + k] = w^(i*k), 1 980 entries, the same values. A plain pointer is
// the 2000-entry table itself.
template <class V> struct TwIK {
    const V* t2;
    const V* t3;
};
template <int NS, class V>
__device__ __forceinline__ V tw_get(const V* tw, int, int, int m) { return tw[m]; }
template <int NS, class V>
__device__ __forceinline__ V tw_get(const TwIK<V>& tw, int i, int k, int m)
{
    static_assert(NS == 20 || NS == 200, "split twiddles: the radix-20-first stages");
    return NS == 20 ? tw.t2[(i - 1) * 20 + k] : tw.t3[(i - 1) * 200 + k];
}
constexpr int kTwIK = 9 * 20 + 9 * 200;  // entries of the split layout
// (every load of the block's prologue issued before the first LDS store: a loop of load ->
// wait -> store paid one L2 round trip per iteration, 8 per table, GNSS_STAGED_LOADS 0)
#ifndef GNSS_STAGED_LOADS
#define GNSS_STAGED_LOADS 1
#endif
template <class V>
__device__ __forceinline__ TwIK<V> load_row_tw_ik(V* s_t, const V* tw_row, int tid)
{
    auto src = [&](int e) {
        const bool t2 = e < 9 * 20;
        const int f = t2 ? e : e - 9 * 20;
        const int i = t2 ? f / 20 + 1 : f / 200 + 1, k = t2 ? f % 20 : f % 200;
        return t2 ? 10 * i * k : i * k;
    };
    if constexpr (GNSS_STAGED_LOADS) {
        constexpr int NIT = (kTwIK + kRowThreads - 1) / kRowThreads;
        V r[NIT];
#pragma unroll
        for (int q = 0; q < NIT; q++) {
            const int e0 = tid + q * kRowThreads;
            r[q] = tw_row[src(e0 < kTwIK ? e0 : kTwIK - 1)];
        }
#pragma unroll
        for (int q = 0; q < NIT; q++)
            if (tid + q * kRowThreads < kTwIK) s_t[tid + q * kRowThreads] = r[q];
    } else {
        for (int e = tid; e < kTwIK; e += kRowThreads) s_t[e] = tw_row[src(e)];
    }
    return TwIK<V>{s_t, s_t + 9 * 20};
}

// ---- BATCH 2000-point transforms side by side in LDS (transform b at a + b*2000), one
// radix-R Stockham stage; every butterfly of the batch is spread over the block's threads.
// SW = 1 (the Ns = 1 radix-20 stage of a single transform): outputs stored padded, element
// 20*j + i at 21*j + i, so the 16 lanes of an LDS cycle hit 16 different 16-B bank slots
// (the plain order's 320-B lane stride put 4 lanes on each: 35 % of the fp64 row pass's LDS
// cycles were conflicts, profiles/r02_acq_counters.json; 140 store cycles per transform
// instead of 500 by the 16-lane model); SW = 2: the stage after it, reading that layout,
// element x = j' + 200*i at (j' + j'/20) + 210*i (one division per thread, none per element).
// The buffer holds kRowPad elements.
template <int DIR, int R, int NS, int BATCH, class V, class TW, int SW = 0>
__device__ __forceinline__ void stage_batch(V* a, const TW& tw, int tid)
{
    constexpr int NB = kRow / R, TOT = NB * BATCH, PER = (TOT + kRowThreads - 1) / kRowThreads;
    static_assert(SW == 0 || (BATCH == 1 && ((SW == 1 && R == 20 && NS == 1) || (SW == 2 && R == 10 && NS == 20))),
                  "padded layout");
    V v[PER][R];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int u0 = tid + q * kRowThreads, u = u0 < TOT ? u0 : TOT - 1;
        const int b = u / NB, j = u - b * NB, k = j % NS;
        const V* src = a + b * kRow;
        if constexpr (SW == 2) {
            const V* s0 = src + j + j / 20;
#pragma unroll
            for (int i = 0; i < R; i++) v[q][i] = s0[210 * i];
        } else {
#pragma unroll
            for (int i = 0; i < R; i++) v[q][i] = src[j + i * NB];
        }
        if constexpr (NS > 1) {
#pragma unroll
            for (int i = 1; i < R; i++) v[q][i] = twid<DIR>(v[q][i], tw_get<NS>(tw, i, k, i * k * (kRow / (NS * R))));
        }
        dft_r<R, DIR>(v[q]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int u = tid + q * kRowThreads;
        if (u < TOT) {
            const int b = u / NB, j = u - b * NB, k = j % NS, d = (j / NS) * NS * R + k;
            V* dst = a + b * kRow;
            if constexpr (SW == 1) {
#pragma unroll
                for (int i = 0; i < R; i++) dst[d + j + i] = v[q][i];
            } else {
#pragma unroll
                for (int i = 0; i < R; i++) dst[d + i * NS] = v[q][i];
            }
        }
    }
    __syncthreads();
}

// 2000 = 10 x 10 x 20: three LDS passes per batch of transforms (natural order at the end).
template <int DIR, int BATCH, class V, class TW>
__device__ __forceinline__ void fft2000_batch(V* a, const TW& tw, int tid)
{
    stage_batch<DIR, 10, 1, BATCH>(a, tw, tid);
    stage_batch<DIR, 10, 10, BATCH>(a, tw, tid);
    stage_batch<DIR, 20, 100, BATCH>(a, tw, tid);
}

// 2000 = 20 x 10 x 10 with the radix-20 pass first (Ns = 1: no twiddles), so the widest
// butterfly never holds twiddles in registers (the fp64 row kernels stay within 256 VGPRs);
// one transform in `a` (kRowPad elements: its first stage's outputs padded, SW above). The
// last stage's outputs go to put(i, t, value), not back to LDS: thread j < 200 computes
// outputs t = j + 200*i (i < 10) and the caller consumes them from registers (one LDS
// write and read of the row and a barrier less per transform). Ends with a barrier (the
// caller may rewrite `a`).
constexpr int kR20Out = 10;  // outputs per thread of the last radix-10 stage
template <int DIR, class V, class TW, class Put>
__device__ __forceinline__ void fft2000_r20first_put(V* a, const TW& tw, int tid, Put put)
{
    stage_batch<DIR, 20, 1, 1, V, TW, 1>(a, tw, tid);
    stage_batch<DIR, 10, 20, 1, V, TW, 2>(a, tw, tid);
    constexpr int R = 10, NB = kRow / R;  // NS = 200: k = j, outputs at j + 200*i
    const bool on = tid < NB;
    const int j = on ? tid : NB - 1;
    V v[R];
#pragma unroll
    for (int i = 0; i < R; i++) v[i] = a[j + i * NB];
#pragma unroll
    for (int i = 1; i < R; i++) v[i] = twid<DIR>(v[i], tw_get<NB>(tw, i, j, i * j));
    dft10<DIR>(v);
    if (on) {
#pragma unroll
        for (int i = 0; i < R; i++) put(i, j + i * NB, v[i]);
    }
    __syncthreads();
}

// The fp64 correlator's inverse row transform with |.|^2 / S^2 accumulated per output in
// registers: acc[i] of thread j < 200 is output j + 200*i, summed over the ms in order
// (acquisition.m:53-61).
constexpr int kInvOut = kR20Out;
template <class TW>
__device__ __forceinline__ void inv_row_power_f64(double2* a, const TW& s_tw, double scale,
                                                  double (&acc)[kInvOut], int tid)
{
    fft2000_r20first_put<1>(a, s_tw, tid, [&](int i, int, double2 v) {
        acc[i] = __builtin_fma(__builtin_fma(v.x, v.x, v.y * v.y), scale, acc[i]);
    });
}

// a value read once (the column pass's intermediate): non-temporal load
__device__ __forceinline__ double2 ld_nt(const double2* p)
{
    double2 v;
    v.x = __builtin_nontemporal_load(&p->x);
    v.y = __builtin_nontemporal_load(&p->y);
    return v;
}

template <class V>
__device__ __forceinline__ void load_row_tw(V* s_tw, const V* tw_row, int tid)
{
    for (int i = tid; i < kRow; i += kRowThreads) s_tw[i] = tw_row[i];
}

// ============================== correlator ========================================
// V = float2: the fast fp32 mode; V = double2: the reference's precision (acquisition.m's
// MATLAB FFTs are fp64), every product, transform and power sum in fp64.

// ---- F1: forward rows. Transform s < nsig: rawsignal(ms) .* carrier(bin) (acquisition.m:41-44,56);
// s >= nsig: the code replica of PRN s - nsig (acquisition.m:49-51). Row n2 holds
// x[P*n1 + n2]; output B[s][n2][k1] * w_S^(-n2*k1).
// The forward transforms of one launch: the nprn code transforms first when `codes`, then the
// signal transforms of bins [bin0, bin0 + nbc) of every ms (the whole pass: bin0 = 0, nbc = nbins);
// launch-local index y -> transform s (s = ms * nbins + bin for signals, nsig + p for codes).
struct FwdSet {
    int nbins, nsig, nprn, bin0, nbc, codes;
    __device__ __forceinline__ int transform(int y) const
    {
        if (codes && y < nprn) return nsig + y;
        const int u = y - (codes ? nprn : 0), idx = u / nbc;
        return idx * nbins + bin0 + (u - idx * nbc);
    }
};

template <int P, class Src, class V>
__global__ __launch_bounds__(kRowThreads) void fwd_rows_kernel(
    const Src src, FwdSet fs, double IF, double freqMin, double freqStep,
    double Fs, const float* __restrict__ ca, double code_step, const V* __restrict__ tw_row,
    const V* __restrict__ tw_col, V* __restrict__ B)
{
    using R = Re<V>;
    constexpr int64_t S = (int64_t)P * kRow;
    __shared__ V s_a[kRowPad], s_tw[kTwIK];
    const int nbins = fs.nbins, nsig = fs.nsig;
    const int n2 = blockIdx.x, s = fs.transform(blockIdx.y), tid = threadIdx.x;
    const TwIK<V> twk = load_row_tw_ik(s_tw, tw_row, tid);
    constexpr int NIT = (kRow + kRowThreads - 1) / kRowThreads;
    if (s < nsig) {
        const int idx = s / nbins, bin = s - idx * nbins;
        const double f = (IF + (freqMin + freqStep * (double)bin)) / Fs;  // cycles per sample
        auto put = [&](int n1, double2 r) {
            const int64_t n = (int64_t)P * n1 + n2;
            double cyc = f * (double)(n + 1);  // n is 1-based in the reference
            cyc -= floor(cyc);
            R c, sn;
            if constexpr (sizeof(R) == 4) {
                const float ph = (float)cyc;
                c = __builtin_amdgcn_cosf(ph);
                sn = __builtin_amdgcn_sinf(ph);
            } else {
                sincospi(2.0 * cyc, &sn, &c);
            }
            const R xr = (R)r.x, xi = (R)r.y;
            s_a[n1] = mk<V>(fma2(xr, c, -(xi * sn)), fma2(xr, sn, xi * c));
        };
        if constexpr (GNSS_STAGED_LOADS) {
            double2 raw[NIT];
#pragma unroll
            for (int q = 0; q < NIT; q++) {
                const int m0 = tid + q * kRowThreads, n1 = m0 < kRow ? m0 : kRow - 1;
                raw[q] = src.at((int64_t)idx * S + (int64_t)P * n1 + n2);
            }
#pragma unroll
            for (int q = 0; q < NIT; q++)
                if (tid + q * kRowThreads < kRow) put(tid + q * kRowThreads, raw[q]);
        } else {
            for (int n1 = tid; n1 < kRow; n1 += kRowThreads) put(n1, src.at((int64_t)idx * S + (int64_t)P * n1 + n2));
        }
    } else {
        const float* cp = ca + (int64_t)(s - nsig) * 1023;
        auto chip = [&](int n1) {
            const int64_t n = (int64_t)P * n1 + n2;
            const int64_t ci = (int64_t)ceil((double)(n + 1) * code_step);  // 1-based into [CA CA]
            return (ci - 1) % 1023;
        };
        if constexpr (GNSS_STAGED_LOADS) {
            float cv[NIT];
#pragma unroll
            for (int q = 0; q < NIT; q++) {
                const int m0 = tid + q * kRowThreads;
                cv[q] = cp[chip(m0 < kRow ? m0 : kRow - 1)];
            }
#pragma unroll
            for (int q = 0; q < NIT; q++)
                if (tid + q * kRowThreads < kRow) s_a[tid + q * kRowThreads] = mk<V>((R)cv[q], (R)0);
        } else {
            for (int n1 = tid; n1 < kRow; n1 += kRowThreads) s_a[n1] = mk<V>((R)cp[chip(n1)], (R)0);
        }
    }
    __syncthreads();
    V* o = B + ((int64_t)s * P + n2) * kRow;
    const V* twc = tw_col + (int64_t)n2 * kRow;
    fft2000_r20first_put<-1>(s_a, twk, tid, [&](int, int k1, V v) { o[k1] = cmul(v, twc[k1]); });
}

// ---- F2: forward columns: X[s][k1 + 2000*k2] = DFT_P over n2 of B[s][n2][k1]
template <int P, class V>
__global__ __launch_bounds__(kColThreads) void fwd_cols_kernel(FwdSet fs, const V* __restrict__ B, V* __restrict__ X)
{
    const int k1 = blockIdx.x * kColThreads + threadIdx.x, s = fs.transform(blockIdx.y);
    if (k1 >= kRow) return;
    const V* b = B + (int64_t)s * P * kRow + k1;
    V v[P];
#pragma unroll
    for (int i = 0; i < P; i++) v[i] = b[(int64_t)i * kRow];
    V* x = X + (int64_t)s * P * kRow + k1;
    dft_prime<P, -1>(v, [&](int k, V y) { x[(int64_t)k * kRow] = y; });
}

// ---- I1: inverse columns of Z = C_p .* conj(X_{ms,bin}) for transform t = (pair, ms)
// of this batch; pair q = first_pair + t / datalen -> bin = q / nprn, p = q % nprn.
// one V (complex fp64 / fp32) by a raw buffer load
template <class V> __device__ __forceinline__ V buf_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff);
template <> __device__ __forceinline__ double2 buf_ld<double2>(__amdgpu_buffer_rsrc_t r, int voff, int soff)
{
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
    return make_double2(__hiloint2double((int)v.y, (int)v.x), __hiloint2double((int)v.w, (int)v.z));
}
template <> __device__ __forceinline__ float2 buf_ld<float2>(__amdgpu_buffer_rsrc_t r, int voff, int soff)
{
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    const u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
}
#ifndef GNSS_COLS_BUF
#define GNSS_COLS_BUF 1  // (A/B: 0 = the column pass's plain loads)
#endif
#ifndef GNSS_COLS_GROUP
#define GNSS_COLS_GROUP 8  // (A/B: signal-spectrum rows per load group of the column pass)
#endif
#ifndef GNSS_TW_ROWS
#define GNSS_TW_ROWS 1  // (A/B: 0 = the column pass multiplies by the four-step twiddle)
#endif
#ifndef GNSS_INVCOLS_WPE
#define GNSS_INVCOLS_WPE 0  // (A/B: waves per EU asked of inv_cols; 0 = the compiler's choice)
#endif
// (the body takes its block coordinates: inv_cols_kernel and the paired launch run it)
template <int P, class V>
__device__ __forceinline__ void inv_cols_body(
    int bx, int t, const V* __restrict__ C, const V* __restrict__ X, int nbins, int nprn, int datalen,
    int first_pair, const V* __restrict__ tw_col, V* __restrict__ A)
{
    const int k1 = bx * kColThreads + threadIdx.x;
    if (k1 >= kRow) return;
    const int q = first_pair + t / datalen, idx = t % datalen;
    const int bin = q / nprn, p = q - bin * nprn;
    V v[P];
    if (GNSS_COLS_BUF == 2) {
        // (A/B) code and signal rows loaded together, G rows at a time with the next G in
        // flight: fewer registers held than all code rows first
        constexpr int kB = P * kRow * (int)sizeof(V), G = GNSS_COLS_GROUP;
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(C + (int64_t)p * P * kRow), (short)0, kB, 0x00020000);
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(X + ((int64_t)idx * nbins + bin) * P * kRow), (short)0, kB, 0x00020000);
        const int vo = k1 * (int)sizeof(V);
        V ca[G], xa[G];
#pragma unroll
        for (int i = 0; i < G; i++) {
            const int r = (i < P ? i : P - 1) * kRow * (int)sizeof(V);
            ca[i] = buf_ld<V>(rc, vo, r);
            xa[i] = buf_ld<V>(rx, vo, r);
        }
#pragma unroll
        for (int g = 0; g < P; g += G) {
            V cb[G], xb[G];
#pragma unroll
            for (int i = 0; i < G; i++)
                if (g + G + i < P) {
                    cb[i] = buf_ld<V>(rc, vo, (g + G + i) * kRow * (int)sizeof(V));
                    xb[i] = buf_ld<V>(rx, vo, (g + G + i) * kRow * (int)sizeof(V));
                }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < G; i++)
                if (g + i < P) v[g + i] = cmulc(ca[i], xa[i]);
#pragma unroll
            for (int i = 0; i < G; i++) { ca[i] = cb[i]; xa[i] = xb[i]; }
        }
    } else if (GNSS_COLS_BUF) {
        // buffer loads (row offsets in SGPRs: no per-load 64-bit address arithmetic), every
        // code-spectrum value first, then the signal spectrum 8 rows at a time with the next 8
        // in flight: the lane waits for L2 about 4 times, not once per row as the compiler's
        // interleaved schedule did
        constexpr int kB = P * kRow * (int)sizeof(V), G = GNSS_COLS_GROUP;
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(C + (int64_t)p * P * kRow), (short)0, kB, 0x00020000);
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(X + ((int64_t)idx * nbins + bin) * P * kRow), (short)0, kB, 0x00020000);
        const int vo = k1 * (int)sizeof(V);
#pragma unroll
        for (int i = 0; i < P; i++) v[i] = buf_ld<V>(rc, vo, i * kRow * (int)sizeof(V));
        V xa[G];
#pragma unroll
        for (int i = 0; i < G; i++) xa[i] = buf_ld<V>(rx, vo, (i < P ? i : P - 1) * kRow * (int)sizeof(V));
#pragma unroll
        for (int g = 0; g < P; g += G) {
            V xb[G];
#pragma unroll
            for (int i = 0; i < G; i++)
                if (g + G + i < P) xb[i] = buf_ld<V>(rx, vo, (g + G + i) * kRow * (int)sizeof(V));
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < G; i++)
                if (g + i < P) v[g + i] = cmulc(v[g + i], xa[i]);
#pragma unroll
            for (int i = 0; i < G; i++) xa[i] = xb[i];
        }
    } else {
        const V* c = C + (int64_t)p * P * kRow + k1;
        const V* x = X + ((int64_t)idx * nbins + bin) * P * kRow + k1;
#pragma unroll
        for (int i = 0; i < P; i++) v[i] = cmulc(c[(int64_t)i * kRow], x[(int64_t)i * kRow]);
    }
    V* a = A + (int64_t)t * P * kRow + k1;
    const V* tw = tw_col + k1;
    // A is streamed once (to the row pass): non-temporal stores keep C and X in the caches.
    // GNSS_TW_ROWS: the four-step twiddle w^(k1 k2) is applied by the row pass as it loads
    // the row (the same product of the same operands: same bits), so this pass issues no
    // load after its first store -- on gfx9 a load's vmcnt wait also waits for every store
    // issued before it, and the twiddle reads between the stores serialised them.
    dft_prime<P, 1>(v, [&](int k, V y) {
        const V z = GNSS_TW_ROWS ? y : cmulc(y, tw[(int64_t)k * kRow]);
        __builtin_nontemporal_store(z.x, &a[(int64_t)k * kRow].x);
        __builtin_nontemporal_store(z.y, &a[(int64_t)k * kRow].y);
    });
}

template <int P, class V>
__global__ __launch_bounds__(kColThreads)
#if GNSS_INVCOLS_WPE > 0
__attribute__((amdgpu_waves_per_eu(GNSS_INVCOLS_WPE, GNSS_INVCOLS_WPE)))
#endif
void inv_cols_kernel(
    const V* __restrict__ C, const V* __restrict__ X, int nbins, int nprn, int datalen,
    int first_pair, const V* __restrict__ tw_col, V* __restrict__ A)
{
    inv_cols_body<P, V>(blockIdx.x, blockIdx.y, C, X, nbins, nprn, datalen, first_pair, tw_col, A);
}

// ---- I2: inverse rows, |.|^2/S^2 summed over the ms in order, stored tau2-major. Two
// ms per pass (their 2000-point transforms side by side, fft2000_batch): half the
// barriers per transform, every lane busy in the radix-20 pass.
template <int P>
__global__ __launch_bounds__(kRowThreads) void inv_rows_kernel(
    const float2* __restrict__ A, int nprn, int datalen, int first_pair, float scale,
    const float2* __restrict__ tw_row, const float2* __restrict__ tw_col, float* __restrict__ corr, int nbins)
{
    constexpr int Q = (kRow + kRowThreads - 1) / kRowThreads;
    constexpr int V4 = kRow / 2;  // float4 = two complex
    constexpr int QV = (V4 + kRowThreads - 1) / kRowThreads;
    static_assert(QV == 4, "row copy is written for 4 float4 per lane");
    __shared__ float4 s_a4[2 * V4];
    __shared__ float2 s_tw[kRow];
    float2* s_a = reinterpret_cast<float2*>(s_a4);
    const int tau2 = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
    load_row_tw(s_tw, tw_row, tid);
    float acc[Q];
#pragma unroll
    for (int i = 0; i < Q; i++) acc[i] = 0.f;
    const float4* src = reinterpret_cast<const float4*>(A + ((int64_t)g * datalen * P + tau2) * kRow);
    // row `idx` (clamped to the last ms: an odd datalen's spare transform is not summed);
    // named registers (an array here ends up in scratch)
    auto ld = [&](int idx, int i) {
        const int e = tid + i * kRowThreads;
        const int r = idx < datalen ? idx : datalen - 1;
        const float4* q = src + (int64_t)r * P * V4 + (e < V4 ? e : V4 - 1);
        float4 v;  // (read once: non-temporal)
        v.x = __builtin_nontemporal_load(&q->x);
        v.y = __builtin_nontemporal_load(&q->y);
        v.z = __builtin_nontemporal_load(&q->z);
        v.w = __builtin_nontemporal_load(&q->w);
        return v;
    };
    // (GNSS_TW_ROWS) this row's four-step twiddles w^(tau2 k1), k1 = 2e, 2e + 1, held for every ms
    float4 tw4[QV];
#pragma unroll
    for (int i = 0; i < QV; i++) {
        const int e = tid + i * kRowThreads;
        tw4[i] = reinterpret_cast<const float4*>(tw_col + (int64_t)tau2 * kRow)[e < V4 ? e : V4 - 1];
    }
    auto st = [&](int h, int i, float4 v) {
        const int e = tid + i * kRowThreads;
        if (GNSS_TW_ROWS) {
            const float2 lo = cmulc(make_float2(v.x, v.y), make_float2(tw4[i].x, tw4[i].y));
            const float2 hi = cmulc(make_float2(v.z, v.w), make_float2(tw4[i].z, tw4[i].w));
            v = make_float4(lo.x, lo.y, hi.x, hi.y);
        }
        if (e < V4) s_a4[h * V4 + e] = v;
    };
    float4 a0 = ld(0, 0), a1 = ld(0, 1), a2 = ld(0, 2), a3 = ld(0, 3);
    float4 b0 = ld(1, 0), b1 = ld(1, 1), b2 = ld(1, 2), b3 = ld(1, 3);
    for (int idx = 0; idx < datalen; idx += 2) {
        st(0, 0, a0); st(0, 1, a1); st(0, 2, a2); st(0, 3, a3);
        st(1, 0, b0); st(1, 1, b1); st(1, 2, b2); st(1, 3, b3);
        if (idx + 2 < datalen) {  // prefetch the next two ms while these transform
            a0 = ld(idx + 2, 0); a1 = ld(idx + 2, 1); a2 = ld(idx + 2, 2); a3 = ld(idx + 2, 3);
            b0 = ld(idx + 3, 0); b1 = ld(idx + 3, 1); b2 = ld(idx + 3, 2); b3 = ld(idx + 3, 3);
        }
        __syncthreads();
        fft2000_batch<1, 2>(s_a, s_tw, tid);
        const bool second = idx + 1 < datalen;
#pragma unroll
        for (int i = 0; i < Q; i++) {  // the ms in order (acquisition.m:53-61)
            const int t1 = tid + i * kRowThreads, t = t1 < kRow ? t1 : kRow - 1;
            const float2 v = s_a[t], w = s_a[kRow + t];
            acc[i] += fma2(v.x, v.x, v.y * v.y) * scale;
            if (second) acc[i] += fma2(w.x, w.x, w.y * w.y) * scale;
        }
        __syncthreads();
    }
    const int q = first_pair + g;
    const int bin = q / nprn, p = q - bin * nprn;
    float* o = corr + (((int64_t)p * nbins + bin) * P + tau2) * kRow;
#pragma unroll
    for (int i = 0; i < Q; i++) {
        const int t1 = tid + i * kRowThreads;
        if (t1 < kRow) o[t1] = acc[i];
    }
}

// The fp64 inverse rows: the same sum order, one ms per pass (two fp64 rows and their
// table would take 96 KB of LDS), the next ms's row prefetched into registers while this
// one transforms, radices 10-10-20 (three LDS passes; 5-5-5-16: correlation 19.7 ->
// 18.5 ms at config 2). Measured and dropped: twiddles from the global table (634 -> 721
// us per batch); a 90-entry split table w^m = w^(m mod 50) w^(50 (m div 50)) (33 KB of
// LDS, twice the blocks per CU; the extra complex product per twiddle: 19.7 -> 29.0 ms);
// a padded layout x -> x + x/20 against the radix-20 pass's 2-way store conflicts (28 %
// of the LDS cycles by SQ_LDS_BANK_CONFLICT): 350 -> 481 us per launch (index divisions);
// radix 10-10-20 (conflict-free first pass, twiddles in the radix-20 pass): 350 -> 367 us.
template <int P>
__device__ __forceinline__ void inv_rows_f64_body(
    int tau2, int g, const double2* __restrict__ A, int nprn, int datalen, int first_pair, double scale,
    const double2* __restrict__ tw_row, const double2* __restrict__ tw_col, double* __restrict__ corr, int nbins)
{
    constexpr int Q = (kRow + kRowThreads - 1) / kRowThreads;
    __shared__ double2 s_a[kRowPad], s_tw[kTwIK];
    const int tid = threadIdx.x;
    const TwIK<double2> twk = load_row_tw_ik(s_tw, tw_row, tid);
    double acc[kInvOut];
#pragma unroll
    for (int i = 0; i < kInvOut; i++) acc[i] = 0.0;
    const double2* src = A + ((int64_t)g * datalen * P + tau2) * kRow;
    // the next ms's row in named registers (an indexed array here is kept in scratch)
    static_assert(Q == 8, "row prefetch is written for 8 values per lane");
    const int e7 = tid + 7 * kRowThreads < kRow ? tid + 7 * kRowThreads : kRow - 1;
    double2 n0, n1, n2, n3, n4, n5, n6, n7;
#define GNSS_LD(IDX)                                                                         \
    {                                                                                        \
        const double2* r = src + (int64_t)(IDX) * P * kRow + tid;                              \
        n0 = ld_nt(r); n1 = ld_nt(r + kRowThreads); n2 = ld_nt(r + 2 * kRowThreads);           \
        n3 = ld_nt(r + 3 * kRowThreads); n4 = ld_nt(r + 4 * kRowThreads);                      \
        n5 = ld_nt(r + 5 * kRowThreads); n6 = ld_nt(r + 6 * kRowThreads); n7 = ld_nt(r + e7 - tid); \
    }
    // (GNSS_TW_ROWS) this row's four-step twiddles w^(tau2 k1) for the lane's 8 elements, held
    // for every ms: the column pass's product cmulc(y, w), moved here
    double2 w0, w1, w2, w3, w4, w5, w6, w7;
    if (GNSS_TW_ROWS) {
        const double2* t = tw_col + (int64_t)tau2 * kRow + tid;
        w0 = t[0]; w1 = t[kRowThreads]; w2 = t[2 * kRowThreads]; w3 = t[3 * kRowThreads];
        w4 = t[4 * kRowThreads]; w5 = t[5 * kRowThreads]; w6 = t[6 * kRowThreads]; w7 = t[e7 - tid];
    }
    GNSS_LD(0)
    for (int idx = 0; idx < datalen; idx++) {
        if (GNSS_TW_ROWS) {
            n0 = cmulc(n0, w0); n1 = cmulc(n1, w1); n2 = cmulc(n2, w2); n3 = cmulc(n3, w3);
            n4 = cmulc(n4, w4); n5 = cmulc(n5, w5); n6 = cmulc(n6, w6); n7 = cmulc(n7, w7);
        }
        s_a[tid] = n0; s_a[tid + kRowThreads] = n1; s_a[tid + 2 * kRowThreads] = n2;
        s_a[tid + 3 * kRowThreads] = n3; s_a[tid + 4 * kRowThreads] = n4;
        s_a[tid + 5 * kRowThreads] = n5; s_a[tid + 6 * kRowThreads] = n6;
        if (tid + 7 * kRowThreads < kRow) s_a[tid + 7 * kRowThreads] = n7;
        if (idx + 1 < datalen) GNSS_LD(idx + 1)
#undef GNSS_LD
        __syncthreads();
        inv_row_power_f64(s_a, twk, scale, acc, tid);  // (ends with a barrier)
    }
    const int q = first_pair + g;
    const int bin = q / nprn, p = q - bin * nprn;
    double* o = corr + (((int64_t)p * nbins + bin) * P + tau2) * kRow;
    if (tid < kRow / kInvOut) {
#pragma unroll
        for (int i = 0; i < kInvOut; i++) o[tid + i * (kRow / kInvOut)] = acc[i];
    }
}

template <int P>
__global__ __launch_bounds__(kRowThreads) void inv_rows_kernel_f64(
    const double2* __restrict__ A, int nprn, int datalen, int first_pair, double scale,
    const double2* __restrict__ tw_row, const double2* __restrict__ tw_col, double* __restrict__ corr, int nbins)
{
    inv_rows_f64_body<P>(blockIdx.x, blockIdx.y, A, nprn, datalen, first_pair, scale, tw_row, tw_col, corr, nbins);
}

// ---- The two passes in one launch (fp64, GNSS_OPT_ACQ_PIPE 3): launch k holds the column
// pass of batch k and the row pass of batch k-1, their blocks interleaved in the grid, so a
// CU runs a column block (bound by the intermediate's streaming stores) beside a row block
// (bound by its fp64 LDS transforms) instead of two of a kind. Block i is a row block iff
// floor((i+1) nr / F) > floor(i nr / F) for i < F (F = front * grid / 100: the long row blocks
// are all dispatched in the grid's first `front` percent, none left for the launch's tail);
// its index is floor(i nr / F), a column block's is i minus the row blocks before it. Each
// block runs the plain kernels' body unchanged: the bits are the two-launch path's.
template <int P>
__global__ __launch_bounds__(kRowThreads) void inv_pair_kernel_f64(
    const double2* __restrict__ C, const double2* __restrict__ X, int nbins, int nprn, int datalen,
    int cols_first, int cols_n, double2* __restrict__ Acols, int rows_first, int rows_n,
    const double2* __restrict__ Arows, double scale, const double2* __restrict__ tw_row,
    const double2* __restrict__ tw_col, double* __restrict__ corr, int front)
{
    constexpr int kCx = (kRow + kColThreads - 1) / kColThreads;
    const int64_t nr = (int64_t)P * rows_n, T = nr + (int64_t)kCx * cols_n * datalen;
    const int64_t F = nr ? std::max<int64_t>(nr, T * front / 100) : 1;
    const int64_t i = blockIdx.x;
    const int64_t r0 = i < F ? i * nr / F : nr, r1 = i < F ? (i + 1) * nr / F : nr;
    if (r1 > r0) {
        const int g = (int)(r0 / P), tau2 = (int)(r0 - (int64_t)g * P);
        inv_rows_f64_body<P>(tau2, g, Arows, nprn, datalen, rows_first, scale, tw_row, tw_col, corr, nbins);
    } else {
        const int c = (int)(i - r0), t = c / kCx;
        inv_cols_body<P, double2>(c - t * kCx, t, C, X, nbins, nprn, datalen, cols_first, tw_col, Acols);
    }
}

// ---- I1 + I2 fused (fp64): one persistent launch, the intermediate kept in each XCD's L2.
// The two-kernel path streams every transform's P x 2000 intermediate A (928 KB at config 2)
// out to HBM and back, 2.2x the correlator's model bytes (profiles/acq_bound_r02.json). Here
// each XCD (read from HW_REG_XCC_ID, not assumed from blockIdx) runs its own pipeline over
// its share of the (bin, PRN) pairs, transform j = (pair, ms) of that share at a time:
//   column workers  I1 of transform j, one 256-column chunk per item, into ring slot j % R
//                   of the XCD's own region (plain stores: the lines stay in its L2);
//   row workers     one row tau2 each for the whole launch; per transform they copy
//                   their row out of the slot (L1-bypassing sc1 loads, served by the same
//                   L2), free the slot, and run I2 (2000-point inverse + |.|^2 sum over the
//                   ms in order).
// Hand-off inside one L2: every storing wave drains its stores (s_waitcnt vmcnt(0)) before
// the workgroup's counter add, and the reader polls the counter and then reads the bytes
// with loads that bypass its L1; producer and consumer are on the same XCD by construction
// (both read HW_REG_XCC_ID). The arithmetic is I1's and I2's, operation for operation: the
// surface equals the two-kernel path's bit for bit (tests/test_gpu_acquisition.py).
constexpr int kFuseX = 8;      // XCC_ID values
constexpr int kFuseSlots = 4;  // ring slots per XCD, at most
constexpr int kFuseLine = 32;  // counter stride (128 B: one counter per L2 line)
constexpr int kFuseChunks = (kRow + kColThreads - 1) / kColThreads;  // column items per transform
constexpr unsigned kFuseSpin = 1u << 22;  // polls (~1 us each, s_sleep'd) before giving up
struct FuseSync {
    unsigned arrive[kFuseX * kFuseLine];           // workgroups per XCC_ID
    unsigned total[kFuseLine];                     // all workgroups
    unsigned err[kFuseLine];                       // != 0: a wait timed out (the surface is void)
    unsigned ready[kFuseX * kFuseSlots * kFuseLine];  // column items stored, per (XCD, slot)
    unsigned freed[kFuseX * kFuseSlots * kFuseLine];  // row workers done copying, per (XCD, slot)
};

__device__ __forceinline__ unsigned ld_sc1(const unsigned* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add_dev(unsigned* p, unsigned v)
{
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane 0: poll until *p >= want (bounded); false on timeout (err set)
__device__ __forceinline__ bool wait_ge(const unsigned* p, unsigned want, FuseSync* sy)
{
    for (unsigned n = 0; n < kFuseSpin; n++) {
        if (ld_sc1(p) >= want) return true;
        if (ld_sc1(sy->err)) return false;
        __builtin_amdgcn_s_sleep(8);
    }
    add_dev(sy->err, 1u);
    return false;
}

template <int P>
__global__ __launch_bounds__(kRowThreads, 2) void inv_fused_kernel_f64(
    const double2* __restrict__ C, const double2* __restrict__ X, int nbins, int nprn, int datalen,
    int npairs, int nslot, double scale, const double2* __restrict__ tw_row, const double2* __restrict__ tw_col,
    double2* __restrict__ ring, FuseSync* __restrict__ sy, double* __restrict__ corr)
{
    constexpr int Q = (kRow + kRowThreads - 1) / kRowThreads;
    constexpr int64_t S = (int64_t)P * kRow;
    __shared__ double2 s_a[kRowPad], s_tw[kTwIK];
    __shared__ int s_role[6];  // xcc, rank, team size, XCD position, active XCDs, ok
    const int tid = threadIdx.x;
    // ---- census: this workgroup's XCD and rank in it, then wait for every workgroup
    if (tid == 0) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        xcc &= kFuseX - 1;
        const unsigned rank = add_dev(&sy->arrive[xcc * kFuseLine], 1u);
        add_dev(sy->total, 1u);
        int ok = wait_ge(sy->total, gridDim.x, sy) ? 1 : 0;
        // an XCD takes part when its team holds a row worker per row and at least 4
        // column workers; pairs are dealt round-robin over those XCDs
        int na = 0, xa = -1, nw = 0;
        for (int x = 0; x < kFuseX; x++) {
            const int w = (int)ld_sc1(&sy->arrive[x * kFuseLine]);
            if (w >= P + 4) {
                if (x == (int)xcc) { xa = na; nw = w; }
                na++;
            }
        }
        if (na == 0) ok = 0;
        if (!ok && rank == 0 && xcc == 0) add_dev(sy->err, 1u);  // (no team: the surface is void)
        s_role[0] = (int)xcc; s_role[1] = (int)rank; s_role[2] = nw; s_role[3] = xa; s_role[4] = na;
        s_role[5] = ok;
    }
    __syncthreads();
    const int xcc = s_role[0], rank = s_role[1], nw = s_role[2], xa = s_role[3], na = s_role[4];
    if (!s_role[5] || xa < 0) return;
    const int nr = P, nc = nw - P;                  // row workers (one per row), column workers
    const int npx = (npairs - xa + na - 1) / na;    // this XCD's pairs: xa, xa + na, ...
    const int ntr = npx * datalen;                  // ... and transforms (pair-major, ms minor)
    unsigned* ready = &sy->ready[xcc * kFuseSlots * kFuseLine];
    unsigned* freed = &sy->freed[xcc * kFuseSlots * kFuseLine];
    double2* ring_x = ring + (int64_t)xcc * kFuseSlots * S;

    if (rank >= nr) {
        // ---- column worker (I1, inv_cols_kernel's arithmetic)
        const int w = rank - nr;
        for (int it = w; it < ntr * kFuseChunks; it += nc) {
            const int j = it / kFuseChunks, ch = it - j * kFuseChunks, slot = j % nslot;
            if (tid == 0) s_role[5] = wait_ge(&freed[slot * kFuseLine], (unsigned)(j / nslot * nr), sy);
            __syncthreads();
            if (!s_role[5]) return;
            const int pi = j / datalen, ms = j - pi * datalen;
            const int q = xa + pi * na, bin = q / nprn, p = q - bin * nprn;
            const int k1 = ch * kColThreads + tid;
            if (k1 < kRow) {
                const double2* c = C + (int64_t)p * S + k1;
                const double2* x = X + ((int64_t)ms * nbins + bin) * S + k1;
                double2 v[P];
#pragma unroll
                for (int i = 0; i < P; i++) v[i] = cmulc(c[(int64_t)i * kRow], ld_nt(x + (int64_t)i * kRow));
                double2* a = ring_x + (int64_t)slot * S + k1;
                const double2* tw = tw_col + k1;
                dft_prime<P, 1>(v, [&](int k, double2 y) {
                    a[(int64_t)k * kRow] = GNSS_TW_ROWS ? y : cmulc(y, tw[(int64_t)k * kRow]);
                });
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores are in L2
            __syncthreads();
            if (tid == 0) add_dev(&ready[slot * kFuseLine], 1u);
        }
        return;
    }
    // ---- row worker: row tau2 = rank of every transform (I2's arithmetic)
    const int tau2 = rank;
    const TwIK<double2> twk = load_row_tw_ik(s_tw, tw_row, tid);
    double acc[kInvOut];
#pragma unroll
    for (int i = 0; i < kInvOut; i++) acc[i] = 0.0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        ring_x, (short)0, (int)(kFuseSlots * S * sizeof(double2)), 0x00020000);
    for (int j = 0; j < ntr; j++) {
        const int slot = j % nslot;
        if (tid == 0) s_role[5] = wait_ge(&ready[slot * kFuseLine], (unsigned)((j / nslot + 1) * kFuseChunks), sy);
        __syncthreads();
        if (!s_role[5]) return;
        const int row0 = (int)(((int64_t)slot * S + (int64_t)tau2 * kRow) * 16);
#pragma unroll
        for (int i = 0; i < Q; i++) {
            const int e = tid + i * kRowThreads;
            if (e < kRow) {
                typedef unsigned u4 __attribute__((ext_vector_type(4)));
                const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, row0 + e * 16, 0, 16 /* sc1 */);
                const double2 y = make_double2(__hiloint2double((int)v.y, (int)v.x), __hiloint2double((int)v.w, (int)v.z));
                s_a[e] = GNSS_TW_ROWS ? cmulc(y, tw_col[(int64_t)tau2 * kRow + e]) : y;
            }
        }
        __syncthreads();  // the row is in LDS: the slot may be refilled
        if (tid == 0) add_dev(&freed[slot * kFuseLine], 1u);
        inv_row_power_f64(s_a, twk, scale, acc, tid);  // (ends with a barrier: s_a free)
        const int pi = j / datalen, ms = j - pi * datalen;
        if (ms == datalen - 1) {
            const int q = xa + pi * na, bin = q / nprn, p = q - bin * nprn;
            double* o = corr + (((int64_t)p * nbins + bin) * P + tau2) * kRow;
#pragma unroll
            for (int i = 0; i < kInvOut; i++) {
                if (tid < kRow / kInvOut) o[tid + i * (kRow / kInvOut)] = acc[i];
                acc[i] = 0.0;
            }
        }
    }
}

// ============================== fine frequency (fp64) =============================
// x[n] = longrawsignal(S-cd + n) .* CA(rem(floor((n+1)/Fs*fc), 1023)+1), n < M = L*S
// (acquisition.m:103-106); X[k] = DFT_N of x zero-padded to N = M*D (:108), D = datalen.
// X[D*q + r] = DFT_M(y_r)[q], y_r[n] = x[n] w_N^(-n r). M = P*T*R (T = L = 10, R = 2000):
//   n = P*T*m1 + P*m2 + n2, q = j1 + R*j2 + T*R*k2.
// FR (rows): DFT_R over m1 of y_r[P*T*m1 + P*m2 + n2] (w_N^(-n r) = w_{R*D}^(-m1 r) *
//            w_N^(-(P*m2 + n2) r), the second factor applied after the DFT), * w_{T*R}^(-m2*j1)
//            -> E[r][n2][m2][j1]
// FC (cols): per (n2, j1) DFT_T over m2, * w_M^(-n2*(j1 + R*j2)); per (j1, j2) DFT_P over n2
//            -> |X| and the first maximum in fftshift order (:110-116)

constexpr int kFineT = 10;
constexpr int kFineJC = 16;  // j1 columns per FC block

// t[x] = w_div^(m), m = x (row = 0) or (x / row) * (x % row) (the [n2][k] product table)
__global__ void fine_twiddle_kernel(double2* __restrict__ t, int64_t len, int64_t div, int64_t row)
{
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= len) return;
    const int64_t m = row ? (x / row) * (x % row) : x;
    double s, c;
    sincospi(-2.0 * (double)m / (double)div, &s, &c);
    t[x] = make_double2(c, s);
}

// t[e] = the split layout's entry e of the w_2000 table (load_row_tw_ik's order), in global memory
__global__ void fine_twik_kernel(const double2* __restrict__ tw_row, double2* __restrict__ t)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kTwIK) return;
    const bool t2 = e < 9 * 20;
    const int f = t2 ? e : e - 9 * 20;
    const int i = t2 ? f / 20 + 1 : f / 200 + 1, k = t2 ? f % 20 : f % 200;
    t[e] = tw_row[t2 ? 10 * i * k : i * k];
}

// CA chip index of sample n of CarrSignal (acquisition.m:104: rem(floor((n+1)/Fs*fc), 1023))
__device__ __forceinline__ int64_t fine_code_of(int64_t n, double invFs, double invFc, double codelength)
{
    const double cvi = floor((invFs * (double)(n + 1)) / invFc);
    return (int64_t)fmod(cvi, codelength);
}

// A row of the fine search reads the samples n = P*T*m1 + rho, m1 < 2000: a lane stride of
// P*T samples, one cache line per lane for 2 bytes of it, and each of the D row passes of a
// column rho reads them again. GNSS_FINE_PREP: one pass per SV first copies CarrSignal's
// samples (unconverted) and their chips (the CA table's float at the chip index) into the
// row order [rho][m1] through an LDS tile (TM consecutive m1 x every rho: a contiguous run of
// the record), so the row pass reads both contiguously and with no dependent table read;
// the values are the ones it computed itself.
#ifndef GNSS_FINE_PREP
#define GNSS_FINE_PREP 1
#endif
#ifndef GNSS_FINE_TWIK
#define GNSS_FINE_TWIK 1
#endif
template <class Src> struct SrcElem;
template <> struct SrcElem<SrcIQ8> {
    using T = char2;
    static constexpr int kTM = 32;  // m1 per prep tile: 32 x 290 x (2 + 4) B = 56 KB of LDS
    __device__ static T get(const SrcIQ8& s, int64_t n) { return reinterpret_cast<const char2*>(s.p)[n]; }
    static SrcIQ8 wrap(const T* p) { return SrcIQ8{reinterpret_cast<const int8_t*>(p)}; }
};
template <> struct SrcElem<SrcC64> {
    using T = double2;
    static constexpr int kTM = 8;  // 8 x 290 x (16 + 4) B = 46 KB
    __device__ static T get(const SrcC64& s, int64_t n) { return s.p[n]; }
    static SrcC64 wrap(const T* p) { return SrcC64{p}; }
};
template <int P, class Src>
__global__ __launch_bounds__(kRowThreads) void fine_prep_kernel(
    const Src src, const int32_t* __restrict__ cd, int64_t S, double invFs, double invFc, double codelength,
    const float* __restrict__ ca0, typename SrcElem<Src>::T* __restrict__ xt0, float* __restrict__ ct0)
{
    using T = typename SrcElem<Src>::T;
    constexpr int PT = P * kFineT, TM = SrcElem<Src>::kTM;
    constexpr int64_t M = (int64_t)PT * kRow;
    __shared__ T s_x[TM * PT];
    __shared__ float s_c[TM * PT];
    const float* ca = ca0 + (int64_t)blockIdx.y * 1023;
    const int m0 = blockIdx.x * TM, tid = threadIdx.x;
    const int tm = kRow - m0 < TM ? kRow - m0 : TM;
    const int64_t base = S - cd[blockIdx.y] - 1, n0 = (int64_t)PT * m0;
    for (int e = tid; e < tm * PT; e += kRowThreads) {  // e = (m1 - m0)*PT + rho: the record in order
        s_x[e] = SrcElem<Src>::get(src, base + n0 + e);
        s_c[e] = ca[fine_code_of(n0 + e, invFs, invFc, codelength)];
    }
    __syncthreads();
    T* xt = xt0 + (int64_t)blockIdx.y * M;
    float* ct = ct0 + (int64_t)blockIdx.y * M;
    for (int e = tid; e < tm * PT; e += kRowThreads) {  // e = rho*tm + c: tm consecutive m1 of a row
        const int rho = e / tm, c = e - rho * tm;
        xt[(int64_t)rho * kRow + m0 + c] = s_x[c * PT + rho];
        ct[(int64_t)rho * kRow + m0 + c] = s_c[c * PT + rho];
    }
}

// (blockIdx.z = the SV of a batched launch: its code delay, code table and transform slab)
// GNSS_FINE_PREP: `src` is the prep pass's [sv][rho][m1] copy and ct its chips.
template <int P, class Src>
__global__ __launch_bounds__(kRowThreads) void fine_rows_kernel(
    const Src src, const float* __restrict__ ct, const int32_t* __restrict__ cd, int64_t S,
    const float* __restrict__ ca0, double invFs, double invFc, double codelength, int D, int64_t N,
    const double2* __restrict__ tw_row, const double2* __restrict__ twik, const double2* __restrict__ tabA,
    const double2* __restrict__ tabB, double2* __restrict__ E0)
{
    constexpr int T = kFineT;
    const int64_t base = S - cd[blockIdx.z] - 1;  // 0-based sample of CarrSignal(1) (acquisition.m:105)
    const float* ca = ca0 + (int64_t)blockIdx.z * 1023;
    double2* E = E0 + (int64_t)blockIdx.z * N;
    // twiddles read from the (L2-resident) global table: 32 KB of LDS per block instead of
    // 64, five blocks per CU instead of two
    __shared__ double2 s_a[kRowPad];
    const int rho = blockIdx.x, r = blockIdx.y, tid = threadIdx.x;
    const int m2 = rho / P, n2 = rho - m2 * P;
    auto sample = [&](int m1) { return (int64_t)P * T * m1 + (int64_t)P * m2 + n2; };
    auto code_of = [&](int64_t n) { return fine_code_of(n, invFs, invFc, codelength); };
    if constexpr (GNSS_FINE_PREP) {
        constexpr int NIT = (kRow + kRowThreads - 1) / kRowThreads;
        const int64_t row0 = ((int64_t)blockIdx.z * P * T + rho) * kRow;
        double2 raw[NIT], ta[NIT];
        float cv[NIT];
#pragma unroll
        for (int q = 0; q < NIT; q++) {
            const int m10 = tid + q * kRowThreads, m1 = m10 < kRow ? m10 : kRow - 1;
            cv[q] = ct[row0 + m1];
            raw[q] = src.at(row0 + m1);
            ta[q] = tabA[(int64_t)r * kRow + m1];
        }
#pragma unroll
        for (int q = 0; q < NIT; q++) {
            const int m1 = tid + q * kRowThreads;
            const double code = (double)cv[q];
            const double2 x = make_double2(raw[q].x * code, raw[q].y * code);
            if (m1 < kRow) s_a[m1] = cmul(x, ta[q]);
        }
    } else if constexpr (GNSS_STAGED_LOADS) {
        constexpr int NIT = (kRow + kRowThreads - 1) / kRowThreads;
        double2 raw[NIT], ta[NIT];
        float cv[NIT];
#pragma unroll
        for (int q = 0; q < NIT; q++) {
            const int m10 = tid + q * kRowThreads, m1 = m10 < kRow ? m10 : kRow - 1;
            const int64_t n = sample(m1);
            cv[q] = ca[code_of(n)];
            raw[q] = src.at(base + n);
            ta[q] = tabA[(int64_t)r * kRow + m1];
        }
#pragma unroll
        for (int q = 0; q < NIT; q++) {
            const int m1 = tid + q * kRowThreads;
            const double code = (double)cv[q];
            const double2 x = make_double2(raw[q].x * code, raw[q].y * code);
            if (m1 < kRow) s_a[m1] = cmul(x, ta[q]);  // w_RD^(-m1*r), [r][m1]: coalesced
        }
    } else {
        for (int m1 = tid; m1 < kRow; m1 += kRowThreads) {
            const int64_t n = sample(m1);
            const double code = (double)ca[code_of(n)];
            const double2 raw = src.at(base + n);
            const double2 x = make_double2(raw.x * code, raw.y * code);
            s_a[m1] = cmul(x, tabA[(int64_t)r * kRow + m1]);  // w_RD^(-m1*r), [r][m1]: coalesced
        }
    }
    __syncthreads();
    double sn, cs;
    const int64_t e = ((int64_t)(P * m2 + n2) * r) % N;
    sincospi(-2.0 * (double)e / (double)N, &sn, &cs);
    const double2 cb = make_double2(cs, sn);
    double2* o = E + (((int64_t)r * P + n2) * T + m2) * kRow;
    const double2* tb = tabB + m2 * kRow;  // w_{T*2000}^(-m2*j1), [m2][j1]
    auto put = [&](int, int j1, double2 v) { o[j1] = cmul(cmul(v, cb), tb[j1]); };
    // GNSS_FINE_TWIK: the stages' twiddles from the global split table (coalesced: lanes read
    // consecutive entries) instead of the plain table (a gather at a lane stride of i or 10 i
    // entries: up to a cache line per lane); the same values
    if constexpr (GNSS_FINE_TWIK)
        fft2000_r20first_put<-1>(s_a, TwIK<double2>{twik, twik + 9 * 20}, tid, put);
    else
        fft2000_r20first_put<-1>(s_a, tw_row, tid, put);
}

struct FineBest {
    double m;
    int64_t i;
};

__device__ __forceinline__ void best_merge(double& m, int64_t& i, double m2, int64_t i2)
{
    if (m2 > m || (m2 == m && i2 < i)) { m = m2; i = i2; }
}

template <int P>
__global__ __launch_bounds__(kColThreads) void fine_cols_kernel(
    const double2* __restrict__ E0, int D, int64_t N, int shifted, const double2* __restrict__ tabK,
    const double2* __restrict__ tabS, FineBest* __restrict__ part0)
{
    constexpr int T = kFineT, JC = kFineJC;
    const double2* E = E0 + (int64_t)blockIdx.z * N;
    FineBest* part = part0 + (int64_t)blockIdx.z * gridDim.x * gridDim.y;
    // 29 x 10 x 16 x 16 B = 74 KB of LDS: two blocks per CU on gfx950's 160 KiB (above the
    // 64 KiB per-workgroup limit of earlier gfx9 parts; this file is built for gfx950 only)
    static_assert(P * T * JC * sizeof(double2) + (kColThreads / 64) * sizeof(double) * 2 <= 80 * 1024,
                  "fine_cols LDS tile: two blocks per CU of gfx950's 160 KiB");
    __shared__ double2 s_e[P * T * JC];  // [n2][m2 -> j2][jj]
    __shared__ FineBest s_b[kColThreads / 64];
    const int r = blockIdx.y, j10 = blockIdx.x * JC, tid = threadIdx.x;
    auto at = [&](int e) {
        const int jj = e % JC, nm = e / JC;  // nm = n2*T + m2
        return E + ((int64_t)r * P * T + nm) * kRow + j10 + jj;
    };
    if constexpr (GNSS_STAGED_LOADS) {
        constexpr int NE = P * T * JC, NIT = (NE + kColThreads - 1) / kColThreads;
        double2 st[NIT];
#pragma unroll
        for (int q = 0; q < NIT; q++) {
            const int e0 = tid + q * kColThreads;
            st[q] = *at(e0 < NE ? e0 : NE - 1);
        }
#pragma unroll
        for (int q = 0; q < NIT; q++)
            if (tid + q * kColThreads < NE) s_e[tid + q * kColThreads] = st[q];
    } else {
        for (int e = tid; e < P * T * JC; e += kColThreads) s_e[e] = *at(e);
    }
    __syncthreads();
    // DFT_T over m2 for each (n2, jj), twiddle w_M^(-n2*k1), k1 = k + 2000*j2:
    // w_M^(-n2*k) (the [n2][k] table, 16 consecutive k per block: coalesced) times
    // w_{P*T}^(-n2*j2) (a 290-entry table). (A gather from the full w_M table fetched
    // ~4x the bytes of E from L2 / MALL.)
    for (int pr = tid; pr < P * JC; pr += kColThreads) {
        const int n2 = pr / JC, jj = pr - n2 * JC;
        double2 v[T];
#pragma unroll
        for (int m2 = 0; m2 < T; m2++) v[m2] = s_e[(n2 * T + m2) * JC + jj];
        dft10<-1>(v);
        const double2 tk = tabK[n2 * kRow + j10 + jj];
#pragma unroll
        for (int j2 = 0; j2 < T; j2++)
            s_e[(n2 * T + j2) * JC + jj] = cmul(v[j2], j2 ? cmul(tk, tabS[(n2 * j2) % (P * T)]) : tk);
    }
    __syncthreads();
    double bm = -1.0;
    int64_t bi = INT64_MAX;
    const int64_t half = N / 2;
    for (int pr = tid; pr < T * JC; pr += kColThreads) {
        const int j2 = pr / JC, jj = pr - j2 * JC;
        double2 v[P];
#pragma unroll
        for (int n2 = 0; n2 < P; n2++) v[n2] = s_e[(n2 * T + j2) * JC + jj];
        const int64_t k1 = j10 + jj + (int64_t)kRow * j2;
        dft_prime<P, -1>(v, [&](int k2, double2 y) {
            const int64_t q = k1 + (int64_t)T * kRow * k2;
            const int64_t k = (int64_t)D * q + r;  // natural bin of the N-point FFT
            int64_t i = k;
            if (shifted == 1) { i = k + half; if (i >= N) i -= N; }
            // 2: real CarrSignal (dataType 1): MATLAB's fft is exactly conjugate-symmetric,
            // a mirror pair ties and its first (lower) index wins
            else if (shifted == 2 && N - k < k) i = N - k;
            best_merge(bm, bi, hypot(y.x, y.y), i);
        });
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double m2 = __shfl_xor(bm, o, 64);
        const int64_t i2 = __shfl_xor(bi, o, 64);
        best_merge(bm, bi, m2, i2);
    }
    if ((tid & 63) == 0) s_b[tid >> 6] = FineBest{bm, bi};
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kColThreads / 64; w++) best_merge(bm, bi, s_b[w].m, s_b[w].i);
        part[(int64_t)r * gridDim.x + blockIdx.x] = FineBest{bm, bi};
    }
}

__global__ void fine_best_final_kernel(const FineBest* __restrict__ part0, int nblk,
                                       int64_t* __restrict__ kbest0)
{
    const FineBest* part = part0 + (int64_t)blockIdx.x * nblk;  // (one block per SV)
    int64_t* kbest = kbest0 + blockIdx.x;
    double bm = -1.0;
    int64_t bi = INT64_MAX;
    for (int k = threadIdx.x; k < nblk; k += blockDim.x) best_merge(bm, bi, part[k].m, part[k].i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double m2 = __shfl_xor(bm, o, 64);
        const int64_t i2 = __shfl_xor(bi, o, 64);
        best_merge(bm, bi, m2, i2);
    }
    __shared__ FineBest s_b[4];
    if ((threadIdx.x & 63) == 0) s_b[threadIdx.x >> 6] = FineBest{bm, bi};
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) best_merge(bm, bi, s_b[w].m, s_b[w].i);
        *kbest = bi + 1;  // 1-based FreqPeakIndex
    }
}

}  // namespace

bool acq_fft_supported(int64_t S) { return S == 13 * kRow || S == 29 * kRow; }

// The forward spectra: X[s] for s < nsig ((ms, bin) signals, s = ms*nbins + bin) and the
// code spectra C[p] (stored after them: X + nsig*S). V = float2 or double2.
template <class V>
hipError_t launch_acq_fft_forward(const int8_t* iq, const double2* xs, int64_t S, int datalen, int nbins,
                                  double IF, double freqMin, double freqStep, double Fs, const float* ca,
                                  int nprn, double codeFreqBasis, const V* tw_row,
                                  const V* tw_col, V* B, V* X, hipStream_t s, int bin0, int nbc, bool codes)
{
    const int nsig = datalen * nbins;
    if (nbc < 0) nbc = nbins - bin0;
    if (bin0 < 0 || nbc < 0 || bin0 + nbc > nbins) return hipErrorInvalidValue;
    const FwdSet fs{nbins, nsig, nprn, bin0, nbc > 0 ? nbc : 1, codes ? 1 : 0};
    const int ntr = (codes ? nprn : 0) + datalen * nbc;
    if (ntr == 0) return hipSuccess;
    const double step = codeFreqBasis / Fs;
#define GNSS_FWD(P_)                                                                            \
    if (S == (int64_t)P_ * kRow) {                                                              \
        if (xs)                                                                                 \
            hipLaunchKernelGGL((fwd_rows_kernel<P_, SrcC64, V>), dim3(P_, ntr), dim3(kRowThreads), 0, s, \
                               SrcC64{xs}, fs, IF, freqMin, freqStep, Fs, ca, step, tw_row, tw_col, B); \
        else                                                                                    \
            hipLaunchKernelGGL((fwd_rows_kernel<P_, SrcIQ8, V>), dim3(P_, ntr), dim3(kRowThreads), 0, s, \
                               SrcIQ8{iq}, fs, IF, freqMin, freqStep, Fs, ca, step, tw_row, tw_col, B); \
        hipLaunchKernelGGL((fwd_cols_kernel<P_, V>), dim3((kRow + kColThreads - 1) / kColThreads, ntr), \
                           dim3(kColThreads), 0, s, fs, B, X);                                  \
        return hipGetLastError();                                                               \
    }
    GNSS_FWD(13) GNSS_FWD(29)
#undef GNSS_FWD
    return hipErrorInvalidValue;
}
template hipError_t launch_acq_fft_forward<float2>(const int8_t*, const double2*, int64_t, int, int, double,
                                                   double, double, double, const float*, int, double,
                                                   const float2*, const float2*, float2*, float2*, hipStream_t, int,
                                                   int, bool);
template hipError_t launch_acq_fft_forward<double2>(const int8_t*, const double2*, int64_t, int, int, double,
                                                    double, double, double, const float*, int, double,
                                                    const double2*, const double2*, double2*, double2*,
                                                    hipStream_t, int, int, bool);

// Correlation of (bin, PRN) pairs [first_pair, first_pair + npair) (pair = bin*nprn + p)
// over every ms: corr[p][bin] (tau2-major) = sum_ms |ifft(C_p .* conj(X_{ms,bin}))|^2.
hipError_t launch_acq_fft_correlate(const float2* C, const float2* X, int64_t S, int datalen,
                                    int nbins, int nprn, int first_pair, int npair,
                                    const float2* tw_row, const float2* tw_col, float2* A,
                                    float* corr, hipStream_t s, int parts)
{
    const float scale = (float)(1.0 / ((double)S * (double)S));  // ifft's 1/N, squared
#define GNSS_INV(P_)                                                                            \
    if (S == (int64_t)P_ * kRow) {                                                              \
        if (parts & kAcqCols)                                                                   \
        hipLaunchKernelGGL((inv_cols_kernel<P_, float2>),                                       \
                           dim3((kRow + kColThreads - 1) / kColThreads, npair * datalen),       \
                           dim3(kColThreads), 0, s, C, X, nbins, nprn, datalen, first_pair,     \
                           tw_col, A);                                                          \
        if (parts & kAcqRows)                                                                   \
        hipLaunchKernelGGL(inv_rows_kernel<P_>, dim3(P_, npair), dim3(kRowThreads), 0, s, A, nprn, \
                           datalen, first_pair, scale, tw_row, tw_col, corr, nbins);            \
        return hipGetLastError();                                                               \
    }
    GNSS_INV(13) GNSS_INV(29)
#undef GNSS_INV
    return hipErrorInvalidValue;
}

hipError_t launch_acq_fft_correlate(const double2* C, const double2* X, int64_t S, int datalen,
                                    int nbins, int nprn, int first_pair, int npair,
                                    const double2* tw_row, const double2* tw_col, double2* A,
                                    double* corr, hipStream_t s, int parts)
{
    const double scale = 1.0 / ((double)S * (double)S);
#define GNSS_INV(P_)                                                                            \
    if (S == (int64_t)P_ * kRow) {                                                              \
        if (parts & kAcqCols)                                                                   \
        hipLaunchKernelGGL((inv_cols_kernel<P_, double2>),                                      \
                           dim3((kRow + kColThreads - 1) / kColThreads, npair * datalen),       \
                           dim3(kColThreads), 0, s, C, X, nbins, nprn, datalen, first_pair,     \
                           tw_col, A);                                                          \
        if (parts & kAcqRows)                                                                   \
        hipLaunchKernelGGL(inv_rows_kernel_f64<P_>, dim3(P_, npair), dim3(kRowThreads), 0, s, A, nprn, \
                           datalen, first_pair, scale, tw_row, tw_col, corr, nbins);            \
        return hipGetLastError();                                                               \
    }
    GNSS_INV(13) GNSS_INV(29)
#undef GNSS_INV
    return hipErrorInvalidValue;
}

// One paired launch (fp64): the column pass of pairs [cols_first, +cols_n) into Acols and the
// row pass of [rows_first, +rows_n) from Arows (a different intermediate: the previous launch's).
hipError_t launch_acq_fft_pair(const double2* C, const double2* X, int64_t S, int datalen, int nbins, int nprn,
                               int cols_first, int cols_n, double2* Acols, int rows_first, int rows_n,
                               const double2* Arows, const double2* tw_row, const double2* tw_col, double* corr,
                               int front, hipStream_t s)
{
    if (front < 1 || front > 100 || cols_n < 0 || rows_n < 0) return hipErrorInvalidValue;
    const double scale = 1.0 / ((double)S * (double)S);
    constexpr int kCx = (kRow + kColThreads - 1) / kColThreads;
#define GNSS_PAIR(P_)                                                                           \
    if (S == (int64_t)P_ * kRow) {                                                              \
        const int64_t nblk = (int64_t)P_ * rows_n + (int64_t)kCx * cols_n * datalen;             \
        if (nblk == 0) return hipSuccess;                                                       \
        if (nblk > INT32_MAX) return hipErrorInvalidConfiguration;                              \
        hipLaunchKernelGGL(inv_pair_kernel_f64<P_>, dim3((unsigned)nblk), dim3(kRowThreads), 0, s, C, X, nbins, \
                           nprn, datalen, cols_first, cols_n, Acols, rows_first, rows_n, Arows, scale, tw_row, \
                           tw_col, corr, front);                                                \
        return hipGetLastError();                                                               \
    }
    static_assert(kColThreads == kRowThreads, "the paired launch runs both bodies in one block shape");
    GNSS_PAIR(13) GNSS_PAIR(29)
#undef GNSS_PAIR
    return hipErrorInvalidValue;
}

size_t acq_fused_sync_bytes() { return sizeof(FuseSync); }
size_t acq_fused_err_offset() { return offsetof(FuseSync, err); }
size_t acq_fused_ring_bytes(int64_t S) { return sizeof(double2) * (size_t)kFuseX * kFuseSlots * (size_t)S; }

// All (bin, PRN) pairs in one persistent launch (I1 + I2 fused, fp64). `sync` holds
// acq_fused_sync_bytes() and `ring` acq_fused_ring_bytes(S); the launch zeroes `sync`.
// Its err word is non-zero afterwards if a wait timed out (a grid that was not resident).
hipError_t launch_acq_fft_correlate_fused(const double2* C, const double2* X, int64_t S, int datalen, int nbins,
                                          int nprn, int nslot, const double2* tw_row, const double2* tw_col,
                                          double2* ring, void* sync, double* corr, hipStream_t s)
{
    if (nslot < 2 || nslot > kFuseSlots) return hipErrorInvalidValue;
    const double scale = 1.0 / ((double)S * (double)S);
    int dev = 0, ncu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipMemsetAsync(sync, 0, sizeof(FuseSync), s);
    if (e != hipSuccess) return e;
    FuseSync* sy = static_cast<FuseSync*>(sync);
#define GNSS_FUSED(P_)                                                                          \
    if (S == (int64_t)P_ * kRow) {                                                              \
        int occ = 0;                                                                            \
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, inv_fused_kernel_f64<P_>, kRowThreads, 0); \
        if (e != hipSuccess) return e;                                                          \
        const int grid = ncu * std::min(occ, 2);                                                \
        if (grid < 1) return hipErrorInvalidConfiguration;                                      \
        hipLaunchKernelGGL(inv_fused_kernel_f64<P_>, dim3(grid), dim3(kRowThreads), 0, s, C, X, nbins, nprn, \
                           datalen, nbins * nprn, nslot, scale, tw_row, tw_col, ring, sy, corr); \
        return hipGetLastError();                                                               \
    }
    GNSS_FUSED(13) GNSS_FUSED(29)
#undef GNSS_FUSED
    return hipErrorInvalidValue;
}

bool fine_fft_supported(int64_t S, int L) { return acq_fft_supported(S) && L == kFineT; }

// Scratch of the fine search: the twiddle tables, then per SV of a batch its N-point slab of
// transform values and its column blocks' arg-max candidates.
namespace {
struct FineLayout {
    int64_t M, N, tabs, slab, part;  // element counts (double2) / offsets
};
FineLayout fine_layout(int64_t S, int L, int datalen)
{
    FineLayout f;
    f.M = (int64_t)L * S;
    f.N = f.M * datalen;
    f.tabs = kRow + (int64_t)kRow * datalen + (int64_t)kFineT * kRow + S + f.M / kRow + kTwIK;
    f.slab = f.N;
    f.part = (int64_t)datalen * (kRow / kFineJC);  // FineBest entries per SV
    return f;
}
}  // namespace

// (GNSS_FINE_PREP) the row-order copies after the candidates: nsv x M samples (sized for the
// widest source, complex fp64), then nsv x M chips (float)
static size_t fine_prep_offset(const FineLayout& f, int nsv)
{
    const size_t b = sizeof(double2) * (size_t)(f.tabs + (int64_t)nsv * f.slab) + sizeof(FineBest) * (size_t)(nsv * f.part);
    return (b + 255) & ~(size_t)255;
}
size_t fine_fft_scratch_bytes(int64_t S, int L, int datalen, int nsv)
{
    const FineLayout f = fine_layout(S, L, datalen);
    if (!GNSS_FINE_PREP) return fine_prep_offset(f, nsv);
    return fine_prep_offset(f, nsv) + (size_t)nsv * f.M * (sizeof(double2) + sizeof(float));
}

// Twiddle tables of the fine search, once per call: w_2000, w_{2000*D}, w_{T*2000}, w_M, w_{P*T}.
hipError_t launch_fine_fft_tables(int64_t S, int L, int datalen, void* scratch, hipStream_t s)
{
    const int64_t M = (int64_t)L * S;
    double2* tw_row = static_cast<double2*>(scratch);
    double2* tabA = tw_row + kRow;
    double2* tabB = tabA + (int64_t)kRow * datalen;
    double2* tabK = tabB + (int64_t)kFineT * kRow;  // [P][2000] w_M^(-n2*k), then w_{P*T}
    double2* tabS = tabK + S;
    // tabA[r][m1] = w_{2000 D}^(m1 r), tabB[m2][j1] = w_{T 2000}^(m2 j1), tabK[n2][k] = w_M^(n2 k):
    // the exponent products laid out so a row pass reads them contiguously (the same
    // values as a gather from the plain tables: the same m through the same formula)
    const int64_t lens[5] = {kRow, (int64_t)kRow * datalen, (int64_t)kFineT * kRow, S, M / kRow};
    const int64_t divs[5] = {kRow, (int64_t)kRow * datalen, (int64_t)kFineT * kRow, M, M / kRow};
    const int64_t rows[5] = {0, kRow, kRow, kRow, 0};
    double2* tabs[5] = {tw_row, tabA, tabB, tabK, tabS};
    for (int t = 0; t < 5; t++)
        hipLaunchKernelGGL(fine_twiddle_kernel, dim3((unsigned)((lens[t] + 255) / 256)), dim3(256), 0,
                           s, tabs[t], lens[t], divs[t], rows[t]);
    // the row transforms' twiddles in the split layout (TwIK: a stage's lanes read consecutive
    // entries), copied from w_2000 after it (the same stream)
    hipLaunchKernelGGL(fine_twik_kernel, dim3((kTwIK + 255) / 256), dim3(256), 0, s, tw_row, tabS + M / kRow);
    return hipGetLastError();
}

// First fftshift-ed argmax (1-based) of |fft(CarrSignal, N)| for nsv SVs in one batch of
// launches (acquisition.m:103-116): SV k's code delay cd[k] (device), its code table
// ca + 1023 k, its result kbest[k]. Every SV's arithmetic is the one-SV launch's.
hipError_t launch_fine_fft_argmax(const int8_t* iq, const double2* xs, int64_t S, int L, int datalen,
                                  const int32_t* cd, int nsv, const float* ca, double Fs, double codeFreqBasis,
                                  double codelength, int shifted, void* scratch, int64_t* kbest, hipStream_t s)
{
    if (nsv < 1 || nsv > 65535) return hipErrorInvalidValue;
    const FineLayout f = fine_layout(S, L, datalen);
    const int64_t N = f.N;
    double2* tw_row = static_cast<double2*>(scratch);
    double2* tabA = tw_row + kRow;
    double2* tabB = tabA + (int64_t)kRow * datalen;
    double2* tabK = tabB + (int64_t)kFineT * kRow;
    double2* tabS = tabK + S;
    double2* E = tw_row + f.tabs;
    FineBest* part = reinterpret_cast<FineBest*>(E + (int64_t)nsv * f.slab);
    char* prep = static_cast<char*>(scratch) + fine_prep_offset(f, nsv);
    float* ct = reinterpret_cast<float*>(prep + (size_t)nsv * f.M * sizeof(double2));
    const int nblk = kRow / kFineJC;
    // the row pass over source Src: from the record itself, or (GNSS_FINE_PREP) from its row-order copy
    auto rows = [&](auto src, auto* xt, auto kern, auto prep_kern, int tm) {
        using SrcT = decltype(src);
        if (GNSS_FINE_PREP) {
            hipLaunchKernelGGL(prep_kern, dim3((kRow + tm - 1) / tm, nsv), dim3(kRowThreads), 0, s, src, cd, S, 1 / Fs,
                               1 / codeFreqBasis, codelength, ca, xt, ct);
            src = SrcElem<SrcT>::wrap(xt);
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)(f.M / kRow), datalen, nsv), dim3(kRowThreads), 0, s, src, ct, cd, S,
                           ca, 1 / Fs, 1 / codeFreqBasis, codelength, datalen, N, tw_row, tabS + f.M / kRow, tabA,
                           tabB, E);
    };
#define GNSS_FINE(P_)                                                                           \
    if (S == (int64_t)P_ * kRow) {                                                              \
        if (xs)                                                                                 \
            rows(SrcC64{xs}, reinterpret_cast<double2*>(prep), fine_rows_kernel<P_, SrcC64>,    \
                 fine_prep_kernel<P_, SrcC64>, SrcElem<SrcC64>::kTM);                           \
        else                                                                                    \
            rows(SrcIQ8{iq}, reinterpret_cast<char2*>(prep), fine_rows_kernel<P_, SrcIQ8>,      \
                 fine_prep_kernel<P_, SrcIQ8>, SrcElem<SrcIQ8>::kTM);                           \
        hipLaunchKernelGGL(fine_cols_kernel<P_>, dim3(nblk, datalen, nsv), dim3(kColThreads), 0, s, E, \
                           datalen, N, shifted, tabK, tabS, part);                                    \
        hipLaunchKernelGGL(fine_best_final_kernel, dim3(nsv), dim3(256), 0, s, part, nblk * datalen, \
                           kbest);                                                              \
        return hipGetLastError();                                                               \
    }
    GNSS_FINE(13) GNSS_FINE(29)
#undef GNSS_FINE
    return hipErrorInvalidValue;
}

}  // namespace gnss
