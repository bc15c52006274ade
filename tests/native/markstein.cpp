// Host check: div_const (csrc/gnss_internal.h), the tracking tail's quotient by a divisor
// known ahead -- Markstein's correction q1 = RN(q + r * RN(1/b)) followed by the exact-
// remainder rounding test -- equals the IEEE quotient x / b bit for bit, on random operands
// of every kind the tail divides (codeFreq, 2*pi*f, integer sample counts, atan outputs,
// phases, small corrections, random bit patterns) and on quotients within a few ulps of a
// rounding midpoint (the hard cases), for the divisors in use (Fs values, 2*pi) and for
// random Fs in [1, 100] MHz; and the rounding test alone (div_round_fix) given the quotient's
// neighbours on either side (powers of two among them, case 4). Also counts where Markstein's
// step alone (div_markstein) is off.
// argv[1] = operands per divisor (default 2e6).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../assignment-for-aae6102_gnss-sdr_amd/csrc/gnss_internal.h"

static uint64_t s = 88172645463325252ull;
static inline uint64_t xr() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline double uni(double lo, double hi) { return lo + (hi - lo) * ((xr() >> 11) * (1.0 / 9007199254740992.0)); }

// x with x/b within a few ulps of the midpoint above a random quotient
static double near_midpoint(double b)
{
    uint64_t u = (xr() >> 12) | 0x3ff0000000000000ull;
    double q;
    memcpy(&q, &u, 8);
    q = ldexp(q, (int)(xr() % 60) - 30);
    const long double m = (long double)q + 0.5L * ((long double)nextafter(q, INFINITY) - q);
    double x = (double)(m * (long double)b);
    for (int t = (int)(xr() % 5) - 2; t != 0; t += t < 0 ? 1 : -1) x = nextafter(x, t < 0 ? -INFINITY : INFINITY);
    return (xr() & 1) ? -x : x;
}

int main(int argc, char** argv)
{
    using namespace gnss;
    double bs[7 + 20] = {58e6, 26e6, kTwoPi, 16.3676e6, 38.192e6, 5e6, 40e6};
    for (int i = 7; i < 27; i++) bs[i] = std::round(uni(1e6, 1e8));  // other sample rates
    const long N = argc > 1 ? atol(argv[1]) : 2000000;
    long bad = 0, mk_off = 0, total = 0;
    for (double b : bs) {
        const double rb = b == kTwoPi ? kInvTwoPi : 1.0 / b;
        long nb = 0;
        for (long k = 0; k < N; k++) {
            double x;
            switch (k & 7) {
            case 0: x = uni(1.0225e6, 1.0235e6); break;      // codeFreq
            case 1: x = uni(-3.2e7, 3.2e7); break;           // 2*pi*f
            case 2: x = (double)(xr() % 1200000); break;     // sample counts
            case 3: x = uni(-1.6, 1.6); break;               // atan outputs
            case 4: x = (k & 8) ? ldexp(b, (int)(xr() % 40) - 20) : ldexp(uni(1, 2), (int)(xr() % 200) - 100); break;
            case 5: x = near_midpoint(b); break;             // the hard cases
            case 6: {
                uint64_t u = xr();
                memcpy(&x, &u, 8);
                if (!std::isfinite(x) || fabs(x) > 1e300 || fabs(x) < 1e-280) x = 1.5;
            } break;
            default: x = uni(0, 3e5); break;                 // carrier phases
            }
            total++;
            if (div_markstein(x, b, rb) != x / b) mk_off++;
            // the rounding test itself: a quotient one step off on either side is repaired
            const double qe = x / b;
            if (qe != 0) {
                const double lo = nextafter(qe, -INFINITY), hi = nextafter(qe, INFINITY);
                if (div_round_fix(x, b, lo) != qe || div_round_fix(x, b, hi) != qe || div_round_fix(x, b, qe) != qe) {
                    if (++nb < 4) printf("fix: b=%.17g x=%.17g\n", b, x);
                }
            }
            if (x / b != div_const(x, b, rb)) {
                if (++nb < 4) printf("b=%.17g x=%.17g ieee=%.17g div_const=%.17g\n", b, x, x / b, div_const(x, b, rb));
            }
        }
        bad += nb;
    }
    printf("markstein step alone off on %ld; mismatches %ld of %ld\n", mk_off, bad, total);
    return bad != 0;
}
