// Host check: div_const (csrc/gnss_internal.h), the tracking tail's quotient by a divisor
// known ahead -- q = RN(x * RN(1/b)), r = x - q*b by FMA, q' = RN(q + r * RN(1/b)) (Markstein)
// -- equals the IEEE quotient x / b bit for bit, on random operands of every kind the tail
// divides (codeFreq, 2*pi*f, integer sample counts, atan outputs, phases, small
// corrections, random bit patterns) for the divisors in use (Fs values, 2*pi).
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

int main(int argc, char** argv)
{
    using namespace gnss;
    const double bs[] = {58e6, 26e6, kTwoPi, 16.3676e6, 38.192e6, 5e6, 40e6};
    const long N = argc > 1 ? atol(argv[1]) : 2000000;
    long bad = 0;
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
            case 4: x = ldexp(uni(1, 2), (int)(xr() % 200) - 100); break;
            case 5: x = uni(-1e-6, 1e-6); break;             // small corrections
            case 6: {
                uint64_t u = xr();
                memcpy(&x, &u, 8);
                if (!std::isfinite(x) || fabs(x) > 1e300 || fabs(x) < 1e-290) x = 1.5;
            } break;
            default: x = uni(0, 3e5); break;                 // carrier phases
            }
            if (x / b != div_const(x, b, rb)) {
                if (++nb < 4) printf("b=%.17g x=%.17g ieee=%.17g div_const=%.17g\n", b, x, x / b, div_const(x, b, rb));
            }
        }
        bad += nb;
    }
    printf("mismatches %ld of %ld\n", bad, 7 * N);
    return bad != 0;
}
