// Host check: fmod_pos (the record's one-FMA remainder, codedelay2 = mod(absoluteSample /
// dataBytesPerSample, Fs*ms), trackingCT.m:170) equals C fmod bit for bit, on the
// record's ranges and on adversarial quotients next to integers.
#include <cmath>
#include <cstdio>
#include <random>

#include "../../assignment-for-aae6102_gnss-sdr_amd/csrc/gnss_internal.h"

int main()
{
    using namespace gnss;
    std::mt19937_64 rng(6102);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long bad = 0, n = 0;
    const double ys[] = {58000.0, 26000.0, 58e6 * 0.001, 26e6 * 0.001, 16368.0, 5e6 * 0.001, 0.1, 3.7};
    for (int it = 0; it < 4000000; it++) {
        const double y = ys[it % 8];
        double x;
        if (it % 4 == 0) x = std::floor(U(rng) * 2e10) / 2;                 // sample positions
        else if (it % 4 == 1) x = std::nextafter(std::floor(U(rng) * 1e6) * y, it % 8 < 4 ? 0.0 : 1e300);
        else if (it % 4 == 2) x = std::floor(U(rng) * 1e6) * y;             // on a multiple
        else x = U(rng) * 1e12;
        const double a = fmod_pos(x, y), b = std::fmod(x, y);
        n++;
        if (a != b || std::signbit(a) != std::signbit(b)) {
            if (bad < 5) printf("x=%.17g y=%.17g fmod_pos=%.17g fmod=%.17g\n", x, y, a, b);
            bad++;
        }
    }
    printf("checked %ld mismatches %ld\n", n, bad);
    return bad != 0;
}
