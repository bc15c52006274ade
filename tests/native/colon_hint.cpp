// Host check: colon_make_hint (the step kernel's division-free colon) builds the same
// a:d:b as colon_make (MathWorks' colonop) on the ranges trackingCT.m forms
// (trackingCT.m:96-98: a = spacing + remChip, b = (n-1)*cps + spacing + remChip).
#include <cstdio>
#include <random>

#include "../../assignment-for-aae6102_gnss-sdr_amd/csrc/gnss_internal.h"

int main()
{
    using namespace gnss;
    std::mt19937_64 rng(6102);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long bad = 0, n_checked = 0;
    for (int it = 0; it < 2000000; it++) {
        const double Fs = it % 3 == 0 ? 26e6 : 58e6;
        const double cf = 1.023e6 + (U(rng) - 0.5) * 40.0;
        const double cps = cf / Fs;
        const int pdi = it % 2 ? 10 : 1;
        const double rc = (U(rng) - 0.5) * 0.05;
        const double taps[] = {-0.5, -0.3, -0.1, 0.0, 0.1, 0.5};
        const double tap = taps[it % 6];
        const int64_t n = (int64_t)round((1023.0 * pdi - rc) / cps) + (int64_t)(it % 5) - 2;
        const double a = (0 + tap) + rc;
        const double b = ((double)(n - 1) * cps + tap) + rc;
        const Colon x = colon_make(a, cps, b), y = colon_make_hint(a, cps, b, n - 1);
        n_checked++;
        if (x.n != y.n || x.c != y.c || x.a != y.a) bad++;
    }
    printf("checked %ld mismatches %ld\n", n_checked, bad);
    return bad != 0;
}
