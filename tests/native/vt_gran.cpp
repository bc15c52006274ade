// Host-side checks of the VT loop mode's helpers (gnss_internal.h), host code only:
//  - vt_gran_put / vt_gran_get: a granule's value comes back with its tag, a granule whose two
//    halves carry different tags (caught mid-write) is rejected, and under a concurrent writer
//    every accepted read is one the writer wrote (value tied to tag);
//  - vt_remchip_next equals the remChip vt_finish leaves in the channel state (the next read's
//    size is what gnss_tracking_vt computes the next orbit for a step ahead).
// Prints "mismatches N".
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>

#include "../../assignment-for-aae6102_gnss-sdr_amd/csrc/gnss_internal.h"

using namespace gnss;

static uint64_t value_of(unsigned tag) { return 0x9e3779b97f4a7c15ull * (uint64_t)(tag + 1); }

int main()
{
    long bad = 0;
    std::mt19937_64 rng(7);
    // round trip
    VtGran g;
    for (int i = 0; i < 100000; i++) {
        const uint64_t bits = rng();
        const unsigned tag = (unsigned)rng();
        vt_gran_put(&g, bits, tag);
        uint64_t got = 0;
        if (!vt_gran_get(&g, tag, &got) || got != bits) bad++;
        if (vt_gran_get(&g, tag + 1, &got)) bad++;
    }
    // halves from two writes (a granule read mid-rewrite): rejected under either tag
    {
        VtGran a, b;
        vt_gran_put(&a, 0x1111222233334444ull, 5);
        vt_gran_put(&b, 0x5555666677778888ull, 6);
        VtGran t{a.lo, b.hi};
        uint64_t got;
        if (vt_gran_get(&t, 5, &got) || vt_gran_get(&t, 6, &got)) bad++;
    }
    // a concurrent writer: every accepted read carries the value its tag was written with
    {
        VtGran c;
        vt_gran_put(&c, value_of(0), 0);
        std::atomic<bool> done{false};
        std::thread w([&] {
            for (unsigned t = 1; t < 2000000; t++) vt_gran_put(&c, value_of(t), t);
            done = true;
        });
        long seen = 0;
        while (!done) {
            const uint64_t lo = __atomic_load_n(&c.lo, __ATOMIC_ACQUIRE);
            const unsigned tag = (unsigned)(lo >> 32);
            uint64_t got;
            if (vt_gran_get(&c, tag, &got)) {
                seen++;
                if (got != value_of(tag)) bad++;
            }
        }
        w.join();
        printf("concurrent reads accepted %ld\n", seen);
    }
    // vt_remchip_next == vt_finish's remChip
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const double Fs = 58e6, ms = 1e-3;
    for (int i = 0; i < 20000; i++) {
        gnss_vt_chan c{};
        c.remChip = U(rng) * 0.9 - 0.45;
        c.codeFreq = 1.023e6 * (1 + (U(rng) - 0.5) * 1e-5);
        c.carrFreq = (U(rng) - 0.5) * 1e4;
        c.snrIndex = 1;
        const double cf_new = 1.023e6 * (1 + (U(rng) - 0.5) * 1e-5);
        const int pdi = 1;
        const VtPrep p = vt_prepare(Fs, 1023.0, pdi, c.remChip, c.codeFreq, cf_new);
        if (p.bad) continue;
        const double rc = vt_remchip_next(Fs, pdi, c.remChip, cf_new, p.n);
        gnss_vt_out o{};
        const int code[3] = {1, 1, 1};
        if (vt_finish(Fs, ms, pdi, 2, 1.0, 1.0, &c, p, code, cf_new, 1.0, 0.5, &o) != GNSS_OK) continue;
        if (std::memcmp(&rc, &c.remChip, sizeof rc) != 0) bad++;
    }
    printf("mismatches %ld\n", bad);
    return bad != 0;
}
