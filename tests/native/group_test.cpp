// Host check of the multi-device context's bookkeeping (csrc/group.h): the round-robin deal,
// the merge of the members' Acquired / diag rows back into PRN-list order, and the status a
// sharded call returns, each against the one-context answer computed directly.
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <random>
#include <thread>
#include <vector>

#include "../../assignment-for-aae6102_gnss-sdr_amd/csrc/group.h"

using namespace gnss;

static int bad = 0;
#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            if (bad < 10) printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            bad++;                                                 \
        }                                                          \
    } while (0)

// one context over the whole PRN list: a PRN is acquired iff snr >= 12 (acquisition.m:70-74).
// The detector's outputs are functions of the PRN alone (the same record for every PRN), so a
// repeated PRN gives repeated rows: the synthetic model below keeps that.
static void serial_acq(const std::vector<int32_t>& prns, const std::vector<double>& snr_of, gnss_acquired* out,
                       gnss_acq_diag* diag)
{
    memset(out, 0, sizeof(*out));
    memset(diag, 0, sizeof(*diag));
    for (size_t i = 0; i < prns.size(); i++) {
        const int p = prns[i];
        const double snr = snr_of[(size_t)p];
        const int k = diag->n++;
        diag->prn[k] = p;
        diag->SNR[k] = snr;
        diag->fbin[k] = p % 29 + 1;
        diag->codePhase[k] = 100 + 7 * p;
        diag->peak[k] = 2 * snr;
        diag->peak2[k] = snr;
        if (snr >= 12) {
            const int a = out->n++;
            out->sv[a] = p;
            out->SNR[a] = snr;
            out->Doppler[a] = -7000 + 500.0 * (double)(p % 29);
            out->codedelay[a] = 1000 * p;
            out->fineFreq[a] = 4.58e6 + (double)p;
        }
    }
}

// the channel loop's status rule over per-channel statuses in channel order (tracking_impl)
static int serial_status(const std::vector<int>& st)
{
    int s = GNSS_OK;
    for (int t : st)
        if (t && (s == GNSS_OK || t == GNSS_ENODATA)) s = t;
    return s;
}

int main()
{
    std::mt19937 rng(6102);
    // deal: every item once, member k gets k, k + m, ...
    for (int n = 0; n < 70; n++)
        for (int m = 1; m <= 9; m++) {
            const auto d = group::deal(n, m);
            std::vector<int> seen((size_t)n, 0);
            CHECK((int)d.size() == m);
            for (int k = 0; k < m; k++)
                for (size_t j = 0; j < d[(size_t)k].size(); j++) {
                    const int i = d[(size_t)k][j];
                    CHECK(i == k + (int)j * m);
                    seen[(size_t)i]++;
                }
            for (int c : seen) CHECK(c == 1);
        }
    // merge_acquired: the members' rows back in list order == the one-context result
    for (int it = 0; it < 2000; it++) {
        const int np = 1 + (int)(rng() % 40), m = 1 + (int)(rng() % 9);
        std::vector<int32_t> prns;
        for (int i = 0; i < np; i++) prns.push_back(it % 2 ? 1 + (int)(rng() % 51) : i + 1);
        std::vector<double> snr(52);
        for (int p = 0; p < 52; p++) snr[(size_t)p] = (double)(rng() % 300) / 10.0;
        gnss_acquired one;
        gnss_acq_diag one_d;
        serial_acq(prns, snr, &one, &one_d);
        const auto shards = group::deal(np, m);
        std::vector<gnss_acquired> outs((size_t)m);
        std::vector<gnss_acq_diag> diags((size_t)m);
        std::vector<int> st((size_t)m);
        for (int k = 0; k < m; k++) {
            std::vector<int32_t> p;
            for (int i : shards[(size_t)k]) p.push_back(prns[(size_t)i]);
            serial_acq(p, snr, &outs[(size_t)k], &diags[(size_t)k]);
            st[(size_t)k] = outs[(size_t)k].n > 0 ? GNSS_OK : GNSS_ENODATA;
        }
        gnss_acquired merged;
        gnss_acq_diag merged_d;
        memset(&merged, 0x7f, sizeof merged);
        CHECK(group::merge_acquired(prns, shards, outs, &diags, &merged, &merged_d));
        CHECK(merged.n == one.n && merged_d.n == one_d.n);
        for (int a = 0; a < one.n; a++) {
            CHECK(merged.sv[a] == one.sv[a] && merged.SNR[a] == one.SNR[a] && merged.Doppler[a] == one.Doppler[a]);
            CHECK(merged.codedelay[a] == one.codedelay[a] && merged.fineFreq[a] == one.fineFreq[a]);
        }
        for (int a = 0; a < one_d.n; a++)
            CHECK(merged_d.prn[a] == one_d.prn[a] && merged_d.fbin[a] == one_d.fbin[a] &&
                  merged_d.codePhase[a] == one_d.codePhase[a] && merged_d.peak2[a] == one_d.peak2[a]);
        CHECK(group::acquisition_status(st, merged.n) == (one.n > 0 ? GNSS_OK : GNSS_ENODATA));
        // a member reporting a PRN it was not given is caught
        if (m > 1 && outs[0].n > 0) {
            outs[0].sv[0] = 99;
            CHECK(!group::merge_acquired(prns, shards, outs, nullptr, &merged, nullptr));
        }
    }
    CHECK(group::acquisition_status({GNSS_ENODATA, GNSS_EIO, GNSS_OK}, 3) == GNSS_EIO);
    // tracking_status: members' (status, first failing channel) == the one-context rule
    for (int it = 0; it < 20000; it++) {
        const int n = 1 + (int)(rng() % 33), m = 1 + (int)(rng() % 9);
        std::vector<int> st((size_t)n, GNSS_OK);
        for (int c = 0; c < n; c++) {
            const unsigned r = rng() % 20;
            st[(size_t)c] = r == 0 ? GNSS_ENODATA : r == 1 ? GNSS_EIO : r == 2 ? GNSS_EINDEX : GNSS_OK;
        }
        const auto shards = group::deal(n, m);
        std::vector<group::TrackStatus> ts;
        for (int k = 0; k < m; k++) {
            std::vector<int> sub;
            int first = -1;
            for (int c : shards[(size_t)k]) {
                sub.push_back(st[(size_t)c]);
                if (st[(size_t)c] && first < 0) first = c;
            }
            ts.push_back({serial_status(sub), first});
        }
        CHECK(group::tracking_status(ts) == serial_status(st));
    }
    // the same with the call's channel list permuted (tr->chan need not be ascending): each
    // member reports the CHANNEL id that failed first, converted to its list position
    // (fail_position); the one-context rule is the first failing channel in LIST order
    for (int it = 0; it < 20000; it++) {
        const int n = 1 + (int)(rng() % 33), m = 1 + (int)(rng() % 9);
        std::vector<int32_t> chans((size_t)n);
        for (int i = 0; i < n; i++) chans[(size_t)i] = i;
        std::shuffle(chans.begin(), chans.end(), rng);
        std::vector<int> st_of((size_t)n, GNSS_OK);  // status by channel id
        for (int c = 0; c < n; c++) {
            const unsigned r = rng() % 12;
            st_of[(size_t)c] = r == 0 ? GNSS_EIO : r == 1 ? GNSS_EINDEX : r == 2 ? GNSS_EDEVICE : GNSS_OK;
        }
        std::vector<int> in_order;
        for (int32_t c : chans) in_order.push_back(st_of[(size_t)c]);
        const auto shards = group::deal(n, m);
        std::vector<group::TrackStatus> ts;
        for (int k = 0; k < m; k++) {
            std::vector<int> sub;
            int fail_chan = -1;
            for (int i : shards[(size_t)k]) {
                const int c = chans[(size_t)i];
                sub.push_back(st_of[(size_t)c]);
                if (st_of[(size_t)c] && fail_chan < 0) fail_chan = c;
            }
            ts.push_back({serial_status(sub), group::fail_position(shards[(size_t)k], chans, fail_chan)});
        }
        CHECK(group::tracking_status(ts) == serial_status(in_order));
    }
    // reciprocal_exact_cached from many threads at once (the group's member threads): one
    // answer per key, equal to the uncached check (run under -fsanitize=thread by the test)
    {
        const double fs[4] = {58e6, 26e6, 38.192e6, 5.714e6};
        std::vector<int> got(32, -1);
        std::vector<std::thread> th;
        for (int t = 0; t < 32; t++)
            th.emplace_back([&, t]() { got[(size_t)t] = group::reciprocal_exact_cached(fs[t % 4], 20000 + 1000 * (t % 4)); });
        for (auto& x : th) x.join();
        for (int t = 0; t < 32; t++) CHECK(got[(size_t)t] == group::reciprocal_exact(fs[t % 4], 20000 + 1000 * (t % 4)));
        CHECK(group::reciprocal_exact(58e6, 600000) == 1);
    }
    // ResidentCache (a member's resident copies of dev_data records): hit only with the same
    // pointer and length; a re-put releases the old copy; writes drop every overlapping record
    {
        int released = 0;
        auto rel = [&](int c) { released += c; };
        group::ResidentCache<int> rc;
        char rec[4096];
        CHECK(rc.find(rec, 1000) == nullptr);
        rc.put(rec, 1000, 7, rel);
        CHECK(rc.find(rec, 1000) && *rc.find(rec, 1000) == 7);
        CHECK(rc.find(rec, 999) == nullptr && rc.find(rec + 1, 1000) == nullptr);
        rc.put(rec, 999, 8, rel);  // same pointer, other length: the old copy is released
        CHECK(released == 7 && rc.m.size() == 1 && *rc.find(rec, 999) == 8);
        rc.put(rec + 2000, 100, 100, rel);
        CHECK(rc.drop_overlapping(rec + 1500, 500, rel) == 0);           // between the two records
        CHECK(rc.drop_overlapping(rec + 2099, 1, rel) == 1 && released == 107);  // the last byte of the second
        CHECK(rc.drop_overlapping(rec + 998, 0, rel) == 1 && released == 115);   // a pointer inside the first
        CHECK(rc.m.empty());
        rc.put(rec, 10, 1, rel);
        rc.put(rec + 10, 10, 2, rel);
        CHECK(rc.drop(rec + 5, rel) == 0 && rc.drop(rec + 10, rel) == 1 && released == 117);
        rc.clear(rel);
        CHECK(rc.m.empty() && released == 118);
    }
    // by_device: first-appearance order, members of a device in order
    {
        const auto g = group::by_device({0, 1, 0, 2, 1, 0});
        CHECK(g.size() == 3);
        CHECK((g[0] == std::vector<int>{0, 2, 5}) && (g[1] == std::vector<int>{1, 4}) && (g[2] == std::vector<int>{3}));
    }
    // combine_timing: durations the slowest member's, counts summed
    {
        gnss_timing a{}, b{};
        a.track_ms = 3;
        b.track_ms = 5;
        a.track_channel_samples = 7;
        b.track_channel_samples = 11;
        const gnss_timing c = group::combine_timing({a, b});
        CHECK(c.track_ms == 5 && c.track_channel_samples == 18);
    }
    printf("mismatches %d\n", bad);
    return bad ? 1 : 0;
}
