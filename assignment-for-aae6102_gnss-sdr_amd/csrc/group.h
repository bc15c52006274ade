// group.h — the bookkeeping of a multi-device context (gnss_ctx_create_multi), host C++ only
// (no HIP: tests/native/group_test.cpp compiles it on the CPU).
//
// The reference runs the PRN loop of acquisition.m:47-80 and the channel loop of
// trackingCT.m:22-528 one item after the other; items share no state (quirk A.11's global
// svindex / nsv aside, which every shard keeps), so a multi-device context deals them
// round-robin over its member contexts and merges the members' results back into the
// caller's arrays in the reference's order. Everything here is that dealing and merging.
#ifndef GNSS_GROUP_H
#define GNSS_GROUP_H

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/gnss_mi355x.h"

namespace gnss {
namespace group {

// items 0..n-1 dealt round-robin over m members: member k gets k, k + m, k + 2m, ...
inline std::vector<std::vector<int>> deal(int n, int m)
{
    std::vector<std::vector<int>> s((size_t)(m > 0 ? m : 0));
    for (int i = 0; i < n && m > 0; i++) s[(size_t)(i % m)].push_back(i);
    return s;
}

// Member results of one acquisition call merged into the reference's output: `prns` is the
// call's PRN list (acquisition.m:47 order), shards[k] the list positions member k searched,
// outs[k] / diags[k] its results (its own PRNs, in its list order). Acquired rows and diag
// rows come out in PRN-list order, as the serial loop appends them (:70-74). Returns false
// if a member's output names a PRN it was not given (a bookkeeping error).
inline bool merge_acquired(const std::vector<int32_t>& prns, const std::vector<std::vector<int>>& shards,
                           const std::vector<gnss_acquired>& outs, const std::vector<gnss_acq_diag>* diags,
                           gnss_acquired* out, gnss_acq_diag* diag)
{
    const size_t m = shards.size();
    std::vector<int> owner(prns.size(), -1);
    for (size_t k = 0; k < m; k++)
        for (int i : shards[k]) owner[(size_t)i] = (int)k;
    std::vector<int> ia(m, 0), id(m, 0);  // next unread row of each member's out / diag
    out->n = 0;
    if (diag) diag->n = 0;
    for (size_t i = 0; i < prns.size(); i++) {
        const int k = owner[i];
        if (k < 0) return false;
        const gnss_acquired& o = outs[(size_t)k];
        if (ia[(size_t)k] < o.n && o.sv[ia[(size_t)k]] == prns[i]) {
            const int r = ia[(size_t)k]++, w = out->n++;
            out->sv[w] = o.sv[r];
            out->SNR[w] = o.SNR[r];
            out->Doppler[w] = o.Doppler[r];
            out->codedelay[w] = o.codedelay[r];
            out->fineFreq[w] = o.fineFreq[r];
        }
        if (diag && diags) {
            const gnss_acq_diag& d = (*diags)[(size_t)k];
            if (id[(size_t)k] >= d.n || d.prn[id[(size_t)k]] != prns[i]) return false;
            const int r = id[(size_t)k]++, w = diag->n++;
            diag->prn[w] = d.prn[r];
            diag->SNR[w] = d.SNR[r];
            diag->fbin[w] = d.fbin[r];
            diag->codePhase[w] = d.codePhase[r];
            diag->peak[w] = d.peak[r];
            diag->peak2[w] = d.peak2[r];
        }
    }
    for (size_t k = 0; k < m; k++)
        if (ia[k] != outs[k].n) return false;  // a row of a PRN the member was not given
    return true;
}

// The status of a sharded acquisition: a member whose PRNs yield nothing returns
// GNSS_ENODATA ("No satellites acquired", acquisition.m:84-85), which holds for the call
// only when the merged result is empty; any other failure is the first member's in order.
inline int acquisition_status(const std::vector<int>& st, int merged_n)
{
    for (int s : st)
        if (s != GNSS_OK && s != GNSS_ENODATA) return s;
    return merged_n > 0 ? GNSS_OK : GNSS_ENODATA;
}

// The status of a sharded tracking call. One context decides it over its channels in
// order (gnss_api.cpp, tracking_impl): GNSS_ENODATA ("Not enough raw data") if any channel
// ran short, else the status of the first failing channel. Member k reports its status and
// the position, in the call's channel list, of the channel that set it (-1: failed before any
// channel ran, i.e. an argument error that every member shares). The same rule over the members' reports gives
// the one-context answer.
struct TrackStatus {
    int status;
    int chan;
};
// A member tracks the channels chans[shard[i]] in shard order and reports the channel id that
// failed first (fail_chan, -1: none); its position in the call's list is what the rule compares.
inline int fail_position(const std::vector<int>& shard, const std::vector<int32_t>& chans, int fail_chan)
{
    for (int i : shard)
        if (chans[(size_t)i] == fail_chan) return i;
    return -1;
}
inline int tracking_status(const std::vector<TrackStatus>& st)
{
    int best = GNSS_OK, best_chan = 0;
    for (const TrackStatus& t : st) {
        if (t.status == GNSS_OK) continue;
        if (t.status == GNSS_ENODATA) return GNSS_ENODATA;
    }
    for (const TrackStatus& t : st) {
        if (t.status == GNSS_OK) continue;
        if (best == GNSS_OK || t.chan < best_chan) {
            best = t.status;
            best_chan = t.chan;
        }
    }
    return best;
}

// CarrTime = k/Fs as the tracking kernels form it (k * RN(1/Fs) plus one FMA correction)
// equals the IEEE quotient for every k in [0, kmax] (exhaustive; gnss_api.cpp caches it per
// (Fs, kmax) behind a mutex, since a group's member threads reach it concurrently).
inline int reciprocal_exact(double Fs, int64_t kmax)
{
    const double y = 1.0 / Fs;
    for (int64_t k = 0; k <= kmax; k++) {
        const double a = (double)k;
        const double q = a * y;
        const double e = std::fma(-q, Fs, a);
        if (std::fma(e, y, q) != a / Fs) return 0;
    }
    return 1;
}

// reciprocal_exact, cached per (Fs, kmax). A multi-device context reaches it from one host
// thread per device (gnss_api.cpp, for_members), so the cache is guarded: the check
// runs outside the lock (a pure function of the key: two threads that miss together compute
// the same answer), the lookup and the insert under it.
inline int reciprocal_exact_cached(double Fs, int64_t kmax)
{
    static std::mutex mu;
    static std::map<std::pair<double, int64_t>, int> cache;
    const auto key = std::make_pair(Fs, kmax);
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    const int ok = reciprocal_exact(Fs, kmax);
    std::lock_guard<std::mutex> lk(mu);
    cache.emplace(key, ok);
    return ok;
}

// A member's resident copies of IF records that live on another device (gnss_file.dev_data on
// devices[0]): one peer copy per record, kept across calls. Keyed by the record's device pointer;
// an entry also holds the record's length (a call naming the same pointer with another length
// re-copies) and the member-side copy (`copy`, owned by the caller: release(copy) frees it). A
// library write into a record's bytes (gnss_dev_upload, gnss_synth_if_device, gnss_dev_free)
// drops every copy that overlaps it; gnss_ctx_drop_record drops one record or all.
template <class Copy>
struct ResidentCache {
    struct Entry {
        uint64_t len;
        Copy copy;
    };
    std::map<uintptr_t, Entry> m;
    // the copy of [key, key + len) if resident with that length, else nullptr
    const Copy* find(const void* key, uint64_t len) const
    {
        auto it = m.find(reinterpret_cast<uintptr_t>(key));
        return it != m.end() && it->second.len == len ? &it->second.copy : nullptr;
    }
    // the entry of `key` (its old copy, if any, released first)
    template <class Release>
    void put(const void* key, uint64_t len, Copy copy, Release release)
    {
        drop(key, release);
        m.emplace(reinterpret_cast<uintptr_t>(key), Entry{len, copy});
    }
    template <class Release>
    int drop(const void* key, Release release)
    {
        auto it = m.find(reinterpret_cast<uintptr_t>(key));
        if (it == m.end()) return 0;
        release(it->second.copy);
        m.erase(it);
        return 1;
    }
    // drop every record whose bytes overlap [p, p + n) (n == 0: the records containing p)
    template <class Release>
    int drop_overlapping(const void* p, uint64_t n, Release release)
    {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = a + (n ? n : 1);
        int k = 0;
        for (auto it = m.begin(); it != m.end();) {
            const uintptr_t lo = it->first, hi = it->first + (it->second.len ? it->second.len : 1);
            if (lo < b && a < hi) {
                release(it->second.copy);
                it = m.erase(it);
                k++;
            } else {
                ++it;
            }
        }
        return k;
    }
    template <class Release>
    void clear(Release release)
    {
        for (auto& kv : m) release(kv.second.copy);
        m.clear();
    }
};

// Timing of a group call: the members ran side by side, so durations are the slowest
// member's and counts are summed.
inline gnss_timing combine_timing(const std::vector<gnss_timing>& t)
{
    gnss_timing r{};
    for (const gnss_timing& x : t) {
        r.acq_ms = std::max(r.acq_ms, x.acq_ms);
        r.acq_corr_ms = std::max(r.acq_corr_ms, x.acq_corr_ms);
        r.acq_fine_ms = std::max(r.acq_fine_ms, x.acq_fine_ms);
        r.track_ms = std::max(r.track_ms, x.track_ms);
        r.track_kernel_ms = std::max(r.track_kernel_ms, x.track_kernel_ms);
        r.track_launches += x.track_launches;
        r.track_channel_samples += x.track_channel_samples;
        r.acq_hypothesis_samples += x.acq_hypothesis_samples;
        r.h2d_ms = std::max(r.h2d_ms, x.h2d_ms);
        r.track10_kernel_ms = std::max(r.track10_kernel_ms, x.track10_kernel_ms);
        r.track10_launches += x.track10_launches;
        r.track10_channel_samples += x.track10_channel_samples;
        r.h2d_bytes += x.h2d_bytes;
        r.track_segments += x.track_segments;
    }
    return r;
}

// Members grouped by device: members on one device run one after the other (two persistent
// tracking grids on one GPU would not both be resident), devices side by side. Returns, per
// distinct device in first-appearance order, the member indices on it.
inline std::vector<std::vector<int>> by_device(const std::vector<int>& devices)
{
    std::vector<int> seen;
    std::vector<std::vector<int>> g;
    for (size_t k = 0; k < devices.size(); k++) {
        auto it = std::find(seen.begin(), seen.end(), devices[k]);
        if (it == seen.end()) {
            seen.push_back(devices[k]);
            g.push_back({(int)k});
        } else {
            g[(size_t)(it - seen.begin())].push_back((int)k);
        }
    }
    return g;
}

}  // namespace group
}  // namespace gnss

#endif
