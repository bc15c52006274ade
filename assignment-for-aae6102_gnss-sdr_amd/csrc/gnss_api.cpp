// gnss_api.cpp — host side of the C-ABI (include/gnss_mi355x.h).
//
// Owns the HIP stream, device buffers, rocFFT plans and step-graphs of one
// device; stages the IF window into HBM once (or uses a caller-resident record)
// and drives the kernels in track.hip / acq.hip. Orchestration mirrors the
// reference's control flow:
//   acquisition.m  : read block -> PRN search -> threshold -> fine frequency
//   trackingCT.m   : phase A (1 ms) -> bit-edge search -> phase B (= A continued,
//                    quirk A.9) -> phase C (10 ms) per channel, channels batched.
#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <functional>
#include <thread>
#include <vector>
#include <fcntl.h>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <unistd.h>
#include <vector>

#include "gnss_internal.h"
#include "group.h"

using namespace gnss;

struct gnss_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;       // the acquisition's row passes beside the column passes
    hipEvent_t ev_cols[2] = {}, ev_rows[2] = {};  // their hand-offs, per intermediate buffer
    std::string err;
    gnss_timing timing{};
    int profiling = 0;
    std::map<std::tuple<size_t, size_t, int, int>, rocfft_plan> plans;
    void* fft_work = nullptr;
    size_t fft_work_size = 0;
    // device scratch kept across calls (hipMalloc/hipFree per call cost ~1 ms and hipFree
    // synchronises): name -> (pointer, bytes)
    std::map<std::string, std::pair<void*, size_t>> pool;
    // pinned host staging kept across calls (the per-step records' download): name ->
    // (pointer, bytes); a pageable std::vector re-faults and bounces every call
    std::map<std::string, std::pair<void*, size_t>> pinned;
    int64_t acq_tw_S = 0;  // the acquisition twiddle tables in the pool are for this S
    int acq_tw_dbl = -1;   //   ... and this precision
    int acq_fp64 = 1;      // acquisition correlation precision: 1 = fp64 (reference), 0 = fp32
    uint64_t window = 0;   // trackingCT: max IF bytes resident in HBM (0: the whole read range)
    int64_t opt[GNSS_OPT_COUNT] = {};  // gnss_ctx_set_option (test hooks; all 0 by default)
    // multi-device context (gnss_ctx_create_multi): the member contexts (empty: a plain one);
    // the group itself is also a context on devices[0], for the entry points that do not shard
    std::vector<gnss_ctx*> members;
    bool member = false;  // a group's member: dev_data on another device is copied in (xGMI)
    int fail_chan = -1;   // tracking: the channel whose status the last call returned (group.h)
    // (a member) its resident copies of dev_data records on another device: one peer copy per
    // record, kept across calls (group.h ResidentCache; the copy is a hipMalloc of this device)
    gnss::group::ResidentCache<void*> resident;
};

// frees a member's resident record copy (on that member's device)
static void release_resident(void* p)
{
    if (p) (void)hipFree(p);
}

// drops the resident copies of every member of ctx that overlap [p, p + n) (n == 0: the records
// containing p; p == nullptr: all of them); returns how many were dropped
static int drop_resident(gnss_ctx* ctx, const void* p, uint64_t n)
{
    int k = 0;
    for (gnss_ctx* m : ctx->members) {
        (void)hipSetDevice(m->device);
        if (m->stream) (void)hipStreamSynchronize(m->stream);  // (no kernel still reads a copy)
        if (!p) {
            k += (int)m->resident.m.size();
            m->resident.clear(release_resident);
        } else {
            k += m->resident.drop_overlapping(p, n, release_resident);
        }
    }
    (void)hipSetDevice(ctx->device);
    return k;
}

// Timing-probe hooks read from the environment in probe builds only (tools/build_probe.sh
// passes -DGNSS_PROBE_BUILD=1); the product library reads no environment variable.
#ifndef GNSS_PROBE_BUILD
#define GNSS_PROBE_BUILD 0
#endif
static const char* probe_env(const char* name)
{
    return GNSS_PROBE_BUILD ? getenv(name) : nullptr;
}

namespace {
// The acquisition's split correlator pipelines its batches over two streams by default
// (GNSS_OPT_ACQ_PIPE; config-2 fp64 correlation 10.10-10.18 -> 9.75-9.88 ms on MI355X,
// profiles/r03_ab_acq_pipe.txt).
constexpr int kAcqPipeDefault = 2;
// the pipeline's forward spectra in bin chunks, each before the first column pass that reads it
#ifndef GNSS_ACQ_FWD_SPLIT
#define GNSS_ACQ_FWD_SPLIT 1
#endif
constexpr bool kAcqFwdSplit = GNSS_ACQ_FWD_SPLIT;
// the paired launch's row blocks sit in the grid's first kAcqPairFront percent (acq_fft.hip)
constexpr int kAcqPairFront = 60;
// steps of gnss_tracking_vt per staged IF window of a host record (GNSS_OPT_VT_SPAN: fewer)
constexpr int kVtSpan = 2000;
// SVs per launch of the fine-frequency search (scratch ~186 MB per SV at config 2)
constexpr int kFineBatch = 16;

// The context's pinned host buffer `key`, at least `bytes` (contents undefined).
// (`flags`: hipHostMalloc's; a key is always asked for with the same flags)
template <class T>
T* pinned_buffer(gnss_ctx* ctx, const char* key, size_t count, unsigned flags = hipHostMallocDefault)
{
    auto& e = ctx->pinned[key];
    const size_t want = std::max<size_t>(count * sizeof(T), 16);
    if (e.second < want) {
        if (e.first) (void)hipHostFree(e.first);
        e = {nullptr, 0};
        if (hipHostMalloc(&e.first, want, flags) != hipSuccess) return nullptr;
        e.second = want;
    }
    return static_cast<T*>(e.first);
}
}  // namespace

namespace {

int fail(gnss_ctx* ctx, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(gnss_ctx* ctx, int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(ctx, GNSS_EDEVICE, "%s:%d %s: %s", __FILE__, __LINE__, #expr,          \
                        hipGetErrorString(e_));                                                \
    } while (0)

// RAII device buffer
struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    bool pooled = false;  // borrowed from the context's pool: not freed here
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release()
    {
        if (p && !pooled) (void)hipFree(p);
        p = nullptr;
        pooled = false;
    }
    hipError_t alloc(size_t bytes)
    {
        release();
        n = bytes;
        return hipMalloc(&p, bytes ? bytes : 16);
    }
    // The context's buffer `key` (grown when too small; contents undefined, as hipMalloc).
    // One key per live buffer; calls on a context are serialised on its stream.
    hipError_t alloc(gnss_ctx* ctx, const char* key, size_t bytes)
    {
        release();
        auto& e = ctx->pool[key];
        const size_t want = bytes ? bytes : 16;
        if (e.second < want) {
            if (e.first) (void)hipFree(e.first);
            e = {nullptr, 0};
            const hipError_t r = hipMalloc(&e.first, want);
            if (r != hipSuccess) {
                e.first = nullptr;
                return r;
            }
            e.second = want;
        }
        p = e.first;
        n = bytes;
        pooled = true;
        return hipSuccess;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// f(0..n-1) over up to 16 host threads (the output expansion writes tens of MB into
// fresh pages; one thread is bound by page faults and a single core's bandwidth).
template <class F>
void parallel_for(int n, F f)
{
    const int nt = std::max(1, std::min({n, 16, (int)std::thread::hardware_concurrency()}));
    if (nt <= 1) {
        for (int i = 0; i < n; i++) f(i);
        return;
    }
    std::vector<std::thread> th;
    th.reserve((size_t)nt);
    for (int t = 0; t < nt; t++)
        th.emplace_back([&, t]() {
            for (int i = t; i < n; i += nt) f(i);
        });
    for (auto& x : th) x.join();
}

struct Events {
    hipEvent_t a = nullptr, b = nullptr;
    Events() { (void)hipEventCreate(&a); (void)hipEventCreate(&b); }
    ~Events() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
    double ms() const { float f = 0; (void)hipEventElapsedTime(&f, a, b); return f; }
};

int64_t file_length(const gnss_file* f)
{
    if (f->dev_data || f->data) return (int64_t)f->nbytes;
    if (!f->path) return -1;
    int fd = open(f->path, O_RDONLY);
    if (fd < 0) return -1;
    int64_t s = lseek(fd, 0, SEEK_END);
    close(fd);
    return s;
}

// The IF bytes [lo, hi) resident in HBM; base = file byte at ptr[0] (16-B aligned).
struct IfWindow {
    DevBuf own;
    const int8_t* ptr = nullptr;
    int64_t base = 0, len = 0;
};

// The file bytes [lo, hi) into device memory dst (returns once they have landed). Streaming staging (trackingCT.m:84-93 reads each step's block from the file;
// here windows are staged whole): chunks of kStageChunk bytes through two pinned host buffers
// of the context -- the disk read (or host copy) of chunk i+1 runs while the DMA engine moves
// chunk i into HBM; a buffer is refilled only after its previous DMA has completed.
int stage_into(gnss_ctx* ctx, const gnss_file* f, int64_t lo, int64_t hi, int8_t* dst)
{
    const int64_t n = hi - lo;
    if (n <= 0) return GNSS_OK;
    Events ev;
    HIP_TRY(hipEventRecord(ev.a, ctx->stream));
    constexpr int64_t kStageChunk = (int64_t)64 << 20;
    int8_t* pb[2] = {pinned_buffer<int8_t>(ctx, "stage.0", (size_t)kStageChunk),
                     pinned_buffer<int8_t>(ctx, "stage.1", (size_t)kStageChunk)};
    if (!pb[0] || !pb[1]) return fail(ctx, GNSS_EDEVICE, "pinned staging buffers");
    hipEvent_t done[2] = {nullptr, nullptr};
    HIP_TRY(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
    struct EvGuard {
        hipEvent_t* e;
        ~EvGuard() { (void)hipEventDestroy(e[0]); (void)hipEventDestroy(e[1]); }
    } guard{done};
    // the descriptor is closed on every return; an early return (a failed HIP call or a short
    // read) first drains the stream, so no DMA still reads a pinned buffer the next call refills
    struct FdGuard {
        int fd;
        hipStream_t s;
        bool drained;
        ~FdGuard()
        {
            if (fd >= 0) close(fd);
            if (!drained) (void)hipStreamSynchronize(s);
        }
    } fg{-1, ctx->stream, false};
    if (!f->data) {
        fg.fd = open(f->path, O_RDONLY);
        if (fg.fd < 0) return fail(ctx, GNSS_EIO, "cannot open '%s'", f->path);
    }
    const int fd = fg.fd;
    int64_t off = 0;
    for (int i = 0; off < n; i++, off += kStageChunk) {
        const int64_t len = std::min(kStageChunk, n - off);
        int8_t* buf = pb[i & 1];
        if (i >= 2) HIP_TRY(hipEventSynchronize(done[i & 1]));  // its last DMA has drained
        if (f->data) {
            memcpy(buf, f->data + lo + off, (size_t)len);
        } else {
            int64_t got = 0;
            while (got < len) {
                const ssize_t r = pread(fd, buf + got, (size_t)(len - got), lo + off + got);
                if (r <= 0) break;
                got += r;
            }
            if (got != len) return fail(ctx, GNSS_EIO, "short read of '%s'", f->path);
        }
        HIP_TRY(hipMemcpyAsync(dst + off, buf, (size_t)len, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipEventRecord(done[i & 1], ctx->stream));
    }
    ctx->timing.h2d_bytes += n;
    HIP_TRY(hipEventRecord(ev.b, ctx->stream));
    HIP_TRY(hipEventSynchronize(ev.b));
    fg.drained = true;
    ctx->timing.h2d_ms += ev.ms();
    return GNSS_OK;
}

// The HIP device a device pointer belongs to (-1 if HIP does not know it).
int pointer_device(const void* p)
{
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return a.device;
}

int stage_window(gnss_ctx* ctx, const gnss_file* f, int64_t lo, int64_t hi, IfWindow& w)
{
    const int64_t flen = file_length(f);
    if (flen < 0) return fail(ctx, GNSS_EIO, "cannot open IF record '%s'", f->path ? f->path : "");
    lo = std::max<int64_t>(0, lo & ~(int64_t)15);
    hi = std::min<int64_t>(hi, flen);
    if (hi <= lo) { hi = lo; }
    if (f->dev_data) {
        if ((reinterpret_cast<uintptr_t>(f->dev_data) & 15) != 0)
            return fail(ctx, GNSS_EARG, "dev_data must be 16-byte aligned");
        const int pd = ctx->member ? pointer_device(f->dev_data) : ctx->device;
        if (pd == ctx->device && !(ctx->member && ctx->opt[GNSS_OPT_FORCE_PEER])) {
            w.ptr = static_cast<const int8_t*>(f->dev_data);
            w.base = 0;
            w.len = flen;
            return GNSS_OK;
        }
        // a group member whose record lives on another device of the node (devices[0]): the
        // whole record into this device's HBM by one peer copy over xGMI, on the first call that
        // reads it; it stays resident for the later calls (group.h ResidentCache) until the
        // library writes into the record or the caller drops it (gnss_ctx_drop_record)
        const void* const* hit = ctx->resident.find(f->dev_data, (uint64_t)flen);
        if (!hit) {
            void* copy = nullptr;
            HIP_TRY(hipMalloc(&copy, (size_t)flen + 64));
            Events ev;
            HIP_TRY(hipEventRecord(ev.a, ctx->stream));
            if (flen > 0 && hipMemcpyPeerAsync(copy, ctx->device, f->dev_data, pd < 0 ? ctx->device : pd,
                                               (size_t)flen, ctx->stream) != hipSuccess) {
                (void)hipStreamSynchronize(ctx->stream);
                (void)hipFree(copy);
                return fail(ctx, GNSS_EDEVICE, "peer copy of the IF record (%lld bytes)", (long long)flen);
            }
            HIP_TRY(hipEventRecord(ev.b, ctx->stream));
            HIP_TRY(hipEventSynchronize(ev.b));
            ctx->timing.h2d_bytes += flen;
            ctx->timing.h2d_ms += ev.ms();
            ctx->resident.put(f->dev_data, (uint64_t)flen, copy, release_resident);
            hit = ctx->resident.find(f->dev_data, (uint64_t)flen);
        }
        w.ptr = static_cast<const int8_t*>(*hit);
        w.base = 0;
        w.len = flen;
        return GNSS_OK;
    }
    const int64_t n = hi - lo;
    HIP_TRY(w.own.alloc((size_t)n + 64));
    const int st = stage_into(ctx, f, lo, hi, w.own.as<int8_t>());
    if (st) return st;
    w.ptr = w.own.as<int8_t>();
    w.base = lo;
    w.len = n;
    return GNSS_OK;
}

int get_plan(gnss_ctx* ctx, size_t len, size_t batch, int dbl, int inverse, rocfft_plan* out)
{
    auto key = std::make_tuple(len, batch, dbl, inverse);
    auto it = ctx->plans.find(key);
    if (it != ctx->plans.end()) { *out = it->second; return GNSS_OK; }
    rocfft_plan plan = nullptr;
    rocfft_status st = rocfft_plan_create(
        &plan, rocfft_placement_inplace,
        inverse ? rocfft_transform_type_complex_inverse : rocfft_transform_type_complex_forward,
        dbl ? rocfft_precision_double : rocfft_precision_single, 1, &len, batch, nullptr);
    if (st != rocfft_status_success)
        return fail(ctx, GNSS_EDEVICE, "rocfft_plan_create(len=%zu, batch=%zu) failed: %d", len, batch, (int)st);
    size_t ws = 0;
    rocfft_plan_get_work_buffer_size(plan, &ws);
    if (ws > ctx->fft_work_size) {
        if (ctx->fft_work) (void)hipFree(ctx->fft_work);
        ctx->fft_work = nullptr;
        HIP_TRY(hipMalloc(&ctx->fft_work, ws));
        ctx->fft_work_size = ws;
    }
    ctx->plans[key] = plan;
    *out = plan;
    return GNSS_OK;
}

int run_fft(gnss_ctx* ctx, void* data, size_t len, size_t batch, int dbl, int inverse)
{
    rocfft_plan plan;
    int st = get_plan(ctx, len, batch, dbl, inverse, &plan);
    if (st) return st;
    rocfft_execution_info info = nullptr;
    rocfft_execution_info_create(&info);
    rocfft_execution_info_set_stream(info, ctx->stream);
    if (ctx->fft_work_size) rocfft_execution_info_set_work_buffer(info, ctx->fft_work, ctx->fft_work_size);
    void* bufs[1] = {data};
    rocfft_status rs = rocfft_execute(plan, bufs, nullptr, info);
    rocfft_execution_info_destroy(info);
    if (rs != rocfft_status_success) return fail(ctx, GNSS_EDEVICE, "rocfft_execute failed: %d", (int)rs);
    return GNSS_OK;
}

// The kernels form CarrTime = k/Fs (trackingCT.m:104) as q = k*RN(1/Fs) corrected by
// one FMA; that equals the IEEE quotient for every k we check here (exhaustive over
// the step's sample range, cached per Fs). Otherwise they divide.
int fast_div_exact(double Fs, int64_t kmax) { return group::reciprocal_exact_cached(Fs, kmax); }

void generate_ca(int prn, float* out);

// C/A chips as 32 words of bits (bit i set <-> chip i is -1), read by the kernels
// through lane shuffles
void ca_bits(int prn, unsigned* out32)
{
    float f[1023];
    generate_ca(prn, f);
    for (int w = 0; w < 32; w++) out32[w] = 0;
    for (int i = 0; i < 1023; i++)
        if (f[i] < 0) out32[i >> 5] |= 1u << (i & 31);
}

// generateCAcode.m:16-64 (host copy; the oracle has its own independent one)
void generate_ca(int prn, float* out)
{
    static const int g2s[51] = {5,   6,   7,   8,   17,  18,  139, 140, 141, 251, 252, 254, 255,
                                256, 257, 258, 469, 470, 471, 472, 473, 474, 509, 512, 513, 514,
                                515, 516, 859, 860, 861, 862, 145, 175, 52,  21,  237, 235, 886,
                                657, 634, 762, 355, 1012, 176, 603, 130, 359, 595, 68,  386};
    int g1[1023], g2[1023];
    unsigned r1 = 0x3FF, r2 = 0x3FF;  // bit i = stage i+1, all stages start at "-1" (= 1 here)
    for (int i = 0; i < 1023; i++) {
        g1[i] = (r1 >> 9) & 1;
        g2[i] = (r2 >> 9) & 1;
        unsigned f1 = ((r1 >> 2) ^ (r1 >> 9)) & 1;
        unsigned f2 = ((r2 >> 1) ^ (r2 >> 2) ^ (r2 >> 5) ^ (r2 >> 7) ^ (r2 >> 8) ^ (r2 >> 9)) & 1;
        r1 = ((r1 << 1) | f1) & 0x3FF;
        r2 = ((r2 << 1) | f2) & 0x3FF;
    }
    // +-1 product of "-1" states == XOR of bits; CA = -(g1 .* g2) -> +1 when bits differ... in
    // the reference's -1 -> bit 1 mapping: value(x) = -1 if bit 1 else +1.
    const int s = g2s[prn - 1];
    for (int i = 0; i < 1023; i++) {
        const int src = (i < s) ? (1023 - s + i) : (i - s);
        const int v1 = g1[i] ? -1 : 1, v2 = g2[src] ? -1 : 1;
        out[i] = (float)(-(v1 * v2));
    }
}

}  // namespace

namespace {
template <class V> struct CplxReal;
template <> struct CplxReal<float2> { using T = float; };
template <> struct CplxReal<double2> { using T = double; };

// The PRN x bin x ms search of acquisition.m:47-61 into corr[p][bin][.] (sum over the ms of
// |ifft(fft(code) .* conj(fft(signal .* carrier)))|^2), V = float2 (fast mode) or double2
// (the reference's precision): the own P x 2000 FFT correlator (acq_fft.hip) where S = P * 2000,
// batched rocFFT otherwise. e_all.a is recorded when the timed work starts; *perm = P for
// the own correlator's tau2-major surface, 0 for natural order.
template <class V>
int acq_search(gnss_ctx* ctx, const int8_t* blk, const double2* xa, int64_t S, int dl, int nb, int np,
               const gnss_signal* sg, const gnss_acq* acq, const float* ca, typename CplxReal<V>::T* corr,
               Events& e_all, int* perm, DevBuf& fsync)
{
    const int dbl = sizeof(V) == sizeof(double2) ? 1 : 0;
    const size_t csz = sizeof(V);
    const int nsig = dl * nb;
    int st = GNSS_OK;
    if (acq_fft_supported(S) && !ctx->opt[GNSS_OPT_ACQ_ROCFFT]) {
        DevBuf d_twr, d_twc, B, X, A;  // (freed after the stream drains)
        const int P = (int)(S / 2000);
        *perm = P;
        // twiddles (fp64 on the host; rounded to fp32 in the fast mode), kept in the
        // context per S and precision
        const bool have_tw = ctx->acq_tw_S == S && ctx->acq_tw_dbl == dbl;
        HIP_TRY(d_twr.alloc(ctx, "acq.d_twr", 2000 * csz));
        HIP_TRY(d_twc.alloc(ctx, "acq.d_twc", (size_t)P * 2000 * csz));
        if (!have_tw) {
            std::vector<V> twr(2000), twc((size_t)P * 2000);
            for (int m = 0; m < 2000; m++) {
                const double a = -2.0 * M_PI * (double)m / 2000.0;
                twr[m].x = std::cos(a);
                twr[m].y = std::sin(a);
            }
            for (int m = 0; m < P; m++)
                for (int k = 0; k < 2000; k++) {
                    const double a = -2.0 * M_PI * (double)((int64_t)m * k % S) / (double)S;
                    twc[(size_t)m * 2000 + k].x = std::cos(a);
                    twc[(size_t)m * 2000 + k].y = std::sin(a);
                }
            HIP_TRY(hipMemcpyAsync(d_twr.p, twr.data(), twr.size() * csz, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(hipMemcpyAsync(d_twc.p, twc.data(), twc.size() * csz, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));  // (the host vectors go out of scope)
            ctx->acq_tw_S = S;
            ctx->acq_tw_dbl = dbl;
        }
        const size_t ntr = (size_t)nsig + np;
        HIP_TRY(B.alloc(ctx, "acq.B", csz * ntr * S));
        HIP_TRY(X.alloc(ctx, "acq.X", csz * ntr * S));
        const int npairs = nb * np;
        if (dbl && ctx->opt[GNSS_OPT_ACQ_FUSED]) {
            // fp64: one persistent launch, the intermediate in each XCD's L2 (acq_fft.hip);
            // the caller reads fsync's error word once the stream has drained
            DevBuf ring;
            const int nslot = ctx->opt[GNSS_OPT_ACQ_RING] ? (int)ctx->opt[GNSS_OPT_ACQ_RING] : 3;
            HIP_TRY(ring.alloc(ctx, "acq.ring", acq_fused_ring_bytes(S)));
            HIP_TRY(fsync.alloc(ctx, "acq.fsync", acq_fused_sync_bytes()));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            HIP_TRY(hipEventRecord(e_all.a, ctx->stream));
            HIP_TRY(launch_acq_fft_forward<V>(blk, xa, S, dl, nb, sg->IF, acq->freqMin, acq->freqStep, sg->Fs, ca,
                                              np, sg->codeFreqBasis, d_twr.as<V>(), d_twc.as<V>(), B.as<V>(),
                                              X.as<V>(), ctx->stream));
            const V* C = X.as<V>() + (size_t)nsig * S;
            HIP_TRY(launch_acq_fft_correlate_fused(reinterpret_cast<const double2*>(C), X.as<double2>(), S, dl, nb,
                                                   np, nslot, d_twr.as<double2>(), d_twc.as<double2>(),
                                                   ring.as<double2>(), fsync.p, reinterpret_cast<double*>(corr),
                                                   ctx->stream));
            return GNSS_OK;
        }
        // (bin, PRN) pairs per batch: the inverse intermediate leaves the L2 either way (PMC
        // FETCH / WRITE, which count Infinity-Cache hits too, profiles/acq_traffic_r01.json),
        // and smaller batches measured slower, so batches of ~1 GiB, balanced (no
        // small tail batch that leaves the chip idle): config 2 (fp32) measured 7.94 ms of
        // correlation at 28 pairs per batch (256 MB), 7.09-7.29 at 112, 7.15-7.30 at 232
        // (tools/gpu_acq_batch.sh). Pairs are independent: the bits do not depend on it.
        const int target = (int)std::max<int64_t>(1, ((int64_t)1 << 30) / ((int64_t)dl * S * (int64_t)csz));
        const int nbat = (npairs + target - 1) / target;
        int batch = (npairs + nbat - 1) / nbat;
        // the test hook, clamped before the narrowing (2^32 would become 0)
        if (ctx->opt[GNSS_OPT_ACQ_BATCH] > 0)
            batch = (int)std::min<int64_t>(ctx->opt[GNSS_OPT_ACQ_BATCH], (int64_t)npairs);
        batch = std::max(1, std::min(batch, npairs));
        // Two streams: batch b's row pass (LDS-bound fp64 transforms, reading the intermediate)
        // runs beside batch b+1's column pass (bound by the intermediate's writes), each batch
        // in its own half of a double intermediate; the column pass of b+2 waits for the rows
        // of b. Every pair is in one batch and its corr entries are written by its row pass
        // alone, so the surface is bit-identical to the one-stream order.
        // Paired launches (fp64, = 3): one launch per batch boundary holding batch b's column
        // blocks and batch b-1's row blocks interleaved, so the two passes share every CU.
        const int64_t pipe = ctx->opt[GNSS_OPT_ACQ_PIPE] ? ctx->opt[GNSS_OPT_ACQ_PIPE] : kAcqPipeDefault;
        const bool pair = dbl && pipe == 3 && npairs > batch;
        const bool two = (pipe == 2 || (pipe == 3 && !dbl)) && npairs > batch;
        hipStream_t s_cols = ctx->stream, s_rows = ctx->stream2;
        const size_t abuf = (size_t)batch * dl * S;
        HIP_TRY(A.alloc(ctx, "acq.A", csz * abuf * (two || pair ? 2 : 1)));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        HIP_TRY(hipEventRecord(e_all.a, ctx->stream));
        // the forward spectra: all at once, or (the two-stream pipeline, GNSS_ACQ_FWD_SPLIT) the
        // codes and the bins batch 0 reads first and each later batch's new bins just before its
        // column pass, on the column stream, where they run beside the previous batch's row pass
        // (the column stream waits on the rows anyway); every spectrum is the same transform of the
        // same data, so the bits do not change
        const bool fwd_split = kAcqFwdSplit && two;
        auto fwd = [&](int bin0, int nbc, bool codes) {
            return launch_acq_fft_forward<V>(blk, xa, S, dl, nb, sg->IF, acq->freqMin, acq->freqStep, sg->Fs, ca, np,
                                             sg->codeFreqBasis, d_twr.as<V>(), d_twc.as<V>(), B.as<V>(), X.as<V>(),
                                             ctx->stream, bin0, nbc, codes);
        };
        int fwd_bins = 0;  // bins [0, fwd_bins) transformed so far
        if (fwd_split) {
            const int need = std::min(nb, (std::min(batch, npairs) - 1) / np + 1);
            HIP_TRY(fwd(0, need, true));
            fwd_bins = need;
        } else {
            HIP_TRY(fwd(0, -1, true));
            fwd_bins = nb;
        }
        const V* C = X.as<V>() + (size_t)nsig * S;
        if (pair) {
            const char* fe = probe_env("GNSS_PAIR_FRONT");  // (probe builds: the A/B knob)
            const int front = fe ? atoi(fe) : kAcqPairFront;
            const int nbt = (npairs + batch - 1) / batch;
            double2* Ah[2] = {reinterpret_cast<double2*>(A.p), reinterpret_cast<double2*>(A.p) + abuf};
            for (int b = 0; b <= nbt; b++) {
                const int cq = b * batch, rq = (b - 1) * batch;
                const int nc = b < nbt ? std::min(batch, npairs - cq) : 0;
                const int nr = b > 0 ? std::min(batch, npairs - rq) : 0;
                HIP_TRY(launch_acq_fft_pair(reinterpret_cast<const double2*>(C), X.as<double2>(), S, dl, nb, np, cq,
                                            nc, Ah[b & 1], rq, nr, Ah[(b + 1) & 1], d_twr.as<double2>(),
                                            d_twc.as<double2>(), reinterpret_cast<double*>(corr), front,
                                            ctx->stream));
            }
            return GNSS_OK;
        }
        if (!two) {
            for (int q0 = 0; q0 < npairs; q0 += batch) {
                const int nq = std::min(batch, npairs - q0);
                HIP_TRY(launch_acq_fft_correlate(C, X.as<V>(), S, dl, nb, np, q0, nq, d_twr.as<V>(),
                                                 d_twc.as<V>(), A.as<V>(), corr, ctx->stream));
            }
            return GNSS_OK;
        }
        // A launch error part way leaves row passes queued on stream2 that still write acq.A /
        // corr: drain it before the error returns, so the next call's pooled buffers are free.
        auto pipelined = [&]() -> int {
            int last = 0;
            for (int q0 = 0, b = 0; q0 < npairs; q0 += batch, b++) {
                const int nq = std::min(batch, npairs - q0);
                const int h = b & 1;
                V* Ah = A.as<V>() + (size_t)h * abuf;
                if (fwd_split) {  // this batch's bins not transformed yet (pairs q0 .. q0 + nq - 1)
                    const int need = std::min(nb, (q0 + nq - 1) / np + 1);
                    if (need > fwd_bins) HIP_TRY(fwd(fwd_bins, need - fwd_bins, false));
                    fwd_bins = std::max(fwd_bins, need);
                }
                if (b >= 2) HIP_TRY(hipStreamWaitEvent(s_cols, ctx->ev_rows[h], 0));  // rows of b-2 read Ah
                HIP_TRY(launch_acq_fft_correlate(C, X.as<V>(), S, dl, nb, np, q0, nq, d_twr.as<V>(), d_twc.as<V>(),
                                                 Ah, corr, s_cols, kAcqCols));
                HIP_TRY(hipEventRecord(ctx->ev_cols[h], s_cols));
                HIP_TRY(hipStreamWaitEvent(s_rows, ctx->ev_cols[h], 0));
                HIP_TRY(launch_acq_fft_correlate(C, X.as<V>(), S, dl, nb, np, q0, nq, d_twr.as<V>(), d_twc.as<V>(),
                                                 Ah, corr, s_rows, kAcqRows));
                HIP_TRY(hipEventRecord(ctx->ev_rows[h], s_rows));
                last = h;
            }
            // the caller's stream owns the result again (stream2 is in order: its last event covers all)
            HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_rows[last], 0));
            return GNSS_OK;
        };
        const int pst = pipelined();
        if (pst != GNSS_OK) (void)hipStreamSynchronize(s_rows);
        return pst;
    }
    // batched rocFFT (sample counts that are not P x 2000)
    *perm = 0;
    DevBuf sig, code, y;
    HIP_TRY(sig.alloc(ctx, "acq.sig", csz * (size_t)nsig * S));
    HIP_TRY(code.alloc(ctx, "acq.code", csz * (size_t)np * S));
    // PRN chunk so the product/IFFT buffer stays <= ~4 GB
    const size_t per_prn = csz * (size_t)nsig * S;
    const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)np, ((size_t)4 << 30) / per_prn));
    HIP_TRY(y.alloc(ctx, "acq.y", per_prn * (size_t)chunk));
    // plans outside the timed region
    rocfft_plan pl;
    if ((st = get_plan(ctx, S, nsig, dbl, 0, &pl))) return st;
    if ((st = get_plan(ctx, S, np, dbl, 0, &pl))) return st;
    for (int p0 = 0; p0 < np; p0 += chunk) {
        const int pc = std::min(chunk, np - p0);
        if ((st = get_plan(ctx, S, (size_t)pc * nsig, dbl, 1, &pl))) return st;
    }
    HIP_TRY(hipEventRecord(e_all.a, ctx->stream));
    HIP_TRY(launch_acq_wipe(blk, xa, S, dl, nb, sg->IF, acq->freqMin, acq->freqStep, sg->Fs, sig.as<V>(), ctx->stream));
    if ((st = run_fft(ctx, sig.p, S, nsig, dbl, 0))) return st;
    HIP_TRY(launch_acq_code(ca, nullptr, np, S, sg->codeFreqBasis, sg->Fs, code.as<V>(), ctx->stream));
    if ((st = run_fft(ctx, code.p, S, np, dbl, 0))) return st;
    for (int p0 = 0; p0 < np; p0 += chunk) {
        const int pc = std::min(chunk, np - p0);
        HIP_TRY(launch_acq_mul(code.as<V>() + (size_t)p0 * S, sig.as<V>(), pc, nsig, S, y.as<V>(), ctx->stream));
        if ((st = run_fft(ctx, y.p, S, (size_t)pc * nsig, dbl, 1))) return st;
        HIP_TRY(launch_acq_power(y.as<V>(), pc, nb, dl, S, 0, corr + (size_t)p0 * nb * S, ctx->stream));
    }
    return GNSS_OK;
}
}  // namespace

// The sibling loop of trackingCT_POS_updated.m (its tracking half): steps and countinx.
struct PosCfg {
    int32_t ctPOS;            // track.ctPOS (datalength, trackingCT_POS_updated.m:50)
    const int32_t* countinx;  // countinx(svIndex) of countinx.mat (:29), by channel position
    // 0: trackingCT_POS_updated.m. 1 or 10: trackingCT_POS_updated_multicorrelator.m, every
    // step at this pdi (track.pdi, :46), 25 taps, ctPOS = datalength/pdi steps (:170)
    int32_t mc_pdi;
};

// trackingCT_multiCorr-GIVEN.m (function trackingCT_multiCorr): `datalength` 1-ms steps
// per channel (:27, hard-coded 50000 there), trackingCT conventions otherwise
struct GivenCfg {
    int32_t datalength;
};

// ---------------------------------------------------------------------------
// Multi-device contexts (gnss_ctx_create_multi): the group's member contexts run their
// shards side by side, one host thread per device (group.h has the dealing and merging).
// ---------------------------------------------------------------------------
namespace {

template <class F>
void for_members(gnss_ctx* g, F fn)
{
    std::vector<int> devs;
    for (gnss_ctx* m : g->members) devs.push_back(m->device);
    std::vector<std::thread> th;
    for (const std::vector<int>& ks : group::by_device(devs))
        th.emplace_back([&fn, ks]() {
            for (int k : ks) fn(k);
        });
    for (auto& t : th) t.join();
}

}  // namespace

extern "C" int gnss_acquisition(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg,
                                const gnss_acq* acq, gnss_acquired* out, gnss_acq_diag* diag);

// acquisition.m's PRN loop (:47-80) dealt over the members; Acquired / diag merged in list order
static int group_acquisition(gnss_ctx* g, const gnss_file* file, const gnss_signal* sg, const gnss_acq* acq,
                             gnss_acquired* out, gnss_acq_diag* diag)
{
    if (!file || !sg || !acq || !out) return GNSS_EARG;
    memset(out, 0, sizeof(*out));
    if (diag) memset(diag, 0, sizeof(*diag));
    g->timing = gnss_timing{};
    std::vector<int32_t> prns;
    if (acq->n_prn > 0 && acq->prn_list) prns.assign(acq->prn_list, acq->prn_list + acq->n_prn);
    else for (int i = 1; i <= 32; i++) prns.push_back(i);  // acquisition.m:47
    if (prns.size() > GNSS_MAX_SV) return fail(g, GNSS_EARG, "too many PRNs");
    const int M = (int)g->members.size();
    const auto shards = group::deal((int)prns.size(), M);
    std::vector<std::vector<int32_t>> plist((size_t)M);
    for (int k = 0; k < M; k++)
        for (int i : shards[(size_t)k]) plist[(size_t)k].push_back(prns[(size_t)i]);
    std::vector<gnss_acquired> outs((size_t)M);
    std::vector<gnss_acq_diag> diags((size_t)M);
    std::vector<int> st((size_t)M, GNSS_ENODATA);
    std::vector<char> ran((size_t)M, 0);
    for_members(g, [&](int k) {
        memset(&outs[(size_t)k], 0, sizeof(gnss_acquired));
        memset(&diags[(size_t)k], 0, sizeof(gnss_acq_diag));
        if (plist[(size_t)k].empty()) return;  // (more members than PRNs)
        gnss_acq a = *acq;
        a.n_prn = (int32_t)plist[(size_t)k].size();
        a.prn_list = plist[(size_t)k].data();
        st[(size_t)k] = gnss_acquisition(g->members[(size_t)k], file, sg, &a, &outs[(size_t)k],
                                         diag ? &diags[(size_t)k] : nullptr);
        ran[(size_t)k] = 1;
    });
    std::vector<gnss_timing> tm;
    for (int k = 0; k < M; k++)
        if (ran[(size_t)k]) tm.push_back(g->members[(size_t)k]->timing);
    g->timing = group::combine_timing(tm);
    for (int k = 0; k < M; k++)
        if (st[(size_t)k] != GNSS_OK && st[(size_t)k] != GNSS_ENODATA)
            return fail(g, st[(size_t)k], "member %d (device %d): %s", k, g->members[(size_t)k]->device,
                        g->members[(size_t)k]->err.c_str());
    if (!group::merge_acquired(prns, shards, outs, diag ? &diags : nullptr, out, diag))
        return fail(g, GNSS_EDEVICE, "multi-device acquisition: member results do not match their PRN shards");
    const int status = group::acquisition_status(st, out->n);
    if (status == GNSS_ENODATA) return fail(g, GNSS_ENODATA, "No satellites acquired");  // :84-85
    return status;
}

static int tracking_impl(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr,
                         const gnss_acquired* acq, gnss_track_out* out, const PosCfg* pos,
                         const GivenCfg* gv, const int32_t* dev_slot);

// trackingCT.m's channel loop (:22-528) dealt over the members. Host outputs: every member
// writes its channels' rows of the caller's arrays (disjoint). GNSS_OUT_DEVICE: a member on
// the output's device expands into it directly; another expands into a buffer of its own HBM
// and copies each channel's contiguous row block over xGMI.
static int group_tracking(gnss_ctx* g, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr,
                          const gnss_acquired* acq, gnss_track_out* out, const PosCfg* pos)
{
    if (!file || !sg || !tr || !acq || !out) return GNSS_EARG;
    g->timing = gnss_timing{};
    const int nsv = acq->n;
    std::vector<int32_t> chans;
    if (tr->chan && tr->n_chan > 0) chans.assign(tr->chan, tr->chan + tr->n_chan);
    else for (int i = 0; i < nsv; i++) chans.push_back(i);
    bool ok = nsv > 0 && nsv <= GNSS_MAX_SV;
    for (int c : chans) ok = ok && c >= 0 && c < nsv;
    if (!ok) return tracking_impl(g, file, sg, tr, acq, out, pos, nullptr, nullptr);  // (its own error)
    const int M = (int)g->members.size();
    const auto shards = group::deal((int)chans.size(), M);
    const bool odev = (out->flags & GNSS_OUT_DEVICE) != 0;
    int outdev = g->device;
    if (odev && (out->rec || out->taps)) {
        const int d = pointer_device(out->rec ? (const void*)out->rec : (const void*)out->taps);
        if (d >= 0) outdev = d;
    }
    const int ntaps = pos ? (pos->mc_pdi ? GNSS_MC_TAPS : 3) : (tr->n_taps > 0 ? tr->n_taps : 3);
    const int64_t ML = out->max_len;
    const size_t rec_blk = (size_t)GNSS_NFIELDS * (size_t)ML, tap_blk = (size_t)2 * ntaps * (size_t)ML;
    std::vector<group::TrackStatus> ts((size_t)M, group::TrackStatus{GNSS_OK, 0});
    std::vector<int32_t> rows((size_t)M, 0);
    std::vector<char> ran((size_t)M, 0);
    for_members(g, [&](int k) {
        gnss_ctx* m = g->members[(size_t)k];
        std::vector<int32_t> mine;
        for (int i : shards[(size_t)k]) mine.push_back(chans[(size_t)i]);
        if (mine.empty()) return;
        ran[(size_t)k] = 1;
        gnss_track t = *tr;
        t.chan = mine.data();
        t.n_chan = (int32_t)mine.size();
        gnss_track_out o = *out;
        const bool remote = odev && (m->device != outdev || m->opt[GNSS_OPT_FORCE_PEER] != 0);
        DevBuf lrec, ltap;
        std::vector<int32_t> slot(mine.size());
        auto set_err = [&](int st, const char* what) {
            ts[(size_t)k] = group::TrackStatus{st, -1};
            m->err = what;
        };
        if (remote) {
            for (size_t i = 0; i < mine.size(); i++) slot[i] = (int32_t)i;
            if (hipSetDevice(m->device) != hipSuccess ||
                (out->rec && lrec.alloc(m, "grp.rec", sizeof(double) * rec_blk * mine.size()) != hipSuccess) ||
                (out->taps && ltap.alloc(m, "grp.taps", sizeof(double) * tap_blk * mine.size()) != hipSuccess)) {
                set_err(GNSS_EDEVICE, "multi-device tracking: member output buffers");
                return;
            }
            o.rec = out->rec ? lrec.as<double>() : nullptr;
            o.taps = out->taps ? ltap.as<double>() : nullptr;
        }
        const int st = tracking_impl(m, file, sg, &t, acq, &o, pos, nullptr, remote ? slot.data() : nullptr);
        // the failing channel's POSITION in the call's channel list (the one-context rule picks the
        // first failing channel in tr->chan order, which need not be ascending)
        ts[(size_t)k] = group::TrackStatus{st, group::fail_position(shards[(size_t)k], chans, m->fail_chan)};
        rows[(size_t)k] = o.cn0_rows;
        if (st != GNSS_OK || !remote) return;
        bool copied = true;
        for (size_t i = 0; i < mine.size() && copied; i++) {
            const int64_t c = mine[i];
            if (out->rec)
                copied = hipMemcpyPeerAsync(out->rec + c * (int64_t)rec_blk, outdev, lrec.as<double>() + i * rec_blk,
                                            m->device, sizeof(double) * rec_blk, m->stream) == hipSuccess;
            if (copied && out->taps)
                copied = hipMemcpyPeerAsync(out->taps + c * (int64_t)tap_blk, outdev, ltap.as<double>() + i * tap_blk,
                                            m->device, sizeof(double) * tap_blk, m->stream) == hipSuccess;
        }
        if (!copied || hipStreamSynchronize(m->stream) != hipSuccess) set_err(GNSS_EDEVICE, "multi-device tracking: peer copy of the rows");
    });
    std::vector<gnss_timing> tm;
    for (int k = 0; k < M; k++)
        if (ran[(size_t)k]) tm.push_back(g->members[(size_t)k]->timing);
    g->timing = group::combine_timing(tm);
    const int status = group::tracking_status(ts);
    if (status != GNSS_OK) {
        if (out->len) for (int c : chans) out->len[c] = 0;
        for (int k = 0; k < M; k++)
            if (ts[(size_t)k].status == status)
                return fail(g, status, "member %d (device %d): %s", k, g->members[(size_t)k]->device,
                            g->members[(size_t)k]->err.c_str());
        return fail(g, status, "multi-device tracking failed");
    }
    int32_t r = 0;
    for (int k = 0; k < M; k++)
        if (ran[(size_t)k]) r = std::max(r, rows[(size_t)k]);
    out->cn0_rows = r;
    return GNSS_OK;
}

extern "C" {

int gnss_abi_version(void) { return GNSS_ABI_VERSION; }

const char* gnss_strerror(int s)
{
    switch (s) {
    case GNSS_OK: return "ok";
    case GNSS_ENODATA: return "no data (no satellites acquired / not enough raw data)";
    case GNSS_EIO: return "I/O error or read past end of IF record";
    case GNSS_EARG: return "invalid or unsupported argument";
    case GNSS_EDEVICE: return "HIP/rocFFT device error";
    case GNSS_EINDEX: return "index out of range (MATLAB would raise an error)";
    default: return "unknown status";
    }
}

int gnss_ctx_create(int device, gnss_ctx** out)
{
    if (!out) return GNSS_EARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return GNSS_EDEVICE;
    if (device < 0 || device >= n) return GNSS_EARG;
    if (hipSetDevice(device) != hipSuccess) return GNSS_EDEVICE;
    gnss_ctx* ctx = new gnss_ctx();
    ctx->device = device;
    bool ok = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; i < 2 && ok; i++)
        ok = hipEventCreateWithFlags(&ctx->ev_cols[i], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&ctx->ev_rows[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        gnss_ctx_destroy(ctx);
        return GNSS_EDEVICE;
    }
    rocfft_setup();
    *out = ctx;
    return GNSS_OK;
}

int gnss_ctx_create_multi(const int* devices, int n, gnss_ctx** out)
{
    if (!out) return GNSS_EARG;
    *out = nullptr;
    if (!devices || n < 1 || n > GNSS_MAX_DEVICES) return GNSS_EARG;
    gnss_ctx* g = nullptr;
    int st = gnss_ctx_create(devices[0], &g);
    if (st) return st;
    for (int k = 0; k < n; k++) {
        gnss_ctx* m = nullptr;
        if ((st = gnss_ctx_create(devices[k], &m))) {
            gnss_ctx_destroy(g);
            return st;
        }
        m->member = true;
        g->members.push_back(m);
    }
    // peer access between the distinct devices (the xGMI copies of records and rows; a pair
    // without it still copies, staged by the runtime)
    std::vector<int> ds(devices, devices + n);
    std::sort(ds.begin(), ds.end());
    ds.erase(std::unique(ds.begin(), ds.end()), ds.end());
    for (int a : ds)
        for (int b : ds) {
            int can = 0;
            if (a == b || hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
            if (hipSetDevice(a) == hipSuccess) (void)hipDeviceEnablePeerAccess(b, 0);
            (void)hipGetLastError();  // (hipErrorPeerAccessAlreadyEnabled is fine)
        }
    (void)hipSetDevice(devices[0]);
    *out = g;
    return GNSS_OK;
}

int gnss_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int gnss_ctx_members(const gnss_ctx* ctx)
{
    if (!ctx) return 0;
    return ctx->members.empty() ? 1 : (int)ctx->members.size();
}

void gnss_ctx_destroy(gnss_ctx* ctx)
{
    if (!ctx) return;
    for (gnss_ctx* m : ctx->members) gnss_ctx_destroy(m);
    ctx->members.clear();
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    ctx->resident.clear(release_resident);
    if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
    for (auto& kv : ctx->plans) rocfft_plan_destroy(kv.second);
    if (ctx->fft_work) (void)hipFree(ctx->fft_work);
    for (auto& kv : ctx->pool)
        if (kv.second.first) (void)hipFree(kv.second.first);
    for (auto& kv : ctx->pinned)
        if (kv.second.first) (void)hipHostFree(kv.second.first);
    for (int i = 0; i < 2; i++) {
        if (ctx->ev_cols[i]) (void)hipEventDestroy(ctx->ev_cols[i]);
        if (ctx->ev_rows[i]) (void)hipEventDestroy(ctx->ev_rows[i]);
    }
    if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* gnss_last_error(const gnss_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int gnss_last_timing(const gnss_ctx* ctx, gnss_timing* out)
{
    if (!ctx || !out) return GNSS_EARG;
    *out = ctx->timing;
    return GNSS_OK;
}

int gnss_ctx_set_profiling(gnss_ctx* ctx, int enable)
{
    if (!ctx) return GNSS_EARG;
    ctx->profiling = enable;
    for (gnss_ctx* m : ctx->members) m->profiling = enable;
    return GNSS_OK;
}

int gnss_ctx_set_window(gnss_ctx* ctx, uint64_t bytes)
{
    if (!ctx) return GNSS_EARG;
    ctx->window = bytes;
    for (gnss_ctx* m : ctx->members) m->window = bytes;
    return GNSS_OK;
}

int gnss_ctx_set_option(gnss_ctx* ctx, int key, int64_t value)
{
    if (!ctx || key < 0 || key >= GNSS_OPT_COUNT) return GNSS_EARG;
    if (key == GNSS_OPT_VT_BLOCKS && (value < 0 || value > GNSS_VT_MAX_BLOCKS))
        return fail(ctx, GNSS_EARG, "GNSS_OPT_VT_BLOCKS outside 0..%d", GNSS_VT_MAX_BLOCKS);
    if (key == GNSS_OPT_VT_SPAN && (value < 0 || value > kVtSpan))
        return fail(ctx, GNSS_EARG, "GNSS_OPT_VT_SPAN outside 0..%d", kVtSpan);
    ctx->opt[key] = value;
    for (gnss_ctx* m : ctx->members) m->opt[key] = value;
    return GNSS_OK;
}

int gnss_ctx_set_acq_precision(gnss_ctx* ctx, int fp64)
{
    if (!ctx || (fp64 != 0 && fp64 != 1)) return GNSS_EARG;
    ctx->acq_fp64 = fp64;
    for (gnss_ctx* m : ctx->members) m->acq_fp64 = fp64;
    return GNSS_OK;
}

int gnss_dev_alloc(gnss_ctx* ctx, uint64_t nbytes, void** dev_ptr)
{
    if (!ctx || !dev_ptr) return GNSS_EARG;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMalloc(dev_ptr, nbytes ? nbytes : 16));
    return GNSS_OK;
}

int gnss_ctx_drop_record(gnss_ctx* ctx, const void* dev_ptr)
{
    if (!ctx) return GNSS_EARG;
    drop_resident(ctx, dev_ptr, 0);
    return GNSS_OK;
}

int gnss_ctx_resident_records(const gnss_ctx* ctx)
{
    if (!ctx) return 0;
    int k = 0;
    for (const gnss_ctx* m : ctx->members) k += (int)m->resident.m.size();
    return k;
}

int gnss_dev_free(gnss_ctx* ctx, void* p)
{
    if (!ctx) return GNSS_EARG;
    drop_resident(ctx, p, 0);  // (the pointer may be handed out again by a later allocation)
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipFree(p));
    return GNSS_OK;
}

int gnss_dev_upload(gnss_ctx* ctx, void* dst, const void* src, uint64_t n)
{
    if (!ctx) return GNSS_EARG;
    drop_resident(ctx, dst, n);  // (a member's copy of these bytes is stale now)
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return GNSS_OK;
}

int gnss_dev_download(gnss_ctx* ctx, void* dst, const void* src, uint64_t n)
{
    if (!ctx) return GNSS_EARG;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return GNSS_OK;
}

// ---------------------------------------------------------------------------
// acquisition.m
// ---------------------------------------------------------------------------
int gnss_acquisition(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg,
                     const gnss_acq* acq, gnss_acquired* out, gnss_acq_diag* diag)
{
    if (!ctx || !file || !sg || !acq || !out) return GNSS_EARG;
    if (!ctx->members.empty()) return group_acquisition(ctx, file, sg, acq, out, diag);
    memset(out, 0, sizeof(*out));
    if (diag) memset(diag, 0, sizeof(*diag));
    ctx->timing = gnss_timing{};
    HIP_TRY(hipSetDevice(ctx->device));
    const int prec = file->dataPrecision, dtyp = file->dataType;
    if ((prec != 1 && prec != 2) || (dtyp != 1 && dtyp != 2))
        return fail(ctx, GNSS_EARG, "dataPrecision must be 1 (int8) or 2 (int16), dataType 1 (I) or 2 (I/Q)");
    // int16 values are de-interleaved into I/Q whatever dataType says (acquisition.m:28-32):
    // with dataType 1 the block holds half the samples and rawsignal(..idx*Sample) fails
    if (prec == 2 && dtyp == 1)
        return fail(ctx, GNSS_EINDEX, "int16 real record: rawsignal has Sample*datalen/2 samples (MATLAB index error)");
    const int64_t bps = (int64_t)prec * dtyp;  // file bytes per sample
    const bool iq8 = prec == 1 && dtyp == 2;   // the kernels' native input
    const int64_t S = sg->Sample;
    const int nb = acq->freqNum, dl = acq->datalen, L = acq->L;
    if (S <= 0 || nb <= 0 || dl <= 0 || L <= 0) return fail(ctx, GNSS_EARG, "bad acquisition sizes");

    std::vector<int32_t> prns;
    if (acq->n_prn > 0 && acq->prn_list) prns.assign(acq->prn_list, acq->prn_list + acq->n_prn);
    else for (int i = 1; i <= 32; i++) prns.push_back(i);  // acquisition.m:47
    if (prns.size() > GNSS_MAX_SV) return fail(ctx, GNSS_EARG, "too many PRNs");
    for (int p : prns) if (p < 1 || p > 51) return fail(ctx, GNSS_EARG, "PRN %d out of range", p);
    const int np = (int)prns.size();

    const int64_t off = file->skip * S * file->dataPrecision * file->dataType;  // :27
    const int64_t need = S * bps * std::max<int64_t>(dl, L + 1);
    const int64_t flen = file_length(file);
    if (flen < off + S * bps * dl) return fail(ctx, GNSS_EIO, "IF record too short for acquisition");
    IfWindow w;
    int st = stage_window(ctx, file, off, off + need, w);
    if (st) return st;
    const int8_t* blk = w.ptr + (off - w.base);
    // other formats: the samples of each fread as fp64 complex (ifmt.hip): the 20-ms block
    // (:28-37) and, with its own means, the (L+1)-ms fine block (:90-99)
    DevBuf xs_acq, xs_fine, xs_sums;
    Events e_conv;
    if (!iq8) {
        const int64_t nfine = flen >= off + S * bps * (L + 1) ? S * (L + 1) : 0;
        HIP_TRY(xs_acq.alloc(ctx, "acq.xs", sizeof(double2) * (size_t)(S * dl)));
        if (nfine) HIP_TRY(xs_fine.alloc(ctx, "acq.xs_fine", sizeof(double2) * (size_t)nfine));
        HIP_TRY(xs_sums.alloc(ctx, "acq.xs_sums", 32));
        HIP_TRY(hipEventRecord(e_conv.a, ctx->stream));
        HIP_TRY(launch_stage_cpx(blk, prec, dtyp, S * dl, xs_acq.as<double2>(), xs_sums.as<unsigned long long>(),
                                 ctx->stream));
        if (nfine)
            HIP_TRY(launch_stage_cpx(blk, prec, dtyp, nfine, xs_fine.as<double2>(),
                                     xs_sums.as<unsigned long long>() + 2, ctx->stream));
        HIP_TRY(hipEventRecord(e_conv.b, ctx->stream));
    }
    const double2* xa = iq8 ? nullptr : xs_acq.as<double2>();
    const double2* xf = iq8 ? nullptr : xs_fine.as<double2>();

    std::vector<float> cah((size_t)np * 1023);
    for (int i = 0; i < np; i++) generate_ca(prns[i], &cah[(size_t)i * 1023]);
    DevBuf ca, corr, peaks, scratch;
    HIP_TRY(ca.alloc(ctx, "acq.ca", cah.size() * sizeof(float)));
    HIP_TRY(hipMemcpyAsync(ca.p, cah.data(), cah.size() * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    // correlation precision: fp64 = the reference's (MATLAB's fft / ifft / abs().^2 in
    // double, acquisition.m:56-61), the default; fp32 = the fast mode
    // (gnss_ctx_set_acq_precision)
    const int dbl = ctx->acq_fp64 ? 1 : 0;
    HIP_TRY(corr.alloc(ctx, "acq.corr", (dbl ? sizeof(double) : sizeof(float)) * (size_t)np * nb * S));
    HIP_TRY(peaks.alloc(ctx, "acq.peaks", sizeof(AcqPeak) * (size_t)np));
    HIP_TRY(scratch.alloc(ctx, "acq.scratch", acq_scratch_bytes(np, np)));
    Events e_all, e_corr;  // e_corr.b marks the end of the PRN search
    int perm = 0;
    DevBuf fsync;  // the fused correlator's counters (its error word is read below)
    if (dbl)
        st = acq_search<double2>(ctx, blk, xa, S, dl, nb, np, sg, acq, ca.as<float>(), corr.as<double>(), e_all,
                                 &perm, fsync);
    else
        st = acq_search<float2>(ctx, blk, xa, S, dl, nb, np, sg, acq, ca.as<float>(), corr.as<float>(), e_all,
                                &perm, fsync);
    if (st) return st;
    const int cshift = (int)std::ceil(sg->Fs / sg->codeFreqBasis);  // :66
    if (dbl)
        HIP_TRY(launch_acq_peak(corr.as<double>(), np, nb, S, cshift, perm, peaks.as<AcqPeak>(), scratch.p,
                                ctx->stream));
    else
        HIP_TRY(launch_acq_peak(corr.as<float>(), np, nb, S, cshift, perm, peaks.as<AcqPeak>(), scratch.p,
                                ctx->stream));
    HIP_TRY(hipEventRecord(e_corr.b, ctx->stream));
    std::vector<AcqPeak> ph((size_t)np);
    HIP_TRY(hipMemcpyAsync(ph.data(), peaks.p, sizeof(AcqPeak) * (size_t)np, hipMemcpyDeviceToHost, ctx->stream));
    unsigned fused_err = 0;
    if (fsync.p)
        HIP_TRY(hipMemcpyAsync(&fused_err, static_cast<char*>(fsync.p) + acq_fused_err_offset(), sizeof(unsigned),
                               hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (fused_err)
        return fail(ctx, GNSS_EDEVICE, "fused correlator: a pipeline wait timed out (grid not resident)");
    ctx->timing.acq_hypothesis_samples = (int64_t)np * nb * dl * S;

    std::vector<int> acq_idx;
    for (int i = 0; i < np; i++) {
        if (diag) {
            int k = diag->n++;
            diag->prn[k] = prns[i];
            diag->SNR[k] = ph[i].snr;
            diag->fbin[k] = ph[i].fbin + 1;
            diag->codePhase[k] = ph[i].cp + 1;
            diag->peak[k] = ph[i].peak;
            diag->peak2[k] = ph[i].peak2;
        }
        if (ph[i].snr >= 12) {  // :70-74
            int k = out->n++;
            out->sv[k] = prns[i];
            out->SNR[k] = ph[i].snr;
            out->Doppler[k] = acq->freqMin + acq->freqStep * (double)ph[i].fbin;
            out->codedelay[k] = ph[i].cp;  // codePhase - 1
            acq_idx.push_back(i);
        }
    }
    if (out->n == 0) {
        HIP_TRY(hipEventRecord(e_all.b, ctx->stream));
        HIP_TRY(hipEventSynchronize(e_all.b));
        ctx->timing.acq_ms = e_all.ms();
        ctx->timing.acq_corr_ms = ctx->timing.acq_ms;
        return fail(ctx, GNSS_ENODATA, "No satellites acquired");  // :84-85
    }

    // fine frequency (:89-126)
    if (flen < off + S * bps * (L + 1)) return fail(ctx, GNSS_EIO, "IF record too short for fine search");
    const int fshift = dtyp == 2 ? 1 : 2;  // fftshift (:109) / real: first of a mirror pair
    const int na = out->n;
    const int64_t N = (int64_t)L * S * dl;  // :108
    if (N % 2) return fail(ctx, GNSS_EINDEX, "odd fftlength: MATLAB indexes past the end (:116)");
    std::vector<float> caf((size_t)na * 1023);
    std::vector<int32_t> cdh((size_t)na);
    for (int k = 0; k < na; k++) {
        generate_ca(out->sv[k], &caf[(size_t)k * 1023]);
        cdh[k] = out->codedelay[k];
    }
    DevBuf fca, fcd, fx, kb;
    HIP_TRY(fca.alloc(ctx, "acq.fca", caf.size() * sizeof(float)));
    HIP_TRY(fcd.alloc(ctx, "acq.fcd", cdh.size() * sizeof(int32_t)));
    HIP_TRY(kb.alloc(ctx, "acq.kb", sizeof(int64_t) * (size_t)na));
    HIP_TRY(hipMemcpyAsync(fca.p, caf.data(), caf.size() * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(fcd.p, cdh.data(), cdh.size() * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    const bool own_fine = fine_fft_supported(S, L) && !ctx->opt[GNSS_OPT_FINE_ROCFFT];
    Events e_fine;
    if (own_fine) {
        // per-SV zero-padded FFT as datalen three-level transforms (acq_fft.hip), up to
        // kFineBatch SVs per launch (each SV's N-point slab, 186 MB at config 2, in one scratch)
        const int fb = std::min(na, kFineBatch);
        HIP_TRY(fx.alloc(ctx, "acq.fx", fine_fft_scratch_bytes(S, L, dl, fb)));
        HIP_TRY(hipEventRecord(e_fine.a, ctx->stream));
        HIP_TRY(launch_fine_fft_tables(S, L, dl, fx.p, ctx->stream));
        for (int k0 = 0; k0 < na; k0 += fb) {
            const int nk = std::min(fb, na - k0);
            HIP_TRY(launch_fine_fft_argmax(blk, xf, S, L, dl, fcd.as<int32_t>() + k0, nk,
                                           fca.as<float>() + (size_t)k0 * 1023, sg->Fs, sg->codeFreqBasis,
                                           sg->codelength, fshift, fx.p, kb.as<int64_t>() + k0, ctx->stream));
        }
    } else {
        HIP_TRY(fx.alloc(ctx, "acq.fx", sizeof(double2) * (size_t)na * N));
        rocfft_plan pl;
        if ((st = get_plan(ctx, N, na, 1, 0, &pl))) return st;
        HIP_TRY(hipEventRecord(e_fine.a, ctx->stream));
        HIP_TRY(launch_fine_build(blk, xf, S, L, fcd.as<int32_t>(), fca.as<float>(), na, sg->Fs, sg->codeFreqBasis,
                                  sg->codelength, N, fx.as<double2>(), ctx->stream));
        if ((st = run_fft(ctx, fx.p, N, na, 1, 0))) return st;
        DevBuf fscr;
        HIP_TRY(fscr.alloc(ctx, "acq.fscr", acq_scratch_bytes(1, na)));
        HIP_TRY(launch_fine_argmax(fx.as<double2>(), na, N, fshift, fscr.p, kb.as<int64_t>(), ctx->stream));
    }
    HIP_TRY(hipEventRecord(e_fine.b, ctx->stream));
    HIP_TRY(hipEventRecord(e_all.b, ctx->stream));
    std::vector<int64_t> kh((size_t)na);
    HIP_TRY(hipMemcpyAsync(kh.data(), kb.p, sizeof(int64_t) * (size_t)na, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (int k = 0; k < na; k++) {
        const double K = (double)kh[k];
        out->fineFreq[k] = (file->dataType == 2) ? (-K * (sg->Fs / (double)N) + sg->Fs / 2) : (K * (sg->Fs / (double)N));
    }
    {
        float f = 0;
        (void)hipEventElapsedTime(&f, e_all.a, e_corr.b);
        ctx->timing.acq_corr_ms = f;
    }
    ctx->timing.acq_fine_ms = e_fine.ms();
    ctx->timing.acq_ms = e_all.ms() + (iq8 ? 0.0 : e_conv.ms());
    return GNSS_OK;
}

// ---------------------------------------------------------------------------
// trackingCT.m
// ---------------------------------------------------------------------------
namespace {

struct StepGraph {
    hipGraphExec_t exec = nullptr;
    hipGraph_t graph = nullptr;
    int count = 0;
    ~StepGraph()
    {
        if (exec) (void)hipGraphExecDestroy(exec);
        if (graph) (void)hipGraphDestroy(graph);
    }
};

}  // namespace

// trackingCT.m (pos == gv == nullptr), the tracking loop of trackingCT_POS_updated.m (pos)
// or of trackingCT_multiCorr-GIVEN.m (gv)
// dev_slot (a group member whose GNSS_OUT_DEVICE rows go through a buffer of its own): channel
// i of the call expands into row block dev_slot[i] of out->rec / out->taps instead of chans[i].
static int tracking_impl(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr,
                         const gnss_acquired* acq, gnss_track_out* out, const PosCfg* pos,
                         const GivenCfg* gv = nullptr, const int32_t* dev_slot = nullptr)
{
    if (ctx) ctx->fail_chan = -1;
    // GNSS_HOSTPROF: host-side phases of this call on stderr
    const bool hp = probe_env("GNSS_HOSTPROF") != nullptr;
    const auto h0 = std::chrono::steady_clock::now();
    auto hms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count(); };
    if (!ctx || !file || !sg || !tr || !acq || !out) return GNSS_EARG;
    HIP_TRY(hipSetDevice(ctx->device));
    ctx->timing = gnss_timing{};
    const int prec = file->dataPrecision, dtyp = file->dataType;
    if ((prec != 1 && prec != 2) || (dtyp != 1 && dtyp != 2))
        return fail(ctx, GNSS_EARG, "dataPrecision must be 1 (int8) or 2 (int16), dataType 1 (I) or 2 (I/Q)");
    if (pos && prec != 1)
        // trackingCT_POS_updated.m:196,207 reads numSample*dataType int16 values but advances
        // file_ptr by numSample*dataType BYTES: overlapping, misaligned reads (not reproduced)
        return fail(ctx, GNSS_EARG, "trackingCT_POS_updated: int8 records only");
    if (gv && (prec != 1 || dtyp != 2 || gv->datalength <= 0 || tr->n_taps != 0 || (tr->chan && tr->n_chan > 0)))
        // :47-48 forms every int8 record as I/Q pairs; codedelay sums the other channels' rows
        // (the whole channel set, below)
        return fail(ctx, GNSS_EARG, "trackingCT_multiCorr: int8 I/Q, datalength > 0, all channels");
    if (pos && (pos->ctPOS <= 0 || (!pos->countinx && !pos->mc_pdi) || tr->n_taps != 0))
        return fail(ctx, GNSS_EARG, "trackingCT_POS_updated: ctPOS > 0, countinx and E/P/L taps required");
    if (prec == 2 && dtyp == 1) {
        // fread(numSample, 'int16') de-interleaved as I/Q (trackingCT.m:84-88): an odd
        // numSample gives I and Q halves of unequal length (MATLAB raises), an even one
        // numSample/2 samples against numSample carrier values -> "Not enough raw data"
        // (:108-112). Every channel's first step has remChip 0 and codeFreq = codeFreqBasis.
        const double n0 = std::round((sg->codelength * 1 - 0.0) / (sg->codeFreqBasis / sg->Fs));
        if (out->len) for (int c = 0; c < acq->n; c++) out->len[c] = 0;
        if (std::fmod(n0, 2.0) != 0) return fail(ctx, GNSS_EINDEX, "int16 real record: odd numSample (MATLAB error)");
        return fail(ctx, GNSS_ENODATA, "Not enough raw data");
    }
    const int nsv = acq->n;
    if (nsv <= 0 || nsv > GNSS_MAX_SV) return fail(ctx, GNSS_EARG, "no channels");
    const int64_t S = sg->Sample;
    const int N1 = gv ? gv->datalength : tr->msToProcessCT_1ms;
    const int n10 = (pos || gv) ? 0 : tr->msToProcessCT_10ms / 10;
    if (!pos && !gv && N1 < 24) return fail(ctx, GNSS_EARG, "msToProcessCT_1ms must be >= 24 (bit-edge search window)");
    if (N1 < 0) return fail(ctx, GNSS_EARG, "msToProcessCT_1ms < 0");
    if (out->max_len < (pos ? (int64_t)pos->ctPOS : gv ? (int64_t)N1 : (int64_t)N1 + 19 + (int64_t)tr->msToProcessCT_10ms))
        return fail(ctx, GNSS_EARG, "max_len too small");
    const bool odev = (out->flags & GNSS_OUT_DEVICE) != 0;  // rec / taps in device memory
    if (odev && gv) return fail(ctx, GNSS_EARG, "GNSS_OUT_DEVICE: not for trackingCT_multiCorr (host codedelay pass)");
    // trackingCT_POS_updated.m: per channel, steps 1..n1 at 1 ms (msIndex <= 1000 +
    // countinx(svIndex), :183), then 10 ms up to ctPOS steps (:294)
    auto pos_n1 = [&](int c) -> int64_t {
        if (pos->mc_pdi) return pos->mc_pdi == 1 ? pos->ctPOS : 0;
        return std::max<int64_t>(0, std::min<int64_t>(pos->ctPOS, (int64_t)N1 + pos->countinx[c]));
    };
    if (8.0 * (sg->codeFreqBasis * 1.01) / sg->Fs >= 1.0)
        return fail(ctx, GNSS_EARG, "Fs too low for the 8-sample lane groups (need Fs > 8.2 MHz)");

    // taps (trackingCT.m:24; ACF taps per trackingCT_multiCorr-GIVEN.m:25)
    TrkParams P{};
    double taps3[3] = {-tr->CorrelatorSpacing, 0, tr->CorrelatorSpacing};
    const double* taps = taps3;
    int ntaps = 3;
    // trackingCT_POS_updated.m:42,210-217: Spacing = 0.6:-0.05:-0.6 (colon values 0.5, 0,
    // -0.5 exactly at 3, 13, 23); Early at Spacing(3) = +0.5, Late at Spacing(23) = -0.5,
    // Prompt Code(ceil(t + 0.05) + 1)
    const double taps_pos[3] = {0.5, 0.0, -0.5};
    // trackingCT_POS_updated_multicorrelator.m:41,207-258: all 25 Spacing values as taps,
    // Code(ceil(t) + 2) with Code = [CA(end) CA.. CA(1) CA(2)] (:94,233), no +0.05 on the
    // prompt; E/P/L = Spacing(3)/(13)/(23) feed the loops (:348-359)
    double taps_mc[25];
    if (pos && pos->mc_pdi) {
        const Colon sp = colon_make(0.6, -0.05, -0.6);
        if (sp.n != 24) return fail(ctx, GNSS_EDEVICE, "Spacing colon");
        for (int k = 0; k < 25; k++) taps_mc[k] = colon_elem(sp, k);
        taps = taps_mc;
        ntaps = 25;
        P.conv = 1;
        P.chip_off = 1;
    } else if (gv) {  // Spacing = -0.6:0.05:0.6 (:25), E/P/L = Spacing(3)/(13)/(23) (:94,106,118)
        const Colon sp = colon_make(-0.6, 0.05, 0.6);
        if (sp.n != 24) return fail(ctx, GNSS_EDEVICE, "Spacing colon");
        for (int k = 0; k < 25; k++) taps_mc[k] = colon_elem(sp, k);
        taps = taps_mc;
        ntaps = 25;
        P.given = 1;
    } else if (pos) {
        taps = taps_pos;
        P.conv = 1;
        P.tap_post[1] = 0.05;
    } else if (tr->n_taps > 0) {
        if (!tr->tap_offsets) return fail(ctx, GNSS_EARG, "tap_offsets missing");
        ntaps = tr->n_taps;
        taps = tr->tap_offsets;
    }
    // 25: the taps of trackingCT_multiCorr-GIVEN.m:25 (-0.6:0.05:0.6) and of
    // trackingCT_POS_updated_multicorrelator.m (int8 records: the step kernel's 25-tap build)
    if (ntaps != 3 && ntaps != 11 && ntaps != 25) return fail(ctx, GNSS_EARG, "n_taps must be 3, 11 or 25");
    if (ntaps == 25 && prec != 1) return fail(ctx, GNSS_EARG, "25 taps: int8 records only");
    P.iE = P.iP = P.iL = -1;
    for (int s = 0; s < ntaps; s++) {
        P.taps[s] = taps[s];
        if (pos) continue;
        if (taps[s] == -tr->CorrelatorSpacing && P.iE < 0) P.iE = s;
        if (taps[s] == 0 && P.iP < 0) P.iP = s;
        if (taps[s] == tr->CorrelatorSpacing && P.iL < 0) P.iL = s;
    }
    if (pos) { P.iE = 0; P.iP = 1; P.iL = 2; }
    if ((pos && pos->mc_pdi) || gv) { P.iE = 2; P.iP = 12; P.iL = 22; }
    if (P.iE < 0 || P.iP < 0 || P.iL < 0) return fail(ctx, GNSS_EARG, "taps must contain -spacing, 0, +spacing");
    bool wide_taps = false;
    {
        double lo_t = 1e300, hi_t = -1e300;
        for (int s = 0; s < ntaps; s++) {
            lo_t = std::min(lo_t, taps[s] + P.tap_post[s]);
            hi_t = std::max(hi_t, taps[s] + P.tap_post[s]);
        }
        // the persistent loop's tap window needs every tap's chip at a lane start within one
        // 32-chip run; a wider tap set runs on the per-step path (a path choice, not
        // an argument error)
        wide_taps = !(hi_t - lo_t <= kTapSpan);
    }
    P.ntaps = ntaps;

    std::vector<int32_t> chans;
    if (tr->chan && tr->n_chan > 0) chans.assign(tr->chan, tr->chan + tr->n_chan);
    else for (int i = 0; i < nsv; i++) chans.push_back(i);
    for (int c : chans) if (c < 0 || c >= nsv) return fail(ctx, GNSS_EARG, "channel index out of range");
    const int nch = (int)chans.size();

    // loop coefficients, calcLoopCoef.m:41-45 (trackingCT.m:26-27)
    auto coef = [](double LBW, double zeta, double k, double& t1, double& t2) {
        double Wn = LBW * 8 * zeta / (4 * (zeta * zeta) + 1);
        t1 = k / (Wn * Wn);
        t2 = 2.0 * zeta / Wn;
    };
    coef(tr->DLLBW, tr->DLLDamp, tr->DLLGain, P.tau1code, P.tau2code);
    coef(tr->PLLBW, tr->PLLDamp, tr->PLLGain, P.tau1carr, P.tau2carr);
    {   // the loop filters' constant quotients (device: loop_update_i); T as the kernel forms it
        // (multicorrelator: (pdi*t)/tau1, :352,361)
        const double T1 = pos ? (pos->mc_pdi ? 1 * sg->ms : sg->ms) : 0.001 * 1;
        const double T10 = pos ? (pos->mc_pdi ? 10 * sg->ms : sg->ms) : 0.001;
        P.dll_r = P.tau2code / P.tau1code;
        P.pll_r = P.tau2carr / P.tau1carr;
        P.dll_t1 = T1 / P.tau1code;
        P.dll_t10 = T10 / P.tau1code;
        P.pll_t1 = T1 / P.tau1carr;
        P.pll_t10 = T10 / P.tau1carr;
    }
    P.Fs = sg->Fs;
    P.codeFreqBasis = sg->codeFreqBasis;
    P.ms = sg->ms;
    P.codelength = sg->codelength;
    P.S = (double)S;
    P.dataBytesPerSample = (double)(file->dataPrecision * file->dataType);
    P.bps = prec * dtyp;
    P.fmt = prec == 2 ? 1 : 0;  // int16 I/Q: staged as is with mean removal; int8 real: as I/Q
    P.inv_Fs = 1.0 / sg->Fs;
    P.exact_div = fast_div_exact(sg->Fs, (int64_t)(S * 10 * 1.02) + 64) ? 0 : 1;
    P.nsv = pos ? 1 : nsv;  // (POS: codedelay sums the channel's own row)
    P.nch = nch;
    P.rec_cap = pos ? pos->ctPOS : N1 + 19 + n10;
    P.cn0_cap = pos ? pos->ctPOS / 20 + 1 : std::max(N1 + 19, n10) / 20 + 1;

    // IF window resident in HBM: from the earliest channel start to the latest
    // possible phase-C end (countinx <= 18, numSample within 1%)
    const int64_t bps = file->dataPrecision * file->dataType;
    int64_t lo = INT64_MAX, hi = 0, hiA = 0;  // hiA: the end of the 1-ms phases' reads
    for (int c : chans) {
        const int64_t cd = acq->codedelay[c];
        lo = std::min(lo, (S - cd + 1 + file->skip * S) * bps);
        if (gv) {  // fseek(S - codedelay - 1 + skip*S) (:57), then one continuous read
            const int64_t a0 = (S - cd - 1 + file->skip * S) * bps;
            lo = std::min(lo, a0);
            hi = std::max(hi, a0 + (int64_t)((double)N1 * S * 1.01 + 4096) * bps);
            continue;
        }
        if (pos) {  // one continuous read: n1 1-ms steps, then 10-ms steps (no re-seek)
            const int64_t n1 = pos_n1(c);
            const double ns = (double)n1 * S + (double)(pos->ctPOS - n1) * 10.0 * S;
            hi = std::max(hi, (S - cd + 1 + file->skip * S) * bps + (int64_t)(ns * 1.01 + 4096) * bps);
            continue;
        }
        const int64_t c0 = (S - cd + 1 + (file->skip + N1 + 18) * S) * bps;
        const int64_t a1 = (S - cd + 1 + file->skip * S) * bps + (int64_t)((N1 + 18) * S * 1.01 + 64) * bps;
        hi = std::max(hi, std::max(c0 + (int64_t)(n10 * 10 * S * 1.01 + 4096) * bps, a1));
        hiA = std::max(hiA, a1);
    }
    P.file_len = file_length(file);
    if (P.file_len < 0) return fail(ctx, GNSS_EIO, "cannot open IF record");
    IfWindow w;
    lo &= ~(int64_t)31;  // whole 8-sample groups of any format
    // Streaming (gnss_ctx_set_window): with a window budget below the read range, the 1-ms
    // phases' range is staged first and the 10-ms phase in segments, each staged (through the
    // pinned double buffer) into the same HBM window before its launch
    const bool seg = ctx->window > 0 && !file->dev_data && !pos && !gv && prec == 1 && dtyp == 2 && n10 > 0 &&
                     (uint64_t)(hi - lo) > ctx->window;
    int st;
    if (seg) {
        if ((uint64_t)(hiA - lo) > ctx->window || ctx->window < (uint64_t)(12 * S * bps * 1.01 + 8192))
            return fail(ctx, GNSS_EARG, "window budget below the 1-ms phases' span");
        HIP_TRY(w.own.alloc(ctx->window + 64));
        w.ptr = w.own.as<int8_t>();
        w.base = lo;
        w.len = std::min<int64_t>(hiA, P.file_len) - lo;
        if ((st = stage_into(ctx, file, w.base, w.base + w.len, w.own.as<int8_t>()))) return st;
    } else if ((st = stage_window(ctx, file, lo, hi, w))) {
        return st;
    }
    const int8_t* iq_dev = w.ptr;
    P.buf_base = w.base;
    P.buf_len = w.len;
    // formats (ifmt.hip): the correlator reads int8 I/Q pairs (fmt 0) or int16 I/Q pairs
    // (fmt 1); staged byte of sample k = 2k / 4k
    DevBuf d_conv, d_pref, d_pscr;
    {
        const int64_t s0 = std::max<int64_t>(lo, w.base);             // file bytes
        const int64_t s1 = std::min<int64_t>(hi, w.base + w.len);
        const int8_t* src = w.ptr + (s0 - w.base);
        if (prec == 1 && dtyp == 1) {  // samples = bytes; staged as (x, 0) pairs
            const int64_t n = std::max<int64_t>(s1 - s0, 0);
            HIP_TRY(d_conv.alloc(ctx, "trk.d_conv", (size_t)(2 * n + 64)));
            HIP_TRY(launch_real8_to_iq8(src, n, d_conv.as<int8_t>(), ctx->stream));
            iq_dev = d_conv.as<int8_t>();
            P.buf_base = 2 * s0;
            P.buf_len = 2 * n;
        } else if (prec == 2) {  // int16 I/Q: the file bytes, plus group prefix sums
            iq_dev = src;
            P.buf_base = s0;
            P.buf_len = std::max<int64_t>(s1 - s0, 0);
            const int64_t ng = P.buf_len / 32;
            HIP_TRY(d_pref.alloc(ctx, "trk.d_pref", 2 * sizeof(long long) * (size_t)(ng + 1)));
            const size_t scr = prefix16_scratch_bytes(ng);
            HIP_TRY(d_pscr.alloc(ctx, "trk.d_pscr", scr));
            long long* pi = d_pref.as<long long>();
            HIP_TRY(launch_prefix16(reinterpret_cast<const short*>(src), ng, pi, pi + ng + 1, d_pscr.p, scr,
                                    ctx->stream));
            P.pref_i = pi;
            P.pref_q = pi + ng + 1;
            P.stage16 = reinterpret_cast<const short*>(iq_dev - P.buf_base);
        }
    }

    // geometry: SUB x 8 contiguous samples per lane, 256 lanes per block, bpc blocks per
    // channel; SUB grows with the step's total work (more per-lane amortisation once the
    // grid fills the chip)
    // a lane's 8*SUB samples may hold at most one chip boundary per tap: 8*SUB*codeFreq/Fs
    // < 1 with margin for the DLL's excursions (the kernel flags a violating step)
    const double cps_max = 1.1 * sg->codeFreqBasis / sg->Fs;
    auto sub_ok = [&](int sub) { return 8.0 * sub * cps_max < 1.0 && (sub == 1 || !P.exact_div); };
    // The lane span depends on the step length only (not on the channel set or the path),
    // so a channel's sums are bit-identical however the channels are sharded. 1-ms steps
    // are latency-bound -> the shortest lanes; 10-ms steps: 24-sample lanes, 96 blocks per
    // channel at Opensky rates, which loads the CUs evenly at 8 channels per GPU (3 blocks
    // per CU; a step lasts as long as its slowest block).
    auto sub_for = [&](int pdi) {
        int sub = pdi >= 10 ? 3 : 1;
        while (sub > 1 && !sub_ok(sub)) sub--;
        if ((P.fmt == 1 || ntaps == 25) && sub != 3) sub = 1;  // (int16, 25 taps: 8- and 24-sample lanes)
        return sub;
    };
    int sub1 = sub_for(1), sub10 = sub_for(10);
    if (const char* fs = probe_env("GNSS_FORCE_SUB10")) {  // probe hook: the 10-ms lane span alone
        const int v = atoi(fs);
        if (v >= 1 && v <= 4 && sub_ok(v) && P.fmt == 0 && ntaps != 25) sub10 = v;
    }
    if (const char* fs = probe_env("GNSS_FORCE_SUB1")) {  // probe hook: the 1-ms lane span alone
        const int v = atoi(fs);
        if (v >= 1 && v <= 4 && sub_ok(v) && P.fmt == 0 && ntaps != 25) sub1 = v;
    }
    if (const int v = (int)ctx->opt[GNSS_OPT_FORCE_SUB]) {  // test hook: exercise every kernel variant
        if (v >= 1 && v <= 4 && sub_ok(v) && ((P.fmt == 0 && ntaps != 25) || v == 1 || v == 3)) sub1 = sub10 = v;
    }
    auto bpc_for = [&](int pdi, int sub) {
        const double groups = (S * pdi * 1.01 + 64) / 8.0 + 2;
        return (int)std::ceil(groups / ((double)kTrkThreads * sub));
    };
    // Persistent step loop (track_run_kernel) when every block of its grid can be
    // resident: one launch per phase run. Residency from the occupancy query; the kernel's
    // own census confirms it (the query can over-report, guide section 1) and a launch
    // that finds a block missing changes nothing and is re-run one launch per step, as is
    // everything with GNSS_NO_PERSIST. Both paths give the same bits.
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    // Virtual blocks per resident block (vpb): where nch x bpc blocks cannot all be
    // resident (config 5: 32 channels x 11 taps), each block correlates vpb of the step's
    // blocks in turn -- the lane geometry and so the bits stay those of bpc blocks.
    // GNSS_OPT_FORCE_VPB (test hook) asks for at least that many.
    // above 3 taps the persistent loop's lanes keep at most kQcapMax interior tap boundaries
    // (lane_correlate's capture queue): checked here for code rates up to cps_max, and a step
    // beyond that rate stops the channel with GNSS_EINDEX in the kernel (as d*M >= 1 does)
    P.qcap_dmax = cps_max;
    auto qcap_ok = [&](int sub) {
        return !GNSS_QCAP || P.ntaps <= 3 ||
               max_taps_in_lane(P.taps, P.tap_post, P.ntaps, 8 * sub, cps_max) <= kQcapMax;
    };
    auto vpb_for = [&](int pdi, int sub) {
        if (ctx->opt[GNSS_OPT_NO_PERSIST] || P.fmt != 0 || wide_taps || bpc_for(pdi, sub) > run_bpc_cap(P.ntaps) ||
            !qcap_ok(sub))
            return 0;
        const int bpc = bpc_for(pdi, sub);
        int v0 = 1;
        if (ctx->opt[GNSS_OPT_FORCE_VPB] > 0) v0 = (int)std::min<int64_t>(ctx->opt[GNSS_OPT_FORCE_VPB], kMaxVpb);
        const int occ1 = std::min(track_run_blocks_per_cu(P, sub, false), 4);
        if (v0 == 1 && occ1 >= 1 && (int64_t)nch * bpc <= (int64_t)occ1 * cus) return 1;
        const int occv = std::min(track_run_blocks_per_cu(P, sub, true), 4);  // 0: no such form
        if (occv < 1) return 0;
        for (int v = std::max(v0, 2); v <= kMaxVpb; v++)
            if ((int64_t)nch * ((bpc + v - 1) / v) <= (int64_t)occv * cus) return v;
        return 0;
    };
    const int vpb1 = vpb_for(1, sub1), vpb10 = vpb_for(10, sub10);
    bool persist1 = vpb1 > 0, persist10 = vpb10 > 0;
    if (const char* pr = probe_env("GNSS_PROBE")) P.probe = atoi(pr);
    const int bpc1 = bpc_for(1, sub1), bpc10 = bpc_for(10, sub10);
    if (bpc10 > kMaxBpc) return fail(ctx, GNSS_EARG, "Sample too large for the step geometry");

    // device state
    std::vector<TrkChan> ch0((size_t)nch);
    std::vector<unsigned> cab((size_t)nch * 32);
    for (int i = 0; i < nch; i++) {
        const int c = chans[i];
        TrkChan& t = ch0[i];
        memset(&t, 0, sizeof(t));
        t.codeFreq = sg->codeFreqBasis;  // trackingCT.m:56-58
        t.carrierFreqBasis = acq->fineFreq[c];
        t.carrierFreq = acq->fineFreq[c];
        t.codedelay0 = acq->codedelay[c];
        t.pos = (S - acq->codedelay[c] + 1 + file->skip * S) * bps;  // :63
        t.snrIndex = 1;
        t.sv1 = c + 1;
        t.prn = acq->sv[c];
        t.n1_target = N1;
        if (pos) {  // trackingCT_POS_updated.m:108-110,290 (file_ptr; codedelay base S - cd + 1)
            t.pos = (int64_t)(((double)S - acq->codedelay[c] + 1 + (double)file->skip * sg->Fs * sg->ms) * bps);
            t.codedelay0 = S - acq->codedelay[c] + 1;
            t.sv1 = 1;
            t.n1_target = pos_n1(c);
            t.countinx = pos->countinx ? pos->countinx[c] : 0;
        }
        if (gv) t.pos = (S - acq->codedelay[c] - 1 + file->skip * S) * bps;  // :57 (Codedelay = cd, :55)
        if (acq->sv[c] < 1 || acq->sv[c] > 51) return fail(ctx, GNSS_EARG, "bad PRN");
        ca_bits(acq->sv[c], &cab[(size_t)i * 32]);
    }
    DevBuf d_chan, d_snap, d_desc, d_ca, d_part, d_arrive, d_rec, d_taps, d_cn1, d_cn10, d_dv, d_pi;
    HIP_TRY(d_chan.alloc(ctx, "trk.d_chan", sizeof(TrkChan) * nch));
    HIP_TRY(d_snap.alloc(ctx, "trk.d_snap", sizeof(TrkChan) * nch));
    HIP_TRY(d_desc.alloc(ctx, "trk.d_desc", sizeof(StepDesc) * nch));
    HIP_TRY(d_ca.alloc(ctx, "trk.d_ca", sizeof(unsigned) * cab.size()));
    HIP_TRY(d_part.alloc(ctx, "trk.d_part", sizeof(double) * (size_t)nch * kMaxBpc * 2 * ntaps));
    const size_t arrive_bytes = sizeof(unsigned) * kArrivePerChan * kArriveStride * nch;
    HIP_TRY(d_arrive.alloc(ctx, "trk.d_arrive", arrive_bytes));
    HIP_TRY(d_rec.alloc(ctx, "trk.d_rec", sizeof(double) * (size_t)nch * P.rec_cap * GNSS_NFIELDS));
    if (out->taps) HIP_TRY(d_taps.alloc(ctx, "trk.d_taps", sizeof(double) * (size_t)nch * P.rec_cap * 2 * ntaps));
    HIP_TRY(d_cn1.alloc(ctx, "trk.d_cn1", sizeof(double) * (size_t)nch * P.cn0_cap));
    HIP_TRY(d_cn10.alloc(ctx, "trk.d_cn10", sizeof(double) * (size_t)nch * P.cn0_cap));
    HIP_TRY(d_dv.alloc(ctx, "trk.d_dv", sizeof(int64_t) * (size_t)nch * (P.rec_cap + 1)));
    HIP_TRY(d_pi.alloc(ctx, "trk.d_pi", sizeof(double) * (size_t)nch * N1));
    HIP_TRY(hipMemcpyAsync(d_chan.p, ch0.data(), sizeof(TrkChan) * nch, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(d_ca.p, cab.data(), sizeof(unsigned) * cab.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemsetAsync(d_arrive.p, 0, arrive_bytes, ctx->stream));
    HIP_TRY(hipMemsetAsync(d_cn1.p, 0, d_cn1.n, ctx->stream));
    HIP_TRY(hipMemsetAsync(d_cn10.p, 0, d_cn10.n, ctx->stream));
    HIP_TRY(hipMemsetAsync(d_dv.p, 0, d_dv.n, ctx->stream));
    HIP_TRY(hipMemsetAsync(d_rec.p, 0, d_rec.n, ctx->stream));

    TrkBuffers B{};
    B.iq = iq_dev;
    B.chan = d_chan.as<TrkChan>();
    B.snap = d_snap.as<TrkChan>();
    B.desc = d_desc.as<StepDesc>();
    B.ca_bits = d_ca.as<unsigned>();
    B.partial = d_part.as<double>();
    B.arrive = d_arrive.as<unsigned>();
    B.rec = d_rec.as<double>();
    B.taps_rec = out->taps ? d_taps.as<double>() : nullptr;
    B.cn0_1 = d_cn1.as<double>();
    B.cn0_10 = d_cn10.as<double>();
    B.dvpre = d_dv.as<int64_t>();
    B.p_i_1ms = d_pi.as<double>();
    B.n1 = N1;

    DevBuf d_stamps;  // timing probe: per-launch wall-clock stamps of channel 0
    const char* stamp_path = probe_env("GNSS_STAMPS");
    if (stamp_path) {
        HIP_TRY(d_stamps.alloc(ctx, "trk.d_stamps", sizeof(unsigned long long) * ((size_t)kStampSlots * (8 + 3 * kMaxBpc) + 1)));
        HIP_TRY(hipMemsetAsync(d_stamps.p, 0, d_stamps.n, ctx->stream));
        B.stamps = d_stamps.as<unsigned long long>();
    }

    DevBuf d_pgran, d_err;
    if (persist1 || persist10) {
        HIP_TRY(d_pgran.alloc(ctx, "trk.d_pgran", sizeof(unsigned long long) * 2 * (size_t)nch * gran_per_chan(ntaps)));
        HIP_TRY(d_err.alloc(ctx, "trk.d_err", 16));
        HIP_TRY(hipMemsetAsync(d_pgran.p, 0, d_pgran.n, ctx->stream));
        HIP_TRY(hipMemsetAsync(d_err.p, 0, 16, ctx->stream));
        B.pgran = d_pgran.as<unsigned long long>();
        B.run_err = d_err.as<unsigned>();
    }
    unsigned tag = 0;  // hand-off tags grow across the launches of this call

    DevBuf d_args;  // the kernels' TrkParams / TrkBuffers
    HIP_TRY(d_args.alloc(ctx, "trk.d_args", sizeof(TrkParams) + sizeof(TrkBuffers)));
    HIP_TRY(hipMemcpyAsync(d_args.p, &P, sizeof(TrkParams), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(static_cast<char*>(d_args.p) + sizeof(TrkParams), &B, sizeof(TrkBuffers),
                           hipMemcpyHostToDevice, ctx->stream));
    const TrkDev TD{d_args.as<TrkParams>(),
                    reinterpret_cast<const TrkBuffers*>(static_cast<char*>(d_args.p) + sizeof(TrkParams))};


    // step launches: one persistent launch per phase run, else K-launch graphs replayed
    // (no host launch cost per step); in profiling mode every launch is bracketed by events.
    std::vector<hipEvent_t> pev;
    std::vector<char> pev10;  // launch of the 10-ms phase
    int64_t launches = 0;
    std::function<int(int, int)> run_steps_ref;
    auto run_steps = [&](int pdi, int count) -> int {
        const int bpc = pdi == 1 ? bpc1 : bpc10, sub = pdi == 1 ? sub1 : sub10;
        if (count <= 0) return GNSS_OK;
        ctx->timing.track_channel_samples += (int64_t)count * nch * (int64_t)S * pdi;
        if (pdi == 1 ? persist1 : persist10) {
            hipEvent_t a = nullptr, b = nullptr;
            if (ctx->profiling) {
                HIP_TRY(hipEventCreate(&a));
                HIP_TRY(hipEventCreate(&b));
                HIP_TRY(hipEventRecord(a, ctx->stream));
            }
            HIP_TRY(hipMemsetAsync(d_err.p, 0, 16, ctx->stream));  // timeout word + census
            HIP_TRY(launch_track_run(P, B, TD, bpc, pdi == 1 ? vpb1 : vpb10, sub, count, tag, ctx->stream));
            tag += (unsigned)count + 1;
            unsigned err[3] = {0, 0, 0};
            HIP_TRY(hipMemcpyAsync(err, d_err.p, sizeof err, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            if (err[0] == 2) {  // census: not every block was resident -> one launch per step
                (pdi == 1 ? persist1 : persist10) = false;
                if (a) (void)hipEventDestroy(a);
                ctx->timing.track_channel_samples -= (int64_t)count * nch * (int64_t)S * pdi;
                return run_steps_ref(pdi, count);
            }
            if (err[0]) return fail(ctx, GNSS_EDEVICE, "persistent tracking kernel: a hand-off wait timed out");
            launches += 1;
            if (ctx->profiling) {
                HIP_TRY(hipEventRecord(b, ctx->stream));
                pev.push_back(a);
                pev.push_back(b);
                pev10.push_back(pdi == 10);
                if (pdi == 10) {
                    ctx->timing.track10_launches += 1;
                    ctx->timing.track10_channel_samples += (int64_t)count * nch * (int64_t)S * pdi;
                }
            }
            return GNSS_OK;
        }
        launches += count;
        if (ctx->profiling) {
            for (int i = 0; i < count; i++) {
                hipEvent_t a, b;
                HIP_TRY(hipEventCreate(&a));
                HIP_TRY(hipEventCreate(&b));
                HIP_TRY(hipEventRecord(a, ctx->stream));
                HIP_TRY(launch_track_step(P, B, TD, bpc, sub, ctx->stream));
                HIP_TRY(hipEventRecord(b, ctx->stream));
                pev.push_back(a);
                pev.push_back(b);
                pev10.push_back(pdi == 10);
            }
            if (pdi == 10) {
                ctx->timing.track10_launches += count;
                ctx->timing.track10_channel_samples += (int64_t)count * nch * (int64_t)S * pdi;
            }
            return GNSS_OK;
        }
        const int K = 50;
        if (count >= K) {
            StepGraph g;
            HIP_TRY(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < K; i++) {
                hipError_t e = launch_track_step(P, B, TD, bpc, sub, ctx->stream);
                if (e != hipSuccess) {
                    hipGraph_t junk;
                    (void)hipStreamEndCapture(ctx->stream, &junk);
                    if (junk) (void)hipGraphDestroy(junk);
                    return fail(ctx, GNSS_EDEVICE, "capture: %s", hipGetErrorString(e));
                }
            }
            HIP_TRY(hipStreamEndCapture(ctx->stream, &g.graph));
            HIP_TRY(hipGraphInstantiate(&g.exec, g.graph, nullptr, nullptr, 0));
            for (int r = 0; r < count / K; r++) HIP_TRY(hipGraphLaunch(g.exec, ctx->stream));
            for (int i = 0; i < count % K; i++) HIP_TRY(launch_track_step(P, B, TD, bpc, sub, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));  // graph objects die with this scope
        } else {
            for (int i = 0; i < count; i++) HIP_TRY(launch_track_step(P, B, TD, bpc, sub, ctx->stream));
        }
        return GNSS_OK;
    };
    run_steps_ref = run_steps;

    Events e_all;
    if (hp) { HIP_TRY(hipStreamSynchronize(ctx->stream)); fprintf(stderr, "hostprof setup %.3f ms\n", hms()); }
    HIP_TRY(hipEventRecord(e_all.a, ctx->stream));
    std::vector<TrkChan> chh((size_t)nch);
    if (gv) {
        // trackingCT_multiCorr-GIVEN.m:52-314: datalength 1-ms steps, no bit-edge search, no
        // 10-ms phase
        HIP_TRY(launch_track_prepare(P, B, TD, 1, 0, ctx->stream));
        if ((st = run_steps(1, N1))) return st;
    } else if (pos) {
        // trackingCT_POS_updated.m:179-413: every channel continues from its own state and
        // file pointer; 1-ms steps while msIndex <= 1000 + countinx(svIndex), then 10 ms
        int64_t n1max = 0, n1min = INT64_MAX;
        for (int c : chans) { n1max = std::max(n1max, pos_n1(c)); n1min = std::min(n1min, pos_n1(c)); }
        HIP_TRY(launch_track_prepare(P, B, TD, 1, 0, ctx->stream));
        if ((st = run_steps(1, (int)n1max))) return st;
        if (n1min < pos->ctPOS) {
            HIP_TRY(hipMemcpyAsync(chh.data(), d_chan.p, sizeof(TrkChan) * nch, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            for (auto& t : chh) t.n1_target = pos->ctPOS;  // (Index + 1 per step: the last step)
            HIP_TRY(hipMemcpyAsync(d_chan.p, chh.data(), sizeof(TrkChan) * nch, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(launch_track_prepare(P, B, TD, 10, 0, ctx->stream));
            if ((st = run_steps(10, (int)(pos->ctPOS - n1min)))) return st;
        }
    } else {
        // phase A: steps 1..N1-1, snapshot (for countinx = -1), step N1, bit-edge search
        HIP_TRY(launch_track_prepare(P, B, TD, 1, 0, ctx->stream));
        if ((st = run_steps(1, N1 - 1))) return st;
        HIP_TRY(launch_track_snapshot(P, B, TD, ctx->stream));
        if ((st = run_steps(1, 1))) return st;
        HIP_TRY(launch_track_bitedge(P, B, TD, ctx->stream));
        HIP_TRY(hipMemcpyAsync(chh.data(), d_chan.p, sizeof(TrkChan) * nch, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        int cxmax = 0;
        for (auto& t : chh) cxmax = std::max(cxmax, t.countinx);
        if (hp)
            for (auto& t : chh)
                fprintf(stderr, "hostprof bitedge prn %d status %d countinx %d n1_target %lld\n", t.prn, t.status,
                        t.countinx, (long long)t.n1_target);
        // phase B continues phase A up to 1000 + countinx (inactive channels skip)
        if ((st = run_steps(1, cxmax))) return st;
        HIP_TRY(launch_track_phase_c_init(P, B, TD, file->skip, ctx->stream));
        // phase C
        if (!seg) {
            if ((st = run_steps(10, n10))) return st;
        } else {
            // segments: from the channels' file positions, as many 10-ms steps as the window
            // holds (numSample <= 10*S*1.01 + 64 per step, the kernels' own bound), staged
            // into the window before their launch (the stream orders the previous launch's
            // reads before the new bytes land)
            const int64_t per_step = (int64_t)(10 * S * 1.01 + 64) * bps;
            for (int done = 0; done < n10;) {
                HIP_TRY(hipMemcpyAsync(chh.data(), d_chan.p, sizeof(TrkChan) * nch, hipMemcpyDeviceToHost,
                                       ctx->stream));
                HIP_TRY(hipStreamSynchronize(ctx->stream));
                int64_t pmin = INT64_MAX, pmax = 0;
                for (auto& t : chh) {
                    if (t.status != GNSS_OK) continue;
                    pmin = std::min(pmin, t.pos);
                    pmax = std::max(pmax, t.pos);
                }
                if (pmin == INT64_MAX) break;  // no channel left
                const int64_t base = (pmin & ~(int64_t)31);
                const int64_t room = (int64_t)ctx->window - (pmax - base) - 4096;
                int k = (int)std::min<int64_t>(n10 - done, room / per_step);
                if (k < 1) return fail(ctx, GNSS_EARG, "window budget below one 10-ms step of every channel");
                const int64_t end = std::min<int64_t>(P.file_len, pmax + (int64_t)k * per_step + 4096);
                if ((st = stage_into(ctx, file, base, end, w.own.as<int8_t>()))) return st;
                P.buf_base = base;
                P.buf_len = end - base;
                B.iq = w.own.as<int8_t>();
                HIP_TRY(hipMemcpyAsync(d_args.p, &P, sizeof(TrkParams), hipMemcpyHostToDevice, ctx->stream));
                HIP_TRY(hipMemcpyAsync(static_cast<char*>(d_args.p) + sizeof(TrkParams), &B, sizeof(TrkBuffers),
                                       hipMemcpyHostToDevice, ctx->stream));
                // the pending descriptors were checked against the previous window: rebuild
                // them from the channels' state (the same fields, the new staging check)
                HIP_TRY(launch_track_prepare(P, B, TD, 10, 1, ctx->stream));
                if ((st = run_steps(10, k))) return st;
                done += k;
                ctx->timing.track_segments += 1;
            }
        }
    }
    HIP_TRY(hipEventRecord(e_all.b, ctx->stream));
    HIP_TRY(hipEventSynchronize(e_all.b));
    ctx->timing.track_ms = e_all.ms();

    ctx->timing.track_launches = launches;
    double ksum = 0, ksum10 = 0;
    for (size_t i = 0; i + 1 < pev.size(); i += 2) {
        float f = 0;
        (void)hipEventElapsedTime(&f, pev[i], pev[i + 1]);
        ksum += f;
        if (pev10[i / 2]) ksum10 += f;
    }
    ctx->timing.track10_kernel_ms = ksum10;
    for (auto e : pev) (void)hipEventDestroy(e);
    ctx->timing.track_kernel_ms = ksum;
    if (stamp_path) {
        std::vector<unsigned long long> st(d_stamps.n / sizeof(unsigned long long));
        HIP_TRY(hipMemcpy(st.data(), d_stamps.p, d_stamps.n, hipMemcpyDeviceToHost));
        if (FILE* fp = fopen(stamp_path, "wb")) {
            fwrite(st.data(), sizeof(unsigned long long), st.size(), fp);
            fclose(fp);
        }
    }

    // results
    if (hp) fprintf(stderr, "hostprof kernels done %.3f ms\n", hms());
    HIP_TRY(hipMemcpyAsync(chh.data(), d_chan.p, sizeof(TrkChan) * nch, hipMemcpyDeviceToHost, ctx->stream));
    const size_t nrec = (size_t)nch * P.rec_cap * GNSS_NFIELDS;
    const size_t ntp = out->taps ? (size_t)nch * P.rec_cap * 2 * ntaps : 0;
    double* rec = odev ? nullptr : pinned_buffer<double>(ctx, "trk.h_rec", nrec);
    double* tp = ntp && !odev ? pinned_buffer<double>(ctx, "trk.h_taps", ntp) : nullptr;
    if (!odev && (!rec || (ntp && !tp))) return fail(ctx, GNSS_EDEVICE, "hipHostMalloc of the record staging failed");
    std::vector<double> cn1((size_t)nch * P.cn0_cap), cn10((size_t)nch * P.cn0_cap);
    if (!odev) {
        HIP_TRY(hipMemcpyAsync(rec, d_rec.p, nrec * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
        if (out->taps) HIP_TRY(hipMemcpyAsync(tp, d_taps.p, ntp * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipMemcpyAsync(cn1.data(), d_cn1.p, cn1.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(cn10.data(), d_cn10.p, cn10.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));

    if (hp) fprintf(stderr, "hostprof d2h done %.3f ms\n", hms());
    int status = GNSS_OK;
    for (int i = 0; i < nch; i++) {
        const TrkChan& t = chh[i];
        if (t.status && ctx->fail_chan < 0) ctx->fail_chan = chans[i];  // (the first failing channel)
        if (t.status && (status == GNSS_OK || t.status == GNSS_ENODATA)) status = t.status;
    }
    if (status != GNSS_OK) {
        if (out->len) for (int c : chans) out->len[c] = 0;
        return fail(ctx, status, status == GNSS_ENODATA ? "Not enough raw data" : "tracking failed: %s",
                    gnss_strerror(status));
    }

    const int64_t ML = out->max_len;
    int rows = pos ? pos->ctPOS / 20 : N1 / 20;
    // series length before the 10-ms values (POS: every step has its own row)
    auto n1_of = [&](int i) -> int64_t { return pos ? (int64_t)pos->ctPOS : (int64_t)N1 + chh[i].countinx; };
    for (int i = 0; i < nch; i++) {
        const int c = chans[i];
        const TrkChan& t = chh[i];
        const int cx = t.countinx;
        const int64_t n1 = n1_of(i);
        if (out->len) out->len[c] = n1 + 10LL * n10;
        if (out->countinx) out->countinx[c] = cx;
        rows = std::max(rows, (int)(n1 / 20));
    }
    // the MATLAB layout: one row per millisecond, each 10-ms step's value on its ten rows
    const int nrf = out->rec ? GNSS_NFIELDS : 0, ntf = out->taps ? 2 * ntaps : 0;
    if (odev) {  // expanded on the GPU straight into the caller's device arrays
        std::vector<int64_t> job(2 * (size_t)nch);
        for (int i = 0; i < nch; i++) {
            job[2 * i] = n1_of(i);
            job[2 * i + 1] = dev_slot ? dev_slot[i] : chans[i];
        }
        DevBuf d_job;
        HIP_TRY(d_job.alloc(ctx, "trk.d_job", sizeof(int64_t) * job.size()));
        HIP_TRY(hipMemcpyAsync(d_job.p, job.data(), sizeof(int64_t) * job.size(), hipMemcpyHostToDevice, ctx->stream));
        if (nrf)
            HIP_TRY(launch_track_expand(d_rec.as<double>(), P.rec_cap, GNSS_NFIELDS, GNSS_NFIELDS, nch,
                                        d_job.as<int64_t>(), out->rec, ML, n10, 0, ctx->stream));
        if (ntf)
            HIP_TRY(launch_track_expand(d_taps.as<double>(), P.rec_cap, 2 * ntaps, 2 * ntaps, nch,
                                        d_job.as<int64_t>(), out->taps, ML, n10, ntaps, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    } else parallel_for(nch * (nrf + ntf), [&](int task) {
        const int i = task / (nrf + ntf), f = task % (nrf + ntf);
        const int c = chans[i];
        const int64_t n1 = n1_of(i);
        double* dst;
        const double* src;
        int64_t stride;
        if (f < nrf) {
            dst = out->rec + ((int64_t)c * GNSS_NFIELDS + f) * ML;
            src = rec + (size_t)i * P.rec_cap * GNSS_NFIELDS + f;
            stride = GNSS_NFIELDS;
        } else {
            const int tq = f - nrf, sidx = tq / 2, iq = tq % 2;
            dst = out->taps + (((int64_t)c * 2 + iq) * ntaps + sidx) * ML;
            src = tp + (size_t)i * P.rec_cap * 2 * ntaps + tq;
            stride = 2 * ntaps;
        }
        for (int64_t k = 0; k < n1; k++) dst[k] = src[k * stride];
        for (int64_t q = 0; q < n10; q++) {
            const double v = src[(n1 + q) * stride];
            for (int r = 0; r < 10; r++) dst[n1 + 10 * q + r] = v;
        }
        for (int64_t k = n1 + 10 * n10; k < ML; k++) dst[k] = 0;  // (a reused buffer's tail)
    });
    if (hp) fprintf(stderr, "hostprof expanded %.3f ms\n", hms());
    if (gv && out->rec) {
        // codedelay = Codedelay + sum(delayValue(1:msIndex)) (trackingCT_multiCorr-GIVEN.m:297):
        // delayValue is ONE nsv x datalength matrix (:29) filled channel after channel, so the
        // linear (column-major) sum takes the earlier channels' rows whole and this channel's
        // own row up to msIndex (rows of later channels are still zero)
        for (int c = 0; c < nsv; c++) {
            double* cdr = out->rec + ((int64_t)c * GNSS_NFIELDS + GNSS_F_codedelay) * ML;
            double sum = 0;
            for (int64_t k = 0; k < N1; k++) {  // linear position k + 1
                const int r = (int)(k % nsv);
                if (r <= c) sum += out->rec[((int64_t)r * GNSS_NFIELDS + GNSS_F_delayValue) * ML + k / nsv];
                cdr[k] = (double)acq->codedelay[c] + sum;
            }
        }
    }
    rows = std::max(rows, n10 / 20);
    out->cn0_rows = rows;  // (POS: CN0_CT, one row per 20 steps of either pdi)
    if (out->CN0_Eph) {
        for (int i = 0; i < nch; i++) {
            const int c = chans[i];
            const int cx = chh[i].countinx;
            const int r1 = pos ? rows : std::max(N1, N1 + cx) / 20, r10 = n10 / 20;
            for (int r = 0; r < out->cn0_cap; r++) {
                double v = 0;
                if (r < r10) v = cn10[(size_t)i * P.cn0_cap + r];
                else if (r < r1) v = cn1[(size_t)i * P.cn0_cap + r];
                out->CN0_Eph[(int64_t)r * nsv + c] = v;
            }
        }
    }
    return GNSS_OK;
}

int gnss_tracking_ct(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr,
                     const gnss_acquired* acq, gnss_track_out* out)
{
    if (ctx && !ctx->members.empty()) return group_tracking(ctx, file, sg, tr, acq, out, nullptr);
    return tracking_impl(ctx, file, sg, tr, acq, out, nullptr);
}

int gnss_tracking_ct_pos(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr,
                         const gnss_acquired* acq, int32_t ctPOS, const int32_t* countinx, gnss_track_out* out)
{
    const PosCfg pc{ctPOS, countinx, 0};
    if (ctx && !ctx->members.empty()) return group_tracking(ctx, file, sg, tr, acq, out, &pc);
    return tracking_impl(ctx, file, sg, tr, acq, out, &pc);
}

int gnss_tracking_ct_multicorr(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg,
                               const gnss_track* tr, const gnss_acquired* acq, int32_t datalength,
                               gnss_track_out* out)
{
    const GivenCfg g{datalength};
    return tracking_impl(ctx, file, sg, tr, acq, out, nullptr, &g);
}

int gnss_tracking_ct_mc(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr,
                        const gnss_acquired* acq, int32_t msPosCT, int32_t pdi, gnss_track_out* out)
{
    if (!ctx) return GNSS_EARG;
    if (pdi != 1 && pdi != 10) return fail(ctx, GNSS_EARG, "multicorrelator: pdi must be 1 or 10");
    if (msPosCT < pdi) return fail(ctx, GNSS_EARG, "multicorrelator: msPosCT/pdi must be >= 1");
    const PosCfg pc{msPosCT / pdi, nullptr, pdi};  // msIndex = 1:datalength/pdi (:170)
    if (!ctx->members.empty()) return group_tracking(ctx, file, sg, tr, acq, out, &pc);
    return tracking_impl(ctx, file, sg, tr, acq, out, &pc);
}

int gnss_correlate_step(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, int prn, int pdi,
                        double remChip, double codeFreq, double carrierFreq, double remPhase,
                        int64_t pos_bytes, int n_taps, const double* taps, double* sums_out,
                        int64_t* numSample_out)
{
    if (!ctx || !file || !sg || !taps || !sums_out || (n_taps != 3 && n_taps != 11) || prn < 1 || prn > 51)
        return GNSS_EARG;
    if (pdi != 1 && pdi != 10) return GNSS_EARG;
    HIP_TRY(hipSetDevice(ctx->device));
    const int64_t S = sg->Sample;
    TrkParams P{};
    P.Fs = sg->Fs;
    P.codeFreqBasis = sg->codeFreqBasis;
    P.ms = sg->ms;
    P.codelength = sg->codelength;
    P.S = (double)S;
    P.dataBytesPerSample = 2;
    P.bps = 2;  // int8 I/Q records only
    P.fmt = 0;
    P.inv_Fs = 1.0 / sg->Fs;
    P.exact_div = fast_div_exact(sg->Fs, (int64_t)(S * 10 * 1.02) + 64) ? 0 : 1;
    P.ntaps = n_taps;
    P.iE = 0; P.iP = n_taps / 2; P.iL = n_taps - 1;
    for (int s = 0; s < n_taps; s++) P.taps[s] = taps[s];
    P.nsv = P.nch = 1;
    P.rec_cap = 1;
    P.cn0_cap = 1;
    P.file_len = file_length(file);
    IfWindow w;
    int st = stage_window(ctx, file, pos_bytes, pos_bytes + (int64_t)(2.1 * S * pdi) + 64, w);
    if (st) return st;
    P.buf_base = w.base;
    P.buf_len = w.len;
    TrkChan c{};
    c.remChip = remChip;
    c.codeFreq = codeFreq;
    c.carrierFreq = carrierFreq;
    c.remPhase = remPhase;
    c.pos = pos_bytes;
    c.n1_target = 1 << 30;
    c.sv1 = 1;
    c.prn = prn;
    unsigned cab[32];
    ca_bits(prn, cab);
    int sub = 1;
    if (const int v = (int)ctx->opt[GNSS_OPT_FORCE_SUB]) {
        if (v >= 2 && v <= 4 && !P.exact_div && 8.0 * v * codeFreq / sg->Fs < 1.0) sub = v;
    }
    const int bpc = (int)std::ceil(((S * pdi * 1.01 + 64) / 8.0 + 2) / ((double)kTrkThreads * sub));
    DevBuf d_chan, d_desc, d_ca, d_part, d_arrive, d_sums;
    HIP_TRY(d_chan.alloc(sizeof(TrkChan)));
    HIP_TRY(d_desc.alloc(sizeof(StepDesc)));
    HIP_TRY(d_ca.alloc(sizeof(cab)));
    HIP_TRY(d_part.alloc(sizeof(double) * kMaxBpc * 2 * n_taps));
    HIP_TRY(d_arrive.alloc(sizeof(unsigned) * kArrivePerChan * kArriveStride));
    HIP_TRY(d_sums.alloc(sizeof(double) * 2 * n_taps));
    HIP_TRY(hipMemcpyAsync(d_chan.p, &c, sizeof c, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(d_ca.p, cab, sizeof cab, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemsetAsync(d_arrive.p, 0, sizeof(unsigned) * kArrivePerChan * kArriveStride, ctx->stream));
    TrkBuffers B{};
    B.iq = w.ptr;
    B.chan = d_chan.as<TrkChan>();
    B.desc = d_desc.as<StepDesc>();
    B.ca_bits = d_ca.as<unsigned>();
    B.partial = d_part.as<double>();
    B.arrive = d_arrive.as<unsigned>();
    B.dbg_sums = d_sums.as<double>();
    DevBuf d_args;  // the kernels' TrkParams / TrkBuffers
    HIP_TRY(d_args.alloc(sizeof(TrkParams) + sizeof(TrkBuffers)));
    HIP_TRY(hipMemcpyAsync(d_args.p, &P, sizeof(TrkParams), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(static_cast<char*>(d_args.p) + sizeof(TrkParams), &B, sizeof(TrkBuffers),
                           hipMemcpyHostToDevice, ctx->stream));
    const TrkDev TD{d_args.as<TrkParams>(),
                    reinterpret_cast<const TrkBuffers*>(static_cast<char*>(d_args.p) + sizeof(TrkParams))};

    HIP_TRY(launch_track_prepare(P, B, TD, pdi, 0, ctx->stream));
    HIP_TRY(launch_track_step(P, B, TD, bpc, sub, ctx->stream));
    HIP_TRY(hipMemcpyAsync(sums_out, d_sums.p, sizeof(double) * 2 * n_taps, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(&c, d_chan.p, sizeof c, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (c.status) return fail(ctx, c.status, "correlate step failed");
    if (numSample_out) {
        const double cps = codeFreq / sg->Fs;
        *numSample_out = (int64_t)round((sg->codelength * pdi - remChip) / cps);
    }
    return GNSS_OK;
}

}  // extern "C"

// generateCAcode.m chips for the other host translation units (vt.cpp)
void gnss::ca_chips(int prn, float* out) { generate_ca(prn, out); }

extern "C" {

// trackingVT_POS_updated.m:157-349, one step of n channels (include/gnss_mi355x.h): the
// reads and replica chips sized on the host (gnss_vt_prepare), the carrier-wiped sums on
// the GPU (vt.hip), the NCO / PLL / DLL discriminator on the host (gnss_vt_nco_step).
int gnss_tracking_vt_run(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr,
                         int32_t pdi, int32_t n, int32_t nsteps, gnss_vt_chan* chans, const double* codeFreq_new,
                         gnss_vt_out* out)
{
    if (!ctx || !file || !sg || !tr || !chans || !codeFreq_new || !out || n < 1 || n > GNSS_MAX_SV || pdi < 1 ||
        nsteps < 1 || !(sg->Fs > 0) || !(sg->codeFreqBasis > 0))
        return fail(ctx, GNSS_EARG, "bad arguments");
    ctx->err.clear();
    ctx->timing = gnss_timing{};
    HIP_TRY(hipSetDevice(ctx->device));
    // formats of trackingVT_POS_updated.m:163-176: int8 I/Q, int8 real, int16 I/Q (means removed)
    const int prec = file->dataPrecision, dtyp = file->dataType;
    if (!((prec == 1 && (dtyp == 1 || dtyp == 2)) || (prec == 2 && dtyp == 2)))
        return fail(ctx, GNSS_EARG, "vector tracking: int8 I/Q, int8 real or int16 I/Q records");
    const int bps = prec * dtyp;
    const int64_t flen = file_length(file);
    if (flen < 0) return fail(ctx, GNSS_EIO, "cannot open IF record");
    // the read range of every step: from the earliest file_ptr, at most nsteps reads of the
    // largest size any step can ask for (the slowest code frequency of the series)
    double cf_min = 1e300;
    for (int i = 0; i < n; i++) {
        if (chans[i].prn < 1 || chans[i].prn > 51) return fail(ctx, GNSS_EARG, "bad PRN");
        if (chans[i].file_ptr < 0 || chans[i].file_ptr % bps) return fail(ctx, GNSS_EARG, "file_ptr");
        if (chans[i].index_int < 0 || chans[i].index_int > 19 || chans[i].snrIndex < 1)
            return fail(ctx, GNSS_EARG, "C/N0 state (index_int 0..19, snrIndex >= 1)");
        cf_min = std::min(cf_min, chans[i].codeFreq);
    }
    for (int64_t k = 0; k < (int64_t)nsteps * n; k++) cf_min = std::min(cf_min, codeFreq_new[k]);
    if (!(cf_min > 0)) return fail(ctx, GNSS_EARG, "code frequencies must be positive");
    const double nmax = std::ceil((sg->codelength * pdi + 2.0) / (cf_min / sg->Fs)) + 2;
    int64_t lo = INT64_MAX, hi = 0;
    for (int i = 0; i < n; i++) {
        lo = std::min(lo, chans[i].file_ptr);
        hi = std::max(hi, chans[i].file_ptr + (int64_t)(nsteps * nmax) * bps);
    }
    IfWindow w;
    int st = stage_window(ctx, file, lo, std::min(hi, flen), w);
    if (st) return st;
    std::vector<unsigned> cab((size_t)n * 32);
    for (int i = 0; i < n; i++) ca_bits(chans[i].prn, &cab[(size_t)i * 32]);
    DevBuf d_chan, d_cf, d_out, d_ca;
    const size_t nrec = (size_t)nsteps * n;
    HIP_TRY(d_chan.alloc(ctx, "vt.chan", sizeof(gnss_vt_chan) * (size_t)n));
    HIP_TRY(d_cf.alloc(ctx, "vt.cf", sizeof(double) * nrec));
    HIP_TRY(d_out.alloc(ctx, "vt.out", sizeof(gnss_vt_out) * nrec));
    HIP_TRY(d_ca.alloc(ctx, "vt.ca", sizeof(unsigned) * cab.size()));
    HIP_TRY(hipMemcpyAsync(d_chan.p, chans, sizeof(gnss_vt_chan) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(d_cf.p, codeFreq_new, sizeof(double) * nrec, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(d_ca.p, cab.data(), sizeof(unsigned) * cab.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemsetAsync(d_out.p, 0, sizeof(gnss_vt_out) * nrec, ctx->stream));
    double t1, t2;
    calc_loop_coef(tr->PLLBW, tr->PLLDamp, tr->PLLGain, t1, t2);
    VtRunArgs A{};
    A.rec = reinterpret_cast<const uint8_t*>(w.ptr);
    A.base = w.base;
    A.len = w.len;
    A.file_len = flen;
    A.chans = d_chan.as<gnss_vt_chan>();
    A.codeFreq = d_cf.as<double>();
    A.out = d_out.as<gnss_vt_out>();
    A.ca_bits = d_ca.as<unsigned>();
    A.Fs = sg->Fs;
    A.ms = sg->ms;
    A.codelength = sg->codelength;
    A.tau1carr = t1;
    A.tau2carr = t2;
    A.n = n;
    A.nsteps = nsteps;
    A.pdi = pdi;
    A.prec = prec;
    A.dtype = dtyp;
    Events ev;
    HIP_TRY(hipEventRecord(ev.a, ctx->stream));
    HIP_TRY(launch_vt_run(A, ctx->stream));
    HIP_TRY(hipEventRecord(ev.b, ctx->stream));
    HIP_TRY(hipMemcpyAsync(out, d_out.p, sizeof(gnss_vt_out) * nrec, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(chans, d_chan.p, sizeof(gnss_vt_chan) * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->timing.track_ms = ev.ms();
    ctx->timing.track_kernel_ms = ctx->timing.track_ms;
    ctx->timing.track_launches = 1;
    int first = GNSS_OK;
    for (int s = 0; s < nsteps; s++)
        for (int i = 0; i < n; i++) {
            const gnss_vt_out& o = out[(size_t)s * n + i];
            if (o.status) {
                if (!first) first = o.status;
            } else if (o.numSample > 0) {
                ctx->timing.track_channel_samples += o.numSample;
            }
        }
    if (first) return fail(ctx, first, "a channel stopped (its record's status): replica index / read past EOF");
    return GNSS_OK;
}

int gnss_tracking_vt_step(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr,
                          int32_t pdi, int32_t n, gnss_vt_chan* chans, const double* codeFreq_new,
                          gnss_vt_out* out)
{
    return gnss_tracking_vt_run(ctx, file, sg, tr, pdi, n, 1, chans, codeFreq_new, out);
}

namespace {
// Wait until VT step `seq` is posted (vt_step_kernel's completion word, coherent host
// memory). The stream is polled now and then, so a grid that ends without posting (a fault)
// surfaces as its error rather than a hang.
hipError_t wait_posted(hipStream_t stream, const unsigned* done, unsigned seq)
{
    auto posted = [&] { return __atomic_load_n(done, __ATOMIC_ACQUIRE) == seq; };
    for (unsigned k = 1;; k++) {
        if (posted()) return hipSuccess;
        __builtin_ia32_pause();
        if ((k & 255) == 0) {
            const hipError_t e = hipStreamQuery(stream);
            if (e == hipErrorNotReady) continue;
            if (e != hipSuccess) return e;
            return posted() ? hipSuccess : hipErrorLaunchFailure;  // (retired: its posts are visible)
        }
    }
}

// The same for the loop mode's sums: until the n granules all carry `seq`, their values to
// `out` (a granule seen once is not read again: the scan resumes where it stopped).
hipError_t wait_granules(hipStream_t stream, const VtGran* g, int n, unsigned seq, double* out)
{
    int i = 0;
    auto posted = [&] {
        uint64_t bits;
        while (i < n && vt_gran_get(g + i, seq, &bits)) {
            std::memcpy(out + i, &bits, sizeof bits);
            i++;
        }
        return i == n;
    };
    for (unsigned k = 1;; k++) {
        if (posted()) return hipSuccess;
        __builtin_ia32_pause();
        if ((k & 255) == 0) {
            const hipError_t e = hipStreamQuery(stream);
            if (e == hipErrorNotReady) continue;
            if (e != hipSuccess) return e;
            return posted() ? hipSuccess : hipErrorLaunchFailure;
        }
    }
}
}  // namespace

// trackingVT_POS_updated.m:157-476, the whole EKF-driven loop: per step, each channel's read
// size (:164) and predicted code frequency (:180-227, gnss_vt_nav_predict, host), the
// correlations of all channels in ONE launch of the VT kernel, each channel's scalar end
// (vt_finish, :284-347), then the EKF (:357-467, gnss_vt_nav_update, host). int8 records: the
// channel states stay on the host and the kernel returns each channel's sums (vt_step_kernel);
// int16 (per-read means first): vt_run_kernel runs the whole step, states in HBM.
int gnss_tracking_vt(gnss_ctx* ctx, const gnss_file* file, const gnss_signal* sg, const gnss_track* tr, int32_t n,
                     int32_t nsteps, gnss_vt_chan* chans, gnss_vt_nav* nav, gnss_vt_out* out, gnss_vt_navsol* sol)
{
    if (!ctx || !file || !sg || !tr || !chans || !nav || !out || n < 1 || n > GNSS_VT_MAX_CH || n != nav->n ||
        nsteps < 0 || !(sg->Fs > 0) || !(sg->codeFreqBasis > 0) || sg->Fs != nav->Fs)
        return fail(ctx, GNSS_EARG, "bad arguments (n in 1..GNSS_VT_MAX_CH and equal to nav->n, signal as at gnss_vt_nav_init)");
    ctx->err.clear();
    ctx->timing = gnss_timing{};
    if (nsteps == 0) return GNSS_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    const int pdi = nav->pdi;
    const int prec = file->dataPrecision, dtyp = file->dataType;
    if (!((prec == 1 && (dtyp == 1 || dtyp == 2)) || (prec == 2 && dtyp == 2)))
        return fail(ctx, GNSS_EARG, "vector tracking: int8 I/Q, int8 real or int16 I/Q records");
    const int bps = prec * dtyp;
    const int64_t flen = file_length(file);
    if (flen < 0) return fail(ctx, GNSS_EIO, "cannot open IF record");
    for (int i = 0; i < n; i++) {
        if (chans[i].prn != nav->prn[i]) return fail(ctx, GNSS_EARG, "chans[i].prn != nav->prn[i]");
        if (chans[i].file_ptr < 0 || chans[i].file_ptr % bps) return fail(ctx, GNSS_EARG, "file_ptr");
        if (chans[i].index_int < 0 || chans[i].index_int > 19 || chans[i].snrIndex < 1)
            return fail(ctx, GNSS_EARG, "C/N0 state (index_int 0..19, snrIndex >= 1)");
        if (!(chans[i].codeFreq > 0)) return fail(ctx, GNSS_EARG, "code frequency must be positive");
    }
    // The IF window: the steps' reads are sized by code frequencies the EKF has not predicted
    // yet, so a window is staged for `span` steps at half the nominal code rate (twice the
    // nominal read) and re-staged when a read would leave it. A resident record is used as is.
    const int64_t nominal = (int64_t)std::ceil(sg->codelength * pdi / (sg->codeFreqBasis / sg->Fs));
    const int64_t span = std::min<int64_t>(nsteps, ctx->opt[GNSS_OPT_VT_SPAN] > 0 ? ctx->opt[GNSS_OPT_VT_SPAN] : kVtSpan);
    IfWindow w;
    auto restage = [&](int64_t lo) -> int {
        const int64_t hi = lo + (span * 2 * nominal + 64) * bps;
        w.own.release();
        w.ptr = nullptr;
        w.base = w.len = 0;
        return stage_window(ctx, file, lo, std::min(hi, flen), w);
    };
    int64_t lo0 = INT64_MAX;
    for (int i = 0; i < n; i++) lo0 = std::min(lo0, chans[i].file_ptr);
    int st = restage(lo0);
    if (st) return st;
    std::vector<unsigned> cab((size_t)n * 32);
    for (int i = 0; i < n; i++) ca_bits(chans[i].prn, &cab[(size_t)i * 32]);
    double t1, t2;
    calc_loop_coef(tr->PLLBW, tr->PLLDamp, tr->PLLGain, t1, t2);
    // int8 records: each step over nb blocks per channel (vt_step_kernel), the step's reads
    // in the kernel arguments and each channel's two sums posted to coherent host memory (no
    // copy commands per step); int16 (per-read means first): one block per channel (vt_run_kernel)
    const bool multi = prec == 1;
    DevBuf d_chan, d_cf, d_out, d_ca, d_part, d_ticket, d_loop;
    double* h_cf = pinned_buffer<double>(ctx, "vt.cf", (size_t)n);
    gnss_vt_out* h_out = pinned_buffer<gnss_vt_out>(ctx, "vt.out", (size_t)n);
    if (!h_cf || !h_out) return fail(ctx, GNSS_EDEVICE, "pinned VT step buffers");
    std::vector<gnss_vt_chan> hc(chans, chans + n);  // (int8: the channel states)
    std::vector<VtPrep> pk((size_t)n);
    std::vector<int> bad((size_t)n, 0);
    VtStepArgs B{};
    int nb = 1;
    int64_t kmax_rfs = 0;
    int loop_cap = 0;  // blocks a loop grid may have (0: no loop mode)
    double rfs = 0;
    if (multi) {
        // blocks per channel, the engine's choice per path (r06_vt_loop_nb*.txt): one launch per
        // step pays a ticket per block, the loop's lead gathers every block's granules at once
        const bool loop_ok = !ctx->profiling && !ctx->opt[GNSS_OPT_NO_PERSIST];
        loop_cap = loop_ok ? vt_loop_resident_blocks(ctx->device) : 0;
        nb = loop_cap >= n ? (int)std::min<int64_t>(std::max<int64_t>(1, (nominal + kVtLoopSamples - 1) / kVtLoopSamples),
                                                    loop_cap / n)
                     : (int)std::min<int64_t>(std::max<int64_t>(1, (nominal + kVtStepSamples - 1) / kVtStepSamples),
                                              GNSS_VT_MAX_BLOCKS);
        if (ctx->opt[GNSS_OPT_VT_BLOCKS] > 0) nb = (int)ctx->opt[GNSS_OPT_VT_BLOCKS];
        B.sums = pinned_buffer<double>(ctx, "vt.sums", 2 * (size_t)n, hipHostMallocCoherent);
        B.done = pinned_buffer<unsigned>(ctx, "vt.done", 1, hipHostMallocCoherent);
        if (!B.sums || !B.done) return fail(ctx, GNSS_EDEVICE, "pinned VT step buffers");
        __atomic_store_n(B.done, 0u, __ATOMIC_RELAXED);
        HIP_TRY(d_ticket.alloc(ctx, "vt.ticket", sizeof(unsigned)));
        HIP_TRY(hipMemsetAsync(d_ticket.p, 0, sizeof(unsigned), ctx->stream));
        B.ticket = d_ticket.as<unsigned>();
        B.Fs = sg->Fs;
        B.real8 = dtyp == 1;
        // k/Fs by Markstein's correction where it is the IEEE quotient (exhaustively verified up
        // to four nominal reads, cached per Fs; a longer read divides)
        kmax_rfs = 4 * nominal;
        rfs = fast_div_exact(sg->Fs, kmax_rfs) ? 1.0 / sg->Fs : 0.0;
        HIP_TRY(d_part.alloc(ctx, "vt.part", sizeof(double) * 2 * (size_t)n * nb));
        B.part = d_part.as<double>();
    } else {
        HIP_TRY(d_chan.alloc(ctx, "vt.chan", sizeof(gnss_vt_chan) * (size_t)n));
        HIP_TRY(d_cf.alloc(ctx, "vt.cf", sizeof(double) * (size_t)n));
        HIP_TRY(d_out.alloc(ctx, "vt.out", sizeof(gnss_vt_out) * (size_t)n));
        HIP_TRY(d_ca.alloc(ctx, "vt.ca", sizeof(unsigned) * cab.size()));
        HIP_TRY(hipMemcpyAsync(d_chan.p, chans, sizeof(gnss_vt_chan) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(d_ca.p, cab.data(), sizeof(unsigned) * cab.size(), hipMemcpyHostToDevice, ctx->stream));
    }
    VtRunArgs A{};
    A.file_len = flen;
    A.chans = d_chan.as<gnss_vt_chan>();
    A.codeFreq = d_cf.as<double>();
    A.out = d_out.as<gnss_vt_out>();
    A.ca_bits = d_ca.as<unsigned>();
    A.Fs = sg->Fs;
    A.ms = sg->ms;
    A.codelength = sg->codelength;
    A.tau1carr = t1;
    A.tau2carr = t2;
    A.n = n;
    A.nsteps = 1;
    A.pdi = pdi;
    A.prec = prec;
    A.dtype = dtyp;
    // Loop mode (int8 records, not profiling, the grid fits on the chip at once): ONE
    // vt_loop_kernel launch runs the steps, each posted through a mailbox in coherent host
    // memory, so a step costs no launch; stopped before a re-staging of the IF window and at
    // the end (also on every early return: `loop_guard`).
    const bool loop_mode = multi && loop_cap > 0 && (int64_t)n * nb <= loop_cap;
    VtGran *mail = nullptr, *gsums = nullptr;
    std::vector<double> loop_sums(2 * (size_t)n);
    bool running = false;
    // the loop's 16-B granules: each channel's relayed read, then every block's two sums
    const size_t gstep_bytes = (size_t)16 * kVtStepWords * n, loop_bytes = gstep_bytes + (size_t)16 * 2 * n * nb;
    uint64_t loop_timeout = 0;
    if (loop_mode) {
        mail = pinned_buffer<VtGran>(ctx, "vt.mail", 2 * (size_t)kVtStepWords * n, hipHostMallocCoherent);
        gsums = pinned_buffer<VtGran>(ctx, "vt.gsums", 2 * (size_t)n, hipHostMallocCoherent);
        if (!mail || !gsums) return fail(ctx, GNSS_EDEVICE, "pinned VT mailbox");
        for (int k = 0; k < 2 * kVtStepWords * n; k++) vt_gran_put(mail + k, 0, 0);
        for (int k = 0; k < 2 * n; k++) vt_gran_put(gsums + k, 0, 0);
        int khz = 0;
        HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
        loop_timeout = (uint64_t)(std::max(khz, 1) * 1e3 * kVtLoopTimeoutS);
        HIP_TRY(d_loop.alloc(ctx, "vt.loop", loop_bytes));
    }
    auto stop_loop = [&]() -> hipError_t {  // (the mailbox's stop tags, then its tags back to 0)
        if (!running) return hipSuccess;
        for (int k = 0; k < 2 * kVtStepWords * n; k++) vt_gran_put(mail + k, 0, kVtLoopStop);
        running = false;
        const hipError_t e = hipStreamSynchronize(ctx->stream);
        for (int k = 0; k < 2 * kVtStepWords * n; k++) vt_gran_put(mail + k, 0, 0);
        return e;
    };
    struct LoopGuard {
        std::function<hipError_t()> stop;
        ~LoopGuard() { (void)stop(); }
    } loop_guard{stop_loop};
    // the host's view of what sizes the next read (:164): remChip / codeFreq / file_ptr of the
    // last step, from the records the kernel returns
    std::vector<double> remChip(n), cf_old(n), codeError(n), carrFreq(n), cf_new(n);
    std::vector<int64_t> fptr(n);
    for (int i = 0; i < n; i++) {
        remChip[i] = chans[i].remChip;
        cf_old[i] = chans[i].codeFreq;
        fptr[i] = chans[i].file_ptr;
    }
    // While a step's kernel runs, the host does the navigation work that needs none of its
    // correlations (bit for bit the work it replaces: the same functions on the same inputs):
    // the EKF's geometry half of this step (vt_nav_gain) and every channel's orbit for the next
    // step, whose read size follows from this step's without its samples (vt_remchip_next).
    // An orbit is used only at the transmit time it was computed for.
    std::vector<VtOrbit> ahead((size_t)n);
    std::vector<char> have_ahead((size_t)n, 0);
    std::unique_ptr<VtGain> gain(new VtGain);
    // Loop mode posts the next step early: of a channel's read only the carrier frequency waits
    // for the step's sums (the PLL, :305-311); its start, size, phase and divisor follow from the
    // step's own read (:161-176, :284-285), so those four words go out while the kernel runs and
    // the frequency right after vt_finish -- the EKF update and the next prediction then run
    // beside the next step's kernel. `early`: step s's words are all out; e_*: what was posted,
    // held against what the step computes when it comes (the same functions: the same bits).
    bool early = false;
    std::vector<int64_t> e_off((size_t)n), e_ns((size_t)n);
    std::vector<double> e_phi0((size_t)n), e_rfs((size_t)n), e_f((size_t)n);
    Events ev;
    double kernel_ms = 0;
    int result = GNSS_OK;
    const auto t_loop = std::chrono::steady_clock::now();
    // (probe builds, GNSS_VT_STAMPS set: the host's share of a step, printed at the end)
    const bool stamps = probe_env("GNSS_VT_STAMPS") != nullptr;
    double st_pre = 0, st_shadow = 0, st_wait = 0, st_post = 0;
    auto now_us = [] {
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    double t_a = stamps ? now_us() : 0;
    DevBuf d_vtst;  // (probe builds with GNSS_VT_STAMPS: the loop kernel's per-step marks)
    if (stamps && loop_mode) {
        const size_t nst = (size_t)kVtStampSteps * (8 + 4 * kVtLoopMaxBlocks);
        HIP_TRY(d_vtst.alloc(ctx, "vt.stamps", sizeof(unsigned long long) * nst));
        HIP_TRY(hipMemsetAsync(d_vtst.p, 0, sizeof(unsigned long long) * nst, ctx->stream));
    }
    for (int s = 0; s < nsteps && result == GNSS_OK; s++) {
        int64_t need_lo = INT64_MAX, need_hi = 0;
        for (int i = 0; i < n; i++) {
            const VtPrep p = vt_prepare(sg->Fs, sg->codelength, pdi, remChip[i], cf_old[i], cf_old[i]);
            if (p.n < 1) {  // ceil(...) <= 0: an index MATLAB rejects
                result = fail(ctx, GNSS_EINDEX, "step %d channel %d: read size %lld", s + 1, i, (long long)p.n);
                break;
            }
            double cf = cf_old[i], dpr = 0, vel[3];
            st = vt_nav_predict_at(nav, i, p.n, have_ahead[(size_t)i] ? &ahead[(size_t)i] : nullptr, &cf, &dpr, vel);
            if (st) {
                result = fail(ctx, st, "step %d channel %d: svPosVel / trop_UNB3 failed", s + 1, i);
                break;
            }
            cf_new[i] = cf;
            h_cf[i] = cf;
            gnss_vt_out& o = out[(size_t)s * n + i];
            o.deltaPr = dpr;
            o.prRate = 0;
            for (int k = 0; k < 3; k++) o.sv_vel[k] = vel[k];
            need_lo = std::min(need_lo, fptr[i]);
            need_hi = std::max(need_hi, fptr[i] + p.n * bps);
        }
        if (result) break;
        if (!file->dev_data && (need_lo < w.base || need_hi > w.base + w.len) && need_hi <= flen) {
            if (early)  // (an early post checked the same reads against this window)
                return fail(ctx, GNSS_EDEVICE, "step %d: posted early, then re-staged", s + 1);
            HIP_TRY(stop_loop());
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            st = restage(need_lo);
            if (st) return st;
            if (need_lo < w.base || need_hi > w.base + w.len)
                return fail(ctx, GNSS_EDEVICE, "step %d: the restaged IF window [%lld, %lld) does not cover the reads [%lld, %lld)",
                            s + 1, (long long)w.base, (long long)(w.base + w.len), (long long)need_lo, (long long)need_hi);
        }
        A.rec = reinterpret_cast<const uint8_t*>(w.ptr);
        A.base = w.base;
        A.len = w.len;
        if (multi) {  // (per-step events only in profiling mode: each is a queue command)
            // the step's reads (:161-176, :217-249): what vt_step_kernel sums, and what stops a
            // channel (a replica index MATLAB rejects, a read past the end of the record)
            for (int i = 0; i < n; i++) {
                const gnss_vt_chan& c = hc[(size_t)i];
                const double cf = cf_new[i];
                const VtPrep p = vt_prepare(sg->Fs, sg->codelength, pdi, c.remChip, c.codeFreq, cf);
                int b = !(cf > 0) ? GNSS_EARG : p.bad;
                if (!b) {
                    const int64_t a0 = c.file_ptr, need = p.n * bps;
                    if (a0 + need > flen) b = GNSS_EIO;
                    else if (a0 < w.base || a0 + need > w.base + w.len) b = GNSS_EIO;  // (outside the window)
                }
                pk[(size_t)i] = p;
                bad[(size_t)i] = b;
                B.ns[i] = b ? 0 : p.n;
                B.off[i] = b ? 0 : c.file_ptr - w.base;
                B.f[i] = c.carrFreq;
                B.phi0[i] = c.remCarrPhase;
                B.rfs[i] = B.ns[i] - 1 <= kmax_rfs ? rfs : 0.0;
            }
            B.rec = A.rec;
            B.seq = (unsigned)s + 1;
            if (loop_mode && early) {  // (the kernel has the step: its words were posted early)
                for (int i = 0; i < n; i++) {
                    if (bad[(size_t)i]) continue;  // (it sums the read; the channel stops below)
                    if (B.off[i] != e_off[(size_t)i] || B.ns[i] != e_ns[(size_t)i] ||
                        std::memcmp(&B.phi0[i], &e_phi0[(size_t)i], 8) || std::memcmp(&B.rfs[i], &e_rfs[(size_t)i], 8))
                        return fail(ctx, GNSS_EDEVICE, "step %d channel %d: the early post differs from the step", s + 1,
                                    i);
                }
            } else if (loop_mode) {
                if (!running) {  // (every device tag back to 0: a stopped launch left kVtLoopStop, a former call its steps)
                    HIP_TRY(hipMemsetAsync(d_loop.p, 0, loop_bytes, ctx->stream));
                    const VtLoopArgs L{B.rec, w.len, B.Fs, B.real8, B.seq, mail, gsums, loop_timeout, d_loop.p,
                                       d_loop.as<char>() + gstep_bytes, d_vtst.as<unsigned long long>()};
                    HIP_TRY(launch_vt_loop(L, n, nb, ctx->stream));
                    running = true;
                }
                // the step's reads as granules tagged with its number (VtBlockStep's word order)
                for (int i = 0; i < n; i++) {
                    VtGran* g = mail + (size_t)kVtStepWords * ((B.seq & 1) * n + i);
                    uint64_t f, phi0, rf;
                    std::memcpy(&f, &B.f[i], 8);
                    std::memcpy(&phi0, &B.phi0[i], 8);
                    std::memcpy(&rf, &B.rfs[i], 8);
                    vt_gran_put(g + 0, (uint64_t)B.off[i], B.seq);
                    vt_gran_put(g + 1, (uint64_t)B.ns[i], B.seq);
                    vt_gran_put(g + 2, f, B.seq);
                    vt_gran_put(g + 3, phi0, B.seq);
                    vt_gran_put(g + 4, rf, B.seq);
                }
            } else {
                if (ctx->profiling) HIP_TRY(hipEventRecord(ev.a, ctx->stream));
                HIP_TRY(launch_vt_step(B, n, nb, ctx->stream));
                if (ctx->profiling) HIP_TRY(hipEventRecord(ev.b, ctx->stream));
            }
        } else {
            HIP_TRY(hipMemcpyAsync(d_cf.p, h_cf, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(hipEventRecord(ev.a, ctx->stream));
            HIP_TRY(launch_vt_run(A, ctx->stream));
            HIP_TRY(hipEventRecord(ev.b, ctx->stream));
            HIP_TRY(hipMemcpyAsync(h_out, d_out.p, sizeof(gnss_vt_out) * (size_t)n, hipMemcpyDeviceToHost,
                                   ctx->stream));
        }
        double t_b = stamps ? now_us() : 0;
        if (stamps) st_pre += t_b - t_a;
        vt_nav_gain(*nav, gain.get());
        for (int i = 0; i < n && s + 1 < nsteps; i++) {
            const int64_t ns = nav->numSample[i];
            const double rc = vt_remchip_next(sg->Fs, pdi, remChip[i], cf_new[i], ns);
            const VtPrep q = vt_prepare(sg->Fs, sg->codelength, pdi, rc, cf_new[i], cf_new[i]);
            have_ahead[(size_t)i] = q.n >= 1;
            if (q.n >= 1) vt_orbit(*nav, i, vt_transmit_next(*nav, i, q.n), &ahead[(size_t)i]);
        }
        // the next step's words that need no sums of this one (`early` above)
        bool early_next = loop_mode && s + 1 < nsteps;
        for (int i = 0; i < n && early_next; i++) {
            const gnss_vt_chan& c = hc[(size_t)i];
            if (bad[(size_t)i]) {
                early_next = false;
                break;
            }
            const int64_t n0 = pk[(size_t)i].n;
            const double rc = vt_remchip_next(sg->Fs, pdi, c.remChip, cf_new[i], n0);
            const VtPrep q = vt_prepare(sg->Fs, sg->codelength, pdi, rc, cf_new[i], cf_new[i]);
            const int64_t a0 = c.file_ptr + n0 * bps, need = q.n * bps;
            if (q.n < 1 || a0 + need > flen || a0 < w.base || a0 + need > w.base + w.len) {
                early_next = false;
                break;
            }
            e_off[(size_t)i] = a0 - w.base;
            e_ns[(size_t)i] = q.n;
            e_phi0[(size_t)i] = vt_rem_carr_phase(c.carrFreq, n0, sg->Fs, c.remCarrPhase);
            e_rfs[(size_t)i] = q.n - 1 <= kmax_rfs ? rfs : 0.0;
        }
        if (early_next) {
            for (int i = 0; i < n; i++) {
                VtGran* g = mail + (size_t)kVtStepWords * (((B.seq + 1) & 1) * n + i);
                uint64_t phi0, rf;
                std::memcpy(&phi0, &e_phi0[(size_t)i], 8);
                std::memcpy(&rf, &e_rfs[(size_t)i], 8);
                vt_gran_put(g + 0, (uint64_t)e_off[(size_t)i], B.seq + 1);
                vt_gran_put(g + 1, (uint64_t)e_ns[(size_t)i], B.seq + 1);
                vt_gran_put(g + 3, phi0, B.seq + 1);
                vt_gran_put(g + 4, rf, B.seq + 1);
            }
        }
        if (stamps) {
            const double t = now_us();
            st_shadow += t - t_b;
            t_b = t;
        }
        if (!multi || ctx->profiling) HIP_TRY(hipStreamSynchronize(ctx->stream));
        if (loop_mode) HIP_TRY(wait_granules(ctx->stream, gsums, 2 * n, (unsigned)s + 1, loop_sums.data()));
        else if (multi) HIP_TRY(wait_posted(ctx->stream, B.done, (unsigned)s + 1));
        if (stamps) {
            t_a = now_us();
            st_wait += t_a - t_b;
        }
        if (ctx->profiling || !multi) kernel_ms += ev.ms();
        // loop mode, the next step posted early: its carrier frequencies first (the PLL alone; the
        // rest of vt_finish and the EKF run beside the next step's kernel)
        early = false;
        if (early_next) {
            for (int i = 0; i < n; i++) {
                const double I = loop_sums[2 * i], Q = loop_sums[2 * i + 1];
                const int cp = vt_code_at(pk[(size_t)i].j[1], pdi, [&](int j) {
                    return ((cab[(size_t)i * 32 + (j >> 5)] >> (j & 31)) & 1u) ? -1 : 1;
                });
                const double f = vt_pll(hc[(size_t)i], pdi, t1, t2, cp * I, cp * Q).carrFreq;
                uint64_t fb;
                std::memcpy(&fb, &f, 8);
                e_f[(size_t)i] = f;
                vt_gran_put(mail + (size_t)kVtStepWords * (((B.seq + 1) & 1) * n + i) + 2, fb, B.seq + 1);
            }
            early = true;
        }
        for (int i = 0; multi && i < n; i++) {  // each channel's scalar end
            gnss_vt_out& h = h_out[i];
            h = gnss_vt_out{};
            if (bad[(size_t)i]) {
                h.status = bad[(size_t)i];
                continue;
            }
            const double* sum = loop_mode ? loop_sums.data() : B.sums;
            const double I = sum[2 * i], Q = sum[2 * i + 1];
            const unsigned* cb = &cab[(size_t)i * 32];
            int code[3];
            for (int t = 0; t < 3; t++)
                code[t] = vt_code_at(pk[(size_t)i].j[t], pdi, [&](int j) { return ((cb[j >> 5] >> (j & 31)) & 1u) ? -1 : 1; });
            const int st2 = vt_finish(sg->Fs, sg->ms, pdi, bps, t1, t2, &hc[(size_t)i], pk[(size_t)i], code, cf_new[i],
                                      I, Q, &h);
            if (st2) h.status = st2;
        }
        for (int i = 0; early && i < n; i++)  // (vt_finish's frequency is the one posted: the same vt_pll)
            if (!h_out[i].status && std::memcmp(&hc[(size_t)i].carrFreq, &e_f[(size_t)i], 8))
                return fail(ctx, GNSS_EDEVICE, "step %d channel %d: the early carrier frequency differs", s + 1, i);
        for (int i = 0; i < n; i++) {
            gnss_vt_out& o = out[(size_t)s * n + i];
            const gnss_vt_out& h = h_out[i];
            const double dpr = o.deltaPr, vel[3] = {o.sv_vel[0], o.sv_vel[1], o.sv_vel[2]};
            o = h;
            o.deltaPr = dpr;
            o.prRate = 0;
            for (int k = 0; k < 3; k++) o.sv_vel[k] = vel[k];
            if (h.status) {
                if (!result) result = fail(ctx, h.status, "step %d channel %d stopped (replica index / read past EOF)",
                                           s + 1, i);
                continue;
            }
            ctx->timing.track_channel_samples += h.numSample;
            remChip[i] = h.remChip;
            cf_old[i] = h.codeFreq;
            fptr[i] = h.absoluteSample;
            codeError[i] = h.codeError;
            carrFreq[i] = h.carrFreq;
        }
        ctx->timing.track_launches += 1;
        if (result) break;
        st = vt_nav_correct(nav, *gain, codeError.data(), cf_new.data(), carrFreq.data(), sol ? sol + s : nullptr);
        if (st) result = fail(ctx, st, "step %d: navigation update failed (singular innovation covariance)", s + 1);
        if (stamps) {
            const double t = now_us();
            st_post += t - t_a;
            t_a = t;
        }
    }
    if (stamps && nsteps > 0)
        fprintf(stderr, "vt stamps (us per step): predict+post %.2f, shadow %.2f, wait %.2f, finish+correct %.2f\n",
                st_pre / nsteps, st_shadow / nsteps, st_wait / nsteps, st_post / nsteps);
    if (stamps && d_vtst.p) {  // the loop kernel's marks (GNSS_VT_PROBE & 4 builds; zeros otherwise)
        HIP_TRY(stop_loop());
        std::vector<unsigned long long> m((size_t)kVtStampSteps * (8 + 4 * kVtLoopMaxBlocks));
        HIP_TRY(hipMemcpy(m.data(), d_vtst.p, m.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        int khz = 0;
        HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
        const double us = 1e3 / std::max(khz, 1);
        double d[6] = {0, 0, 0, 0, 0, 0}, d6 = 0, d7 = 0;
        int cnt = 0;
        // the per-block marks as their maximum over the blocks (the step's last block)
        for (int k = 0; k < std::min(nsteps, kVtStampSteps); k++)
            for (int q = 0; q < 4; q++) {
                unsigned long long mx = 0;
                const unsigned long long* bm = &m[(size_t)kVtStampSteps * 8 + ((size_t)k * 4 + q) * kVtLoopMaxBlocks];
                for (int bl = 0; bl < kVtLoopMaxBlocks; bl++) mx = std::max(mx, bm[bl]);
                m[(size_t)8 * k + (q == 0 ? 2 : q == 1 ? 3 : q == 2 ? 6 : 7)] = mx;
            }
        for (int k = 10; k + 1 < std::min(nsteps, kVtStampSteps); k++) {
            const unsigned long long* r = &m[(size_t)8 * k];
            const unsigned long long* r1 = &m[(size_t)8 * (k + 1)];
            if (!r[0] || !r[5] || !r1[0]) continue;
            for (int j = 0; j < 5; j++) d[j] += (double)(long long)(r[j + 1] - r[j]) * us;
            d[5] += (double)(long long)(r1[0] - r[5]) * us;
            if (r[6] && r[7]) {
                d6 += (double)(long long)(r[6] - r[2]) * us;
                d7 += (double)(long long)(r[7] - r[6]) * us;
            }
            cnt++;
        }
        if (cnt)
            fprintf(stderr, "vt loop marks (us per step, %d steps): relay %.2f, to last block %.2f, to last sums %.2f "
                            "(last terms %.2f after the last block had the step, butterfly %.2f), gather %.2f, "
                            "sums out %.2f, sums out -> next mailbox seen %.2f\n",
                    cnt, d[0] / cnt, d[1] / cnt, d[2] / cnt, d6 / cnt, d7 / cnt, d[3] / cnt, d[4] / cnt, d[5] / cnt);
    }
    HIP_TRY(stop_loop());
    if (!multi) HIP_TRY(hipMemcpyAsync(chans, d_chan.p, sizeof(gnss_vt_chan) * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (multi) std::copy(hc.begin(), hc.end(), chans);
    ctx->timing.track_kernel_ms = kernel_ms;  // (int8 records: summed in profiling mode only)
    ctx->timing.track_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_loop).count();
    return result;
}

int gnss_ca_code(int prn, int8_t* out1023)
{
    if (prn < 1 || prn > 51 || !out1023) return GNSS_EARG;
    float f[1023];
    generate_ca(prn, f);
    for (int i = 0; i < 1023; i++) out1023[i] = (int8_t)f[i];
    return GNSS_OK;
}

int gnss_synth_if_device(gnss_ctx* ctx, const gnss_synth* cfg, uint64_t sample0, uint64_t nsamples,
                         void* dev_dst)
{
    if (!ctx || !cfg || !dev_dst || cfg->n_sv < 0 || cfg->n_sv > GNSS_MAX_SV) return GNSS_EARG;
    drop_resident(ctx, dev_dst, 2 * nsamples);  // (int8 I/Q: a member's copy of these bytes is stale now)
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<float> cah((size_t)std::max(1, cfg->n_sv) * 1023);
    for (int i = 0; i < cfg->n_sv; i++) {
        if (cfg->sv[i].prn < 1 || cfg->sv[i].prn > 51) return GNSS_EARG;
        generate_ca(cfg->sv[i].prn, &cah[(size_t)i * 1023]);
    }
    DevBuf ca;
    HIP_TRY(ca.alloc(cah.size() * sizeof(float)));
    HIP_TRY(hipMemcpyAsync(ca.p, cah.data(), cah.size() * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(launch_synth_if(*cfg, ca.as<float>(), sample0, nsamples, static_cast<int8_t*>(dev_dst), ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return GNSS_OK;
}

}  // extern "C"
