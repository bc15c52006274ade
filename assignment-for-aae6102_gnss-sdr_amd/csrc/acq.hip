// acq.hip — acquisition.m parallel-code-phase search for gfx950 (MI355X).
//
// Reference: SDR_MATLAB-main/acqtckpos/acquisition.m. The reference recomputes
// fft(replica) and the PRN-invariant signal FFT inside its PRN x ms x bin loop
// (quirk A.2); here the signal spectra are computed once per (ms, bin) and the
// code spectra once per PRN, both by batched rocFFT. The kernels below are the
// parts around the transforms: carrier wipe, conj-product, |.|^2 non-coherent
// accumulation (fixed ms order), and the two-level peak / SNR detector with
// MATLAB's first-index semantics. Fine frequency uses an fp64 zero-padded FFT.
#include "gnss_internal.h"

namespace gnss {

namespace {

__device__ __forceinline__ float sin_rev(float x) { return __builtin_amdgcn_sinf(x); }
__device__ __forceinline__ float cos_rev(float x) { return __builtin_amdgcn_cosf(x); }

// The rocFFT path's kernels, in fp32 (fast mode) or fp64 (the reference's precision):
// V = float2 / double2, R its scalar.
template <class V> struct ScalarOf;
template <> struct ScalarOf<float2> { using T = float; };
template <> struct ScalarOf<double2> { using T = double; };

template <class V>
__device__ __forceinline__ V mkv(typename ScalarOf<V>::T x, typename ScalarOf<V>::T y)
{
    V r;
    r.x = x;
    r.y = y;
    return r;
}

// temp1 = rawsignal(ms idx) .* carrier(freqband,:)  (acquisition.m:41-44,56)
// carrier(b, n) = exp(1i*2*pi*(IF + freqMin + freqStep*(b-1))*n/Fs), n = 1..S
template <class Src, class V>
__global__ void acq_wipe_kernel(const Src src, int64_t S, int datalen, int nbins,
                                double IF, double freqMin, double freqStep, double Fs,
                                V* __restrict__ out)
{
    using R = typename ScalarOf<V>::T;
    const int j = blockIdx.y;  // (idx, b) pair: j = idx*nbins + b
    const int idx = j / nbins, b = j - idx * nbins;
    const double f = (IF + (freqMin + freqStep * (double)b)) / Fs;  // cycles per sample
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < S;
         n += (int64_t)gridDim.x * blockDim.x) {
        double cyc = f * (double)(n + 1);
        cyc -= floor(cyc);
        R c, s;
        if constexpr (sizeof(R) == 4) {
            const float ph = (float)cyc;
            c = cos_rev(ph);
            s = sin_rev(ph);
        } else {
            sincospi(2.0 * cyc, &s, &c);
        }
        const double2 x = src.at((int64_t)idx * S + n);
        const R xr = (R)x.x, xi = (R)x.y;
        out[(int64_t)j * S + n] = mkv<V>(xr * c - xi * s, xr * s + xi * c);
    }
}

// scode = [CA CA](ceil(n*(codeFreqBasis/Fs))), n = 1..S  (acquisition.m:49-51)
template <class V>
__global__ void acq_code_kernel(const float* __restrict__ ca, int nprn, int64_t S, double step,
                                V* __restrict__ out)
{
    using R = typename ScalarOf<V>::T;
    const int p = blockIdx.y;
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < S;
         n += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ci = (int64_t)ceil((double)(n + 1) * step);  // 1-based into [CA CA]
        out[(int64_t)p * S + n] = mkv<V>((R)ca[(int64_t)p * 1023 + (ci - 1) % 1023], (R)0);
    }
}

// temp3 .* conj(fft(temp1))  (acquisition.m:57-59): y[p][j][k] = C[p][k] * conj(X[j][k])
template <class V>
__global__ void acq_mul_kernel(const V* __restrict__ C, const V* __restrict__ X,
                               int nsig, int64_t S, V* __restrict__ y)
{
    const int j = blockIdx.y, p = blockIdx.z;
    const V* c = C + (int64_t)p * S;
    const V* x = X + (int64_t)j * S;
    V* o = y + ((int64_t)p * nsig + j) * S;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < S;
         k += (int64_t)gridDim.x * blockDim.x) {
        const V a = c[k], b = x[k];
        // (ar + i ai)(br - i bi)
        o[k] = mkv<V>(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
    }
}

// correlation(b,:) = sum over ms of abs(ifft(.)).^2 (acquisition.m:53-61), ms order fixed
template <class V>
__global__ void acq_power_kernel(const V* __restrict__ y, int nbins, int datalen, int64_t S,
                                 typename ScalarOf<V>::T scale, typename ScalarOf<V>::T* __restrict__ corr)
{
    using R = typename ScalarOf<V>::T;
    const int b = blockIdx.y, p = blockIdx.z;
    const int nsig = nbins * datalen;
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < S;
         n += (int64_t)gridDim.x * blockDim.x) {
        R acc = 0;
        for (int idx = 0; idx < datalen; idx++) {
            const V v = y[((int64_t)p * nsig + (int64_t)idx * nbins + b) * S + n];
            acc += (v.x * v.x + v.y * v.y) * scale;
        }
        corr[((int64_t)p * nbins + b) * S + n] = acc;
    }
}

// (the surface is fp32 in the fast mode, fp64 at the reference's precision)
template <class R> struct PeakPart {
    R m;
    int32_t bin, col;
};

template <class R>
__device__ __forceinline__ void peak_merge(R& m, int& bin, int& col, R m2, int b2, int c2)
{
    if (m2 > m) { m = m2; bin = b2; col = c2; }
    else if (m2 == m) { bin = min(bin, b2); col = min(col, c2); }
}

// [~,fbin] = max(max(corr')); [peak,codePhase] = max(max(corr)) (acquisition.m:62-63):
// the global max; fbin = first bin holding it, codePhase = first column holding it.
// perm = P: the surface is stored tau2-major (acq_fft.hip), storage k -> column
// k / 2000 + P * (k % 2000); perm = 0: natural order.
__device__ __forceinline__ int64_t natural_col(int64_t k, int perm)
{
    return perm ? k / 2000 + (int64_t)perm * (k % 2000) : k;
}


template <class R>
__global__ void acq_peak_part_kernel(const R* __restrict__ corr, int nbins, int64_t S,
                                     int nblk, int perm, PeakPart<R>* __restrict__ part)
{
    const int p = blockIdx.y, blk = blockIdx.x;
    const R* c = corr + (int64_t)p * nbins * S;
    R m = (R)-1;
    int bin = 0x7fffffff, col = 0x7fffffff;
    // (a column's bins loaded 8 at a time before they are merged: the merge keeps the maximum
    // with the lowest bin / column on ties, so its order does not matter; one load per merge
    // waited for each L2 round trip)
    for (int64_t k = (int64_t)blk * blockDim.x + threadIdx.x; k < S; k += (int64_t)nblk * blockDim.x) {
        const int ck = (int)natural_col(k, perm);
        for (int b0 = 0; b0 < nbins; b0 += 8) {
            R v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = c[(int64_t)(b0 + u < nbins ? b0 + u : nbins - 1) * S + k];
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (b0 + u < nbins) peak_merge(m, bin, col, v[u], b0 + u, ck);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const R m2 = __shfl_xor(m, o, 64);
        const int b2 = __shfl_xor(bin, o, 64), c2 = __shfl_xor(col, o, 64);
        peak_merge(m, bin, col, m2, b2, c2);
    }
    __shared__ PeakPart<R> s[16];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) s[wv] = PeakPart<R>{m, bin, col};
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) peak_merge(m, bin, col, s[w].m, s[w].bin, s[w].col);
        part[(int64_t)p * nblk + blk] = PeakPart<R>{m, bin, col};
    }
}

// Merge the partials, then SNR = 10*log10(peak^2 / mean(corr(fbin, off-peak).^2))
// with the off-peak range [1:cp-cshift, cp+cshift:end] (acquisition.m:66-68).
template <class R>
__global__ void acq_peak_final_kernel(const R* __restrict__ corr, int nbins, int64_t S,
                                      int nblk, int cshift, int perm, const PeakPart<R>* __restrict__ part,
                                      AcqPeak* __restrict__ out)
{
    const int p = blockIdx.x;
    __shared__ R s_m;
    __shared__ int s_bin, s_col;
    __shared__ double s_sum[16], s_cnt[16], s_mx[16];
    if (threadIdx.x == 0) {
        R m = (R)-1;
        int bin = 0x7fffffff, col = 0x7fffffff;
        for (int k = 0; k < nblk; k++) {
            const PeakPart<R> q = part[(int64_t)p * nblk + k];
            peak_merge(m, bin, col, q.m, q.bin, q.col);
        }
        s_m = m; s_bin = bin; s_col = col;
    }
    __syncthreads();
    const int fbin = s_bin;
    const int64_t cp1 = (int64_t)s_col + 1;  // 1-based codePhase
    const R* row = corr + ((int64_t)p * nbins + fbin) * S;
    double sum = 0, cnt = 0, mx = 0;
    // in storage order (coalesced; the permuted surface's natural order strides 2 000 entries
    // across a wave), 8 loads in flight
#pragma unroll 8
    for (int64_t q = threadIdx.x; q < S; q += blockDim.x) {
        const int64_t k = natural_col(q, perm) + 1;  // 1-based column
        const double v = (double)row[q];
        const bool off = k <= cp1 - cshift || k >= cp1 + cshift;
        sum += off ? v * v : 0.0;  // (+0.0 leaves a non-negative sum unchanged)
        cnt += off ? 1.0 : 0.0;
        mx = off ? fmax(mx, v) : mx;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o, 64);
        cnt += __shfl_xor(cnt, o, 64);
        mx = fmax(mx, __shfl_xor(mx, o, 64));
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s_sum[wv] = sum; s_cnt[wv] = cnt; s_mx[wv] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
            sum += s_sum[w]; cnt += s_cnt[w]; mx = fmax(mx, s_mx[w]);
        }
        const double pk = (double)s_m;
        AcqPeak r;
        r.peak = (double)s_m;
        r.fbin = fbin;
        r.cp = s_col;
        r.snr = 10.0 * log10((pk * pk) / (sum / cnt));
        r.peak2 = mx;
        out[p] = r;
    }
}

// CarrSignal = longrawsignal(S-cd : S-cd+L*S-1) .* longCaCode, zero-padded to N
// (acquisition.m:103-108); fp64, code index floor((1/Fs*k)/(1/fc)) as the reference.
template <class Src>
__global__ void fine_build_kernel(const Src src, int64_t S, int L,
                                  const int32_t* __restrict__ codedelay,
                                  const float* __restrict__ ca, double invFs, double invFc,
                                  double codelength, int64_t N, double2* __restrict__ out)
{
    const int s = blockIdx.y;
    const int64_t Ls = (int64_t)L * S;
    const int64_t base = S - codedelay[s] - 1;  // 0-based sample of k = 1
    double2* o = out + (int64_t)s * N;
    for (int64_t k0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k0 < N;
         k0 += (int64_t)gridDim.x * blockDim.x) {
        double2 v = make_double2(0.0, 0.0);
        if (k0 < Ls) {
            const double cvi = floor((invFs * (double)(k0 + 1)) / invFc);
            const float code = ca[(int64_t)s * 1023 + (int64_t)fmod(cvi, codelength)];
            const double2 x = src.at(base + k0);
            v = make_double2(x.x * code, x.y * code);
        }
        o[k0] = v;
    }
}

struct FinePart {
    double m;
    int64_t i;
};

// first max of abs(fftshift(F)) (acquisition.m:110-116); shifted index i maps to
// unshifted (i + N/2) mod N.
__global__ void fine_argmax_part_kernel(const double2* __restrict__ F, int64_t N, int shifted,
                                        int nblk, FinePart* __restrict__ part)
{
    const int s = blockIdx.y, blk = blockIdx.x;
    const double2* f = F + (int64_t)s * N;
    double m = -1.0;
    int64_t bi = INT64_MAX;
    const int64_t half = N / 2;
    for (int64_t i = (int64_t)blk * blockDim.x + threadIdx.x; i < N;
         i += (int64_t)nblk * blockDim.x) {
        int64_t j = shifted == 1 ? i + half : i;
        if (j >= N) j -= N;
        const double2 v = f[j];
        const double a = hypot(v.x, v.y);
        // shifted 2: real CarrSignal, exactly conjugate-symmetric in MATLAB -> the lower
        // index of a mirror pair
        const int64_t ii = (shifted == 2 && N - i < i) ? N - i : i;
        if (a > m || (a == m && ii < bi)) { m = a; bi = ii; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double m2 = __shfl_xor(m, o, 64);
        const int64_t i2 = __shfl_xor(bi, o, 64);
        if (m2 > m || (m2 == m && i2 < bi)) { m = m2; bi = i2; }
    }
    __shared__ FinePart sp[16];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sp[wv] = FinePart{m, bi};
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++)
            if (sp[w].m > m || (sp[w].m == m && sp[w].i < bi)) { m = sp[w].m; bi = sp[w].i; }
        part[(int64_t)s * nblk + blk] = FinePart{m, bi};
    }
}

__global__ void fine_argmax_final_kernel(const FinePart* __restrict__ part, int nblk,
                                         int64_t* __restrict__ kbest)
{
    const int s = blockIdx.x;
    if (threadIdx.x) return;
    double m = -1.0;
    int64_t bi = INT64_MAX;
    for (int k = 0; k < nblk; k++) {
        const FinePart q = part[(int64_t)s * nblk + k];
        if (q.m > m || (q.m == m && q.i < bi)) { m = q.m; bi = q.i; }
    }
    kbest[s] = bi + 1;  // 1-based FreqPeakIndex
}

constexpr int kPeakBlocks = 128;
constexpr int kFineBlocks = 512;

}  // namespace

template <class V>
static hipError_t launch_acq_wipe_t(const int8_t* iq, const double2* xs, int64_t S, int datalen, int nbins,
                                    double IF, double freqMin, double freqStep, double Fs, V* out, hipStream_t s)
{
    dim3 grid((unsigned)((S + 255) / 256), (unsigned)(datalen * nbins));
    if (xs)
        hipLaunchKernelGGL((acq_wipe_kernel<SrcC64, V>), grid, dim3(256), 0, s, SrcC64{xs}, S, datalen, nbins, IF,
                           freqMin, freqStep, Fs, out);
    else
        hipLaunchKernelGGL((acq_wipe_kernel<SrcIQ8, V>), grid, dim3(256), 0, s, SrcIQ8{iq}, S, datalen, nbins, IF,
                           freqMin, freqStep, Fs, out);
    return hipGetLastError();
}

template <class V>
static hipError_t launch_acq_code_t(const float* ca, int nprn, int64_t S, double codeFreqBasis, double Fs, V* out,
                                    hipStream_t s)
{
    dim3 grid((unsigned)((S + 255) / 256), (unsigned)nprn);
    hipLaunchKernelGGL(acq_code_kernel<V>, grid, dim3(256), 0, s, ca, nprn, S, codeFreqBasis / Fs, out);
    return hipGetLastError();
}

template <class V>
static hipError_t launch_acq_mul_t(const V* code_spec, const V* sig_spec, int nprn, int nsig, int64_t S, V* out,
                                   hipStream_t s)
{
    dim3 grid((unsigned)((S + 1023) / 1024), (unsigned)nsig, (unsigned)nprn);
    hipLaunchKernelGGL(acq_mul_kernel<V>, grid, dim3(256), 0, s, code_spec, sig_spec, nsig, S, out);
    return hipGetLastError();
}

template <class V>
static hipError_t launch_acq_power_t(const V* y, int nprn, int nbins, int datalen, int64_t S,
                                     typename ScalarOf<V>::T* corr, hipStream_t s)
{
    using R = typename ScalarOf<V>::T;
    dim3 grid((unsigned)((S + 255) / 256), (unsigned)nbins, (unsigned)nprn);
    const R scale = (R)(1.0 / ((double)S * (double)S));  // ifft's 1/N, squared
    hipLaunchKernelGGL(acq_power_kernel<V>, grid, dim3(256), 0, s, y, nbins, datalen, S, scale, corr);
    return hipGetLastError();
}

hipError_t launch_acq_wipe(const int8_t* iq, const double2* xs, int64_t S, int datalen, int nbins, double IF,
                           double freqMin, double freqStep, double Fs, float2* out, hipStream_t s)
{
    return launch_acq_wipe_t(iq, xs, S, datalen, nbins, IF, freqMin, freqStep, Fs, out, s);
}
hipError_t launch_acq_wipe(const int8_t* iq, const double2* xs, int64_t S, int datalen, int nbins, double IF,
                           double freqMin, double freqStep, double Fs, double2* out, hipStream_t s)
{
    return launch_acq_wipe_t(iq, xs, S, datalen, nbins, IF, freqMin, freqStep, Fs, out, s);
}
hipError_t launch_acq_code(const float* ca, const int32_t* /*prn_slot*/, int nprn, int64_t S,
                           double codeFreqBasis, double Fs, float2* out, hipStream_t s)
{
    return launch_acq_code_t(ca, nprn, S, codeFreqBasis, Fs, out, s);
}
hipError_t launch_acq_code(const float* ca, const int32_t* /*prn_slot*/, int nprn, int64_t S,
                           double codeFreqBasis, double Fs, double2* out, hipStream_t s)
{
    return launch_acq_code_t(ca, nprn, S, codeFreqBasis, Fs, out, s);
}
hipError_t launch_acq_mul(const float2* code_spec, const float2* sig_spec, int nprn, int nsig,
                          int64_t S, float2* out, hipStream_t s)
{
    return launch_acq_mul_t(code_spec, sig_spec, nprn, nsig, S, out, s);
}
hipError_t launch_acq_mul(const double2* code_spec, const double2* sig_spec, int nprn, int nsig,
                          int64_t S, double2* out, hipStream_t s)
{
    return launch_acq_mul_t(code_spec, sig_spec, nprn, nsig, S, out, s);
}
hipError_t launch_acq_power(const float2* y, int nprn, int nbins, int datalen, int64_t S,
                            int /*first_ms*/, float* corr, hipStream_t s)
{
    return launch_acq_power_t(y, nprn, nbins, datalen, S, corr, s);
}
hipError_t launch_acq_power(const double2* y, int nprn, int nbins, int datalen, int64_t S,
                            int /*first_ms*/, double* corr, hipStream_t s)
{
    return launch_acq_power_t(y, nprn, nbins, datalen, S, corr, s);
}

template <class R>
static hipError_t launch_acq_peak_t(const R* corr, int nprn, int nbins, int64_t S, int cshift,
                                    int perm, AcqPeak* out, void* scratch, hipStream_t s)
{
    PeakPart<R>* part = reinterpret_cast<PeakPart<R>*>(scratch);
    hipLaunchKernelGGL(acq_peak_part_kernel<R>, dim3(kPeakBlocks, nprn), dim3(256), 0, s, corr, nbins, S,
                       kPeakBlocks, perm, part);
    hipLaunchKernelGGL(acq_peak_final_kernel<R>, dim3(nprn), dim3(256), 0, s, corr, nbins, S,
                       kPeakBlocks, cshift, perm, part, out);
    return hipGetLastError();
}

hipError_t launch_acq_peak(const float* corr, int nprn, int nbins, int64_t S, int cshift,
                           int perm, AcqPeak* out, void* scratch, hipStream_t s)
{
    return launch_acq_peak_t(corr, nprn, nbins, S, cshift, perm, out, scratch, s);
}

hipError_t launch_acq_peak(const double* corr, int nprn, int nbins, int64_t S, int cshift,
                           int perm, AcqPeak* out, void* scratch, hipStream_t s)
{
    return launch_acq_peak_t(corr, nprn, nbins, S, cshift, perm, out, scratch, s);
}

hipError_t launch_fine_build(const int8_t* iq, const double2* xs, int64_t S, int L, const int32_t* codedelay,
                             const float* ca, int nsv, double Fs, double codeFreqBasis,
                             double codelength, int64_t N, double2* out, hipStream_t s)
{
    dim3 grid(4096, (unsigned)nsv);
    if (xs)
        hipLaunchKernelGGL(fine_build_kernel<SrcC64>, grid, dim3(256), 0, s, SrcC64{xs}, S, L, codedelay, ca,
                           1 / Fs, 1 / codeFreqBasis, codelength, N, out);
    else
        hipLaunchKernelGGL(fine_build_kernel<SrcIQ8>, grid, dim3(256), 0, s, SrcIQ8{iq}, S, L, codedelay, ca,
                           1 / Fs, 1 / codeFreqBasis, codelength, N, out);
    return hipGetLastError();
}

hipError_t launch_fine_argmax(const double2* F, int nsv, int64_t N, int shifted, void* scratch,
                              int64_t* kbest, hipStream_t s)
{
    FinePart* part = reinterpret_cast<FinePart*>(scratch);
    hipLaunchKernelGGL(fine_argmax_part_kernel, dim3(kFineBlocks, nsv), dim3(256), 0, s, F, N,
                       shifted, kFineBlocks, part);
    hipLaunchKernelGGL(fine_argmax_final_kernel, dim3(nsv), dim3(64), 0, s, part, kFineBlocks, kbest);
    return hipGetLastError();
}

size_t acq_scratch_bytes(int nprn, int nsv)
{
    size_t a = sizeof(PeakPart<double>) * (size_t)kPeakBlocks * (size_t)nprn;
    size_t b = sizeof(FinePart) * (size_t)kFineBlocks * (size_t)nsv;
    return a > b ? a : b;
}

}  // namespace gnss
