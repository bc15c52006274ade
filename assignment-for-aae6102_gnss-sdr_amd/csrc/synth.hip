// synth.hip — deterministic synthetic GPS L1 C/A IF record, int8 I/Q.
// Same algorithm as the CPU twin in oracle/gnss_oracle.c (or_synth_if): per SV a
// C/A code at rate 1.023e6*(1 + fd/1575.42e6) chips/s, 50 bps nav bits, carrier at
// -(IF + fd) so that the reference's exp(+j*2*pi*(IF+fd)*t) wipes it, plus AWGN
// from a counter-based hash. Used to make multi-GB records directly in HBM for
// the benchmark (no PCIe upload inside or before the timed region).
#include "gnss_internal.h"

namespace gnss {

namespace {

constexpr int kLnavBits = 3000;  // two LNAV frames (60 s), repeated

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct SynthSv {
    double amp, crate, frate, code_phase0, carr_phase0, bit_phase;
    uint64_t bit_seed;
    int32_t lnav, pad;
};

__global__ void synth_kernel(const SynthSv* __restrict__ sv, int nsv, const float* __restrict__ ca,
                             double sigma, uint64_t seed, uint64_t sample0, uint64_t nsamples,
                             int8_t* __restrict__ dst, const int8_t* __restrict__ lnav_bits)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsamples;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t n = sample0 + i;
        double re = 0, im = 0;
        for (int s = 0; s < nsv; s++) {
            const SynthSv v = sv[s];
            const double th = v.code_phase0 + (double)n * v.crate;
            int64_t chip = (int64_t)floor(th) % 1023;
            if (chip < 0) chip += 1023;
            const double bitf = floor((th + v.bit_phase) / 20460.0);
            double D;
            if (v.lnav) {  // LNAV bit b -> (-1)^b (gnss_lnav_bits, kLnavBits-bit cycle)
                int64_t k = (int64_t)bitf % kLnavBits;
                if (k < 0) k += kLnavBits;
                D = lnav_bits[k] ? -1.0 : 1.0;
            } else {
                const uint64_t bh = mix64(v.bit_seed ^ (uint64_t)(int64_t)bitf);
                D = (bh & 1) ? 1.0 : -1.0;
            }
            double ph = v.carr_phase0 - (double)n * v.frate;
            ph -= floor(ph);
            const double a = v.amp * D * (double)ca[s * 1023 + chip];
            double sn, cs;
            sincos(kTwoPi * ph, &sn, &cs);
            re += a * cs;
            im += a * sn;
        }
        const uint64_t h1 = mix64(seed ^ (n * 0xD1B54A32D192ED03ULL));
        const uint64_t h2 = mix64(h1 ^ 0x8CB92BA72F3D8DD7ULL);
        const double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);
        const double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
        const double r = sqrt(-2.0 * log(u1)) * sigma;
        double sn, cs;
        sincos(kTwoPi * u2, &sn, &cs);
        double vi = rint(re + r * cs), vq = rint(im + r * sn);
        vi = fmin(127.0, fmax(-128.0, vi));
        vq = fmin(127.0, fmax(-128.0, vq));
        char2 o;
        o.x = (signed char)vi;
        o.y = (signed char)vq;
        reinterpret_cast<char2*>(dst)[i] = o;
    }
}

}  // namespace

hipError_t launch_synth_if(const gnss_synth& cfg, const float* ca, uint64_t sample0,
                           uint64_t nsamples, int8_t* dst, hipStream_t s)
{
    const double fL1 = 1575.42e6, fc = 1.023e6;
    SynthSv h[GNSS_MAX_SV];
    for (int i = 0; i < cfg.n_sv; i++) {
        const gnss_synth_sv& v = cfg.sv[i];
        const double snr_lin = pow(10.0, v.cn0_dbhz / 10.0);
        h[i].amp = sqrt(2.0 * cfg.noise_sigma * cfg.noise_sigma * snr_lin / cfg.Fs);
        h[i].crate = fc * (1.0 + v.doppler_hz / fL1) / cfg.Fs;
        h[i].frate = (cfg.IF + v.doppler_hz) / cfg.Fs;
        h[i].code_phase0 = v.code_phase0;
        h[i].carr_phase0 = v.carr_phase0;
        h[i].bit_phase = v.bit_phase_chips;
        h[i].bit_seed = v.bit_seed;
        h[i].lnav = v.lnav;
        h[i].pad = 0;
    }
    SynthSv* d = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(SynthSv) * GNSS_MAX_SV + kLnavBits, s);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(d, h, sizeof(SynthSv) * (size_t)(cfg.n_sv > 0 ? cfg.n_sv : 1),
                       hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    static int8_t lnav[kLnavBits];  // (the same message on every SV)
    static bool lnav_ready = false;
    if (!lnav_ready) {
        (void)gnss_lnav_bits(1, kLnavBits, lnav);
        lnav_ready = true;
    }
    int8_t* d_lnav = reinterpret_cast<int8_t*>(d + GNSS_MAX_SV);
    e = hipMemcpyAsync(d_lnav, lnav, kLnavBits, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    const uint64_t blocks = (nsamples + 255) / 256;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0,
                       s, d, cfg.n_sv, ca, cfg.noise_sigma, cfg.seed, sample0, nsamples, dst, d_lnav);
    e = hipGetLastError();
    (void)hipFreeAsync(d, s);
    return e;
}

}  // namespace gnss
