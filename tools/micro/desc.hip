// Tail probe: one wave runs pieces of the tracking tail (prepare_desc role 0, the DLL half
// of loop_update, step_size, colon_make_hint) in dependent loops; wall clock per call.
// Built from track.hip itself (same inlining): hipcc --offload-arch=gfx950 -O3
// -std=c++17 -ffp-contract=off tools/micro/desc.hip -o tools/micro/desc
#include "../../assignment-for-aae6102_gnss-sdr_amd/csrc/track.hip"
#include <cstdio>

namespace gnss {
__global__ void desc_probe(const TrkParams* pp, StepDesc* d, unsigned long long* t, int reps)
{
    const TrkParams& p = *pp;
    const int lane = threadIdx.x;
    NcoState c{0.001, 1.0, 1.023e6 + 0.3, 4.58e6 + 1234.5, 580000, 1000000, 1000};
    TrkChan ch{};
    ch.codeFreq = c.codeFreq;
    unsigned long long w0;
    // 0: prepare_desc role 0 (code side, 3 taps)
    w0 = wall_clock64();
    for (int i = 0; i < reps; i++) {
        prepare_desc_i(p, c, 10, 0, 0, lane, d);
        c.remChip = d->remChip_next * 1e-3;  // dependency through the output
    }
    t[0] = wall_clock64() - w0;
    // 1: DLL half of the loop update
    double e = 1000.0;
    w0 = wall_clock64();
    for (int i = 0; i < reps; i++) {
        const LoopUpd u = loop_update_i(p, ch, e, 2.0, 3.0, 4.0, 900.0, 5.0, 10, 0, 1);
        e = 1000.0 + u.codeFreq * 1e-9;
    }
    t[1] = wall_clock64() - w0;
    // 2: step_size
    w0 = wall_clock64();
    for (int i = 0; i < reps; i++) {
        const StepSize z = step_size(p, c, 10, 0);
        c.remChip = (double)z.n * 1e-9;
    }
    t[2] = wall_clock64() - w0;
    // 3: colon_make_hint + ends
    double a = 0.5 + lane * 1e-3, cps = 1.023e6 / 58e6;
    int64_t n = 580000;
    w0 = wall_clock64();
    for (int i = 0; i < reps; i++) {
        const double bb = ((double)(n - 1) * cps + 0.5) + a;
        const Colon col = colon_make_hint(a, cps, bb, n - 1);
        a = 0.5 + (colon_elem(col, n - 1) - bb) * 1e-3;
    }
    t[3] = wall_clock64() - w0;
    // 4: role 1 (carrier table, sincos per lane)
    w0 = wall_clock64();
    for (int i = 0; i < reps; i++) {
        prepare_desc_i(p, c, 10, 0, 1, lane, d);
        c.carrierFreq = 4.58e6 + d->phi[3] * 1e-9;
    }
    t[4] = wall_clock64() - w0;
    if (lane == 0) t[5] = d->n;
}
}  // namespace gnss

int main()
{
    using namespace gnss;
    TrkParams P{};
    P.Fs = 58e6; P.codeFreqBasis = 1.023e6; P.ms = 1e-3; P.codelength = 1023; P.S = 58000;
    P.tau1code = 0.00703054225877465; P.tau2code = 0.3749245; P.tau1carr = 3.1246854483442903e-4;
    P.tau2carr = 0.04998993333333334; P.dataBytesPerSample = 2; P.inv_Fs = 1 / 58e6;
    P.buf_base = 0; P.buf_len = 1LL << 40; P.file_len = 1LL << 40; P.ntaps = 3; P.iE = 0; P.iP = 1; P.iL = 2;
    P.nsv = 1; P.nch = 1; P.bps = 2; P.taps[0] = -0.5; P.taps[2] = 0.5;
    TrkParams* dP; StepDesc* dD; unsigned long long* dT;
    hipMalloc(&dP, sizeof P); hipMalloc(&dD, sizeof(StepDesc)); hipMalloc(&dT, 8 * sizeof(unsigned long long));
    hipMemcpy(dP, &P, sizeof P, hipMemcpyHostToDevice);
    const int reps = 200;
    unsigned long long t[8];
    for (int it = 0; it < 3; it++) {
        hipLaunchKernelGGL(desc_probe, dim3(1), dim3(64), 0, 0, dP, dD, dT, reps);
        hipDeviceSynchronize();
    }
    hipMemcpy(t, dT, sizeof t, hipMemcpyDeviceToHost);
    const char* nm[] = {"prepare_desc role 0 (code)", "loop_update DLL half", "step_size", "colon_make_hint+end",
                        "prepare_desc role 1 (carrier)"};
    for (int k = 0; k < 5; k++) printf("%-32s %8.1f ns per call\n", nm[k], t[k] * 10.0 / reps);
    printf("n = %llu\n", t[5]);
    return 0;
}
