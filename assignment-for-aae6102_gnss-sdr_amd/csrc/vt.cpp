// vt.cpp — the host half of a vector-tracking step (trackingVT_POS_updated.m:157-349):
// read sizing, the three replica chips of the reference's linear-indexing quirk, the
// remaining code / carrier phase, the C/N0 estimator, the PLL and the DLL discriminator
// (vt_prepare / vt_finish in gnss_internal.h: the same source as the kernel's scalar end,
// vt.hip). Compiled with -ffp-contract=off like the rest of the library, so every
// operation rounds as MATLAB's does.
// Reference: SDR_MATLAB-main/acqtckpos/trackingVT_POS_updated.m (line cites inline).
#include <cmath>

#include "gnss_internal.h"

using namespace gnss;

namespace {

int valid_signal(const gnss_signal* sg, int pdi)
{
    return sg && sg->Fs > 0 && sg->codeFreqBasis > 0 && pdi >= 1;
}

}  // namespace

extern "C" {

int gnss_vt_prepare(const gnss_signal* sg, int32_t pdi, const gnss_vt_chan* c, double codeFreq_new,
                    int32_t code_out[3], int64_t* numSample)
{
    if (!valid_signal(sg, pdi) || !c || !code_out || c->prn < 1 || c->prn > 51 || !(c->codeFreq > 0) ||
        !(codeFreq_new > 0))
        return GNSS_EARG;
    // numSample with the LAST step's codeFreq (:161; the new one is predicted further down
    // the loop body, :211-215, and builds the colons, :217-222)
    const VtPrep p = vt_prepare(sg->Fs, sg->codelength, pdi, c->remChip, c->codeFreq, codeFreq_new);
    if (p.bad) return p.bad;
    if (numSample) *numSample = p.n;
    float ca[1023];
    ca_chips(c->prn, ca);
    for (int s = 0; s < 3; s++)
        code_out[s] = vt_code_at(p.j[s], pdi, [&](int i) { return ca[i] < 0 ? -1 : 1; });
    return GNSS_OK;
}

int gnss_vt_nco_step(const gnss_signal* sg, const gnss_track* tr, int32_t pdi, gnss_vt_chan* c,
                     double codeFreq_new, double sumI, double sumQ, gnss_vt_out* out)
{
    if (!tr || !out || !c) return GNSS_EARG;
    // the C/N0 window index vt_finish writes Zk[index_int] at (:294-295)
    if (c->index_int < 0 || c->index_int > 19 || c->snrIndex < 1) return GNSS_EARG;
    int32_t code[3];
    int64_t n = 0;
    const int st = gnss_vt_prepare(sg, pdi, c, codeFreq_new, code, &n);
    if (st) return st;
    const VtPrep p = vt_prepare(sg->Fs, sg->codelength, pdi, c->remChip, c->codeFreq, codeFreq_new);
    double t1, t2;
    calc_loop_coef(tr->PLLBW, tr->PLLDamp, tr->PLLGain, t1, t2);
    const int cd[3] = {code[0], code[1], code[2]};
    // int8 I/Q byte offsets (dataPrecision * dataType = 2)
    return vt_finish(sg->Fs, sg->ms, pdi, 2, t1, t2, c, p, cd, codeFreq_new, sumI, sumQ, out);
}

}  // extern "C"
