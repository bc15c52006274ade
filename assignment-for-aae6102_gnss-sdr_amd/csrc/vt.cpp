// vt.cpp — the host half of a vector-tracking step (trackingVT_POS_updated.m:157-349):
// read sizing, the three replica chips of the reference's linear-indexing quirk, the
// remaining code / carrier phase, the PLL and the DLL discriminator. Scalar fp64 work of
// a few hundred operations per channel and step; the carrier-wiped sums it consumes are
// the GPU's (gnss_tracking_vt_step, vt.hip). Compiled with -ffp-contract=off like the
// rest of the library, so every operation rounds as MATLAB's does.
// Reference: SDR_MATLAB-main/acqtckpos/trackingVT_POS_updated.m (line cites inline).
#include <cmath>

#include "gnss_internal.h"

using namespace gnss;

namespace {

// Spacing = 0.7:-0.05:-0.7 (:27) as MATLAB's colon builds it; element i (1-based)
double vt_spacing(int i1)
{
    const Colon c = colon_make(0.7, -0.05, -0.7);
    return colon_elem(c, i1 - 1);
}

// calcLoopCoef.m:41-45
void loop_coef(double LBW, double zeta, double k, double& t1, double& t2)
{
    const double Wn = LBW * 8 * zeta / (4 * (zeta * zeta) + 1);
    t1 = k / (Wn * Wn);
    t2 = 2.0 * zeta / Wn;
}

int valid_signal(const gnss_signal* sg, int pdi)
{
    return sg && sg->Fs > 0 && sg->codeFreqBasis > 0 && pdi >= 1;
}

}  // namespace

extern "C" {

int gnss_vt_prepare(const gnss_signal* sg, int32_t pdi, const gnss_vt_chan* c, double codeFreq_new,
                    int32_t code_out[3], int64_t* numSample)
{
    if (!valid_signal(sg, pdi) || !c || !code_out || c->prn < 1 || c->prn > 51 || !(c->codeFreq > 0))
        return GNSS_EARG;
    // numSample = ceil((codelength*pdi - remChip)/(codeFreq/Fs)) with the LAST step's
    // codeFreq (:161; the new one is predicted further down the loop body, :211-215)
    const double ns = std::ceil((sg->codelength * pdi - c->remChip) / (c->codeFreq / sg->Fs));
    if (!(ns >= 1) || ns > 1e9) return GNSS_EINDEX;
    if (numSample) *numSample = (int64_t)ns;
    // Code = [CA(end) repmat(CA,1,pdi) CA(1)] (:110); ceil_mx(idx) is ONE element: the first
    // sample's index ceil(t(1)) + 1 of row idx (t(1) = 0 + Spacing + remChip, :218-222),
    // clamped to 1025 (:240-246, which only ever inspects that element)
    float ca[1023];
    ca_chips(c->prn, ca);
    const int sp[3] = {5, 15, 25};
    const int64_t len = 1023 * (int64_t)pdi + 2;
    (void)codeFreq_new;
    for (int s = 0; s < 3; s++) {
        const double t1 = (0 + vt_spacing(sp[s])) + c->remChip;
        double j = std::ceil(t1) + 1;
        if (j > 1025) j = 1025;
        if (!(j >= 1) || j > (double)len) return GNSS_EINDEX;  // MATLAB index error
        const int64_t ji = (int64_t)j;
        const float v = ji == 1 ? ca[1022] : ji == len ? ca[0] : ca[(ji - 2) % 1023];
        code_out[s] = v < 0 ? -1 : 1;
    }
    return GNSS_OK;
}

int gnss_vt_nco_step(const gnss_signal* sg, const gnss_track* tr, int32_t pdi, gnss_vt_chan* c,
                     double codeFreq_new, double sumI, double sumQ, gnss_vt_out* out)
{
    if (!tr || !out || !(codeFreq_new > 0)) return GNSS_EARG;
    int32_t code[3];
    int64_t n = 0;
    int st = gnss_vt_prepare(sg, pdi, c, codeFreq_new, code, &n);
    if (st) return st;
    const double Fs = sg->Fs;
    // the read: numSample complex samples (int8 I/Q), ftell after it (:162-172, :344)
    const int64_t absS = c->file_ptr + n * 2;
    // codePhaseStep = codeFreq/Fs (:218); t_CodePrompt = (0 + Spacing(15) + remChip) :
    // codePhaseStep : ((numSample - 1)*codePhaseStep + Spacing(15) + remChip) (:220)
    const double cps = codeFreq_new / Fs;
    const double sp = vt_spacing(15);
    const double a = (0 + sp) + c->remChip;
    const double b = ((double)(n - 1) * cps + sp) + c->remChip;
    const Colon col = colon_make(a, cps, b);
    if (col.n != n - 1) return GNSS_EINDEX;  // t_CodePrompt(numSample) past the colon's end
    // remChip = (t_CodePrompt(numSample) + codePhaseStep) - 1023*pdi (:284)
    const double remChip = (colon_elem(col, n - 1) + cps) - 1023 * pdi;
    // Wave(numSample+1) = 2*pi*(carrFreq * (numSample/Fs)) + remCarrPhase (:275-276, :285)
    const double W = kTwoPi * (c->carrFreq * ((double)n / Fs)) + c->remCarrPhase;
    const double remCarrPhase = std::fmod(W, kTwoPi);
    // E / P / L: one chip value times the whole sums (:247-249, :267-272)
    out->E_i = code[0] * sumI;
    out->E_q = code[0] * sumQ;
    out->P_i = code[1] * sumI;
    out->P_q = code[1] * sumQ;
    out->L_i = code[2] * sumI;
    out->L_q = code[2] * sumQ;
    // PLL (:305-311)
    double t1, t2;
    loop_coef(tr->PLLBW, tr->PLLDamp, tr->PLLGain, t1, t2);
    const double carrError = std::atan(out->P_q / out->P_i) / (2.0 * 3.14159265358979323846);
    const double carrNco = c->oldCarrNco + (t2 / t1) * (carrError - c->oldCarrError) +
                           carrError * (pdi * 1e-3 / t1);
    const double carrFreq = c->carrFreqBasis + carrNco;
    // DLL discriminator (:314-316)
    const double E = std::sqrt(out->E_i * out->E_i + out->E_q * out->E_q);
    const double L = std::sqrt(out->L_i * out->L_i + out->L_q * out->L_q);
    out->codeError = -0.5 * (E - L) / (E + L);
    out->carrError = carrError;
    out->carrNco = carrNco;
    out->remChip = remChip;
    out->remCarrPhase = remCarrPhase;
    out->codeFreq = codeFreq_new;
    out->carrFreq = carrFreq;
    out->numSample = n;
    out->absoluteSample = absS;
    // codedelay = mod(absoluteSample/(dataPrecision*dataType), Fs*ms) (:347; int8 I/Q)
    out->codedelay = fmod_pos((double)absS / 2, Fs * sg->ms);
    // the state of the next step
    c->file_ptr = absS;
    c->remChip = remChip;
    c->remCarrPhase = remCarrPhase;
    c->codeFreq = codeFreq_new;
    c->carrFreq = carrFreq;
    c->oldCarrNco = carrNco;
    c->oldCarrError = carrError;
    return GNSS_OK;
}

}  // extern "C"
