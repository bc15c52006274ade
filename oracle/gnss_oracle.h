/*
 * gnss_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU fp64 restatement of the reference hot path (acquisition.m, trackingCT.m,
 * generateCAcode.m, calcLoopCoef.m of KangWelly/Assignment-for-AAE6102_GNSS-SDR)
 * used as the parity checker for the HIP product path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library never links or calls it.
 *
 * Parity pinning: C/A codes against the IS-GPS-200
 * first-10-chip table; the NCO / loop-filter arithmetic against the bit-exact
 * replay of SDR_MATLAB-main/tckRstCT_10ms_Opensky.mat; output structure against
 * countinx.mat / Acquired_Opensky_5000.mat. Correlator sums and FFT values
 * against MATLAB itself are UNPINNED (the IF recordings are absent).
 */
#ifndef GNSS_ORACLE_H
#define GNSS_ORACLE_H
#include "../include/gnss_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* generateCAcode.m:16-64 — 1023 chips of +-1 for PRN 1..51 */
int  or_generate_ca(int prn, int8_t *out1023);
/* calcLoopCoef.m:41-45 */
void or_calc_loop_coef(double LBW, double zeta, double k, double *tau1, double *tau2);

/* MATLAB colon a:d:b (MathWorks' published colonop algorithm). n = number of
 * intervals (elements = n+1); n < 0 -> empty. */
typedef struct or_colon { double a, d, c; int64_t n; } or_colon;
void   or_colon_init(or_colon *r, double a, double d, double b);
double or_colon_elem(const or_colon *r, int64_t k);
int64_t or_colon_len(double a, double d, double b);
void   or_colon_fill(double a, double d, double b, double *out, int64_t cap);

/* Complex FFT (any length, mixed radix), fp64, interleaved re/im.
 * dir = -1 forward (MATLAB fft), +1 inverse with 1/N scale (MATLAB ifft). */
int or_fft(double *inout, int64_t n, int dir);

/* MATLAB round (half away from zero), mod(a,b), rem(a,b) */
double or_round(double x);
double or_mod(double a, double b);

/* acquisition.m:1-127 */
int or_acquisition(const gnss_file *file, const gnss_signal *signal, const gnss_acq *acq,
                   gnss_acquired *out, gnss_acq_diag *diag, int nthreads);

/* trackingCT.m:1-530 (phase B literally re-runs phase A). */
int or_tracking_ct(const gnss_file *file, const gnss_signal *signal, const gnss_track *track,
                   const gnss_acquired *acquired, gnss_track_out *out, int nthreads);

/* The tracking loop of trackingCT_POS_updated.m:92-144,179-413 (see gnss_tracking_ct_pos
 * in include/gnss_mi355x.h for the conventions; positioning is out of scope). */
int or_tracking_ct_pos(const gnss_file *file, const gnss_signal *signal, const gnss_track *track,
                       const gnss_acquired *acquired, int32_t ctPOS, const int32_t *countinx,
                       gnss_track_out *out, int nthreads);
/* trackingCT_multiCorr-GIVEN.m's loop (datalength 1-ms steps, 25 taps); outputs as
 * gnss_tracking_ct_multicorr. */
int or_tracking_ct_given(const gnss_file *file, const gnss_signal *signal, const gnss_track *track,
                         const gnss_acquired *acquired, int32_t datalength, gnss_track_out *out,
                         int nthreads);
/* The tracking loop of trackingCT_POS_updated_multicorrelator.m (25 taps, every step at
 * pdi, msPosCT/pdi steps); outputs as gnss_tracking_ct_mc. */
int or_tracking_ct_mc(const gnss_file *file, const gnss_signal *signal, const gnss_track *track,
                      const gnss_acquired *acquired, int32_t msPosCT, int32_t pdi, gnss_track_out *out,
                      int nthreads);

/* One trackingCT-style correlation step on host bytes (the body of
 * trackingCT.m:96-118 / :429-449 without the negation): sums[2*ntaps] =
 * (I, Q) per tap. Exposed for per-step parity tests. */
void or_set_carrier_mode(int mode);
void or_set_lane_geometry(int w, int a7);
void or_correlate_step(const int8_t *iq, int64_t numSample, double remChip, double codeFreq,
                       double Fs, double carrierFreq, double remPhase, const int8_t *ca1023,
                       int pdi, int ntaps, const double *taps, double *sums);

/* trackingCT.m:178-213: returns countinx (0 if not found), *status = GNSS_EINDEX
 * where MATLAB would raise an index error. */
int or_bit_edge(const double *P_i, int64_t len, int *status);

/* Sibling NCO replay (trackingCT_POS_updated.m:186-262 conventions) for the
 * tckRstCT_10ms_Opensky.mat KAT: given the previous state, produce next
 * numSample (ceil), remChip and remCarrPhase. */
void or_nco_replay(double remChip, double codeFreq, double carrFreq, double remCarrPhase,
                   double Fs, double codelength, int pdi, int use_ceil,
                   int64_t *numSample, double *remChipNext, double *remCarrPhaseNext);
/* trackingCT.m:136-150 loop filter, one update: returns the new output. */
int or_vt_step(const uint8_t *raw, int64_t nbytes, int prec, int dtype, double *st, double codeFreq_new,
               const int8_t *ca, double Fs, double codelength, double ms, int pdi, double tau1carr,
               double tau2carr, const double *sums, double *rec);
double or_loop_filter(double outLast, double discri, double discriLast, double tau1, double tau2,
                      double T);

/* trackingVT_POS_updated.m, the vector half: SDR_MATLAB-main/geo helpers,
 * the code-frequency prediction (:180-227), the EKF (:357-467) and the closed loop. */
#define OR_VT_MAXCH 32
typedef struct or_vtnav {
    int n, pdi, msIndex, counterUptR, counter_r, thresUptR;
    int prn[OR_VT_MAXCH];
    double eph[OR_VT_MAXCH][21];  /* gnss_eph_sv order */
    double ALPHA[4], BETA[4], doy, cSpeed, Fc, Fs, IF, codeFreqBasis, ms, corrUpt;
    double cnslxyz[3];
    double estPos[3], estVel[3], clkBias, clkDrift, total_state[8];
    double Tm[8][8], state_cov[8][8], process_noise[8][8];
    double mesurement_noise[2 * OR_VT_MAXCH][2 * OR_VT_MAXCH];
    double recordR[200][2 * OR_VT_MAXCH];
    double transmitTimeVT[OR_VT_MAXCH], tot_est_tck[OR_VT_MAXCH], tot_est_pos[OR_VT_MAXCH];
    double predictedPr_last[OR_VT_MAXCH], deltaPr[OR_VT_MAXCH], counter_corr[OR_VT_MAXCH];
    double ionodel[OR_VT_MAXCH], tropodel_unb3[OR_VT_MAXCH], el[OR_VT_MAXCH], az[OR_VT_MAXCH];
    double numSample[OR_VT_MAXCH];
} or_vtnav;
void or_xyz2llh(const double *xyz, double *llh);
void or_llh2xyz(const double *llh, double *xyz);
void or_xyz2enu(const double *xyz, const double *orgxyz, double *enu);
void or_erotcorr(const double *svxyz, double pr, double *svxyzr);
double or_ionocorr(double systime, const double *svxyz, const double *usrxyz, const double *ALPHA,
                   const double *BETA);
int or_trop_unb3(double doy, double lat, double alt, double el, double *out);
int or_svposvel(const double *eph, double t, double *sv_xyz, double *sv_vel, double *clkcorr_m,
                double *clkcorr_m_vel, double *grpdel);
size_t or_vtnav_size(void);
int or_vtnav_init(or_vtnav *v, int n, int pdi, const int *prn, const double *eph21, const double *cnslxyz,
                  const double *ALPHA, const double *BETA, double doy, double cSpeed, double Fc, double Fs,
                  double IF, double codeFreqBasis, double ms, const double *usrPos, const double *usrVel,
                  double clkBias, double clkDrift, const double *timeTransmit);
int or_vtnav_predict(or_vtnav *v, int i, int64_t numSample, double *codeFreq, double *deltaPr, double *sv_vel);
int or_vtnav_update(or_vtnav *v, const double *codeError, const double *codeFreq, const double *carrFreq,
                    double *state_out, double *es_out);
int or_tracking_vt(const uint8_t *raw, int64_t nbytes, int prec, int dtype, or_vtnav *v, double *chan_st,
                   const int8_t *ca, double codelength, double tau1carr, double tau2carr, int nsteps, double *rec,
                   double *nav_out);

/* Synthetic IF — CPU twin of the HIP generator. */
void or_synth_if(const gnss_synth *cfg, uint64_t sample0, uint64_t nsamples, int8_t *dst,
                 int nthreads);

#ifdef __cplusplus
}
#endif
#endif
