/*
 * gnss_mi355x.h — C-ABI drop-in boundary for the GPS L1 C/A acquisition +
 * conventional-tracking hot path of KangWelly/Assignment-for-AAE6102_GNSS-SDR,
 * implemented with hand-written CDNA4 (gfx950) HIP kernels.
 *
 * The reference boundary is two MATLAB function calls (no FFI of its own):
 *
 *   Acquired = acquisition(file, signal, acq)
 *       SDR_MATLAB-main/acqtckpos/acquisition.m:1, called from SDR_main.m:22
 *       and Plot_task_1.m:14
 *   [TckResultCT, CN0_Eph, countinx] = trackingCT(file, signal, track, Acquired)
 *       SDR_MATLAB-main/acqtckpos/trackingCT.m:1, called from SDR_main.m:38
 *
 * The structs below carry exactly the MATLAB struct fields those functions read
 * (SDR_MATLAB-main/initParameters.m:20-70), as POD with fixed-width members.
 * Everything is plain pointers and sizes; no torch / HIP types cross this line.
 * The caller allocates every output; all lengths are known in advance.
 *
 * Threading: a gnss_ctx is bound to one HIP device and is not re-entrant
 * (MATLAB calls the MEX from one thread; the ctypes harness follows that rule).
 */
#ifndef GNSS_MI355X_H
#define GNSS_MI355X_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNSS_ABI_VERSION 13

/* ---- status codes (SURVEY §8b "Error conventions") --------------------- */
#define GNSS_OK         0
#define GNSS_ENODATA    1  /* reference's empty-result paths: "No satellites acquired"
                              (acquisition.m:84-85) / "Not enough raw data" ->
                              TckResultCT = [] (trackingCT.m:108-112, 302-306)          */
#define GNSS_EIO        2  /* file cannot be opened/read, or phase-C read past EOF
                              (trackingCT.m:442 has no check: MATLAB raises an error)  */
#define GNSS_EARG       3  /* bad/unsupported argument                                  */
#define GNSS_EDEVICE    4  /* HIP / rocFFT failure                                      */
#define GNSS_EINDEX     5  /* an index MATLAB would reject (e.g. P_i(i+17) past the end
                              in the bit-edge search, trackingCT.m:179-204)             */

#define GNSS_MAX_SV     64   /* generateCAcode.m:16-27 knows 51 PRNs                     */
#define GNSS_MAX_TAPS   32

/* ---- config structs (initParameters.m) ---------------------------------- */

/* file.* (initParameters.m:20-21,35-38). Exactly one of path / data / dev_data
 * is used, in that order of preference reversed (dev_data, then data, then
 * path). All seeks are absolute ('bof'), so positioned reads of `path` are
 * equivalent to MATLAB's fseek/fread on file.fid (SURVEY §8b "File handle"). */
typedef struct gnss_file {
    const char   *path;          /* file.fileRoute, or NULL                          */
    const int8_t *data;          /* host-resident IF record (byte 0 = file byte 0)   */
    const void   *dev_data;      /* IF record already resident in this ctx's HBM     */
    uint64_t      nbytes;        /* bytes in data / dev_data (ignored for path)      */
    int64_t       skip;          /* file.skip, ms                                    */
    int32_t       dataType;      /* file.dataType: 1 = I, 2 = IQ                     */
    int32_t       dataPrecision; /* file.dataPrecision: 1 = int8, 2 = int16          */
} gnss_file;

/* signal.* (initParameters.m:41-48) */
typedef struct gnss_signal {
    double  IF;              /* Hz                                  */
    double  Fs;              /* Hz                                  */
    double  codeFreqBasis;   /* 1.023e6                             */
    double  ms;              /* 1e-3                                */
    int64_t Sample;          /* ceil(Fs*ms)                         */
    double  codelength;      /* codeFreqBasis*ms                    */
} gnss_signal;

/* acq.* (initParameters.m:50-55) */
typedef struct gnss_acq {
    int32_t        freqNum;
    double         freqMin;
    double         freqStep;
    int32_t        datalen;   /* ms of non-coherent 1-ms FFT correlations            */
    int32_t        L;         /* ms used by the fine-frequency FFT                   */
    int32_t        n_prn;     /* 0 -> PRNs 1..32, as acquisition.m:47 hard-codes     */
    const int32_t *prn_list;  /* explicit PRN list (config 1: {3}; rank sharding)    */
} gnss_acq;

/* Acquired (acquisition.m:19-23,71-74,121): row vectors in ascending PRN order. */
typedef struct gnss_acquired {
    int32_t n;
    int32_t sv[GNSS_MAX_SV];
    double  SNR[GNSS_MAX_SV];
    double  Doppler[GNSS_MAX_SV];
    int32_t codedelay[GNSS_MAX_SV];
    double  fineFreq[GNSS_MAX_SV];
} gnss_acquired;

/* Per-PRN detector diagnostics (not part of the reference struct): every tested
 * PRN, acquired or not. peak2 = largest correlation value outside the peak's
 * +-56-sample exclusion window of the peak bin (margin of the argmax). */
typedef struct gnss_acq_diag {
    int32_t n;
    int32_t prn[GNSS_MAX_SV];
    double  SNR[GNSS_MAX_SV];
    int32_t fbin[GNSS_MAX_SV];        /* 1-based, as MATLAB                         */
    int32_t codePhase[GNSS_MAX_SV];   /* 1-based                                    */
    double  peak[GNSS_MAX_SV];
    double  peak2[GNSS_MAX_SV];
} gnss_acq_diag;

/* track.* (initParameters.m:58-70) */
typedef struct gnss_track {
    double  CorrelatorSpacing;      /* chip                                         */
    double  DLLBW, DLLDamp, DLLGain;
    double  PLLBW, PLLDamp, PLLGain;
    int32_t msToProcessCT_1ms;      /* the 1-ms phases A/B (trackingCT.m:29,221)    */
    int32_t msToProcessCT_10ms;     /* the 10-ms phase C (trackingCT.m:384)         */
    /* Multi-correlator ACF taps (config 5; semantics of
     * trackingCT_multiCorr-GIVEN.m:25,92-143). n_taps = 0 -> the three E/P/L taps
     * [-CorrelatorSpacing 0 +CorrelatorSpacing] (trackingCT.m:24). Otherwise
     * tap_offsets[n_taps] (chips) must contain -CorrelatorSpacing, 0 and
     * +CorrelatorSpacing, which feed the DLL/PLL exactly as E/P/L do. n_taps is
     * 3, 11 (config 5: -0.5:0.1:0.5) or 25 (-0.6:0.05:0.6 of the GIVEN file; int8
     * records only).                                                           */
    int32_t        n_taps;
    const double  *tap_offsets;
    /* Channel shard (multi-GPU): process Acquired channels chan[0..n_chan-1]
     * (0-based svindex) only; NULL -> every channel. Outputs of other channels
     * are left untouched. The quirk of trackingCT.m:161 (linear indexing into an
     * nsv x N matrix) uses the GLOBAL svindex and nsv, so shards stay bit-equal.  */
    int32_t        n_chan;
    const int32_t *chan;
} gnss_track;

/* Fields of one TckResultCT(prn) entry, in trackingCT.m:153-170 order. */
enum gnss_track_field {
    GNSS_F_P_i = 0, GNSS_F_P_q, GNSS_F_E_i, GNSS_F_E_q, GNSS_F_L_i, GNSS_F_L_q,
    GNSS_F_PLLdiscri, GNSS_F_DLLdiscri, GNSS_F_codedelay, GNSS_F_remChip,
    GNSS_F_codeFreq, GNSS_F_carrierFreq, GNSS_F_remPhase, GNSS_F_remSample,
    GNSS_F_numSample, GNSS_F_delayValue, GNSS_F_absoluteSample, GNSS_F_codedelay2,
    GNSS_NFIELDS
};

/* gnss_tracking_ct_pos stores trackingCT_POS_updated.m:273-292's fields in the same
 * slots: PLLdiscri = carrError, DLLdiscri = codeError, carrierFreq = carrFreq,
 * remPhase = remCarrPhase, and the remSample slot (that loop has no remSample) holds
 * absoluteSampleCodedelay. */
#define GNSS_F_carrError               GNSS_F_PLLdiscri
#define GNSS_F_codeError               GNSS_F_DLLdiscri
#define GNSS_F_carrFreq                GNSS_F_carrierFreq
#define GNSS_F_remCarrPhase            GNSS_F_remPhase
#define GNSS_F_absoluteSampleCodedelay GNSS_F_remSample

/* Outputs of trackingCT. Caller-allocated:
 *   rec      [nsv][GNSS_NFIELDS][max_len]  TckResultCT series per channel
 *            (series length 1000 + countinx + msToProcessCT_10ms, phase-C values
 *            written 10x as trackingCT.m:507-524 does); may be NULL.
 *   taps     [nsv][2][n_taps][max_len]     I then Q of every ACF tap; NULL unless
 *            wanted (phase-C taps are negated like E/P/L, trackingCT.m:447-449).
 *   len      [nsv]  series length per channel
 *   countinx [nsv]  bit-edge result (trackingCT.m:207)
 *   CN0_Eph  [cn0_cap][nsv] row-major (row = snrIndex-1); rows never written are 0
 *   cn0_rows  out: rows of the MATLAB CN0_Eph matrix
 *   flags     GNSS_OUT_DEVICE: rec and taps are DEVICE pointers (HIP memory of the
 *             ctx's device, e.g. gnss_dev_alloc or a framework tensor); the series are
 *             expanded into them on the GPU and never cross PCIe, so a multi-GPU caller
 *             can all-gather them over RCCL/xGMI as they lie. The call returns after the
 *             writes have completed (ctx stream synchronised). len, countinx and CN0_Eph
 *             stay host arrays. Not for gnss_tracking_ct_multicorr (its codedelay
 *             post-pass runs on the host): GNSS_EARG there.
 * max_len must be >= msToProcessCT_1ms + 19 + msToProcessCT_10ms.             */
#define GNSS_OUT_DEVICE 1
typedef struct gnss_track_out {
    int64_t  max_len;
    double  *rec;
    double  *taps;
    int64_t *len;
    int32_t *countinx;
    double  *CN0_Eph;
    int32_t  cn0_cap;
    int32_t  cn0_rows;
    int32_t  flags;     /* GNSS_OUT_DEVICE or 0 (ABI v7)                           */
    int32_t  reserved;
} gnss_track_out;

/* Device-side timing of the last call (hipEvents on the ctx stream). */
typedef struct gnss_timing {
    double acq_ms;            /* whole acquisition, IF resident in HBM             */
    double acq_corr_ms;       /* wipe + FFT correlation + power accumulation       */
    double acq_fine_ms;       /* fine-frequency FFTs + argmax                      */
    double track_ms;          /* whole trackingCT, IF resident in HBM              */
    double track_kernel_ms;   /* sum of correlator-kernel durations                */
    int64_t track_launches;   /* correlator-kernel launches                        */
    int64_t track_channel_samples;   /* channel-samples correlated (all taps)      */
    int64_t acq_hypothesis_samples;  /* PRN x bin x ms x Sample                     */
    double h2d_ms;            /* host->HBM upload of the IF window, if any         */
    /* profiling mode, the 10-ms phase (trackingCT.m:377-525) alone: the dominant
     * correlator kernel                                                           */
    double  track10_kernel_ms;
    int64_t track10_launches;
    int64_t track10_channel_samples;
    int64_t h2d_bytes;        /* bytes staged host/disk -> HBM in h2d_ms (ABI v8)  */
    int64_t track_segments;   /* 10-ms phase segments staged (gnss_ctx_set_window) */
} gnss_timing;

typedef struct gnss_ctx gnss_ctx;

int         gnss_abi_version(void);
const char *gnss_strerror(int status);

/* Create a context bound to HIP device `device` (owns stream, device buffers,
 * rocFFT plans). Replaces the MEX's persistent state (freed by mexAtExit). */
int  gnss_ctx_create(int device, gnss_ctx **out);
/* Multi-device context (ABI v11): one member context per entry of devices[0..n-1] (a device
 * may repeat; its members then run one after the other), so a MEX caller of SDR_main.m:22,38
 * shards over the GPUs of a node with no MATLAB change. gnss_acquisition deals the PRN list
 * (acquisition.m:47-80) and gnss_tracking_ct / _pos / _mc the channel list (trackingCT.m:22-528)
 * round-robin over the members, one host thread per device; each member keeps the global
 * svindex / nsv (quirk A.11), so every row is bit-identical to the one-context call. Results
 * are merged into the caller's arrays in the reference's order (Acquired and diag in PRN-list
 * order; tracking rows by channel). GNSS_OUT_DEVICE arrays live on devices[0]; a member on
 * another device expands its rows in its own HBM and copies them over xGMI (peer copies), and
 * a gnss_file.dev_data record on another device is copied range by range into each member's
 * HBM the same way. The status is the one-context call's (group.h). Every other entry point
 * runs on devices[0] alone. The setters apply to every member. n in 1..GNSS_MAX_DEVICES. */
#define GNSS_MAX_DEVICES 16
int  gnss_ctx_create_multi(const int *devices, int n, gnss_ctx **out);
/* Record residency of a multi-device context (ABI v12): a member on another device than a
 * gnss_file.dev_data record copies the WHOLE record into its own HBM by one peer copy (xGMI) the
 * first time a call reads it, and keeps that copy for every later call naming the same pointer
 * and length (gnss_timing.h2d_bytes counts the copy once). The library drops the copies that a
 * write of its own makes stale (gnss_dev_upload, gnss_synth_if_device into the record,
 * gnss_dev_free of it); a caller that rewrites the record by other means (its own hipMemcpy, a
 * MATLAB gpuArray) drops it here first. dev_ptr NULL drops every resident copy. The members'
 * copies are freed by gnss_ctx_destroy. No-ops for a one-device context. Replaces nothing in the
 * reference (SDR_main.m:22,38 re-read the file on every call). */
int  gnss_ctx_drop_record(gnss_ctx *ctx, const void *dev_ptr);
/* Resident record copies held by the context's members (0 for a one-device context). */
int  gnss_ctx_resident_records(const gnss_ctx *ctx);
/* HIP devices visible to this process (0 without a GPU or runtime). */
int  gnss_device_count(void);
/* Members of a context (1 for gnss_ctx_create). */
int  gnss_ctx_members(const gnss_ctx *ctx);
void gnss_ctx_destroy(gnss_ctx *ctx);
const char *gnss_last_error(const gnss_ctx *ctx);
int  gnss_last_timing(const gnss_ctx *ctx, gnss_timing *out);
/* Profiling mode: every correlator-step launch is bracketed by hipEvents (no
 * step graphs) so gnss_timing.track_kernel_ms is the sum of kernel durations. */
int  gnss_ctx_set_profiling(gnss_ctx *ctx, int enable);
/* Precision of the acquisition's PRN x bin x ms correlation (ABI v8; replaces nothing in
 * the reference, whose fft/ifft/abs().^2 are MATLAB doubles, acquisition.m:56-61):
 * fp64 = 1 (default) runs it at the reference's precision; fp64 = 0 is the fp32 fast mode
 * (the same decisions in every parity test, SNR within 1e-3 dB). The fine-frequency FFT
 * (acquisition.m:103-116) is fp64 in both. GNSS_EARG for other values. */
int  gnss_ctx_set_acq_precision(gnss_ctx *ctx, int fp64);
/* Streaming (ABI v8): at most `bytes` of IF resident in HBM per trackingCT call (0 = the
 * call's whole read range, the default). A record read from `path` or host `data` whose read
 * range exceeds it is staged in windows: the 1-ms phases' range first, then the 10-ms phase
 * (trackingCT.m:377-525) in segments of as many steps as the window holds, each staged through
 * the context's pinned double buffer before its launch (trackingCT.m:416-426 reads every step
 * from the file; the outputs are bit-identical to the unsegmented call). GNSS_EARG from the
 * call if the budget cannot hold the 1-ms phases' span or one 10-ms step of every channel. */
int  gnss_ctx_set_window(gnss_ctx *ctx, uint64_t bytes);
/* Test hooks (ABI v9; replace nothing in the reference): force one code path of the engine
 * so the parity tests can prove every path gives the reference's results. All default 0
 * (the engine's own choice); GNSS_EARG for an unknown key.                               */
#define GNSS_OPT_FORCE_SUB    0  /* lane span 8*v samples for both tracking phases (1..4) */
#define GNSS_OPT_NO_PERSIST   1  /* != 0: one launch per tracking step (no persistent loop;
                                    gnss_tracking_vt too, ABI v13)                        */
#define GNSS_OPT_FORCE_VPB    2  /* >= 2: virtual blocks per resident block of the loop     */
#define GNSS_OPT_ACQ_ROCFFT   3  /* != 0: rocFFT instead of the own P x 2000 correlator     */
#define GNSS_OPT_FINE_ROCFFT  4  /* != 0: rocFFT for the fine-frequency transform           */
#define GNSS_OPT_ACQ_BATCH    5  /* > 0: (bin, PRN) pairs per correlator batch (split path) */
#define GNSS_OPT_ACQ_FUSED    6  /* != 0: fp64 correlator as one persistent launch with the
                                    intermediate in each XCD's L2 (measured slower, kept
                                    for the record; default: two launches per batch)      */
#define GNSS_OPT_ACQ_RING     7  /* 2..4: ring slots per XCD of the fused correlator (3)    */
#define GNSS_OPT_ACQ_PIPE     8  /* split path: 1 = column and row passes of every batch in
                                    order on one stream, 2 = pipelined over two streams
                                    (batch b's rows beside batch b+1's columns, two
                                    intermediates), 3 = paired launches (fp64: batch
                                    b+1's column blocks and batch b's row blocks in one
                                    grid, interleaved; fp32 runs 2); 0 = the engine's
                                    choice                                                */
#define GNSS_OPT_VT_BLOCKS    9  /* 1..GNSS_VT_MAX_BLOCKS: blocks per channel of
                                    gnss_tracking_vt's step (GNSS_EARG above)             */
#define GNSS_OPT_FORCE_PEER   10 /* != 0 (multi-device contexts): every member treats
                                    dev_data and GNSS_OUT_DEVICE arrays as on another
                                    device (range copies in, row copies out), so one GPU
                                    exercises the peer-copy path                          */
#define GNSS_OPT_VT_SPAN      11 /* 1..2000 (ABI v13): steps per staged IF window of
                                    gnss_tracking_vt on a host record (2000; GNSS_EARG
                                    outside), so a short loop exercises the re-staging   */
#define GNSS_OPT_COUNT        12
int  gnss_ctx_set_option(gnss_ctx *ctx, int key, int64_t value);

/* Device memory owned by the ctx, for callers that keep an IF record resident
 * in HBM (gnss_file.dev_data) across calls. */
int  gnss_dev_alloc(gnss_ctx *ctx, uint64_t nbytes, void **dev_ptr);
int  gnss_dev_free(gnss_ctx *ctx, void *dev_ptr);
int  gnss_dev_upload(gnss_ctx *ctx, void *dev_dst, const void *host_src, uint64_t nbytes);
int  gnss_dev_download(gnss_ctx *ctx, void *host_dst, const void *dev_src, uint64_t nbytes);

/* acquisition.m replacement (acquisition.m:1-127). Returns GNSS_ENODATA with
 * out->n == 0 when nothing is acquired (acquisition.m:84-85). diag may be NULL. */
int gnss_acquisition(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                     const gnss_acq *acq, gnss_acquired *out, gnss_acq_diag *diag);

/* trackingCT.m replacement (trackingCT.m:1-530). The `countinx.mat` side file
 * (trackingCT.m:530) is the wrapper's job (MEX / Python mirror). */
int gnss_tracking_ct(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                     const gnss_track *track, const gnss_acquired *acquired,
                     gnss_track_out *out);

/* The tracking loop of trackingCT_POS_updated.m (its positioning half,
 * :420-565, is out of scope). Replaces the per-channel correlator / NCO / DLL / PLL of
 * trackingCT_POS_updated.m:92-144,179-413:
 *   - file_ptr = (Sample - codedelay + 1 + skip*Sample)*bytes (:108-110), one continuous
 *     read per channel (no re-seek at the 1 -> 10 ms switch);
 *   - steps msIndex = 1..ctPOS (track.ctPOS, :50); pdi = 1 while msIndex <= 1000 +
 *     countinx[svIndex] (:183; 1000 = track.msToProcessCT_1ms, countinx as loaded from
 *     countinx.mat at :29, indexed by channel POSITION), else 10;
 *   - numSample = ceil(...) (:189); E/P/L at Spacing(3) = +0.5, prompt Code(ceil(t+0.05)+1),
 *     Spacing(23) = -0.5 (:42,210-217); no negation; codeFreq = f0 + codeNco (:262);
 *     loop filters with T = signal.ms at every pdi (:257,266);
 *   - C/N0 every 20 steps of either pdi into one CN0_CT (:237-250);
 *   - one record row per step (Index = msIndex), codedelay = Sample - codedelay + 1 +
 *     sum(delayValue(svIndex,1:Index)) (:290).
 * out: rec[nsv][GNSS_NFIELDS][max_len] (max_len >= ctPOS, len = ctPOS), CN0_Eph = CN0_CT
 * (cn0_rows = ctPOS/20), countinx echoed. int8 records only (GNSS_EARG for int16: the
 * reference advances file_ptr by numSample*dataType bytes after reading twice that,
 * :196,207). EOF inside the loop -> GNSS_EIO (MATLAB raises on the short vector).    */
int gnss_tracking_ct_pos(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                         const gnss_track *track, const gnss_acquired *acquired, int32_t ctPOS,
                         const int32_t *countinx, gnss_track_out *out);

/* The tracking loop of trackingCT_POS_updated_multicorrelator.m (the
 * 25-tap sibling; its positioning half, :446-590, is out of scope). Replaces the channel
 * loop of trackingCT_POS_updated_multicorrelator.m:41-136,170-440:
 *   - steps msIndex = 1..msPosCT/pdi (datalength = track.msPosCT, pdi = track.pdi, :46-49,
 *     :170; pdi 1 or 10), every step at that pdi, one continuous read per channel from
 *     file_ptr = (Sample - codedelay + 1 + skip*Sample)*bytes (:101-103);
 *   - GNSS_MC_TAPS taps at Spacing = 0.6:-0.05:-0.6 (:41), replica Code(ceil(t) + 2) with
 *     Code = [CA(end) repmat(CA,1,pdi) CA(1) CA(2)] (:94,233-258), no +0.05 on the prompt;
 *     E/P/L = Spacing(3)/(13)/(23) feed the DLL/PLL; numSample = ceil(...) (:177);
 *     codeFreq = f0 + codeNco; loop filters with T = pdi*t (:351-364);
 *   - C/N0 every 20 steps with 1/(t*pdi) (:333-345);
 *   - one record row per step (the fields of :428-439 in gnss_track_out.rec as for
 *     gnss_tracking_ct_pos), every tap in gnss_track_out.taps[nsv][2][25][max_len] in
 *     Spacing order (E_i_060 ... L_i060 of :374-423).
 * max_len >= msPosCT/pdi; track->n_taps must be 0. int8 records only, EOF -> GNSS_EIO. */
#define GNSS_MC_TAPS 25

/* trackingCT_multiCorr-GIVEN.m (function trackingCT_multiCorr, the multi-correlator loop the
 * assignment hands out). Replaces TckResultCT = trackingCT_multiCorr(file,
 * signal, track, Acquired) (:1): per channel, fseek to (Sample - codedelay - 1 + skip*Sample)
 * bytes*2 (:57) and `datalength` 1-ms steps (:27 hard-codes 50000) read continuously, with
 * trackingCT.m's loop (round -> ceil for numSample, :60; remChip from codeFreqBasis*ms;
 * codeFreq = f0 - code_output; T = 1 ms) on the GNSS_MC_TAPS taps Spacing = -0.6:0.05:0.6
 * (:25), Code(ceil(t) + 1), E/P/L = Spacing(3)/(13)/(23) = -0.5/0/+0.5. Records as
 * gnss_tracking_ct (rec fields of :287-297 in the trackingCT slots, remSample included; every
 * tap in taps[nsv][2][25][max_len], the E_i_060 ... L_q060 of :163-286), one row per step;
 * codedelay = codedelay + sum(delayValue(1:msIndex)) over ONE nsv x datalength matrix filled
 * channel after channel (:29,297: earlier channels' rows count whole). CN0_CT every 20 steps.
 * max_len >= datalength; int8 I/Q records only (:47-48 pairs every record), no channel shard;
 * a short read -> GNSS_EIO (MATLAB raises; the function has no "Not enough raw data" branch). */
int gnss_tracking_ct_multicorr(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                               const gnss_track *track, const gnss_acquired *acquired,
                               int32_t datalength, gnss_track_out *out);
int gnss_tracking_ct_mc(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                        const gnss_track *track, const gnss_acquired *acquired, int32_t msPosCT,
                        int32_t pdi, gnss_track_out *out);

/* ---- naviDecode_updated.m ---------------------------------
 * Navigation-bit decode on the tracking output: bit synchronisation of P_i, preamble
 * search, parity (paritychk_James.m) and subframe 1-3 fields (bin2dec_GPSSDR.m,
 * comp2dec.m), with the reference's behaviour kept (repeat decodes are appended; bit
 * arrays carry over between channels — see csrc/navdecode.cpp).
 * Replaces [ephemeris, ~, for_prest] = naviDecode_updated(Acquired, ALLTckResult)
 * (naviDecode_updated.m:1, called at SDR_main.m:54). Channel c's ephemeris(prn) is
 * eph[c][field][0 .. eph_len[c][field]), prn = acquired->sv[c]. Host code (no GPU). */
enum gnss_eph_field {
    GNSS_E_TOW = 0, GNSS_E_TOW1, GNSS_E_sfb, GNSS_E_sfb1, GNSS_E_weeknum, GNSS_E_N, GNSS_E_health,
    GNSS_E_IODC, GNSS_E_TGD, GNSS_E_toc, GNSS_E_af2, GNSS_E_af1, GNSS_E_af0, GNSS_E_IODE2, GNSS_E_Crs,
    GNSS_E_deltan, GNSS_E_M0, GNSS_E_Cuc, GNSS_E_ecc, GNSS_E_Cus, GNSS_E_sqrta, GNSS_E_toe, GNSS_E_Cic,
    GNSS_E_omegae, GNSS_E_Cis, GNSS_E_i0, GNSS_E_Crc, GNSS_E_w, GNSS_E_omegadot, GNSS_E_IODE3,
    GNSS_E_idot, GNSS_E_updatetime, GNSS_E_updatetime_tow,
    GNSS_EPH_NFIELDS
};

typedef struct gnss_nav_out {
    int32_t  eph_cap;     /* values per field per channel (GNSS_EARG if one overflows) */
    double  *eph;         /* [nsv][GNSS_EPH_NFIELDS][eph_cap]                            */
    int32_t *eph_len;     /* [nsv][GNSS_EPH_NFIELDS]                                     */
    int32_t *updateflag;  /* [nsv] ephemeris(prn).updateflag                             */
    int64_t *nav1;        /* [nsv] for_prest.nav1(prn): first P_i index of the bit stream */
    int64_t *sfb1;        /* [nsv] for_prest.sfb1(prn): first subframe 1 (0 if none)      */
} gnss_nav_out;

/* P_i of channel c at P_i[c*stride + k], k < len[c] (TckResultCT(sv[c]).P_i). */
int gnss_navi_decode(const gnss_acquired *acquired, const double *P_i, const int64_t *len,
                     int64_t stride, gnss_nav_out *out);

/* Per-step parity hook: ONE trackingCT correlation step (trackingCT.m:79-118: numSample
 * from remChip/codeFreq, E/P/L or ACF replicas, carrier wipe, sums; no negation, no
 * loop update) at an arbitrary NCO state, on the same kernel the tracker launches.
 * sums_out[2*n_taps] = (I, Q) per tap; taps as gnss_track.tap_offsets (3 or 11). */
int gnss_correlate_step(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                        int prn, int pdi, double remChip, double codeFreq, double carrierFreq,
                        double remPhase, int64_t pos_bytes, int n_taps, const double *taps,
                        double *sums_out, int64_t *numSample_out);

/* ---- trackingVT_POS_updated.m, the tracking half (ABI v9) -----------
 * Steps of the loop at trackingVT_POS_updated.m:157-349 for n channels: read sizing (:161),
 * the three replica chips, the carrier wipe and sums (:217-281), the remaining code /
 * carrier phase (:284-285), the C/N0 estimator (:292-304), the PLL (:305-311) and the DLL
 * discriminator (:314-316). The vector half -- satellite position, iono / tropo, the
 * predicted code frequency and the Kalman filter (:166-215, :350-420) -- stays with the
 * caller, which passes each step's predicted code frequency.
 * The reference's replica quirk is kept: Code(svindex, ceil_mx(1)) linear-indexes ONE
 * element of the 3 x n matrix ceil_mx (the first sample's chip of each of the E / P / L
 * rows, the 1025 clamp of :240-246 applied to it alone), so E / P / L = that chip times
 * the whole sum(InphaseSignal) / sum(QuadratureSignal). Spacing = 0.7:-0.05:-0.7 (:27):
 * E / P / L at Spacing(5) / (15) / (25) = +0.5 / 0 / -0.5; the three colons must have
 * numSample elements each (ceil_mx's vertical concatenation and t_CodePrompt(numSample),
 * :217-228, :284), else GNSS_EINDEX as MATLAB raises.
 * Formats (:163-176): int8 I/Q (dataPrecision 1, dataType 2), int8 real (1, 1), int16 I/Q
 * with each read's means removed (2, 2); file_ptr in bytes. */
typedef struct gnss_vt_chan {
    int32_t prn;
    int32_t pad;
    int64_t file_ptr;       /* bytes: the fseek position of the next read (:162)          */
    double  remChip;        /* chips (:284)                                               */
    double  remCarrPhase;   /* rad (:285)                                                 */
    double  codeFreq;       /* the last step's code frequency: sizes the next read (:161) */
    double  carrFreq;       /* carrier NCO frequency (:310)                               */
    double  carrFreqBasis;  /* (:121)                                                     */
    double  oldCarrNco, oldCarrError;  /* PLL filter state (:307-308)                    */
    int32_t index_int;      /* C/N0 estimator (:78-81, :293-303): Zk entries filled, 0..19 */
    int32_t snrIndex;       /*   the next CN0_VT row (1-based; starts at 1)                */
    double  Zk[20];         /*   P_i^2 + P_q^2 of the current K = 20 block                 */
} gnss_vt_chan;

/* TckResultVT(prn).*(msIndex) of one channel and step (:319-346) and CN0_VT. */
typedef struct gnss_vt_out {
    double  E_i, E_q, P_i, P_q, L_i, L_q;
    double  carrError, codeError, carrNco;
    double  remChip, remCarrPhase, codeFreq, carrFreq;
    int64_t numSample, absoluteSample;
    double  codedelay;
    double  CN0;            /* CN0_VT(cn0_row, svindex) when cn0_row > 0 (:301)           */
    int32_t cn0_row;        /* 1-based row written by this step, 0: none                  */
    int32_t status;         /* GNSS_OK, or the channel's error at this step (vt_run)      */
    /* ABI v10, written by gnss_tracking_vt (the vector half; 0 from vt_run / vt_step):     */
    double  deltaPr;        /* TckResultVT(prn).deltaPr(msIndex) (:221,351), m/s          */
    double  prRate;         /* TckResultVT(prn).prRate: never assigned in the loop, 0 (:142) */
    double  sv_vel[3];      /* TckResultVT(prn).sv_vel(msIndex,:) (:185,346), m/s ECEF     */
} gnss_vt_out;

/* nsteps steps of the n channels in ONE launch (one workgroup per channel loops over the
 * steps: read sizing, sums in a fixed order, the scalar end, all on the GPU):
 * codeFreq_new[s * n + i] = channel i's code frequency for step s (:211-215; the caller's
 * EKF prediction, or a recorded series), pdi = track.pdi. chans[] are advanced in place;
 * out[s * n + i] = channel i's record of step s. A channel whose step fails (GNSS_EINDEX: a
 * replica index MATLAB would reject; GNSS_EIO: read past EOF) stops there with
 * out[..].status set; the call returns the first such status. */
int gnss_tracking_vt_run(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                         const gnss_track *track, int32_t pdi, int32_t n, int32_t nsteps,
                         gnss_vt_chan *chans, const double *codeFreq_new, gnss_vt_out *out);

/* One step: gnss_tracking_vt_run with nsteps = 1. */
int gnss_tracking_vt_step(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                          const gnss_track *track, int32_t pdi, int32_t n, gnss_vt_chan *chans,
                          const double *codeFreq_new, gnss_vt_out *out);

/* The same step's host half alone (no GPU): from the channel state, this step's code
 * frequency and the step's carrier-wiped sums (sumI = sum(InphaseSignal), sumQ =
 * sum(QuadratureSignal)), the record and the advanced state -- the arithmetic the
 * kernel's scalar end runs (the same source). int8 I/Q byte offsets. */
int gnss_vt_nco_step(const gnss_signal *signal, const gnss_track *track, int32_t pdi,
                     gnss_vt_chan *chan, double codeFreq_new, double sumI, double sumQ,
                     gnss_vt_out *out);

/* The replica chips and read size of a VT step (host, no GPU): code[3] = the E / P / L
 * chip values (+-1) the quirk multiplies the sums by, *numSample = ceil(...) (:161). */
int gnss_vt_prepare(const gnss_signal *signal, int32_t pdi, const gnss_vt_chan *chan,
                    double codeFreq_new, int32_t code_out[3], int64_t *numSample);

/* ---- trackingVT_POS_updated.m, the vector half (ABI v10) -------------
 * The EKF that drives the VT loop's code NCOs: per step and channel, the satellite position
 * at the block's transmit time (svPosVel.m), the iono / tropo corrections every 0.1 s
 * (ionocorr.m, trop_UNB3.m), the predicted pseudorange with the earth-rotation correction
 * (erotcorr.m) and from it the code frequency (:180-227); after the step's correlations the
 * 8-state EKF (position, velocity, clock bias, clock drift) on the 2n code and carrier
 * measurements (:357-442) and the adaptive measurement noise (:444-467). Host C++ (fp64 with
 * MATLAB's operation order, -ffp-contract=off); libm's sin / cos / atan2 / pow and MATLAB's
 * BLAS-backed matrix products and inv() round differently in the last place, so the values
 * match the reference within the ulp bounds stated in tests/test_vt_nav_kat.py. */
#define GNSS_VT_MAX_CH 32
#define GNSS_VT_MAX_BLOCKS 1024  /* blocks per channel of one VT step (GNSS_OPT_VT_BLOCKS)  */

/* ephemeris(prn).*(eph_idx) -- the fields svPosVel.m:23-44 reads (eph_idx = 1, :36). */
typedef struct gnss_eph_sv {
    double sqrta, deltan, toe, M0, ecc, w, Cus, Cuc, Crs, Crc, Cis, Cic, i0, idot, omegae, omegadot;
    double toc, af0, af1, af2, TGD;
} gnss_eph_sv;

/* The inputs of the vector half beyond the tracking structs: cnslxyz, the iono model
 * (initParameters.m:29-31), cmn.doy / cmn.cSpeed, signal.Fc. */
typedef struct gnss_vt_nav_cfg {
    double cnslxyz[3]; /* the cnslxyz argument (SDR_main.m:66: llh2xyz(solu.iniPos)), ECEF m:
                          the ionocorr user position (:200) and the navSolutionsVT ENU
                          origin (:407-415)                                                  */
    double ALPHA[4];   /* global ALPHA, BETA: broadcast iono model (initParameters.m:29-30)  */
    double BETA[4];
    double doy;        /* cmn.doy (trop_UNB3, :201)                                          */
    double cSpeed;     /* cmn.cSpeed, m/s                                                    */
    double Fc;         /* signal.Fc, Hz (the carrier's pseudorange rate, :380)               */
} gnss_vt_nav_cfg;

/* The loop's navigation state (all of trackingVT_POS_updated.m's cross-step variables other
 * than the channels' NCO state, which is gnss_vt_chan). Caller-allocated POD: init fills it,
 * predict / update advance it; it may be copied (a checkpoint) between steps. */
typedef struct gnss_vt_nav {
    int32_t n, pdi;
    int32_t msIndex;            /* the step being run: 1-based, advanced by update        */
    int32_t counterUptR, counter_r;
    int32_t prn[GNSS_VT_MAX_CH];
    gnss_vt_nav_cfg cfg;
    double  Fs, IF, codeFreqBasis, ms;
    double  cnslxyz[3];
    double  total_state[8];     /* [estPos estVel clkBias clkDrift] (:70, :400, :440)     */
    double  state_cov[64];      /* row-major 8 x 8 (:49, :391, :398)                      */
    double  R[2 * GNSS_VT_MAX_CH];     /* diag(mesurement_noise) (:55-56, :447-462)      */
    double  recordR2[2 * GNSS_VT_MAX_CH]; /* sum(recordR.^2) over the rows since the last
                                             noise update (:395, :446)                    */
    double  transmitTime[GNSS_VT_MAX_CH];  /* transmitTimeVT (:131, :181)                 */
    double  tot_est_tck[GNSS_VT_MAX_CH];   /* this step's (:182)                          */
    double  predictedPr_last[GNSS_VT_MAX_CH];
    double  counter_corr[GNSS_VT_MAX_CH];  /* (:86, :189-204)                             */
    double  ionodel[GNSS_VT_MAX_CH], tropodel[GNSS_VT_MAX_CH];
    double  el[GNSS_VT_MAX_CH], az[GNSS_VT_MAX_CH];   /* degrees (:195-196)               */
    int64_t numSample[GNSS_VT_MAX_CH];     /* this step's reads (:164)                    */
    gnss_eph_sv eph[GNSS_VT_MAX_CH];
} gnss_vt_nav;

/* navSolutionsVT.*(msIndex,:) of one step (:418-436). The 2n-long rows hold the code
 * measurements (channels 0..n-1) then the carrier ones (n..2n-1). */
typedef struct gnss_vt_navsol {
    double localTime;
    double usrPos[3], usrVel[3];
    double usrPosENU[3], usrVelENU[3], usrPosLLH[3];   /* LLH: degrees, degrees, m       */
    double clkBias, clkDrift;
    double state[8];              /* error_state after the update (:428)                  */
    double state_cov[8];          /* diag(state_cov) (:431)                               */
    double newZ[2 * GNSS_VT_MAX_CH];
    double meas_inno[2 * GNSS_VT_MAX_CH];
    double satEA[GNSS_VT_MAX_CH], satAZ[GNSS_VT_MAX_CH];  /* el / az, degrees             */
    double predicted_z[2 * GNSS_VT_MAX_CH];  /* H_pos * error_state (:434)               */
    double satePos[3], sateVel[3]; /* svxyzr_pos / sv_vel_pos of the LAST channel (:426-427:
                                      svindex is the loop's last value there)             */
    double svxyz_pos[GNSS_VT_MAX_CH][3];  /* navSolutionsVT.svxyz_pos(:,:,msIndex) (:429)  */
    double kalman_gain[8][2 * GNSS_VT_MAX_CH]; /* (:430), columns 0..2n-1 used           */
    double R[2 * GNSS_VT_MAX_CH]; /* navSolutionsVT.R(counter_r,:) when r_row > 0 (:466) */
    int32_t r_row;                /* 1-based row of navSolutionsVT.R written, 0: none     */
    int32_t reserved;
} gnss_vt_navsol;

/* svPosVel.m: SV position / velocity (ECEF), clock correction (m, m/s) and group delay (s)
 * at transmit time t (GPS seconds of week). Any output pointer may be NULL. */
int gnss_sv_pos_vel(const gnss_eph_sv *eph, double t, double pos[3], double vel[3],
                    double *clkcorr_m, double *clkcorr_m_vel, double *grpdel);
/* The SDR_MATLAB-main/geo helpers the loop uses, exported for their known-answer tests:
 *   GNSS_GEO_XYZ2LLH  in xyz[3]            -> out llh[3] (rad, rad, m)   xyz2llh.m
 *   GNSS_GEO_LLH2XYZ  in llh[3]            -> out xyz[3]                 llh2xyz.m
 *   GNSS_GEO_XYZ2ENU  in xyz[3], org[3]    -> out enu[3]                 xyz2enu.m
 *   GNSS_GEO_EROTCORR in svxyz[3], pr      -> out svxyzr[3]              erotcorr.m
 *   GNSS_GEO_IONO     in t, svxyz[3], usrxyz[3], ALPHA[4], BETA[4] -> out[0] m  ionocorr.m
 *   GNSS_GEO_TROP     in doy, lat (deg), alt (m), el (deg)   -> out[0] m  trop_UNB3.m  */
#define GNSS_GEO_XYZ2LLH  0
#define GNSS_GEO_LLH2XYZ  1
#define GNSS_GEO_XYZ2ENU  2
#define GNSS_GEO_EROTCORR 3
#define GNSS_GEO_IONO     4
#define GNSS_GEO_TROP     5
int gnss_geo(int fn, const double *in, double *out);

/* The loop's initialisation (:39-86, :109-155): the EKF (Transistion_Matrix with pdi * ms,
 * state_cov, process / measurement noise), total_state from the navigation solution of the
 * scalar loop at row skiptimeVT/navSolPeriod (usrPos, usrVel, clkBias, clkDrift, :66-70),
 * transmitTimeVT = navSolutionsCT.timeTransmit(1, :) (:131), counters. prn[n], eph[n] per
 * channel in Acquired.sv order. The channels' NCO state (gnss_vt_chan) comes from
 * TckResultCT at msStartTckVT (:114-124); the caller builds it (sdr.trackingVT_POS_updated).
 * pdi = track.pdi. GNSS_EARG for n outside 1..GNSS_VT_MAX_CH. */
int gnss_vt_nav_init(const gnss_vt_nav_cfg *cfg, const gnss_signal *signal, int32_t pdi, int32_t n,
                     const int32_t *prn, const gnss_eph_sv *eph, const double usrPos[3],
                     const double usrVel[3], double clkBias, double clkDrift,
                     const double *timeTransmit, gnss_vt_nav *nav);

/* The tracking-side prediction for channel i of step nav->msIndex (:180-227): advance the
 * transmit time by numSample / Fs (the step's read, sized with the LAST code frequency, :164),
 * svPosVel at it, the iono / tropo update every corrUpt steps, the predicted pseudorange
 * and, from step 2 on, codeFreq = codeFreqBasis * (1 - deltaPr / c); at step 1 *codeFreq is
 * left as passed (TckResultCT's codeFreq(msStartTckVT), :218-219). Outputs the step's
 * deltaPr and sv_vel. */
int gnss_vt_nav_predict(gnss_vt_nav *nav, int32_t i, int64_t numSample, double *codeFreq,
                        double *deltaPr, double sv_vel[3]);

/* The navigation update after every channel's correlation of step nav->msIndex (:357-467):
 * measurements Z = [codeError * c / codeFreq ; prr_predicted - prr_measured - clkDrift +
 * sv_clk_vel] from each channel's codeError, codeFreq and carrFreq (TckResultVT of this
 * step), the Kalman update, the state prediction for the next step and, every
 * 200 / pdi steps, the measurement-noise update. sol (may be NULL) receives the
 * navSolutionsVT row. Advances nav->msIndex. */
int gnss_vt_nav_update(gnss_vt_nav *nav, const double *codeError, const double *codeFreq,
                       const double *carrFreq, gnss_vt_navsol *sol);

/* The whole loop (trackingVT_POS_updated.m:157-476) for nsteps = msToProcessVT / pdi steps:
 * per step, every channel's read size and predicted code frequency on the host, the
 * correlations and NCO / PLL / DLL / C/N0 of all channels in one launch of the VT kernel
 * (vt.hip; chans stay resident in HBM), then the EKF on the host. chans[n] and *nav advance
 * in place; out[s * n + i] = TckResultVT(Acquired.sv(i)).*(s + 1) incl. deltaPr / prRate /
 * sv_vel; sol[s] (may be NULL) = navSolutionsVT row s + 1. A channel error (a replica index
 * MATLAB rejects, a read past EOF) stops the loop at that step (MATLAB raises): the step's
 * records hold the status, the call returns it. */
int gnss_tracking_vt(gnss_ctx *ctx, const gnss_file *file, const gnss_signal *signal,
                     const gnss_track *track, int32_t n, int32_t nsteps, gnss_vt_chan *chans,
                     gnss_vt_nav *nav, gnss_vt_out *out, gnss_vt_navsol *sol);

/* generateCAcode.m:16-64: the 1023 +-1 chips of PRN 1..51 used by the kernels. */
int gnss_ca_code(int prn, int8_t *out1023);

/* ---- synthetic IF: deterministic int8 I/Q record ------------ */
typedef struct gnss_synth_sv {
    int32_t prn;
    double  doppler_hz;     /* carrier Doppler; code Doppler = fd/1575.42e6      */
    double  code_phase0;    /* chips at absolute sample 0 (unwrapped)            */
    double  carr_phase0;    /* cycles at absolute sample 0                       */
    double  cn0_dbhz;
    uint64_t bit_seed;      /* 50 bps nav-bit stream seed                        */
    double  bit_phase_chips;/* nav-bit edge offset, chips                        */
    int32_t lnav;           /* 1: the bits are the LNAV message of gnss_lnav_bits
                               (bit k of the record = bit k mod 3000) instead of
                               seeded random bits; device generator only          */
    int32_t reserved;
} gnss_synth_sv;

typedef struct gnss_synth {
    double   Fs, IF;
    double   noise_sigma;   /* per I/Q component, LSB                            */
    uint64_t seed;
    int32_t  n_sv;
    gnss_synth_sv sv[GNSS_MAX_SV];
} gnss_synth;

/* The synthetic LNAV message (subframes 1-5, TLM/HOW/parity per IS-GPS-200, the
 * ephemeris fields naviDecode_updated.m reads; csrc/lnav.cpp): nbits transmitted bits
 * (0/1) from the start of a subframe 1 with HOW TOW count 65020. */
int gnss_lnav_bits(int32_t prn, int32_t nbits, int8_t *bits_out);

/* Fill dev_dst (this ctx's HBM) with samples [sample0, sample0 + nsamples) of
 * the record, 2 bytes per sample (I then Q). */
int gnss_synth_if_device(gnss_ctx *ctx, const gnss_synth *cfg, uint64_t sample0,
                         uint64_t nsamples, void *dev_dst);

#ifdef __cplusplus
}
#endif
#endif /* GNSS_MI355X_H */
