/*
 * gnss_oracle.c — TEST INFRASTRUCTURE ONLY (see gnss_oracle.h).
 *
 * Plain-C fp64 restatement of the reference hot path, operation by operation,
 * in MATLAB's evaluation order (left to right, no fused multiply-add: build
 * with -ffp-contract=off). Citations are to /root/reference/SDR_MATLAB-main/.
 */
#define _GNU_SOURCE
#include "gnss_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <unistd.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TWO_PI (2.0 * M_PI) /* MATLAB's 2*pi evaluated first: 6.283185307179586 */

/* ------------------------------------------------------------------------ */
/* generateCAcode.m                                                          */
/* ------------------------------------------------------------------------ */
/* G2 delays, generateCAcode.m:16-27 (32 GPS + 19 SBAS). */
static const int g2s[51] = {
    5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470, 471, 472,
    473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862, 145, 175, 52, 21, 237, 235, 886,
    657, 634, 762, 355, 1012, 176, 603, 130, 359, 595, 68, 386};

int or_generate_ca(int prn, int8_t *out)
{
    if (prn < 1 || prn > 51) return GNSS_EARG;
    int g1[1023], g2[1023], reg[10];
    /* G1: taps 3,10 in +-1 arithmetic (generateCAcode.m:34-42) */
    for (int i = 0; i < 10; i++) reg[i] = -1;
    for (int i = 0; i < 1023; i++) {
        g1[i] = reg[9];
        int save = reg[2] * reg[9];
        for (int j = 9; j > 0; j--) reg[j] = reg[j - 1];
        reg[0] = save;
    }
    /* G2: taps 2,3,6,8,9,10 (generateCAcode.m:49-57) */
    for (int i = 0; i < 10; i++) reg[i] = -1;
    for (int i = 0; i < 1023; i++) {
        g2[i] = reg[9];
        int save = reg[1] * reg[2] * reg[5] * reg[7] * reg[8] * reg[9];
        for (int j = 9; j > 0; j--) reg[j] = reg[j - 1];
        reg[0] = save;
    }
    /* g2 = [g2(1023-s+1:1023) g2(1:1023-s)] ; CA = -(g1.*g2) (:61,64) */
    int s = g2s[prn - 1];
    for (int i = 0; i < 1023; i++) {
        int src = (i < s) ? (1023 - s + i) : (i - s);
        out[i] = (int8_t)(-(g1[i] * g2[src]));
    }
    return GNSS_OK;
}

/* calcLoopCoef.m:41-45 */
void or_calc_loop_coef(double LBW, double zeta, double k, double *tau1, double *tau2)
{
    double Wn = LBW * 8 * zeta / (4 * (zeta * zeta) + 1);
    *tau1 = k / (Wn * Wn);
    *tau2 = 2.0 * zeta / Wn;
}

/* ------------------------------------------------------------------------ */
/* MATLAB scalar semantics                                                   */
/* ------------------------------------------------------------------------ */
double or_round(double x) { return round(x); } /* half away from zero */

double or_mod(double a, double b)
{
    if (b == 0) return a;
    double r = fmod(a, b);
    if (r != 0 && ((r < 0) != (b < 0))) r += b;
    return r;
}

/* Colon operator a:d:b following MathWorks' published colonop algorithm:
 * n from round((b-a)/d) with a 2*eps tolerance, right end snapped to b, and the
 * vector built from both ends toward the midpoint. */
void or_colon_init(or_colon *r, double a, double d, double b)
{
    r->a = a; r->d = d; r->c = b; r->n = -1;
    if (!isfinite(a) || !isfinite(d) || !isfinite(b)) return;
    if (d == 0 || (a < b && d < 0) || (b < a && d > 0)) return;
    double tol = 2.0 * DBL_EPSILON * fmax(fabs(a), fabs(b));
    double sig = (d > 0) ? 1.0 : -1.0;
    double n;
    if (a == floor(a) && d == 1) {
        n = floor(b) - a;
    } else if (a == floor(a) && d == floor(d)) {
        double q = floor(a / d);
        double rr = a - q * d;
        n = floor((b - rr) / d) - q;
    } else {
        n = round((b - a) / d);
        if (sig * (a + n * d - b) > tol) n = n - 1;
    }
    double c = a + n * d;
    if (sig * (c - b) > -tol) c = b;
    r->c = c;
    r->n = (int64_t)n;
}

double or_colon_elem(const or_colon *r, int64_t k)
{
    int64_t n = r->n;
    if (2 * k == n) return (r->a + r->c) / 2;
    if (k <= n / 2) return r->a + (double)k * r->d;
    return r->c - (double)(n - k) * r->d;
}

int64_t or_colon_len(double a, double d, double b)
{
    or_colon r;
    or_colon_init(&r, a, d, b);
    return r.n + 1;
}

void or_colon_fill(double a, double d, double b, double *out, int64_t cap)
{
    or_colon r;
    or_colon_init(&r, a, d, b);
    for (int64_t k = 0; k <= r.n && k < cap; k++) out[k] = or_colon_elem(&r, k);
}

/* ------------------------------------------------------------------------ */
/* Mixed-radix complex FFT (decimation in time, recursive), fp64             */
/* ------------------------------------------------------------------------ */
typedef struct { double re, im; } cpx;

typedef struct fftplan {
    int64_t n;
    int nf;
    int64_t fac[2 * 64]; /* (p, m) pairs */
    cpx *tw;             /* tw[k] = exp(-2*pi*i*k/n) */
    int maxp;
} fftplan;

static int fft_plan_init(fftplan *pl, int64_t n)
{
    pl->n = n; pl->nf = 0; pl->maxp = 1;
    int64_t m = n, p = 4;
    while (m > 1) {
        while (m % p) {
            if (p == 4) p = 2;
            else if (p == 2) p = 3;
            else p += 2;
            if (p * p > m) p = m;
        }
        m /= p;
        pl->fac[2 * pl->nf] = p;
        pl->fac[2 * pl->nf + 1] = m;
        pl->nf++;
        if (p > pl->maxp) pl->maxp = (int)p;
    }
    pl->tw = (cpx *)malloc(sizeof(cpx) * (size_t)(n ? n : 1));
    if (!pl->tw) return -1;
    for (int64_t k = 0; k < n; k++) {
        double ang = -2.0 * M_PI * (double)k / (double)n;
        pl->tw[k].re = cos(ang);
        pl->tw[k].im = sin(ang);
    }
    return 0;
}

static void fft_plan_free(fftplan *pl) { free(pl->tw); pl->tw = NULL; }

static inline cpx cmul(cpx a, cpx b)
{
    cpx r = {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
    return r;
}

static void fft_work(cpx *out, const cpx *in, int64_t fstride, const int64_t *fac,
                     const fftplan *pl, cpx *scratch)
{
    int64_t p = fac[0], m = fac[1];
    if (m == 1) {
        for (int64_t q = 0; q < p; q++) out[q] = in[q * fstride];
    } else {
        for (int64_t q = 0; q < p; q++)
            fft_work(out + q * m, in + q * fstride, fstride * p, fac + 2, pl, scratch);
    }
    const int64_t N = pl->n;
    const int64_t wp = N / p; /* W_p = tw[N/p] */
    for (int64_t u = 0; u < m; u++) {
        for (int64_t q = 0; q < p; q++) {
            cpx v = out[u + q * m];
            scratch[q] = (q == 0 || u == 0) ? v : cmul(v, pl->tw[fstride * q * u]);
        }
        if (p == 2) {
            cpx a = scratch[0], b = scratch[1];
            out[u].re = a.re + b.re; out[u].im = a.im + b.im;
            out[u + m].re = a.re - b.re; out[u + m].im = a.im - b.im;
            continue;
        }
        for (int64_t q1 = 0; q1 < p; q1++) {
            cpx acc = scratch[0];
            for (int64_t q = 1; q < p; q++) {
                int64_t e = (q * q1) % p;
                cpx t = e ? cmul(scratch[q], pl->tw[e * wp]) : scratch[q];
                acc.re += t.re; acc.im += t.im;
            }
            out[u + q1 * m] = acc;
        }
    }
}

static int fft_exec(const fftplan *pl, cpx *data, int dir)
{
    int64_t n = pl->n;
    if (n <= 1) return 0;
    cpx *tmp = (cpx *)malloc(sizeof(cpx) * (size_t)n);
    cpx *scratch = (cpx *)malloc(sizeof(cpx) * (size_t)pl->maxp);
    if (!tmp || !scratch) { free(tmp); free(scratch); return -1; }
    if (dir > 0)
        for (int64_t k = 0; k < n; k++) data[k].im = -data[k].im;
    memcpy(tmp, data, sizeof(cpx) * (size_t)n);
    fft_work(data, tmp, 1, pl->fac, pl, scratch);
    if (dir > 0) {
        double s = 1.0 / (double)n;
        for (int64_t k = 0; k < n; k++) { data[k].re *= s; data[k].im = -data[k].im * s; }
    }
    free(tmp); free(scratch);
    return 0;
}

int or_fft(double *inout, int64_t n, int dir)
{
    fftplan pl;
    if (fft_plan_init(&pl, n)) return GNSS_EARG;
    int r = fft_exec(&pl, (cpx *)inout, dir);
    fft_plan_free(&pl);
    return r ? GNSS_EARG : GNSS_OK;
}

/* ------------------------------------------------------------------------ */
/* IF record access (fseek 'bof' + fread of int8)                            */
/* ------------------------------------------------------------------------ */
/* Copies up to `count` bytes at absolute byte `off` into dst; returns bytes
 * read (fread semantics: short at EOF). */
static int64_t rd_bytes(const gnss_file *f, int64_t off, int64_t count, int8_t *dst)
{
    if (off < 0 || count <= 0) return 0;
    if (f->data) {
        if ((uint64_t)off >= f->nbytes) return 0;
        int64_t avail = (int64_t)f->nbytes - off;
        int64_t n = count < avail ? count : avail;
        memcpy(dst, f->data + off, (size_t)n);
        return n;
    }
    if (!f->path) return -1;
    int fd = open(f->path, O_RDONLY);
    if (fd < 0) return -1;
    int64_t got = 0;
    while (got < count) {
        ssize_t r = pread(fd, dst + got, (size_t)(count - got), off + got);
        if (r <= 0) break;
        got += r;
    }
    close(fd);
    return got;
}

static int64_t file_size(const gnss_file *f)
{
    if (f->data) return (int64_t)f->nbytes;
    if (!f->path) return -1;
    int fd = open(f->path, O_RDONLY);
    if (fd < 0) return -1;
    int64_t s = lseek(fd, 0, SEEK_END);
    close(fd);
    return s;
}

/* The IF samples of one fread, as the reference forms them (acquisition.m:28-37,
 * :90-99; trackingCT.m:84-93, :416-426): `nsamp` samples requested at byte `off`.
 *   int8 (dataPrecision 1): dataType 2 -> I/Q byte pairs, dataType 1 -> real bytes;
 *   int16 (dataPrecision 2): fread(nsamp*dataType, 'int16') de-interleaved into
 *     I = values(1:2:end), Q = values(2:2:end) WHATEVER dataType says, each half
 *     minus its own mean (sum / length, exact for integer-valued doubles).
 * Returns the length MATLAB's rawsignal gets (fewer than nsamp at EOF; nsamp/2 for
 * int16 with dataType 1), -1 on an I/O failure, -2 where MATLAB raises an error
 * (I and Q halves of unequal length: an odd number of values read). *bytes = the
 * bytes fread consumed (the ftell advance). */
static int64_t rd_cpx(const gnss_file *f, int64_t off, int64_t nsamp, cpx *out, int64_t *bytes)
{
    const int prec = f->dataPrecision, type = f->dataType;
    const int64_t want = nsamp * type * prec;
    int8_t *b = (int8_t *)malloc((size_t)(want > 0 ? want : 1));
    if (!b) return -1;
    int64_t got = rd_bytes(f, off, want, b);
    if (got < 0) { free(b); return -1; }
    int64_t m;
    if (prec == 1) {
        *bytes = got;
        if (type == 2) {
            if (got & 1) { free(b); return -2; }
            m = got / 2;
            for (int64_t k = 0; k < m; k++) { out[k].re = b[2 * k]; out[k].im = b[2 * k + 1]; }
        } else {
            m = got;
            for (int64_t k = 0; k < m; k++) { out[k].re = b[k]; out[k].im = 0; }
        }
    } else {
        const int64_t nv = got / 2; /* whole int16 values */
        *bytes = 2 * nv;
        if (nv & 1) { free(b); return -2; }
        m = nv / 2;
        const int16_t *v = (const int16_t *)b; /* little-endian host, as the file */
        double si = 0, sq = 0;
        for (int64_t k = 0; k < m; k++) { si += v[2 * k]; sq += v[2 * k + 1]; }
        const double mi = si / (double)m, mq = sq / (double)m;
        for (int64_t k = 0; k < m; k++) {
            out[k].re = (double)v[2 * k] - mi;
            out[k].im = (double)v[2 * k + 1] - mq;
        }
    }
    free(b);
    return m;
}

/* ------------------------------------------------------------------------ */
/* acquisition.m                                                             */
/* ------------------------------------------------------------------------ */
static int nthreads_of(int n)
{
#ifdef _OPENMP
    return n > 0 ? n : omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

int or_acquisition(const gnss_file *file, const gnss_signal *sg, const gnss_acq *acq,
                   gnss_acquired *out, gnss_acq_diag *diag, int nthreads)
{
    memset(out, 0, sizeof(*out));
    if (diag) memset(diag, 0, sizeof(*diag));
    if ((file->dataPrecision != 1 && file->dataPrecision != 2) || (file->dataType != 1 && file->dataType != 2))
        return GNSS_EARG;
    const int64_t S = sg->Sample;
    const int nb = acq->freqNum, dl = acq->datalen;
    if (S <= 0 || nb <= 0 || dl <= 0 || acq->L <= 0) return GNSS_EARG;

    int prns[GNSS_MAX_SV], np = 0;
    if (acq->n_prn > 0 && acq->prn_list) {
        for (int i = 0; i < acq->n_prn && i < GNSS_MAX_SV; i++) prns[np++] = acq->prn_list[i];
    } else {
        for (int i = 1; i <= 32; i++) prns[np++] = i; /* acquisition.m:47 */
    }

    /* read data (acquisition.m:27,34-37) */
    const int64_t off = file->skip * S * file->dataPrecision * file->dataType;
    cpx *raw = (cpx *)malloc(sizeof(cpx) * (size_t)(S * dl));
    if (!raw) return GNSS_EIO;
    {
        int64_t nb_read = 0;
        const int64_t m = rd_cpx(file, off, S * dl, raw, &nb_read);
        /* rawsignal(1+(idx-1)*Sample : idx*Sample) past the end is MATLAB's index
         * error (int16 with dataType 1 always: half the samples); a short file: EIO */
        if (m == -1) { free(raw); return GNSS_EIO; }
        if (m == -2 || (m < S * dl && file->dataPrecision == 2 && file->dataType == 1)) { free(raw); return GNSS_EINDEX; }
        if (m < S * dl) { free(raw); return GNSS_EIO; }
    }

    /* carrier(freqband,:) = exp(1i*2*pi*(IF+dopplershift)*sampleindex./Fs) (:41-44) */
    cpx *carrier = (cpx *)malloc(sizeof(cpx) * (size_t)(nb * S));
    for (int b = 0; b < nb; b++) {
        double ds = acq->freqMin + acq->freqStep * (double)b;
        double w = TWO_PI * (sg->IF + ds);
        for (int64_t n = 1; n <= S; n++) {
            double th = (w * (double)n) / sg->Fs;
            carrier[b * S + n - 1].re = cos(th);
            carrier[b * S + n - 1].im = sin(th);
        }
    }

    fftplan pl;
    fft_plan_init(&pl, S);

    /* conj(fft(temp1)) is PRN-invariant (quirk A.2): computed once per (ms, bin). */
    cpx *Xc = (cpx *)malloc(sizeof(cpx) * (size_t)(dl * nb * S));
    int nt = nthreads_of(nthreads);
#pragma omp parallel for num_threads(nt) schedule(dynamic)
    for (int j = 0; j < dl * nb; j++) {
        int idx = j / nb, b = j % nb;
        cpx *x = Xc + (int64_t)j * S;
        for (int64_t n = 0; n < S; n++) {
            double xr = raw[idx * S + n].re, xi = raw[idx * S + n].im;
            cpx c = carrier[b * S + n];
            x[n].re = xr * c.re - xi * c.im;
            x[n].im = xr * c.im + xi * c.re;
        }
        fft_exec(&pl, x, -1);
        for (int64_t n = 0; n < S; n++) x[n].im = -x[n].im;
    }

    const int64_t cshift = (int64_t)ceil(sg->Fs / sg->codeFreqBasis); /* :66 */
    double res_snr[GNSS_MAX_SV], res_peak[GNSS_MAX_SV], res_peak2[GNSS_MAX_SV];
    int res_fbin[GNSS_MAX_SV], res_cp[GNSS_MAX_SV];

#pragma omp parallel for num_threads(nt) schedule(dynamic)
    for (int ip = 0; ip < np; ip++) {
        int8_t ca[1023];
        or_generate_ca(prns[ip], ca);
        cpx *C = (cpx *)malloc(sizeof(cpx) * (size_t)S);
        cpx *y = (cpx *)malloc(sizeof(cpx) * (size_t)S);
        double *corr = (double *)calloc((size_t)(nb * S), sizeof(double));
        /* scode = [CA CA](ceil(sampleindex.*(codeFreqBasis/Fs))) (:50-51) */
        double step = sg->codeFreqBasis / sg->Fs;
        for (int64_t n = 1; n <= S; n++) {
            int64_t ci = (int64_t)ceil((double)n * step); /* 1-based into [CA CA] */
            C[n - 1].re = ca[(ci - 1) % 1023];
            C[n - 1].im = 0;
        }
        fft_exec(&pl, C, -1); /* temp3 = fft(replica) (:58) */
        for (int idx = 0; idx < dl; idx++) {
            for (int b = 0; b < nb; b++) {
                const cpx *x = Xc + ((int64_t)idx * nb + b) * S;
                for (int64_t k = 0; k < S; k++) y[k] = cmul(C[k], x[k]);
                fft_exec(&pl, y, +1);
                double *row = corr + (int64_t)b * S;
                for (int64_t k = 0; k < S; k++) { /* abs(...).^2 accumulated (:59) */
                    double a = hypot(y[k].re, y[k].im);
                    row[k] = row[k] + a * a;
                }
            }
        }
        /* [~, fbin] = max(max(abs(correlation'))); [peak, codePhase] = max(max(...)) (:62-63) */
        double peak = -INFINITY;
        for (int64_t i = 0; i < nb * S; i++)
            if (corr[i] > peak) peak = corr[i];
        int fbin = 0;
        int64_t cp = 0;
        for (int b = 0; b < nb && !fbin; b++)
            for (int64_t k = 0; k < S; k++)
                if (corr[b * S + k] == peak) { fbin = b + 1; break; }
        for (int64_t k = 0; k < S && !cp; k++)
            for (int b = 0; b < nb; b++)
                if (corr[b * S + k] == peak) { cp = k + 1; break; }
        /* SNR over corr(fbin, [1:cp-cshift cp+cshift:end]) (:66-68) */
        const double *row = corr + (int64_t)(fbin - 1) * S;
        double ss = 0, p2 = 0;
        int64_t cnt = 0;
        for (int64_t k = 1; k <= cp - cshift; k++) { ss += row[k - 1] * row[k - 1]; cnt++; if (row[k - 1] > p2) p2 = row[k - 1]; }
        for (int64_t k = cp + cshift; k <= S; k++) { ss += row[k - 1] * row[k - 1]; cnt++; if (row[k - 1] > p2) p2 = row[k - 1]; }
        double snr = 10.0 * log10((peak * peak) / (ss / (double)cnt));
        res_snr[ip] = snr; res_peak[ip] = peak; res_peak2[ip] = p2;
        res_fbin[ip] = fbin; res_cp[ip] = (int)cp;
        free(C); free(y); free(corr);
    }

    for (int ip = 0; ip < np; ip++) {
        if (diag) {
            int k = diag->n++;
            diag->prn[k] = prns[ip]; diag->SNR[k] = res_snr[ip]; diag->fbin[k] = res_fbin[ip];
            diag->codePhase[k] = res_cp[ip]; diag->peak[k] = res_peak[ip]; diag->peak2[k] = res_peak2[ip];
        }
        if (res_snr[ip] >= 12) { /* :70-74 */
            int k = out->n++;
            out->sv[k] = prns[ip];
            out->SNR[k] = res_snr[ip];
            out->Doppler[k] = acq->freqMin + acq->freqStep * (double)(res_fbin[ip] - 1);
            out->codedelay[k] = res_cp[ip] - 1;
        }
    }
    free(Xc); free(carrier); free(raw);
    fft_plan_free(&pl);

    if (out->n == 0) return GNSS_ENODATA; /* :84-85 */

    /* fine frequency (:89-126) */
    const int64_t Ls = (int64_t)acq->L * S;
    cpx *lraw = (cpx *)malloc(sizeof(cpx) * (size_t)(S * (acq->L + 1)));
    {
        int64_t nb_read = 0;
        const int64_t m = rd_cpx(file, off, S * (acq->L + 1), lraw, &nb_read);
        if (m == -1) { free(lraw); return GNSS_EIO; }
        if (m == -2) { free(lraw); return GNSS_EINDEX; }
        if (m < S * (acq->L + 1)) { free(lraw); return GNSS_EIO; }
    }
    const int64_t N = Ls * dl; /* fftlength = length(CarrSignal)*acq.datalen (:108) */
    fftplan fp;
    fft_plan_init(&fp, N);
    const double invFs = 1 / sg->Fs, invFc = 1 / sg->codeFreqBasis;
    int status = GNSS_OK;
#pragma omp parallel for num_threads(nt < out->n ? nt : out->n) schedule(dynamic)
    for (int s = 0; s < out->n; s++) {
        int8_t ca[1023];
        or_generate_ca(out->sv[s], ca);
        cpx *x = (cpx *)calloc((size_t)N, sizeof(cpx));
        int64_t start = S - out->codedelay[s]; /* 1-based (:106) */
        for (int64_t k = 1; k <= Ls; k++) {
            double cvi = floor((invFs * (double)k) / invFc);      /* :104 */
            int8_t code = ca[(int64_t)fmod(cvi, sg->codelength)]; /* :105 rem(.,1023)+1 */
            int64_t j = start + k - 1;                            /* 1-based sample */
            x[k - 1].re = lraw[j - 1].re * code;
            x[k - 1].im = lraw[j - 1].im * code;
        }
        fft_exec(&fp, x, -1);
        /* abs(fftshift(.)); max over 1:halffftlength*2 -> first index (:110-116) */
        int64_t half = (N + 1) / 2;
        double best = -1;
        int64_t kbest = 0;
        const int shifted = file->dataType == 2; /* :109-112 */
        for (int64_t i = 0; i < 2 * half && i < N; i++) {
            /* fftshift: shifted[i] = F[(i + floor(N/2)) mod N]. A real CarrSignal
             * (dataType 1) has an exactly conjugate-symmetric fft in MATLAB: |F(N-i)|
             * is |F(i)| bit for bit, so the first index of a tie is the lower bin. */
            int64_t j = shifted ? (i + N / 2) % N : (i <= N - i ? i : N - i);
            double a = hypot(x[j].re, x[j].im);
            if (a > best) { best = a; kbest = i + 1; }
        }
        if (2 * half > N) {
#pragma omp atomic write
            status = GNSS_EINDEX; /* odd fftlength: MATLAB indexes past the end */
        }
        if (shifted)
            out->fineFreq[s] = -(double)kbest * (sg->Fs / (double)N) + sg->Fs / 2; /* :119 */
        else
            out->fineFreq[s] = (double)kbest * (sg->Fs / (double)N); /* :117 */
        free(x);
    }
    fft_plan_free(&fp);
    free(lraw);
    return status;
}

/* ------------------------------------------------------------------------ */
/* trackingCT.m                                                              */
/* ------------------------------------------------------------------------ */
/* Code(ceil(t)+1) with Code = [CA(1023) repmat(CA,1,pdi) CA(1)] (trackingCT.m:68,413):
 * chip c = ceil(t) maps to CA((c-1) mod 1023 + 1). */
static inline int chip_ok(int64_t c, int pdi) { return c >= 0 && c <= 1023 * (int64_t)pdi + 1; }
static inline int ca_index(int64_t c) { return (int)((c + 1022) % 1023); }

static void correlate_cpx(const cpx *x, int64_t n, double remChip, double codeFreq, double Fs,
                          double carrierFreq, double remPhase, const int8_t *ca, int pdi, int ntaps,
                          const double *taps, const double *post, int chip_off, double *sums);

/* Carrier evaluation mode (TEST EXPERIMENT ONLY): 0 = the reference's rounded Wave (default);
 * 1 = the same phase without the per-sample fp64 roundings (long double), to measure how
 * much the closed loop depends on reproducing them. */
static int g_carrier_mode = 0;
void or_set_carrier_mode(int mode) { g_carrier_mode = mode; }
/* mode >= 2 (experiment only): the carrier of the lane-table correlator -- lanes of g_lane_w
 * samples aligned to the 8-sample groups of the file (first lane starts g_lane_a7 = A mod 8
 * samples before the window), e^{i Wave(lane start)} (the reference's rounding) times the
 * table e^{i m delta} quantised to `mode` fractional bits. */
static int g_lane_w = 24, g_lane_a7 = 0;
void or_set_lane_geometry(int w, int a7) { g_lane_w = w; g_lane_a7 = a7; }

void or_correlate_step(const int8_t *iq, int64_t n, double remChip, double codeFreq, double Fs,
                       double carrierFreq, double remPhase, const int8_t *ca, int pdi, int ntaps,
                       const double *taps, double *sums)
{
    cpx *x = (cpx *)malloc(sizeof(cpx) * (size_t)(n > 0 ? n : 1));
    for (int64_t k = 0; k < n; k++) { x[k].re = iq[2 * k]; x[k].im = iq[2 * k + 1]; }
    correlate_cpx(x, n, remChip, codeFreq, Fs, carrierFreq, remPhase, ca, pdi, ntaps, taps, NULL, 0, sums);
    free(x);
}

/* The correlator of trackingCT.m:96-118 on rawsignal0DC (complex doubles). post[s]
 * (NULL = none) is added to tap s's colon element before ceil: the prompt's
 * Code(ceil(t_CodePrompt + 0.05) + indx) of trackingCT_POS_updated.m:216. chip_off = 1:
 * Code(ceil(t) + 2) with Code = [CA(1023) repmat(CA,1,pdi) CA(1) CA(2)]
 * (trackingCT_POS_updated_multicorrelator.m:94,233-258), i.e. CA((ceil(t)) mod 1023 + 1). */
static void correlate_cpx(const cpx *x, int64_t n, double remChip, double codeFreq, double Fs,
                          double carrierFreq, double remPhase, const int8_t *ca, int pdi, int ntaps,
                          const double *taps, const double *post, int chip_off, double *sums)
{
    (void)pdi;
    const double d = codeFreq / Fs;
    or_colon col[GNSS_MAX_TAPS];
    /* sum(Code.*InphaseSignal): the order of MATLAB's summation is not published;
     * accumulate in extended precision so the oracle is the (near-)exact sum. */
    long double acc[2 * GNSS_MAX_TAPS];
    for (int s = 0; s < ntaps; s++) {
        /* t = (0 + Spacing(s) + remChip) : d : ((numSample-1)*d + Spacing(s) + remChip) */
        double a = (0 + taps[s]) + remChip;
        double b = ((double)(n - 1) * d + taps[s]) + remChip;
        or_colon_init(&col[s], a, d, b);
        acc[2 * s] = 0;
        acc[2 * s + 1] = 0;
    }
    for (int64_t k = 0; k < n; k++) {
        /* CarrTime = (0:numSample)./Fs; Wave = (2*pi*(carrierFreq.*CarrTime)) + remPhase */
        double W = TWO_PI * (carrierFreq * ((double)k / Fs)) + remPhase;
        double cw = cos(W), sw = sin(W);
        if (g_carrier_mode == 1) {
            /* experiment only: the carrier phase without MATLAB's per-sample roundings */
            long double Wl = (long double)TWO_PI * (long double)carrierFreq * (long double)k /
                             (long double)Fs + (long double)remPhase;
            cw = (double)cosl(Wl);
            sw = (double)sinl(Wl);
        } else if (g_carrier_mode >= 2) {
            const int64_t L = (k + g_lane_a7) / g_lane_w;
            const int64_t ks = L * g_lane_w - g_lane_a7;
            const double Wb = TWO_PI * (carrierFreq * ((double)ks / Fs)) + remPhase;
            const long double dl = 2.0L * 3.14159265358979323846264338327950288L * (long double)carrierFreq / (long double)Fs;
            const long double sc = ldexpl(1.0L, g_carrier_mode);
            const long double tr = roundl(cosl(dl * (long double)(k - ks)) * sc) / sc;
            const long double ti = roundl(sinl(dl * (long double)(k - ks)) * sc) / sc;
            const long double br = cosl((long double)Wb), bi = sinl((long double)Wb);
            cw = (double)(br * tr - bi * ti);
            sw = (double)(br * ti + bi * tr);
        }
        double xr = x[k].re, xi = x[k].im;
        double I = xr * sw + xi * cw; /* imag(raw.*carrsig) */
        double Q = xr * cw - xi * sw; /* real(raw.*carrsig) */
        for (int s = 0; s < ntaps; s++) {
            double t = or_colon_elem(&col[s], k);
            if (post) t = t + post[s];
            double code = ca[ca_index((int64_t)ceil(t) + chip_off)];
            acc[2 * s] += code * I;
            acc[2 * s + 1] += code * Q;
        }
    }
    for (int s = 0; s < 2 * ntaps; s++) sums[s] = (double)acc[s];
}

int or_bit_edge(const double *P, int64_t len, int *status)
{
    *status = GNSS_OK;
#define SGN(x) (((x) > 0) - ((x) < 0))
    for (int64_t i = 7; i <= len - 1; i++) { /* 1-based i (trackingCT.m:179) */
        int si = SGN(P[i - 1]);
        int ok = 1;
        for (int j = 6; j >= 1 && ok; j--) ok = SGN(P[i - j - 1]) != si;
        for (int j = 1; j <= 17 && ok; j++) {
            if (i + j > len) { *status = GNSS_EINDEX; return 0; }
            ok = SGN(P[i + j - 1]) == si;
        }
        if (ok && i >= 600) return (int)(or_mod((double)i, 20) - 1); /* :207 */
    }
#undef SGN
    return 0;
}

void or_nco_replay(double remChip, double codeFreq, double carrFreq, double remCarrPhase,
                   double Fs, double codelength, int pdi, int use_ceil, int64_t *numSample,
                   double *remChipNext, double *remCarrPhaseNext)
{
    double cps = codeFreq / Fs;
    double ns = (codelength * pdi - remChip) / cps;
    int64_t n = (int64_t)(use_ceil ? ceil(ns) : round(ns));
    *numSample = n;
    /* remChip = t_CodePrompt(numSample) + cps - codelength*pdi, last colon element = b */
    double a = (0 + 0.0) + remChip;
    double b = ((double)(n - 1) * cps + 0.0) + remChip;
    or_colon col;
    or_colon_init(&col, a, cps, b);
    *remChipNext = (or_colon_elem(&col, n - 1) + cps) - codelength * pdi;
    double W = TWO_PI * (carrFreq * ((double)n / Fs)) + remCarrPhase;
    *remCarrPhaseNext = fmod(W, TWO_PI);
}

double or_loop_filter(double outLast, double discri, double discriLast, double tau1, double tau2,
                      double T)
{
    /* code_output = code_outputLast + (tau2/tau1)*(d - dLast) + d*(T/tau1) (trackingCT.m:140) */
    return outLast + (tau2 / tau1) * (discri - discriLast) + discri * (T / tau1);
}

/* ---- trackingVT_POS_updated.m:157-349, the tracking half of one step ----
 * st[0..7] = {file_ptr (bytes), remChip, remCarrPhase, codeFreq (last step), carrFreq,
 * carrFreqBasis, oldCarrNco, oldCarrError}, advanced in place; rec[16] = {E_i, E_q, P_i, P_q,
 * L_i, L_q, carrError, codeError, carrNco, remChip, remCarrPhase, codeFreq, carrFreq, numSample,
 * absoluteSample, codedelay}. iq = the int8 I/Q record from byte 0 (NULL: sums given in
 * sums[2] = {sum I, sum Q}, the replay of a recorded step); ca = the PRN's 1023 chips.
 * Returns GNSS_* (EINDEX: a replica index MATLAB rejects; EIO: read past nbytes). */
static double or_vt_spacing(int i1)
{
    or_colon c;
    or_colon_init(&c, 0.7, -0.05, -0.7); /* Spacing = 0.7:-0.05:-0.7 (:27) */
    return or_colon_elem(&c, i1 - 1);
}

static double cn0_moment(const double *Zk, double T);

/* trackingVT_POS_updated.m:157-349, the tracking half of one step of one channel.
 * st (VT_STATE): [0] file_ptr (bytes), [1] remChip, [2] remCarrPhase, [3] codeFreq (the last
 * step's), [4] carrFreq, [5] carrFreqBasis, [6] oldCarrNco, [7] oldCarrError, [8] index_int,
 * [9] snrIndex, [10..29] Zk; advanced in place. rec (VT_REC, 18): E/P/L I/Q, carrError,
 * codeError, carrNco, remChip, remCarrPhase, codeFreq, carrFreq, numSample, absoluteSample,
 * codedelay, CN0, cn0_row. raw = the record's bytes (prec / dtype: dataPrecision /
 * dataType, :163-176) or NULL with sums = (sum I, sum Q) given. */
int or_vt_step(const uint8_t *raw, int64_t nbytes, int prec, int dtype, double *st, double codeFreq_new,
               const int8_t *ca, double Fs, double codelength, double ms, int pdi, double tau1carr,
               double tau2carr, const double *sums, double *rec)
{
    const double remChip0 = st[1];
    const int64_t n = (int64_t)ceil((codelength * pdi - remChip0) / (st[3] / Fs)); /* :161 */
    if (n < 1) return GNSS_EINDEX;
    const int64_t ptr = (int64_t)st[0];
    const int bps = prec * dtype;
    const double cps = codeFreq_new / Fs; /* :218 */
    /* t_CodeEarly / Prompt / Late (:220-222): each must have numSample elements (ceil_mx's
     * vertical concatenation, :227; t_CodePrompt(numSample), :284).
     * Code = [CA(end) repmat(CA,1,pdi) CA(1)] (:110): ceil_mx(idx) = the first element of
     * row idx = ceil(0 + Spacing + remChip) + 1, the 1025 clamp on it alone (:230-249) */
    int code[3];
    const int sp[3] = {5, 15, 25};
    or_colon col[3];
    for (int s = 0; s < 3; s++) {
        const double spc = or_vt_spacing(sp[s]);
        or_colon_init(&col[s], (0 + spc) + remChip0, cps, ((double)(n - 1) * cps + spc) + remChip0);
        if (col[s].n != n - 1) return GNSS_EINDEX;
        double j = ceil((0 + spc) + remChip0) + 1;
        if (j > 1025) j = 1025;
        const int64_t len = 1023 * (int64_t)pdi + 2, ji = (int64_t)j;
        if (ji < 1 || ji > len) return GNSS_EINDEX;
        code[s] = ji == 1 ? ca[1022] : ji == len ? ca[0] : ca[(ji - 2) % 1023];
    }
    double sI, sQ;
    if (raw) {
        if (ptr < 0 || ptr + (int64_t)bps * n > nbytes) return GNSS_EIO;
        double mi = 0, mq = 0;
        if (prec == 2) { /* rawsignal = (I - mean(I)) + 1i*(Q - mean(Q)) (:166-170) */
            for (int64_t k = 0; k < n; k++) {
                mi += (double)(int16_t)(raw[ptr + 4 * k] | (raw[ptr + 4 * k + 1] << 8));
                mq += (double)(int16_t)(raw[ptr + 4 * k + 2] | (raw[ptr + 4 * k + 3] << 8));
            }
            mi = mi / (double)n;
            mq = mq / (double)n;
        }
        long double aI = 0, aQ = 0;
        for (int64_t k = 0; k < n; k++) {
            /* Wave = (2*pi*(carrFreq .* CarrTime)) + remCarrPhase, CarrTime = (0:n)/Fs (:275-276) */
            const double W = TWO_PI * (st[4] * ((double)k / Fs)) + st[2];
            double xr, xi;
            if (prec == 2) {
                xr = (double)(int16_t)(raw[ptr + 4 * k] | (raw[ptr + 4 * k + 1] << 8)) - mi;
                xi = (double)(int16_t)(raw[ptr + 4 * k + 2] | (raw[ptr + 4 * k + 3] << 8)) - mq;
            } else if (dtype == 1) { /* int8 real (:172-175) */
                xr = (int8_t)raw[ptr + k];
                xi = 0;
            } else {
                xr = (int8_t)raw[ptr + 2 * k];
                xi = (int8_t)raw[ptr + 2 * k + 1];
            }
            aI += xr * sin(W) + xi * cos(W); /* imag(rawsignal .* carrsig) (:279) */
            aQ += xr * cos(W) - xi * sin(W); /* real(...) (:280) */
        }
        sI = (double)aI;
        sQ = (double)aQ;
    } else {
        sI = sums[0];
        sQ = sums[1];
    }
    const double remChip = (or_colon_elem(&col[1], n - 1) + cps) - 1023 * pdi;          /* :284 */
    const double remCarrPhase = fmod(TWO_PI * (st[4] * ((double)n / Fs)) + st[2], TWO_PI); /* :285 */
    const double Ei = code[0] * sI, Eq = code[0] * sQ, Pi = code[1] * sI, Pq = code[1] * sQ;
    const double Li = code[2] * sI, Lq = code[2] * sQ;
    /* C/N0 (:292-304; flag_snr is 1 throughout) */
    double cn0 = 0, cn0_row = 0;
    int index_int = (int)st[8] + 1;
    st[10 + index_int - 1] = Pi * Pi + Pq * Pq;
    if (index_int % 20 == 0) {
        cn0 = cn0_moment(st + 10, 1 * ms * pdi);
        cn0_row = st[9];
        index_int = 0;
        st[9] += 1;
    }
    st[8] = index_int;
    const double carrError = atan(Pq / Pi) / (2.0 * M_PI);                              /* :306 */
    const double carrNco = st[6] + (tau2carr / tau1carr) * (carrError - st[7]) +
                           carrError * (pdi * 1e-3 / tau1carr);                         /* :307 */
    const double carrFreq = st[5] + carrNco;                                            /* :310 */
    const double E = sqrt(Ei * Ei + Eq * Eq), L = sqrt(Li * Li + Lq * Lq);
    const double codeError = -0.5 * (E - L) / (E + L);                                  /* :316 */
    const int64_t absS = ptr + (int64_t)bps * n;                                        /* ftell */
    const double r[18] = {Ei, Eq, Pi, Pq, Li, Lq, carrError, codeError, carrNco, remChip, remCarrPhase,
                          codeFreq_new, carrFreq, (double)n, (double)absS,
                          fmod((double)absS / bps, Fs * ms), cn0, cn0_row};            /* :347 */
    memcpy(rec, r, sizeof r);
    st[0] = (double)absS;
    st[1] = remChip;
    st[2] = remCarrPhase;
    st[3] = codeFreq_new;
    st[4] = carrFreq;
    st[6] = carrNco;
    st[7] = carrError;
    return GNSS_OK;
}

typedef struct chan_state {
    double remChip, remPhase, remSample;
    double carrier_output, carrier_outputLast, PLLdiscriLast;
    double code_output, code_outputLast, DLLdiscriLast;
    double codeFreq, carrierFreqBasis, carrierFreq;
    int64_t numSample;
    int64_t pos; /* file position indicator, bytes */
    int index_int, snrIndex;
    double Zk[20];
} chan_state;

typedef struct trk_ctx {
    const gnss_file *file;
    const gnss_signal *sg;
    const gnss_track *tr;
    int64_t fsize;
    int ntaps, iE, iP, iL;
    const double *taps;
    double tau1code, tau2code, tau1carr, tau2carr;
    int nsv;
    int given; /* trackingCT_multiCorr-GIVEN.m: ceil numSample (:60), a short read raises */
    gnss_track_out *out;
} trk_ctx;

static void chan_init(chan_state *c, const trk_ctx *t, const gnss_acquired *acq, int sv)
{
    memset(c, 0, sizeof(*c));
    c->codeFreq = t->sg->codeFreqBasis;
    c->carrierFreqBasis = acq->fineFreq[sv];
    c->carrierFreq = acq->fineFreq[sv];
    c->snrIndex = 1;
}

/* record one value into rec[ch][field][i0..i1) */
static inline void rec_put(const trk_ctx *t, int ch, int f, int64_t i0, int64_t i1, double v)
{
    if (!t->out->rec) return;
    double *r = t->out->rec + ((int64_t)ch * GNSS_NFIELDS + f) * t->out->max_len;
    for (int64_t i = i0; i < i1 && i < t->out->max_len; i++) r[i] = v;
}

static inline void taps_put(const trk_ctx *t, int ch, int64_t i0, int64_t i1, const double *sums)
{
    if (!t->out->taps) return;
    for (int s = 0; s < t->ntaps; s++)
        for (int iq = 0; iq < 2; iq++) {
            double *r = t->out->taps + (((int64_t)ch * 2 + iq) * t->ntaps + s) * t->out->max_len;
            for (int64_t i = i0; i < i1 && i < t->out->max_len; i++) r[i] = sums[2 * s + iq];
        }
}

/* sum(delayValue(1:Index)) for an nsv x N matrix whose only non-zero row is sv
 * (1-based) holding dv[0..filled-1] (trackingCT.m:161,359,515, quirk A.11). */
static double dv_linear_sum(const int64_t *dv, int64_t filled, int64_t Index, int sv, int nsv)
{
    if (Index < sv) return 0;
    int64_t cols = (Index - sv) / nsv + 1;
    if (cols > filled) cols = filled;
    double s = 0;
    for (int64_t c = 0; c < cols; c++) s += (double)dv[c];
    return s;
}

/* One tracking step (body of trackingCT.m:79-170 / 407-524). Returns status. */
static int trk_step(const trk_ctx *t, chan_state *c, int ch, int sv1, int pdi, int phaseC,
                    int64_t Index, int64_t *dv, int64_t dv_col, double *cn0, cpx *buf,
                    const int8_t *ca, int64_t codedelay0, double *p_i_log)
{
    const gnss_signal *sg = t->sg;
    const double S = (double)sg->Sample;
    int64_t delayValue;
    if (phaseC) {
        delayValue = c->numSample - (int64_t)(S * pdi); /* :411 uses previous numSample */
        c->remSample = (sg->codelength * pdi - c->remChip) / (c->codeFreq / sg->Fs); /* :414 */
        c->numSample = (int64_t)or_round((sg->codelength * pdi - c->remChip) / (c->codeFreq / sg->Fs));
    } else {
        c->remSample = (sg->codelength - c->remChip) / (c->codeFreq / sg->Fs); /* :79 */
        const double q = (sg->codelength * pdi - c->remChip) / (c->codeFreq / sg->Fs);
        c->numSample = (int64_t)(t->given ? ceil(q) : or_round(q)); /* (GIVEN :60 ceil) */
        delayValue = c->numSample - (int64_t)(S * pdi); /* :82 */
    }
    dv[dv_col] = delayValue;
    const int64_t n = c->numSample;
    int64_t got = 0;
    const int64_t m = rd_cpx(t->file, c->pos, n, buf, &got); /* :84-93 / :416-426 */
    if (m == -1) return GNSS_EIO;
    if (m == -2) return GNSS_EINDEX;
    if (m != n) return (phaseC || t->given) ? GNSS_EIO : GNSS_ENODATA; /* :108-112 / :442 */
    c->pos += got; /* ftell */

    /* code range check: MATLAB would raise an index error */
    {
        const double d = c->codeFreq / sg->Fs;
        for (int s = 0; s < t->ntaps; s++) {
            double a = (0 + t->taps[s]) + c->remChip;
            double b = ((double)(n - 1) * d + t->taps[s]) + c->remChip;
            or_colon col;
            or_colon_init(&col, a, d, b);
            if (col.n != n - 1) return GNSS_EINDEX;
            if (!chip_ok((int64_t)ceil(or_colon_elem(&col, 0)), pdi) ||
                !chip_ok((int64_t)ceil(or_colon_elem(&col, n - 1)), pdi))
                return GNSS_EINDEX;
        }
    }

    double sums[2 * GNSS_MAX_TAPS];
    g_lane_w = pdi == 1 ? 8 : 24;
    g_lane_a7 = (int)(((c->pos - got) / (t->file->dataType * t->file->dataPrecision)) & 7);
    correlate_cpx(buf, n, c->remChip, c->codeFreq, sg->Fs, c->carrierFreq, c->remPhase, ca, pdi,
                  t->ntaps, t->taps, NULL, 0, sums);
    if (phaseC)
        for (int s = 0; s < 2 * t->ntaps; s++) sums[s] = -sums[s]; /* :447-449 */

    /* remChip = (t_CodePrompt(numSample) + codeFreq/Fs) - codeFreqBasis*ms*pdi (:102) */
    {
        const double d = c->codeFreq / sg->Fs;
        double a = (0 + t->taps[t->iP]) + c->remChip;
        double b = ((double)(n - 1) * d + t->taps[t->iP]) + c->remChip;
        or_colon col;
        or_colon_init(&col, a, d, b);
        c->remChip = (or_colon_elem(&col, n - 1) + c->codeFreq / sg->Fs) -
                     sg->codeFreqBasis * sg->ms * pdi;
    }
    /* remPhase = rem(Wave(numSample+1), 2*pi) (:104-106) */
    c->remPhase = fmod(TWO_PI * (c->carrierFreq * ((double)n / sg->Fs)) + c->remPhase, TWO_PI);

    const double E_i = sums[2 * t->iE], E_q = sums[2 * t->iE + 1];
    const double P_i = sums[2 * t->iP], P_q = sums[2 * t->iP + 1];
    const double L_i = sums[2 * t->iL], L_q = sums[2 * t->iL + 1];
    if (p_i_log) p_i_log[Index - 1] = P_i;

    /* C/N0 every K = 20 steps (:120-134) */
    c->index_int += 1;
    c->Zk[c->index_int - 1] = P_i * P_i + P_q * P_q;
    if (c->index_int % 20 == 0) {
        double mean = 0;
        for (int k = 0; k < 20; k++) mean += c->Zk[k];
        mean = mean / 20;
        double var = 0;
        for (int k = 0; k < 20; k++) var += (c->Zk[k] - mean) * (c->Zk[k] - mean);
        var = var / 19;
        double m2v = mean * mean - var;
        double cn;
        double scale = 1 / (1 * sg->ms * pdi);
        if (m2v >= 0) {
            double NA2 = sqrt(m2v);
            double varIQ = 0.5 * (mean - NA2);
            cn = fabs(10 * log10(scale * NA2 / (2 * varIQ)));
        } else { /* sqrt of a negative: complex NA2 = i*y; abs(10*log10(z)) */
            double y = sqrt(-m2v);
            /* z = (scale * (i*y)) / (2 * 0.5*(mean - i*y)) */
            double nr = 0, ni = scale * y;
            double dr = 2 * (0.5 * mean), di = 2 * (0.5 * -y);
            double den = dr * dr + di * di;
            double zr = (nr * dr + ni * di) / den, zi = (ni * dr - nr * di) / den;
            double lr = 10 * (log(hypot(zr, zi)) / log(10.0));
            double li = 10 * (atan2(zi, zr) / log(10.0));
            cn = hypot(lr, li);
        }
        if (cn0 && c->snrIndex <= t->out->cn0_cap)
            cn0[(int64_t)(c->snrIndex - 1) * t->nsv + ch] = cn;
        c->index_int = 0;
        c->snrIndex += 1;
    }

    /* DLL (:136-143); phase C keeps T = 0.001 (:473) */
    double E = sqrt(E_i * E_i + E_q * E_q);
    double L = sqrt(L_i * L_i + L_q * L_q);
    double DLLdiscri = 0.5 * (E - L) / (E + L);
    double Tc = phaseC ? 0.001 : (0.001 * pdi);
    c->code_output = or_loop_filter(c->code_outputLast, DLLdiscri, c->DLLdiscriLast, t->tau1code,
                                    t->tau2code, Tc);
    c->DLLdiscriLast = DLLdiscri;
    c->code_outputLast = c->code_output;
    c->codeFreq = sg->codeFreqBasis - c->code_output;
    /* PLL (:145-150) */
    double PLLdiscri = atan(P_q / P_i) / TWO_PI;
    c->carrier_output = or_loop_filter(c->carrier_outputLast, PLLdiscri, c->PLLdiscriLast,
                                       t->tau1carr, t->tau2carr, Tc);
    c->carrier_outputLast = c->carrier_output;
    c->PLLdiscriLast = PLLdiscri;
    c->carrierFreq = c->carrierFreqBasis + c->carrier_output;

    /* record (:153-170; phase C writes Index-9:Index, :507-524) */
    int64_t i1 = Index, i0 = phaseC ? Index - 10 : Index - 1; /* 0-based half-open */
    double absS = (double)c->pos;
    double cd = (double)codedelay0 + dv_linear_sum(dv, dv_col + 1, Index, sv1, t->nsv);
    double vals[GNSS_NFIELDS] = {P_i, P_q, E_i, E_q, L_i, L_q, PLLdiscri, DLLdiscri, cd,
                                 c->remChip, c->codeFreq, c->carrierFreq, c->remPhase,
                                 c->remSample, (double)n, (double)delayValue, absS,
                                 or_mod(absS / (t->file->dataPrecision * t->file->dataType),
                                        sg->Fs * sg->ms)};
    for (int f = 0; f < GNSS_NFIELDS; f++) rec_put(t, ch, f, i0, i1, vals[f]);
    taps_put(t, ch, i0, i1, sums);
    return GNSS_OK;
}

static int track_channel(const trk_ctx *t, const gnss_acquired *acq, int ch, double *cn0,
                         int *countinx_out)
{
    const gnss_signal *sg = t->sg;
    const gnss_file *f = t->file;
    const int64_t S = sg->Sample;
    const int sv1 = ch + 1;
    const int64_t N1 = t->tr->msToProcessCT_1ms, N10 = t->tr->msToProcessCT_10ms;
    const int64_t cd0 = acq->codedelay[ch];
    int8_t ca[1023];
    if (or_generate_ca(acq->sv[ch], ca)) return GNSS_EARG;
    cpx *buf = (cpx *)malloc(sizeof(cpx) * (size_t)(2 * (S * 10 + 4096)));
    int64_t *dv = (int64_t *)calloc((size_t)(N1 + 32 + N10), sizeof(int64_t));
    double *plog = (double *)calloc((size_t)(N1 + 1), sizeof(double));
    chan_state c;
    int st = GNSS_OK;

    /* phase A (:22-171) */
    chan_init(&c, t, acq, ch);
    c.pos = (S - cd0 + 1 + f->skip * S) * f->dataPrecision * f->dataType; /* :63 */
    for (int64_t i = 1; i <= N1 && st == GNSS_OK; i++)
        st = trk_step(t, &c, ch, sv1, 1, 0, i, dv, i - 1, cn0, buf, ca, cd0, plog);
    if (st) goto done;

    /* bit transition (:178-213) on the phase-A P_i (length N1) */
    int cx = or_bit_edge(plog, N1, &st);
    if (st) goto done;
    *countinx_out = cx;

    /* phase B (:215-369): identical re-run for N1 + countinx steps */
    chan_init(&c, t, acq, ch);
    memset(dv, 0, sizeof(int64_t) * (size_t)(N1 + 32 + N10));
    c.pos = (S - cd0 + 1 + f->skip * S) * f->dataPrecision * f->dataType; /* :258 */
    int64_t Index = 0;
    for (int64_t i = 1; i <= N1 + cx && st == GNSS_OK; i++) {
        Index++;
        st = trk_step(t, &c, ch, sv1, 1, 0, Index, dv, i - 1, cn0, buf, ca, cd0, NULL);
    }
    if (st) goto done;

    /* phase C (:377-525) */
    memset(dv, 0, sizeof(int64_t) * (size_t)(N1 + 32 + N10));
    c.index_int = 0;
    c.snrIndex = 1;
    c.pos = (S - cd0 + 1 + (f->skip + N1 + cx) * S) * f->dataPrecision * f->dataType; /* :403 */
    for (int64_t is = 1; is <= N10 / 10 && st == GNSS_OK; is++) {
        Index += 10;
        st = trk_step(t, &c, ch, sv1, 10, 1, Index, dv, is - 1, cn0, buf, ca, cd0, NULL);
    }
    if (!st && t->out->len) t->out->len[ch] = Index;
done:
    free(buf);
    free(dv);
    free(plog);
    return st;
}

int or_tracking_ct(const gnss_file *file, const gnss_signal *sg, const gnss_track *tr,
                   const gnss_acquired *acq, gnss_track_out *out, int nthreads)
{
    if ((file->dataPrecision != 1 && file->dataPrecision != 2) || (file->dataType != 1 && file->dataType != 2))
        return GNSS_EARG;
    trk_ctx t;
    memset(&t, 0, sizeof(t));
    t.file = file; t.sg = sg; t.tr = tr; t.out = out; t.nsv = acq->n;
    t.fsize = file_size(file);
    double taps3[3] = {-tr->CorrelatorSpacing, 0, tr->CorrelatorSpacing}; /* :24 */
    if (tr->n_taps > 0) {
        if (tr->n_taps > GNSS_MAX_TAPS || !tr->tap_offsets) return GNSS_EARG;
        t.ntaps = tr->n_taps; t.taps = tr->tap_offsets;
    } else {
        t.ntaps = 3; t.taps = taps3;
    }
    t.iE = t.iP = t.iL = -1;
    for (int s = 0; s < t.ntaps; s++) {
        if (t.taps[s] == -tr->CorrelatorSpacing && t.iE < 0) t.iE = s;
        if (t.taps[s] == 0 && t.iP < 0) t.iP = s;
        if (t.taps[s] == tr->CorrelatorSpacing && t.iL < 0) t.iL = s;
    }
    if (t.iE < 0 || t.iP < 0 || t.iL < 0) return GNSS_EARG;
    if (out->max_len < (int64_t)tr->msToProcessCT_1ms + 19 + tr->msToProcessCT_10ms) return GNSS_EARG;
    or_calc_loop_coef(tr->DLLBW, tr->DLLDamp, tr->DLLGain, &t.tau1code, &t.tau2code); /* :26-27 */
    or_calc_loop_coef(tr->PLLBW, tr->PLLDamp, tr->PLLGain, &t.tau1carr, &t.tau2carr);

    int nch = tr->chan ? tr->n_chan : acq->n;
    int nt = nthreads_of(nthreads);
    int status = GNSS_OK;
    if (out->CN0_Eph) memset(out->CN0_Eph, 0, sizeof(double) * (size_t)out->cn0_cap * (size_t)acq->n);
#pragma omp parallel for num_threads(nt) schedule(dynamic)
    for (int i = 0; i < nch; i++) {
        int ch = tr->chan ? tr->chan[i] : i;
        int cx = 0;
        int st = track_channel(&t, acq, ch, out->CN0_Eph, &cx);
        if (out->countinx) out->countinx[ch] = cx;
#pragma omp critical
        {
            /* the reference aborts the whole call on the first failing channel;
             * ENODATA dominates (TckResultCT = []), then the hard errors */
            if (st && (status == GNSS_OK || st == GNSS_ENODATA)) status = st;
        }
    }
    /* CN0_Eph rows = max rows written by any phase (quirk A.16) */
    int rows = 0;
    int r1 = tr->msToProcessCT_1ms / 20;
    for (int i = 0; i < nch; i++) {
        int ch = tr->chan ? tr->chan[i] : i;
        int cx = out->countinx ? out->countinx[ch] : 0;
        int rb = (int)((tr->msToProcessCT_1ms + cx) / 20);
        if (rb > rows) rows = rb;
    }
    if (r1 > rows) rows = r1;
    if (tr->msToProcessCT_10ms / 10 / 20 > rows) rows = tr->msToProcessCT_10ms / 10 / 20;
    out->cn0_rows = rows;
    return status;
}

/* ------------------------------------------------------------------------ */
/* trackingCT_multiCorr-GIVEN.m (function trackingCT_multiCorr)              */
/* ------------------------------------------------------------------------ */
/* Per channel (:31-313): fseek to (Sample - codedelay - 1 + skip*Sample)*bytes (:57), then
 * `datalength` 1-ms steps of trackingCT.m's step with ceil numSample (:58-60), 25 taps at
 * Spacing = -0.6:0.05:0.6 (:25), Code(ceil(t)+1) (:140-164), E/P/L = Spacing(3)/(13)/(23).
 * codedelay (:297) = Codedelay + sum(delayValue(1:msIndex)) over the one nsv x datalength
 * matrix of :29, filled channel after channel: a pass after all channels. */
int or_tracking_ct_given(const gnss_file *file, const gnss_signal *sg, const gnss_track *tr,
                         const gnss_acquired *acq, int32_t datalength, gnss_track_out *out,
                         int nthreads)
{
    if (file->dataPrecision != 1 || file->dataType != 2 || datalength <= 0 || tr->n_taps != 0 ||
        (tr->chan && tr->n_chan > 0) || out->max_len < datalength)
        return GNSS_EARG;
    double sp[25];
    or_colon spc;
    or_colon_init(&spc, -0.6, 0.05, 0.6);
    if (spc.n != 24) return GNSS_EARG;
    for (int k = 0; k < 25; k++) sp[k] = or_colon_elem(&spc, k);
    trk_ctx t;
    memset(&t, 0, sizeof(t));
    t.file = file; t.sg = sg; t.tr = tr; t.out = out; t.nsv = acq->n;
    t.fsize = file_size(file);
    t.ntaps = 25; t.taps = sp; t.iE = 2; t.iP = 12; t.iL = 22; t.given = 1;
    or_calc_loop_coef(tr->DLLBW, tr->DLLDamp, tr->DLLGain, &t.tau1code, &t.tau2code); /* :21-22 */
    or_calc_loop_coef(tr->PLLBW, tr->PLLDamp, tr->PLLGain, &t.tau1carr, &t.tau2carr);
    const int nsv = acq->n;
    const int64_t S = sg->Sample;
    int status = GNSS_OK;
    if (out->CN0_Eph) memset(out->CN0_Eph, 0, sizeof(double) * (size_t)out->cn0_cap * (size_t)nsv);
#pragma omp parallel for num_threads(nthreads_of(nthreads)) schedule(dynamic)
    for (int ch = 0; ch < nsv; ch++) {
        int8_t ca[1023];
        int st = or_generate_ca(acq->sv[ch], ca) ? GNSS_EARG : GNSS_OK;
        cpx *buf = (cpx *)malloc(sizeof(cpx) * (size_t)(2 * (S + 4096)));
        int64_t *dv = (int64_t *)calloc((size_t)datalength, sizeof(int64_t));
        const int64_t cd0 = acq->codedelay[ch]; /* Codedelay = AcqCodeDelay (:53,55) */
        chan_state c;
        chan_init(&c, &t, acq, ch);
        c.pos = (S - cd0 - 1 + file->skip * S) * file->dataPrecision * file->dataType; /* :57 */
        for (int64_t i = 1; i <= datalength && st == GNSS_OK; i++)
            st = trk_step(&t, &c, ch, ch + 1, 1, 0, i, dv, i - 1, out->CN0_Eph, buf, ca, cd0, NULL);
        if (!st && out->len) out->len[ch] = datalength;
        if (out->countinx) out->countinx[ch] = 0;
        free(buf);
        free(dv);
#pragma omp critical
        {
            if (st && status == GNSS_OK) status = st;
        }
    }
    if (status == GNSS_OK && out->rec) {
        const int64_t ML = out->max_len;
        for (int ch = 0; ch < nsv; ch++) {
            double *cdr = out->rec + ((int64_t)ch * GNSS_NFIELDS + GNSS_F_codedelay) * ML;
            double sum = 0;
            for (int64_t k = 0; k < datalength; k++) { /* linear position k + 1 */
                int r = (int)(k % nsv);
                if (r <= ch) sum += out->rec[((int64_t)r * GNSS_NFIELDS + GNSS_F_delayValue) * ML + k / nsv];
                cdr[k] = (double)acq->codedelay[ch] + sum;
            }
        }
    }
    out->cn0_rows = datalength / 20;
    return status;
}

/* ------------------------------------------------------------------------ */
/* trackingCT_POS_updated.m: its tracking loop (positioning half out of scope) */
/* ------------------------------------------------------------------------ */

/* The C/N0 moment estimator of trackingCT_POS_updated.m:241-246 (= trackingCT.m:124-131). */
static double cn0_moment(const double *Zk, double T)
{
    double mean = 0;
    for (int k = 0; k < 20; k++) mean += Zk[k];
    mean = mean / 20;
    double var = 0;
    for (int k = 0; k < 20; k++) var += (Zk[k] - mean) * (Zk[k] - mean);
    var = var / 19;
    double m2v = mean * mean - var;
    double scale = 1 / T; /* 1/(1*t*pdi) */
    if (m2v >= 0) {
        double NA2 = sqrt(m2v);
        double varIQ = 0.5 * (mean - NA2);
        return fabs(10 * log10(scale * NA2 / (2 * varIQ)));
    }
    double y = sqrt(-m2v); /* complex NA2 = i*y (quirk A.16) */
    double nr = 0, ni = scale * y;
    double dr = 2 * (0.5 * mean), di = 2 * (0.5 * -y);
    double den = dr * dr + di * di;
    double zr = (nr * dr + ni * di) / den, zi = (ni * dr - nr * di) / den;
    double lr = 10 * (log(hypot(zr, zi)) / log(10.0));
    double li = 10 * (atan2(zi, zr) / log(10.0));
    return hypot(lr, li);
}

/* The two sibling loops: trackingCT_POS_updated.m (mc_pdi = 0: E/P/L, the prompt at
 * ceil(t + 0.05), 1-ms steps up to 1000 + countinx then 10-ms steps, T = t) and
 * trackingCT_POS_updated_multicorrelator.m (mc_pdi = 1 or 10: the 25 Spacing taps,
 * Code(ceil(t) + 2), every step at mc_pdi, T = pdi*t). */
typedef struct {
    int ntaps, iE, iP, iL, chip_off, mc_pdi;
    double taps[GNSS_MAX_TAPS], post[GNSS_MAX_TAPS];
} trkpos_mode;

/* One channel of trackingCT_POS_updated.m:92-118 (init) and :179-408 (the msIndex loop,
 * both pdi branches; the channel loop is independent per svIndex: each channel seeks its
 * own file_ptr before every read); with mc_pdi, of
 * trackingCT_POS_updated_multicorrelator.m:91-136 and :170-440. */
static int trkpos_channel(const trk_ctx *t, const gnss_acquired *acq, int ch, int32_t ctPOS,
                          int32_t cx, double *cn0, const trkpos_mode *md)
{
    const gnss_signal *sg = t->sg;
    const gnss_file *f = t->file;
    const double S = (double)sg->Sample;
    const double *taps = md->taps, *post = md->post;
    int8_t ca[1023];
    if (or_generate_ca(acq->sv[ch], ca)) return GNSS_EARG;
    cpx *buf = (cpx *)malloc(sizeof(cpx) * (size_t)(2 * (sg->Sample * 10 + 4096)));
    int st = GNSS_OK;
    const int64_t AcqCodeDelay = acq->codedelay[ch]; /* (multicorrelator: :95,101-103) */
    int64_t file_ptr = (int64_t)((S - (double)AcqCodeDelay + 1 + (double)f->skip * sg->Fs * sg->ms) *
                                 f->dataPrecision * f->dataType); /* :108-110 */
    const double AcqFreq = acq->fineFreq[ch];                     /* :113-114 */
    double carrFreq = AcqFreq, codeFreq = sg->codeFreqBasis, remChip = 0, remCarrPhase = 0;
    double carrNco = 0, oldCarrNco = 0, oldCarrError = 0, codeNco = 0, code_outputLast = 0,
           DLLdiscriLast = 0;
    double Zk[20] = {0};
    int index_int = 0, snrIndex = 1;
    double dvsum = 0;
    const double tT = sg->ms; /* t = signal.ms (:48) */
    for (int64_t Index = 1; Index <= ctPOS && st == GNSS_OK; Index++) {
        const int pdi = md->mc_pdi ? md->mc_pdi
                                   : (Index <= t->tr->msToProcessCT_1ms + (int64_t)cx) ? 1 : 10; /* :183,:294 */
        const double cps = codeFreq / sg->Fs;                                          /* :188 */
        const int64_t n = (int64_t)ceil((sg->codelength * pdi - remChip) / cps);       /* :189 */
        const int64_t delayValue = n - (int64_t)(S * pdi);                             /* :191 */
        int64_t got = 0;
        const int64_t m = rd_cpx(f, file_ptr, n, buf, &got); /* fseek + fread (:193-205) */
        if (m == -1 || m != n) { st = GNSS_EIO; break; }     /* short read: MATLAB raises */
        if (m == -2) { st = GNSS_EINDEX; break; }
        const int64_t ftell_pos = file_ptr + got;
        file_ptr = file_ptr + n * f->dataType;               /* :207 (int8: = ftell) */
        /* code index range (MATLAB would raise on an out-of-range Code index): ceil(t) + 1 +
         * chip_off within [1, 1023*pdi + 2 + chip_off] */
        for (int s = 0; s < md->ntaps && st == GNSS_OK; s++) {
            double a = (0 + taps[s]) + remChip;
            double b = ((double)(n - 1) * cps + taps[s]) + remChip;
            or_colon col;
            or_colon_init(&col, a, cps, b);
            if (col.n != n - 1 ||
                !chip_ok((int64_t)ceil(or_colon_elem(&col, 0) + post[s]) + md->chip_off, pdi) ||
                !chip_ok((int64_t)ceil(or_colon_elem(&col, n - 1) + post[s]), pdi))
                st = GNSS_EINDEX;
        }
        if (st) break;
        double tsums[2 * GNSS_MAX_TAPS];
        correlate_cpx(buf, n, remChip, codeFreq, sg->Fs, carrFreq, remCarrPhase, ca, pdi, md->ntaps, taps,
                      post, md->chip_off, tsums); /* :210-235 (multicorrelator :207-329) */
        {   /* remChip = t_CodePrompt(numSample) + codePhaseStep - codelength*pdi (:220; mc :262) */
            double a = (0 + taps[md->iP]) + remChip;
            double b = ((double)(n - 1) * cps + taps[md->iP]) + remChip;
            or_colon col;
            or_colon_init(&col, a, cps, b);
            remChip = or_colon_elem(&col, n - 1) + cps - sg->codelength * pdi;
        }
        /* Wave = 2*pi*(carrFreq.*CarrTime) + remCarrPhase; rem(Wave(n+1), 2*pi) (:222-224) */
        remCarrPhase = fmod(TWO_PI * (carrFreq * ((double)n / sg->Fs)) + remCarrPhase, TWO_PI);
        const double E_i = tsums[2 * md->iE], E_q = tsums[2 * md->iE + 1], P_i = tsums[2 * md->iP],
                     P_q = tsums[2 * md->iP + 1], L_i = tsums[2 * md->iL], L_q = tsums[2 * md->iL + 1];
        /* loop T: t (:257,266); multicorrelator (pdi*t) (:352,361) */
        const double Tl = md->mc_pdi ? pdi * tT : tT;
        /* C/N0 (:238-250) */
        index_int += 1;
        Zk[index_int - 1] = P_i * P_i + P_q * P_q;
        if (index_int % 20 == 0) {
            double cn = cn0_moment(Zk, 1 * tT * pdi);
            if (cn0 && snrIndex <= t->out->cn0_cap) cn0[(int64_t)(snrIndex - 1) * t->nsv + ch] = cn;
            index_int = 0;
            snrIndex += 1;
        }
        /* DLL (:253-262) */
        double E = sqrt(E_i * E_i + E_q * E_q);
        double L = sqrt(L_i * L_i + L_q * L_q);
        double codeError = 0.5 * (E - L) / (E + L);
        codeNco = or_loop_filter(code_outputLast, codeError, DLLdiscriLast, t->tau1code, t->tau2code, Tl);
        DLLdiscriLast = codeError;
        code_outputLast = codeNco;
        codeFreq = sg->codeFreqBasis + codeNco;
        /* PLL (:265-270) */
        double carrError = atan(P_q / P_i) / TWO_PI;
        carrNco = or_loop_filter(oldCarrNco, carrError, oldCarrError, t->tau1carr, t->tau2carr, Tl);
        oldCarrNco = carrNco;
        oldCarrError = carrError;
        carrFreq = AcqFreq + carrNco;
        /* record (:273-292) */
        dvsum += (double)delayValue;
        const double absS = (double)ftell_pos;
        const double cd2 = or_mod(absS / (f->dataPrecision * f->dataType), sg->Fs * sg->ms);
        const double codedelay = (S - (double)AcqCodeDelay + 1) + dvsum;
        double vals[GNSS_NFIELDS] = {P_i, P_q, E_i, E_q, L_i, L_q, carrError, codeError, codedelay,
                                     remChip, codeFreq, carrFreq, remCarrPhase, cd2, (double)n,
                                     (double)delayValue, absS, cd2};
        for (int fi = 0; fi < GNSS_NFIELDS; fi++) rec_put(t, ch, fi, Index - 1, Index, vals[fi]);
        taps_put(t, ch, Index - 1, Index, tsums);
    }
    if (!st && t->out->len) t->out->len[ch] = ctPOS;
    free(buf);
    return st;
}

static int trkpos_run(const gnss_file *file, const gnss_signal *sg, const gnss_track *tr,
                      const gnss_acquired *acq, int32_t ctPOS, const int32_t *countinx,
                      gnss_track_out *out, int nthreads, const trkpos_mode *md)
{
    if (file->dataPrecision != 1 || (file->dataType != 1 && file->dataType != 2) || ctPOS <= 0 ||
        (!countinx && !md->mc_pdi) || tr->n_taps != 0 || out->max_len < ctPOS)
        return GNSS_EARG;
    trk_ctx t;
    memset(&t, 0, sizeof(t));
    t.file = file; t.sg = sg; t.tr = tr; t.out = out; t.nsv = acq->n;
    t.fsize = file_size(file);
    t.ntaps = md->ntaps;
    or_calc_loop_coef(tr->DLLBW, tr->DLLDamp, tr->DLLGain, &t.tau1code, &t.tau2code); /* :87-88 */
    or_calc_loop_coef(tr->PLLBW, tr->PLLDamp, tr->PLLGain, &t.tau1carr, &t.tau2carr);
    int nch = tr->chan ? tr->n_chan : acq->n;
    int nt = nthreads_of(nthreads);
    int status = GNSS_OK;
    if (out->CN0_Eph) memset(out->CN0_Eph, 0, sizeof(double) * (size_t)out->cn0_cap * (size_t)acq->n);
#pragma omp parallel for num_threads(nt) schedule(dynamic)
    for (int i = 0; i < nch; i++) {
        int ch = tr->chan ? tr->chan[i] : i;
        const int32_t cx = countinx ? countinx[ch] : 0;
        int st = trkpos_channel(&t, acq, ch, ctPOS, cx, out->CN0_Eph, md);
        if (out->countinx) out->countinx[ch] = cx;
#pragma omp critical
        {
            if (st && status == GNSS_OK) status = st;
        }
    }
    out->cn0_rows = ctPOS / 20;
    return status;
}

int or_tracking_ct_pos(const gnss_file *file, const gnss_signal *sg, const gnss_track *tr,
                       const gnss_acquired *acq, int32_t ctPOS, const int32_t *countinx,
                       gnss_track_out *out, int nthreads)
{
    trkpos_mode md;
    memset(&md, 0, sizeof(md));
    md.ntaps = 3; md.iE = 0; md.iP = 1; md.iL = 2;
    md.taps[0] = 0.5; md.taps[1] = 0.0; md.taps[2] = -0.5; /* Spacing(3), (13), (23) (:42) */
    md.post[1] = 0.05;                                     /* ceil(t_CodePrompt+0.05) (:216) */
    return trkpos_run(file, sg, tr, acq, ctPOS, countinx, out, nthreads, &md);
}

int or_tracking_ct_mc(const gnss_file *file, const gnss_signal *sg, const gnss_track *tr,
                      const gnss_acquired *acq, int32_t msPosCT, int32_t pdi, gnss_track_out *out,
                      int nthreads)
{
    if ((pdi != 1 && pdi != 10) || msPosCT < pdi) return GNSS_EARG;
    trkpos_mode md;
    memset(&md, 0, sizeof(md));
    md.ntaps = 25; md.iE = 2; md.iP = 12; md.iL = 22; md.chip_off = 1; md.mc_pdi = pdi;
    or_colon sp; /* Spacing = 0.6:-0.05:-0.6 (:41) */
    or_colon_init(&sp, 0.6, -0.05, -0.6);
    if (sp.n != 24) return GNSS_EARG;
    for (int k = 0; k < 25; k++) md.taps[k] = or_colon_elem(&sp, k);
    return trkpos_run(file, sg, tr, acq, msPosCT / pdi, NULL, out, nthreads, &md); /* 1:datalength/pdi */
}

/* ------------------------------------------------------------------------ */
/* Synthetic IF                                                 */
/* ------------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void or_synth_if(const gnss_synth *cfg, uint64_t sample0, uint64_t nsamples, int8_t *dst,
                 int nthreads)
{
    const double fL1 = 1575.42e6, fc = 1.023e6;
    int8_t ca[GNSS_MAX_SV][1023];
    double amp[GNSS_MAX_SV], crate[GNSS_MAX_SV], frate[GNSS_MAX_SV];
    for (int s = 0; s < cfg->n_sv; s++) {
        or_generate_ca(cfg->sv[s].prn, ca[s]);
        double snr_lin = pow(10.0, cfg->sv[s].cn0_dbhz / 10.0);
        amp[s] = sqrt(2.0 * cfg->noise_sigma * cfg->noise_sigma * snr_lin / cfg->Fs);
        crate[s] = fc * (1.0 + cfg->sv[s].doppler_hz / fL1) / cfg->Fs;
        frate[s] = (cfg->IF + cfg->sv[s].doppler_hz) / cfg->Fs;
    }
    int nt = nthreads_of(nthreads);
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < (int64_t)nsamples; i++) {
        uint64_t n = sample0 + (uint64_t)i;
        double re = 0, im = 0;
        for (int s = 0; s < cfg->n_sv; s++) {
            const gnss_synth_sv *v = &cfg->sv[s];
            double th = v->code_phase0 + (double)n * crate[s];
            double chipf = floor(th);
            int64_t chip = (int64_t)chipf % 1023;
            if (chip < 0) chip += 1023;
            double bitf = floor((th + v->bit_phase_chips) / 20460.0);
            uint64_t bh = mix64(v->bit_seed ^ (uint64_t)(int64_t)bitf);
            double D = (bh & 1) ? 1.0 : -1.0;
            double ph = v->carr_phase0 - (double)n * frate[s]; /* received at -(IF+fd) */
            ph -= floor(ph);
            double a = amp[s] * D * ca[s][chip];
            re += a * cos(TWO_PI * ph);
            im += a * sin(TWO_PI * ph);
        }
        uint64_t h1 = mix64(cfg->seed ^ (n * 0xD1B54A32D192ED03ULL));
        uint64_t h2 = mix64(h1 ^ 0x8CB92BA72F3D8DD7ULL);
        double u1 = ((double)(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);
        double u2 = (double)(h2 >> 11) * (1.0 / 9007199254740992.0);
        double r = sqrt(-2.0 * log(u1)) * cfg->noise_sigma;
        double vi = rint(re + r * cos(TWO_PI * u2));
        double vq = rint(im + r * sin(TWO_PI * u2));
        if (vi > 127) vi = 127;
        if (vi < -128) vi = -128;
        if (vq > 127) vq = 127;
        if (vq < -128) vq = -128;
        dst[2 * i] = (int8_t)vi;
        dst[2 * i + 1] = (int8_t)vq;
    }
}

/* ===========================================================================================
 * trackingVT_POS_updated.m, the vector half: the geo helpers of
 * SDR_MATLAB-main/geo, the code-frequency prediction (:180-227) and the 8-state EKF
 * (:357-467), restated line by line; the closed loop with or_vt_step's correlator.
 * =========================================================================================== */

/* sin / cos as separate libm calls: MATLAB evaluates sin() and cos() element by element, and
 * gcc would otherwise fuse a sin / cos pair of one argument into glibc's sincos(), which
 * rounds differently in the last place (the product's host code, built by clang, calls sin
 * and cos; oracle and product then agree bit for bit on the navigation half). */
__attribute__((noinline)) static double or_nsin(double x) { return sin(x); }
__attribute__((noinline)) static double or_ncos(double x) { return cos(x); }

/* xyz2llh.m:25-69 */
void or_xyz2llh(const double *xyz, double *llh)
{
    double x = xyz[0], y = xyz[1], z = xyz[2];
    double x2 = x * x, y2 = y * y, z2 = z * z;                 /* x^2 */
    double a = 6378137.0000, b = 6356752.3142;
    double e = sqrt(1 - (b / a) * (b / a));                    /* (b/a).^2 */
    double b2 = b * b, e2 = e * e, ep = e * (a / b);
    double r = sqrt(x2 + y2), r2 = r * r;
    double E2 = a * a - b * b;
    double F = 54 * b2 * z2;
    double G = r2 + (1 - e2) * z2 - e2 * E2;
    double c = (e2 * e2 * F * r2) / (G * G * G);
    double s = pow(1 + c + sqrt(c * c + 2 * c), 1.0 / 3.0);
    double q = s + 1 / s + 1;
    double P = F / (3 * (q * q) * G * G);
    double Q = sqrt(1 + 2 * e2 * e2 * P);
    double ro = -(P * e2 * r) / (1 + Q) + sqrt((a * a / 2) * (1 + 1 / Q) - (P * (1 - e2) * z2) / (Q * (1 + Q)) -
                                               P * r2 / 2);
    double t0 = r - e2 * ro;
    double tmp = t0 * t0;
    double U = sqrt(tmp + z2), V = sqrt(tmp + (1 - e2) * z2);
    double zo = (b2 * z) / (a * V);
    double height = U * (1 - b2 / (a * V));
    double lat = atan((z + ep * ep * zo) / r);
    double temp = atan(y / x), lon;
    if (x >= 0) lon = temp;
    else if (x < 0 && y >= 0) lon = M_PI + temp;
    else lon = temp - M_PI;
    llh[0] = lat;
    llh[1] = lon;
    llh[2] = height;
}

/* llh2xyz.m:20-34 */
void or_llh2xyz(const double *llh, double *xyz)
{
    double re = 6378137.0, eflat = (1.0 / 298.257223563);
    double e2 = (2 - eflat) * eflat;
    double slat = or_nsin(llh[0]), clat = or_ncos(llh[0]);
    double r_N = re / sqrt(1 - e2 * slat * slat);
    xyz[0] = (r_N + llh[2]) * clat * or_ncos(llh[1]);
    xyz[1] = (r_N + llh[2]) * clat * or_nsin(llh[1]);
    xyz[2] = (r_N * (1 - e2) + llh[2]) * slat;
}

/* R * d for a 3x3 R, each row's sum left to right */
static void or_mv3(double R[3][3], const double *d, double *out)
{
    for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int j = 0; j < 3; j++) s = s + R[i][j] * d[j];
        out[i] = s;
    }
}

/* xyz2enu.m:32-47 */
void or_xyz2enu(const double *xyz, const double *orgxyz, double *enu)
{
    double difxyz[3] = {xyz[0] - orgxyz[0], xyz[1] - orgxyz[1], xyz[2] - orgxyz[2]};
    double orgllh[3];
    or_xyz2llh(orgxyz, orgllh);
    double phi = orgllh[0], lam = orgllh[1];
    double sinphi = or_nsin(phi), cosphi = or_ncos(phi), sinlam = or_nsin(lam), coslam = or_ncos(lam);
    double R[3][3] = {{-sinlam, coslam, 0},
                      {-sinphi * coslam, -sinphi * sinlam, cosphi},
                      {cosphi * coslam, cosphi * sinlam, sinphi}};
    or_mv3(R, difxyz, enu);
}

/* erotcorr.m:21-35 */
void or_erotcorr(const double *svxyz, double pr, double *svxyzr)
{
    double omega = 7.2921151467e-5;
    double deltat = pr / 299792458;
    double theta = omega * deltat;
    double rotmat[3][3] = {{or_ncos(theta), or_nsin(theta), 0}, {-or_nsin(theta), or_ncos(theta), 0}, {0, 0, 1}};
    or_mv3(rotmat, svxyz, svxyzr);
}

/* ionocorr.m:21-61 (phiu / lambdau are the SATELLITE's latitude / longitude, :23,33,38) */
double or_ionocorr(double systime, const double *svxyz, const double *usrxyz, const double *ALPHA,
                   const double *BETA)
{
    double svllh[3], svenu[3];
    or_xyz2llh(svxyz, svllh);
    or_xyz2enu(svxyz, usrxyz, svenu);
    double el = atan2(svenu[2], sqrt(svenu[0] * svenu[0] + svenu[1] * svenu[1]));
    double az = atan2(svenu[0], svenu[1]);
    double E = el / M_PI;
    double F = 1 + 16 * ((0.53 - E) * (0.53 - E) * (0.53 - E));
    double psi = 0.00137 / (E + 0.11) - 0.022;
    double phiu = svllh[0] / M_PI;
    double phii = phiu + psi * or_ncos(az);
    if (phii > 0.416) phii = 0.416;
    if (phii < -0.416) phii = -0.416;
    double lambdau = svllh[1] / M_PI;
    double lambdai = lambdau + psi * or_nsin(az) / or_ncos(phii * M_PI);
    double phim = phii + 0.064 * or_ncos((lambdai - 1.616) * M_PI);
    double t = 4.32e4 * lambdai + systime;
    while ((t < 0) | (t >= 86400)) {
        if (t >= 86400) t = t - 86400;
        if (t < 0) t = t + 86400;
    }
    double PER = BETA[0] + BETA[1] * phim + BETA[2] * (phim * phim) + BETA[3] * (phim * phim * phim);
    if (PER < 72000) PER = 72000;
    double x = 2 * M_PI * (t - 50400) / PER;
    double AMP = ALPHA[0] + ALPHA[1] * phim + ALPHA[2] * (phim * phim) + ALPHA[3] * (phim * phim * phim);
    if (AMP < 0) AMP = 0;
    double Tiono;
    if (fabs(x) < 1.57) Tiono = F * (5e-9 + AMP * (1 - (x * x) / 2 + ((x * x) * (x * x)) / 24));
    else Tiono = F * 5e-9;
    return Tiono * 299792458;
}

/* trop_UNB3.m (Get_UNB3_Model.m, Trop_Saastamoinen_UNB3_Components.m, Trop_Black_Eisner_Map.m;
 * MATLAB's cosd reduces by quadrants first). Returns GNSS_EINDEX for |lat| <= 15 (avg(0,:)). */
int or_trop_unb3(double doy, double lat, double alt, double el, double *out)
{
    static const double avg[5][6] = {{15.0, 1013.25, 299.65, 26.31, 0.00630, 2.77},
                                     {30.0, 1017.25, 294.15, 21.79, 0.00605, 3.15},
                                     {45.0, 1015.75, 283.15, 11.66, 0.00558, 2.57},
                                     {60.0, 1011.75, 272.15, 6.78, 0.00539, 1.81},
                                     {75.0, 1013.00, 263.65, 4.11, 0.00453, 1.55}};
    static const double amp[5][6] = {{15.0, 0.00, 0.00, 0.00, 0.00, 0.00},
                                     {30.0, -3.75, 7.00, 8.85, 0.00025, 0.33},
                                     {45.0, -2.25, 11.00, 7.24, 0.00032, 0.46},
                                     {60.0, -1.75, 15.00, 5.36, 0.00081, 0.74},
                                     {75.0, -0.50, 14.50, 3.39, 0.00062, 0.30}};
    double UNB3_GM = 9.80665, UNB3_RD = 287.054, UNB3_K1 = 0.000077604, UNB3_K2 = 0.382;
    double doy2rad = 2 * M_PI / 365.25, ep = UNB3_GM / UNB3_RD;
    if (lat < 0.0) doy = doy - 211.0;
    else doy = doy - 28.0;
    double cosphs = or_ncos(doy * doy2rad);
    lat = fabs(lat);
    int p1, p2;
    double m;
    if (lat >= 75.0) { p1 = 4; p2 = 4; m = 0; }
    else if (lat <= 15.0) return GNSS_EINDEX;
    else {
        p1 = (int)floor((lat - 15) / 15) + 1;
        p2 = p1 + 1;
        m = (lat - avg[p1 - 1][0]) / (avg[p2 - 1][0] - avg[p1 - 1][0]);
    }
#define OR_LI(tb, c) (m * (tb[p2 - 1][c] - tb[p1 - 1][c]) + tb[p1 - 1][c])
    double Pavg = OR_LI(avg, 1), Tavg = OR_LI(avg, 2), WVPavg = OR_LI(avg, 3), Bavg = OR_LI(avg, 4);
    double Lavg = OR_LI(avg, 5);
    double Pamp = OR_LI(amp, 1), Tamp = OR_LI(amp, 2), WVPamp = OR_LI(amp, 3), Bamp = OR_LI(amp, 4);
    double Lamp = OR_LI(amp, 5);
#undef OR_LI
    double T0 = Tavg - Tamp * cosphs, P0 = Pavg - Pamp * cosphs, WVP0 = WVPavg - WVPamp * cosphs;
    double beta = Bavg - Bamp * cosphs, lambda = Lavg - Lamp * cosphs;
    double T = T0 - beta * alt;
    double P = P0 * pow((T / T0), ep / (beta));
    double WVP = WVP0 * pow((T / T0), (ep * ((lambda) + 1) / (beta)) - 1);
    double K_dry = P * UNB3_K1 * UNB3_RD / UNB3_GM;
    double K_wet = WVP * UNB3_K2 * UNB3_RD / ((UNB3_GM * (lambda + 1) - beta * UNB3_RD) * T0);
    /* cosd(el) */
    double nq = round(el / 90), rr = (M_PI / 180) * (el - nq * 90);
    long mq = ((long)nq % 4 + 4) % 4;
    double ce = mq == 0 ? or_ncos(rr) : mq == 1 ? -or_nsin(rr) : mq == 2 ? -or_ncos(rr) : or_nsin(rr);
    double m_dry = 1.0 / sqrt(1.0 - ce * ce / 1.002001);
    double m_wet = m_dry;
    *out = K_dry * m_dry + K_wet * m_wet;
    return GNSS_OK;
}

/* svPosVel.m:21-177; eph[21] in gnss_eph_sv order */
int or_svposvel(const double *eph, double t, double *sv_xyz, double *sv_vel, double *clkcorr_m,
                double *clkcorr_m_vel, double *grpdel)
{
    double SQRTSMA = eph[0], DELTAN = eph[1], TOE = eph[2], MZERO = eph[3], ECCEN = eph[4], ARGPERI = eph[5];
    double CUS = eph[6], CUC = eph[7], CRS = eph[8], CRC = eph[9], CIS = eph[10], CIC = eph[11];
    double IZERO = eph[12], IDOT = eph[13], OMEGAZERO = eph[14], OMEGADOT = eph[15];
    double toc = eph[16], AF0 = eph[17], AF1 = eph[18], AF2 = eph[19], TGD = eph[20];
    double tkc = t - toc;
    int iter = 0;
    while (tkc > 302400) { tkc = tkc - 604800; if (++iter > 3) return GNSS_EARG; }
    iter = 0;
    while (tkc < -302400) { tkc = tkc + 604800; if (++iter > 3) return GNSS_EARG; }
    double F = -4.442807633e-10;
    double clkcorr = (AF0 + AF1 * tkc + AF2 * tkc * tkc) - TGD;
    double gpsPi = 3.1415926535898, mu = 3986005e8, OMGedot = 7.2921151467e-5;
    double tk = (t - clkcorr) - TOE;
    iter = 0;
    while (tk > 302400) { tk = tk - 604800; if (++iter > 3) return GNSS_EARG; }
    iter = 0;
    while (tk < -302400) { tk = tk + 604800; if (++iter > 3) return GNSS_EARG; }
    double A = (SQRTSMA) * (SQRTSMA);
    double n_o = sqrt(mu / (A * A * A));
    double n = n_o + DELTAN;
    double Mk = MZERO + n * tk;
    Mk = fmod(Mk + 2 * gpsPi, 2 * gpsPi);
    double Ek = Mk, sep = 1, oldEk = Ek;
    iter = 0;
    while (sep > 1e-13) {
        Ek = Mk + ECCEN * or_nsin(Ek);
        sep = fabs(Ek - oldEk);
        oldEk = Ek;
        iter = iter + 1;
        if (iter > 10) break;
    }
    Ek = fmod(Ek + 2 * gpsPi, 2 * gpsPi);
    double cos_Ek = or_ncos(Ek), sin_Ek = or_nsin(Ek);
    double c1 = 1 - ECCEN * cos_Ek;
    double Ek_dot = n / c1;
    double c2 = sqrt(1 - ECCEN * ECCEN);
    double sin_vk = (c2 * sin_Ek) / (1 - ECCEN * cos_Ek);
    double cos_vk = (cos_Ek - ECCEN) / (1 - ECCEN * cos_Ek);
    double vk = atan2(sin_vk, cos_vk);
    double vk_dot = Ek_dot * c2 / c1;
    double PHIk = vk + ARGPERI;
    PHIk = fmod(PHIk, 2 * gpsPi);
    double c2phik = or_ncos(2 * PHIk), s2phik = or_nsin(2 * PHIk);
    double delta_uk = CUS * s2phik + CUC * c2phik;
    double delta_rk = CRS * s2phik + CRC * c2phik;
    double delta_ik = CIS * s2phik + CIC * c2phik;
    double uk = PHIk + delta_uk;
    double uk_dot = vk_dot * (1 + 2 * ((CUS * c2phik - CUC * s2phik)));
    double rk = A * (1 - ECCEN * cos_Ek) + delta_rk;
    double rk_dot = A * ECCEN * Ek_dot * sin_Ek + 2 * vk_dot * (CRS * c2phik - CRC * s2phik);
    double ik = IZERO + delta_ik + IDOT * tk;
    double ik_dot = IDOT + vk_dot * 2 * (CIS * c2phik - CIC * s2phik);
    double cos_uk = or_ncos(uk), sin_uk = or_nsin(uk);
    double xxk = rk * cos_uk, yyk = rk * sin_uk;
    double xxk_dot = rk_dot * cos_uk - uk_dot * rk * sin_uk;
    double yyk_dot = rk_dot * sin_uk + uk_dot * rk * cos_uk;
    double OMGk = OMEGAZERO + (OMEGADOT - OMGedot) * (tk) - OMGedot * TOE;
    OMEGADOT = OMEGADOT - OMGedot;
    OMGk = fmod(OMGk + 2 * gpsPi, 2 * gpsPi);
    double cosO = or_ncos(OMGk), sinO = or_nsin(OMGk), cosi = or_ncos(ik), sini = or_nsin(ik);
    sv_xyz[0] = xxk * cosO - yyk * cosi * sinO;
    sv_xyz[1] = xxk * sinO + yyk * cosi * cosO;
    sv_xyz[2] = yyk * sini;
    sv_vel[0] = xxk_dot * cosO - OMEGADOT * xxk * sinO - yyk_dot * cosi * sinO + ik_dot * yyk * sini * sinO -
                OMEGADOT * yyk * cosi * cosO;
    sv_vel[1] = xxk_dot * sinO + OMEGADOT * xxk * cosO + yyk_dot * cosi * cosO - ik_dot * yyk * sini * cosO -
                OMEGADOT * yyk * cosi * sinO;
    sv_vel[2] = yyk_dot * sini + ik_dot * yyk * cosi;
    double c3 = F * ECCEN * SQRTSMA;
    *clkcorr_m = 299792458 * (AF0 + AF1 * tkc + AF2 * tkc * tkc + c3 * sin_Ek);
    *grpdel = TGD;
    *clkcorr_m_vel = 299792458 * (AF1 + 2 * AF2 * tkc + c3 * cos_Ek * Ek_dot);
    return GNSS_OK;
}

/* C(m x n) = A(m x k) * B(k x n), row-major, k summed left to right from 0 */
static void or_mm(const double *A, const double *B, double *Cm, int m, int k, int n)
{
    for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++) {
            double s = 0;
            for (int q = 0; q < k; q++) s = s + A[i * k + q] * B[q * n + j];
            Cm[i * n + j] = s;
        }
}

/* inv(A) (N x N, row-major, overwritten): Gaussian elimination with partial pivoting (first
 * largest |pivot|), multipliers stored in place, then each column of the identity solved
 * forward and back. The reference's inv() is LAPACK's getrf + getri; this fixed order is the
 * restatement's (and the product's, vtnav.cpp inv_lu). Returns 0 if singular. */
static int or_inv(double *A, int N, double *X)
{
    int perm[2 * OR_VT_MAXCH];
    for (int i = 0; i < N; i++) perm[i] = i;
    for (int j = 0; j < N; j++) {
        int p = j;
        for (int i = j + 1; i < N; i++)
            if (fabs(A[i * N + j]) > fabs(A[p * N + j])) p = i;
        if (A[p * N + j] == 0) return 0;
        if (p != j) {
            for (int k = 0; k < N; k++) {
                double t = A[j * N + k];
                A[j * N + k] = A[p * N + k];
                A[p * N + k] = t;
            }
            int t = perm[j];
            perm[j] = perm[p];
            perm[p] = t;
        }
        for (int i = j + 1; i < N; i++) {
            A[i * N + j] = A[i * N + j] / A[j * N + j];
            for (int k = j + 1; k < N; k++) A[i * N + k] = A[i * N + k] - A[i * N + j] * A[j * N + k];
        }
    }
    double y[2 * OR_VT_MAXCH];
    for (int c = 0; c < N; c++) {
        for (int i = 0; i < N; i++) {
            y[i] = (perm[i] == c) ? 1.0 : 0.0;
            for (int k = 0; k < i; k++) y[i] = y[i] - A[i * N + k] * y[k];
        }
        for (int i = N - 1; i >= 0; i--) {
            double s = y[i];
            for (int k = i + 1; k < N; k++) s = s - A[i * N + k] * X[k * N + c];
            X[i * N + c] = s / A[i * N + i];
        }
    }
    return 1;
}

/* :39-86, :131-155 */
int or_vtnav_init(or_vtnav *v, int n, int pdi, const int *prn, const double *eph21, const double *cnslxyz,
                  const double *ALPHA, const double *BETA, double doy, double cSpeed, double Fc, double Fs,
                  double IF, double codeFreqBasis, double ms, const double *usrPos, const double *usrVel,
                  double clkBias, double clkDrift, const double *timeTransmit)
{
    if (n < 1 || n > OR_VT_MAXCH || pdi < 1) return GNSS_EARG;
    memset(v, 0, sizeof *v);
    v->n = n;
    v->pdi = pdi;
    v->msIndex = 1;
    for (int i = 0; i < n; i++) {
        v->prn[i] = prn[i];
        memcpy(v->eph[i], eph21 + 21 * i, 21 * sizeof(double));
        v->transmitTimeVT[i] = timeTransmit[i];             /* :131 */
    }
    memcpy(v->ALPHA, ALPHA, sizeof v->ALPHA);
    memcpy(v->BETA, BETA, sizeof v->BETA);
    v->doy = doy;
    v->cSpeed = cSpeed;
    v->Fc = Fc;
    v->Fs = Fs;
    v->IF = IF;
    v->codeFreqBasis = codeFreqBasis;
    v->ms = ms;
    memcpy(v->cnslxyz, cnslxyz, sizeof v->cnslxyz);            /* the argument (SDR_main.m:66) */
    for (int i = 0; i < 8; i++) v->Tm[i][i] = 1;              /* :40-47 */
    v->Tm[0][3] = v->Tm[1][4] = v->Tm[2][5] = v->Tm[6][7] = pdi * ms;
    const double sc[8] = {1e-1, 1e-1, 1e-1, 1e-1, 1e-1, 1e-1, 1e0, 1e0};
    for (int i = 0; i < 8; i++) v->state_cov[i][i] = 1e5 * sc[i]; /* :49 */
    const double pn[8] = {1e0, 1e0, 1e0, 1e-1, 1e-1, 1e-1, 1e-1, 1e-2};
    for (int i = 0; i < 8; i++) v->process_noise[i][i] = pn[i];   /* :51-54 */
    for (int i = 0; i < n; i++) {                                  /* :55-56 */
        v->mesurement_noise[i][i] = 3e-1;
        v->mesurement_noise[n + i][n + i] = 1e-1;
    }
    v->thresUptR = 200 % pdi == 0 ? 200 / pdi : -1; /* :63 (real 200/pdi: never met otherwise) */
    for (int k = 0; k < 3; k++) {
        v->estPos[k] = usrPos[k];
        v->estVel[k] = usrVel[k];
    }
    v->clkBias = clkBias;
    v->clkDrift = clkDrift;
    for (int k = 0; k < 3; k++) {                                  /* :70 */
        v->total_state[k] = usrPos[k];
        v->total_state[3 + k] = usrVel[k];
    }
    v->total_state[6] = clkBias;
    v->total_state[7] = clkDrift;
    v->corrUpt = 0.1 / (pdi * ms);                                 /* :84-86 */
    for (int i = 0; i < n; i++) v->counter_corr[i] = v->corrUpt - 1 * 1.0;
    return GNSS_OK;
}

/* :181-224 for channel i (numSample already sized, :164); *codeFreq left as passed at msIndex 1 */
int or_vtnav_predict(or_vtnav *v, int i, int64_t numSample, double *codeFreq, double *deltaPr, double *sv_vel)
{
    v->numSample[i] = (double)numSample;
    v->transmitTimeVT[i] = v->transmitTimeVT[i] + (double)numSample / v->Fs;
    v->tot_est_tck[i] = v->transmitTimeVT[i];
    double svxyz[3], vel[3], sv_clk, sv_clk_vel, grpdel;
    int st = or_svposvel(v->eph[i], v->tot_est_tck[i], svxyz, vel, &sv_clk, &sv_clk_vel, &grpdel);
    if (st) return st;
    v->counter_corr[i] = v->counter_corr[i] + 1;
    if (v->counter_corr[i] == v->corrUpt) {
        double svenu[3], temp[3];
        or_xyz2enu(svxyz, v->estPos, svenu);
        double el_rad = atan(svenu[2] / sqrt(svenu[0] * svenu[0] + svenu[1] * svenu[1]));
        double az_rad = atan2(svenu[0], svenu[1]);
        v->az[i] = az_rad * 180 / M_PI;
        v->el[i] = el_rad * 180 / M_PI;
        or_xyz2llh(v->estPos, temp);
        double user_ll[3] = {temp[0] * 180 / M_PI, temp[1] * 180 / M_PI, temp[2]};
        v->ionodel[i] = or_ionocorr(v->tot_est_tck[i], svxyz, v->cnslxyz, v->ALPHA, v->BETA);
        double tr;
        st = or_trop_unb3(v->doy, user_ll[0], user_ll[2], v->el[i], &tr);
        if (st) return st;
        v->tropodel_unb3[i] = fabs(tr);
        v->counter_corr[i] = 0;
    }
    double r = sqrt((svxyz[0] - v->estPos[0]) * (svxyz[0] - v->estPos[0]) +
                    (svxyz[1] - v->estPos[1]) * (svxyz[1] - v->estPos[1]) +
                    (svxyz[2] - v->estPos[2]) * (svxyz[2] - v->estPos[2]));
    double pr = r + v->clkBias + sv_clk - grpdel * v->cSpeed - v->tropodel_unb3[i] - v->ionodel[i];
    double svr[3];
    or_erotcorr(svxyz, pr, svr);
    r = sqrt((svr[0] - v->estPos[0]) * (svr[0] - v->estPos[0]) + (svr[1] - v->estPos[1]) * (svr[1] - v->estPos[1]) +
             (svr[2] - v->estPos[2]) * (svr[2] - v->estPos[2]));
    pr = r + v->clkBias + sv_clk - grpdel * v->cSpeed - v->tropodel_unb3[i] - v->ionodel[i];
    if (v->msIndex != 1) {
        v->deltaPr[i] = (pr - v->predictedPr_last[i]) / (v->pdi * v->ms);
        *codeFreq = v->codeFreqBasis * (1 - v->deltaPr[i] / v->cSpeed);
    }
    v->predictedPr_last[i] = pr;
    *deltaPr = v->deltaPr[i];
    memcpy(sv_vel, vel, sizeof vel);
    return GNSS_OK;
}

/* :321 and :357-467; state_out[8] = estPos, estVel, clkBias, clkDrift after the update (may be
 * NULL), es_out[8] = error_state (may be NULL) */
int or_vtnav_update(or_vtnav *v, const double *codeError, const double *codeFreq, const double *carrFreq,
                    double *state_out, double *es_out)
{
    const int n = v->n, N = 2 * n;
    double Z[2 * OR_VT_MAXCH], H[2 * OR_VT_MAXCH][8];
    memset(H, 0, sizeof H);
    for (int i = 0; i < n; i++) Z[i] = codeError[i] * v->cSpeed / codeFreq[i];        /* :321 */
    double numSample_min = v->numSample[0];
    for (int i = 1; i < n; i++)
        if (v->numSample[i] < numSample_min) numSample_min = v->numSample[i];
    numSample_min = numSample_min - 1;                                                 /* :357 */
    for (int i = 0; i < n; i++) {
        double tot_est_pos = v->tot_est_tck[i] - (v->numSample[i] - numSample_min) / v->Fs;
        v->tot_est_pos[i] = tot_est_pos;
        double svxyz_pos[3], sv_vel_pos[3], sv_clk_pos, sv_clk_vel, grpdel;
        int st = or_svposvel(v->eph[i], tot_est_pos, svxyz_pos, sv_vel_pos, &sv_clk_pos, &sv_clk_vel, &grpdel);
        if (st) return st;
        double d0 = svxyz_pos[0] - v->estPos[0], d1 = svxyz_pos[1] - v->estPos[1], d2 = svxyz_pos[2] - v->estPos[2];
        double r = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        double ppr = r + v->clkBias + sv_clk_pos - grpdel * v->cSpeed - v->tropodel_unb3[i] - v->ionodel[i];
        double svr[3];
        or_erotcorr(svxyz_pos, ppr, svr);
        d0 = svr[0] - v->estPos[0];
        d1 = svr[1] - v->estPos[1];
        d2 = svr[2] - v->estPos[2];
        r = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        double a[3] = {(svr[0] - v->estPos[0]) / r, (svr[1] - v->estPos[1]) / r, (svr[2] - v->estPos[2]) / r};
        for (int k = 0; k < 3; k++) {
            H[i][k] = -a[k];
            H[n + i][3 + k] = -a[k];
        }
        H[i][6] = 1;
        H[n + i][7] = 1;
        double prr_measured = (carrFreq[i] + v->IF) * v->cSpeed / v->Fc;
        double prr_predicted = 0;
        for (int k = 0; k < 3; k++) prr_predicted = prr_predicted + (v->estVel[k] - sv_vel_pos[k]) * a[k];
        Z[n + i] = prr_predicted - prr_measured - v->clkDrift + sv_clk_vel;
    }
    /* :387-404 */
    double es[8] = {0}, Tt[8][8], TP[8][8], TPT[8][8], Ht[8][2 * OR_VT_MAXCH];
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) Tt[r][c] = v->Tm[c][r];
    or_mm(&v->Tm[0][0], &v->state_cov[0][0], &TP[0][0], 8, 8, 8);
    or_mm(&TP[0][0], &Tt[0][0], &TPT[0][0], 8, 8, 8);
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) v->state_cov[r][c] = TPT[r][c] + v->process_noise[r][c];
    double Hc[2 * OR_VT_MAXCH * 8];
    for (int r = 0; r < N; r++)
        for (int c = 0; c < 8; c++) {
            Hc[r * 8 + c] = H[r][c];
            Ht[c][r] = H[r][c];
        }
    double Htc[8 * 2 * OR_VT_MAXCH];
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < N; c++) Htc[r * N + c] = Ht[r][c];
    double PHt[8 * 2 * OR_VT_MAXCH], HP[2 * OR_VT_MAXCH * 8], S[4 * OR_VT_MAXCH * OR_VT_MAXCH];
    double Si[4 * OR_VT_MAXCH * OR_VT_MAXCH], K[8 * 2 * OR_VT_MAXCH];
    or_mm(&v->state_cov[0][0], Htc, PHt, 8, 8, N);
    or_mm(Hc, &v->state_cov[0][0], HP, N, 8, 8);
    or_mm(HP, Htc, S, N, 8, N);
    for (int r = 0; r < N; r++)
        for (int c = 0; c < N; c++) S[r * N + c] = S[r * N + c] + v->mesurement_noise[r][c];
    if (!or_inv(S, N, Si)) return GNSS_EINDEX;
    or_mm(PHt, Si, K, 8, N, N);
    v->counterUptR = v->counterUptR + 1;
    if (v->counterUptR <= 200) /* (rows past 200 are never read: thresUptR <= 200) */
        for (int k = 0; k < N; k++) v->recordR[v->counterUptR - 1][k] = Z[k] - 0.0; /* newZ' - H*0 (:395) */
    double inno[2 * OR_VT_MAXCH];
    for (int k = 0; k < N; k++) inno[k] = Z[k];
    double Kz[8];
    or_mm(K, inno, Kz, 8, N, 1);
    for (int k = 0; k < 8; k++) es[k] = es[k] + Kz[k];
    double KH[64], IKH[64], Pn[64];
    or_mm(K, Hc, KH, 8, N, 8);
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) IKH[r * 8 + c] = (r == c ? 1.0 : 0.0) - KH[r * 8 + c];
    or_mm(IKH, &v->state_cov[0][0], Pn, 8, 8, 8);
    memcpy(&v->state_cov[0][0], Pn, sizeof Pn);
    for (int k = 0; k < 8; k++) v->total_state[k] = v->total_state[k] + es[k];
    for (int k = 0; k < 3; k++) {
        v->estPos[k] = v->total_state[k];
        v->estVel[k] = v->total_state[3 + k];
    }
    v->clkBias = v->total_state[6];
    v->clkDrift = v->total_state[7];
    if (state_out) {
        for (int k = 0; k < 3; k++) {
            state_out[k] = v->estPos[k];
            state_out[3 + k] = v->estVel[k];
        }
        state_out[6] = v->clkBias;
        state_out[7] = v->clkDrift;
    }
    if (es_out) memcpy(es_out, es, sizeof es);
    /* :440-442 */
    double xn[8];
    or_mm(&v->Tm[0][0], v->total_state, xn, 8, 8, 1);
    memcpy(v->total_state, xn, sizeof xn);
    for (int k = 0; k < 3; k++) v->estPos[k] = v->total_state[k];
    v->clkBias = v->total_state[6];
    /* :445-467 */
    if (v->counterUptR == v->thresUptR) {
        double tmpR[2 * OR_VT_MAXCH];
        for (int k = 0; k < N; k++) {
            double s = 0;
            for (int r = 0; r < v->thresUptR; r++) s = s + v->recordR[r][k] * v->recordR[r][k];
            tmpR[k] = 1.0 / v->counterUptR * s;
        }
        for (int i = 0; i < n; i++) {
            v->mesurement_noise[i][i] = tmpR[i] * 10;
            v->mesurement_noise[n + i][n + i] = tmpR[n + i] * 1;
        }
        for (int idx = 0; idx < n; idx++) {
            if (v->mesurement_noise[idx][idx] >= 12000) v->mesurement_noise[idx][idx] = 12000;
            else if (v->mesurement_noise[idx][idx] <= 0.01) v->mesurement_noise[idx][idx] = 0.01;
            if (v->mesurement_noise[idx + n][idx + n] >= 400) v->mesurement_noise[idx + n][idx + n] = 400;
            else if (v->mesurement_noise[idx + n][idx + n] <= 0.01) v->mesurement_noise[idx + n][idx + n] = 0.01;
        }
        v->counterUptR = 0;
        v->counter_r = v->counter_r + 1;
    }
    v->msIndex = v->msIndex + 1;
    return GNSS_OK;
}

size_t or_vtnav_size(void) { return sizeof(or_vtnav); }

/* The closed loop (:160-476): nsteps steps of n channels on an IF record, or_vt_step's
 * correlator (its sums in long double) with the EKF closing the loop. chan_st[n][30] (VT_STATE,
 * advanced), ca[n][1023]. rec[nsteps][n][23] = the VT_REC fields + deltaPr, prRate, sv_vel[3];
 * nav_out[nsteps][8] = estPos, estVel, clkBias, clkDrift after each update. */
int or_tracking_vt(const uint8_t *raw, int64_t nbytes, int prec, int dtype, or_vtnav *v, double *chan_st,
                   const int8_t *ca, double codelength, double tau1carr, double tau2carr, int nsteps, double *rec,
                   double *nav_out)
{
    const int n = v->n;
    for (int s = 0; s < nsteps; s++) {
        double codeError[OR_VT_MAXCH], cfk[OR_VT_MAXCH], carrFreq[OR_VT_MAXCH];
        for (int i = 0; i < n; i++) {
            double *st = chan_st + 30 * i;
            double *r = rec + ((int64_t)s * n + i) * 23;
            int64_t numSample = (int64_t)ceil((codelength * v->pdi - st[1]) / (st[3] / v->Fs)); /* :164 */
            if (numSample < 1) return GNSS_EINDEX;
            double cf = st[3], dpr, vel[3];
            int e = or_vtnav_predict(v, i, numSample, &cf, &dpr, vel);
            if (e) return e;
            e = or_vt_step(raw, nbytes, prec, dtype, st, cf, ca + 1023 * i, v->Fs, codelength, v->ms, v->pdi,
                           tau1carr, tau2carr, NULL, r);
            if (e) return e;
            r[18] = dpr;
            r[19] = 0; /* prRate: never assigned (:142) */
            memcpy(r + 20, vel, sizeof vel);
            codeError[i] = r[7];
            cfk[i] = cf;
            carrFreq[i] = r[12];
        }
        int e = or_vtnav_update(v, codeError, cfk, carrFreq, nav_out ? nav_out + 8 * s : NULL, NULL);
        if (e) return e;
    }
    return GNSS_OK;
}
