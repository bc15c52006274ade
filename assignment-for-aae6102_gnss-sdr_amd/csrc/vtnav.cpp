// vtnav.cpp — the vector half of trackingVT_POS_updated.m: the per-step
// code-frequency prediction of every channel from the EKF's receiver state (:180-227) and the
// 8-state EKF on the channels' code / carrier measurements (:357-467), with the SDR_MATLAB-main
// geo helpers it calls (svPosVel.m, xyz2llh.m, llh2xyz.m, xyz2enu.m, ionocorr.m, trop_UNB3.m
// with Get_UNB3_Model.m / Trop_Saastamoinen_UNB3_Components.m / Trop_Black_Eisner_Map.m,
// erotcorr.m). Host code: a step's navigation work is a few hundred scalar fp64 operations
// and one 2n x 2n inverse, latency-bound and serial across steps, so it stays on the CPU
// beside the VT correlator kernel (vt.hip); gnss_tracking_vt (gnss_api.cpp) alternates the
// two. Built with -ffp-contract=off: every operation rounds separately, in the reference's
// association order (line cites inline).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "gnss_internal.h"

namespace {

constexpr double kPi = 3.14159265358979323846;  // MATLAB pi

// ---- SDR_MATLAB-main/geo ------------------------------------------------------------------

// xyz2llh.m:25-69 (Kaplan's closed form, WGS-84)
void xyz2llh(const double* xyz, double* llh)
{
    const double x = xyz[0], y = xyz[1], z = xyz[2];
    const double x2 = x * x, y2 = y * y, z2 = z * z;
    const double a = 6378137.0000, b = 6356752.3142;
    const double e = std::sqrt(1 - (b / a) * (b / a));
    const double b2 = b * b, e2 = e * e, ep = e * (a / b);
    const double r = std::sqrt(x2 + y2), r2 = r * r;
    const double E2 = a * a - b * b;
    const double F = 54 * b2 * z2;
    const double G = r2 + (1 - e2) * z2 - e2 * E2;
    const double c = (e2 * e2 * F * r2) / (G * G * G);
    const double s = std::pow(1 + c + std::sqrt(c * c + 2 * c), 1.0 / 3.0);
    const double sp = s + 1 / s + 1;
    const double P = F / (3 * (sp * sp) * G * G);
    const double Q = std::sqrt(1 + 2 * e2 * e2 * P);
    const double ro = -(P * e2 * r) / (1 + Q) +
                      std::sqrt((a * a / 2) * (1 + 1 / Q) - (P * (1 - e2) * z2) / (Q * (1 + Q)) - P * r2 / 2);
    const double d = r - e2 * ro;
    const double tmp = d * d;
    const double U = std::sqrt(tmp + z2);
    const double V = std::sqrt(tmp + (1 - e2) * z2);
    const double zo = (b2 * z) / (a * V);
    llh[2] = U * (1 - b2 / (a * V));
    llh[0] = std::atan((z + ep * ep * zo) / r);
    const double t = std::atan(y / x);
    llh[1] = x >= 0 ? t : (y >= 0 ? kPi + t : t - kPi);
}

// llh2xyz.m:20-34
void llh2xyz(const double* llh, double* xyz)
{
    const double re = 6378137.0, eflat = 1.0 / 298.257223563;
    const double e2 = (2 - eflat) * eflat;
    const double slat = std::sin(llh[0]), clat = std::cos(llh[0]);
    const double rN = re / std::sqrt(1 - e2 * slat * slat);
    xyz[0] = (rN + llh[2]) * clat * std::cos(llh[1]);
    xyz[1] = (rN + llh[2]) * clat * std::sin(llh[1]);
    xyz[2] = (rN * (1 - e2) + llh[2]) * slat;
}

// the rotation of xyz2enu.m:37-46 (rows E, N, U) at origin latitude / longitude
void enu_rot(const double* org_llh, double R[3][3])
{
    const double sphi = std::sin(org_llh[0]), cphi = std::cos(org_llh[0]);
    const double slam = std::sin(org_llh[1]), clam = std::cos(org_llh[1]);
    R[0][0] = -slam;        R[0][1] = clam;         R[0][2] = 0;
    R[1][0] = -sphi * clam; R[1][1] = -sphi * slam; R[1][2] = cphi;
    R[2][0] = cphi * clam;  R[2][1] = cphi * slam;  R[2][2] = sphi;
}

// R * v, each row summed left to right (MATLAB's matrix-vector product, :47)
void mat3_vec(const double R[3][3], const double* v, double* out)
{
    for (int i = 0; i < 3; i++) out[i] = R[i][0] * v[0] + R[i][1] * v[1] + R[i][2] * v[2];
}

// xyz2enu.m:32-47
void xyz2enu(const double* xyz, const double* org, double* enu)
{
    const double d[3] = {xyz[0] - org[0], xyz[1] - org[1], xyz[2] - org[2]};
    double llh[3], R[3][3];
    xyz2llh(org, llh);
    enu_rot(llh, R);
    mat3_vec(R, d, enu);
}

// erotcorr.m:28-35: the satellite position rotated by the earth's rotation over the signal's
// flight time pr / c
void erotcorr(const double* sv, double pr, double* out)
{
    const double omega = 7.2921151467e-5;
    const double theta = omega * (pr / 299792458);
    const double c = std::cos(theta), s = std::sin(theta);
    const double R[3][3] = {{c, s, 0}, {-s, c, 0}, {0, 0, 1}};
    mat3_vec(R, sv, out);
}

// ionocorr.m:21-61 (the broadcast Klobuchar model). The reference takes the "user" latitude
// and longitude from the SATELLITE's llh (svllh, :23,33,38): kept.
double ionocorr(double systime, const double* svxyz, const double* usrxyz, const double* ALPHA,
                const double* BETA)
{
    double svllh[3], enu[3];
    xyz2llh(svxyz, svllh);
    xyz2enu(svxyz, usrxyz, enu);
    const double el = std::atan2(enu[2], std::sqrt(enu[0] * enu[0] + enu[1] * enu[1]));
    const double az = std::atan2(enu[0], enu[1]);
    const double E = el / kPi;
    const double e3 = 0.53 - E;
    const double F = 1 + 16 * (e3 * e3 * e3);
    const double psi = 0.00137 / (E + 0.11) - 0.022;
    double phii = svllh[0] / kPi + psi * std::cos(az);
    if (phii > 0.416) phii = 0.416;
    if (phii < -0.416) phii = -0.416;
    const double lambdai = svllh[1] / kPi + psi * std::sin(az) / std::cos(phii * kPi);
    const double phim = phii + 0.064 * std::cos((lambdai - 1.616) * kPi);
    double t = 4.32e4 * lambdai + systime;
    while (t < 0 || t >= 86400) {
        if (t >= 86400) t = t - 86400;
        if (t < 0) t = t + 86400;
    }
    const double pm2 = phim * phim, pm3 = pm2 * phim;
    double PER = BETA[0] + BETA[1] * phim + BETA[2] * pm2 + BETA[3] * pm3;
    if (PER < 72000) PER = 72000;
    const double x = 2 * kPi * (t - 50400) / PER;
    double AMP = ALPHA[0] + ALPHA[1] * phim + ALPHA[2] * pm2 + ALPHA[3] * pm3;
    if (AMP < 0) AMP = 0;
    const double x2 = x * x;
    const double Tiono = std::fabs(x) < 1.57 ? F * (5e-9 + AMP * (1 - x2 / 2 + (x2 * x2) / 24)) : F * 5e-9;
    return Tiono * 299792458;
}

// MATLAB cosd: the argument reduced by quadrants of 90 degrees first (exact), then
// cos / sin of the remainder in radians
double cosd(double x)
{
    const double n = std::round(x / 90);
    const double r = (kPi / 180) * (x - n * 90);
    const long m = ((long)n % 4 + 4) % 4;
    return m == 0 ? std::cos(r) : m == 1 ? -std::sin(r) : m == 2 ? -std::cos(r) : std::sin(r);
}

// trop_UNB3.m + Trop_Saastamoinen_UNB3_Components.m + Get_UNB3_Model.m +
// Trop_Black_Eisner_Map.m: lat in degrees (trackingVT_POS_updated.m:199-201 passes degrees).
// Returns GNSS_EINDEX where MATLAB's table lookup would fail (|lat| <= 15: avg(0, :)).
int trop_unb3(double doy, double lat, double alt, double el, double* out)
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
    const double GM = 9.80665, RD = 287.054, K1 = 0.000077604, K2 = 0.382;
    const double doy2rad = 2 * kPi / 365.25, ep = GM / RD;
    doy = lat < 0.0 ? doy - 211.0 : doy - 28.0;  // Get_UNB3_Model.m:29-33
    const double cosphs = std::cos(doy * doy2rad);
    lat = std::fabs(lat);
    int p1, p2;
    double m;
    if (lat >= 75.0) {  // :40-43: row 4 (60 deg) of the 1-based table, as written
        p1 = p2 = 4;
        m = 0;
    } else if (lat <= 15.0) {  // :44-47: index 0 -> MATLAB raises
        return GNSS_EINDEX;
    } else {
        p1 = (int)std::floor((lat - 15) / 15) + 1;
        p2 = p1 + 1;
        m = (lat - avg[p1 - 1][0]) / (avg[p2 - 1][0] - avg[p1 - 1][0]);
    }
    auto lerp = [&](const double (*tb)[6], int c) { return m * (tb[p2 - 1][c] - tb[p1 - 1][c]) + tb[p1 - 1][c]; };
    const double T0 = lerp(avg, 2) - lerp(amp, 2) * cosphs;
    const double P0 = lerp(avg, 1) - lerp(amp, 1) * cosphs;
    const double WVP0 = lerp(avg, 3) - lerp(amp, 3) * cosphs;
    const double beta = lerp(avg, 4) - lerp(amp, 4) * cosphs;
    const double lambda = lerp(avg, 5) - lerp(amp, 5) * cosphs;
    const double T = T0 - beta * alt;
    const double P = P0 * std::pow(T / T0, ep / beta);
    const double WVP = WVP0 * std::pow(T / T0, (ep * (lambda + 1) / beta) - 1);
    const double Kdry = P * K1 * RD / GM;
    const double Kwet = WVP * K2 * RD / ((GM * (lambda + 1) - beta * RD) * T0);
    const double ce = cosd(el);
    const double mdry = 1.0 / std::sqrt(1.0 - ce * ce / 1.002001);
    *out = Kdry * mdry + Kwet * mdry;
    return GNSS_OK;
}

// svPosVel.m:23-177 at transmit time t
int sv_pos_vel(const gnss_eph_sv& e, double t, double* pos, double* vel, double* clk_m, double* clk_v,
               double* grpdel)
{
    double tkc = t - e.toc;
    for (int it = 0; tkc > 302400; it++) {
        if (it > 3) return GNSS_EARG;  // "Input time should be time of week in seconds"
        tkc = tkc - 604800;
    }
    for (int it = 0; tkc < -302400; it++) {
        if (it > 3) return GNSS_EARG;
        tkc = tkc + 604800;
    }
    const double F = -4.442807633e-10;
    const double clkcorr = (e.af0 + e.af1 * tkc + e.af2 * tkc * tkc) - e.TGD;  // :64
    const double gpsPi = 3.1415926535898, mu = 3986005e8, OMGedot = 7.2921151467e-5;
    double tk = (t - clkcorr) - e.toe;
    for (int it = 0; tk > 302400; it++) {
        if (it > 3) return GNSS_EARG;
        tk = tk - 604800;
    }
    for (int it = 0; tk < -302400; it++) {
        if (it > 3) return GNSS_EARG;
        tk = tk + 604800;
    }
    const double A = e.sqrta * e.sqrta;
    const double n = std::sqrt(mu / (A * A * A)) + e.deltan;
    double Mk = e.M0 + n * tk;
    Mk = std::fmod(Mk + 2 * gpsPi, 2 * gpsPi);
    double Ek = Mk, oldEk = Ek, sep = 1;
    for (int it = 0; sep > 1e-13;) {  // :94-100, at most 11 iterations
        Ek = Mk + e.ecc * std::sin(Ek);
        sep = std::fabs(Ek - oldEk);
        oldEk = Ek;
        if (++it > 10) break;
    }
    Ek = std::fmod(Ek + 2 * gpsPi, 2 * gpsPi);
    const double cosE = std::cos(Ek), sinE = std::sin(Ek);
    const double c1 = 1 - e.ecc * cosE;
    const double Ekd = n / c1;
    const double c2 = std::sqrt(1 - e.ecc * e.ecc);
    const double sin_vk = (c2 * sinE) / (1 - e.ecc * cosE);
    const double cos_vk = (cosE - e.ecc) / (1 - e.ecc * cosE);
    const double vk = std::atan2(sin_vk, cos_vk);
    const double vkd = Ekd * c2 / c1;
    const double PHIk = std::fmod(vk + e.w, 2 * gpsPi);
    const double c2p = std::cos(2 * PHIk), s2p = std::sin(2 * PHIk);
    const double duk = e.Cus * s2p + e.Cuc * c2p;
    const double drk = e.Crs * s2p + e.Crc * c2p;
    const double dik = e.Cis * s2p + e.Cic * c2p;
    const double uk = PHIk + duk;
    const double ukd = vkd * (1 + 2 * ((e.Cus * c2p - e.Cuc * s2p)));
    const double rk = A * (1 - e.ecc * cosE) + drk;
    const double rkd = A * e.ecc * Ekd * sinE + 2 * vkd * (e.Crs * c2p - e.Crc * s2p);
    const double ik = e.i0 + dik + e.idot * tk;
    const double ikd = e.idot + vkd * 2 * (e.Cis * c2p - e.Cic * s2p);
    const double cu = std::cos(uk), su = std::sin(uk);
    const double xx = rk * cu, yy = rk * su;
    const double xxd = rkd * cu - ukd * rk * su;
    const double yyd = rkd * su + ukd * rk * cu;
    double OMGk = e.omegae + (e.omegadot - OMGedot) * tk - OMGedot * e.toe;
    const double OMD = e.omegadot - OMGedot;
    OMGk = std::fmod(OMGk + 2 * gpsPi, 2 * gpsPi);
    const double cO = std::cos(OMGk), sO = std::sin(OMGk), ci = std::cos(ik), si = std::sin(ik);
    if (pos) {
        pos[0] = xx * cO - yy * ci * sO;
        pos[1] = xx * sO + yy * ci * cO;
        pos[2] = yy * si;
    }
    if (vel) {  // :170-172
        vel[0] = xxd * cO - OMD * xx * sO - yyd * ci * sO + ikd * yy * si * sO - OMD * yy * ci * cO;
        vel[1] = xxd * sO + OMD * xx * cO + yyd * ci * cO - ikd * yy * si * cO - OMD * yy * ci * sO;
        vel[2] = yyd * si + ikd * yy * ci;
    }
    const double c3 = F * e.ecc * e.sqrta;
    if (clk_m) *clk_m = 299792458 * (e.af0 + e.af1 * tkc + e.af2 * tkc * tkc + c3 * sinE);
    if (clk_v) *clk_v = 299792458 * (e.af1 + 2 * e.af2 * tkc + c3 * cosE * Ekd);
    if (grpdel) *grpdel = e.TGD;
    return GNSS_OK;
}

double dist3(const double* a, const double* b)  // sqrt(sum((a - b).^2)), left to right
{
    const double d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2];
    return std::sqrt(d0 * d0 + d1 * d1 + d2 * d2);
}

// predictedPr = r + clkBias + sv_clk - grpdel*c - tropo - iono with the earth-rotation
// correction of the satellite position (:208-215 and :369-373, the same two passes)
double predicted_pr(const gnss_vt_nav& v, int i, const double* sv, double clkm, double grpdel, double* svr)
{
    const double* estPos = v.total_state;
    const double clkBias = v.total_state[6];
    const double cS = v.cfg.cSpeed;
    double r = dist3(sv, estPos);
    double pr = r + clkBias + clkm - grpdel * cS - v.tropodel[i] - v.ionodel[i];
    erotcorr(sv, pr, svr);
    r = dist3(svr, estPos);
    return r + clkBias + clkm - grpdel * cS - v.tropodel[i] - v.ionodel[i];
}

// inv(S) for the EKF's 2n x 2n innovation covariance: LU with partial pivoting (the first
// largest pivot), then the columns of the identity solved through L and U. The reference's
// inv() is LAPACK's; this is one fixed order, the oracle's too (or_vt_inv).
bool inv_lu(double* A, int N, double* X)
{
    int piv[2 * GNSS_VT_MAX_CH];
    for (int i = 0; i < N; i++) piv[i] = i;
    for (int j = 0; j < N; j++) {
        int p = j;
        for (int i = j + 1; i < N; i++)
            if (std::fabs(A[i * N + j]) > std::fabs(A[p * N + j])) p = i;
        if (A[p * N + j] == 0) return false;
        if (p != j) {
            for (int k = 0; k < N; k++) std::swap(A[j * N + k], A[p * N + k]);
            std::swap(piv[j], piv[p]);
        }
        for (int i = j + 1; i < N; i++) {
            const double l = A[i * N + j] / A[j * N + j];
            A[i * N + j] = l;
            for (int k = j + 1; k < N; k++) A[i * N + k] = A[i * N + k] - l * A[j * N + k];
        }
    }
    double y[2 * GNSS_VT_MAX_CH];
    for (int c = 0; c < N; c++) {
        for (int i = 0; i < N; i++) {  // L y = P e_c
            double s = piv[i] == c ? 1.0 : 0.0;
            for (int k = 0; k < i; k++) s = s - A[i * N + k] * y[k];
            y[i] = s;
        }
        for (int i = N - 1; i >= 0; i--) {  // U x = y
            double s = y[i];
            for (int k = i + 1; k < N; k++) s = s - A[i * N + k] * X[k * N + c];
            X[i * N + c] = s / A[i * N + i];
        }
    }
    return true;
}

// C = A (m x k) * B (k x n), row-major, each sum left to right
void matmul(const double* A, const double* B, double* C, int m, int k, int n)
{
    for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++) {
            double s = A[i * k] * B[j];
            for (int q = 1; q < k; q++) s = s + A[i * k + q] * B[q * n + j];
            C[i * n + j] = s;
        }
}

void transition(int pdi, double ms, double* T)  // Transistion_Matrix (:40-47)
{
    for (int i = 0; i < 64; i++) T[i] = (i % 9 == 0) ? 1.0 : 0.0;
    const double dt = pdi * ms;
    T[0 * 8 + 3] = T[1 * 8 + 4] = T[2 * 8 + 5] = T[6 * 8 + 7] = dt;
}

}  // namespace

// ---- the vector half, split around the VT kernel (gnss_internal.h) ----------------------------

double gnss::vt_transmit_next(const gnss_vt_nav& v, int i, int64_t numSample)
{
    return v.transmitTime[i] + (double)numSample / v.Fs;  // :181
}

void gnss::vt_orbit(const gnss_vt_nav& v, int i, double t, VtOrbit* o)
{
    o->t = t;
    o->st = sv_pos_vel(v.eph[i], t, o->sv, o->vel, &o->clkm, &o->clkv, &o->grp);  // :185-186
}

// :180-227 for channel i with read size numSample
int gnss::vt_nav_predict_at(gnss_vt_nav* v, int i, int64_t numSample, const VtOrbit* ahead, double* codeFreq,
                            double* deltaPr, double sv_vel[3])
{
    const double T = v->pdi * v->ms;
    v->numSample[i] = numSample;
    v->transmitTime[i] = vt_transmit_next(*v, i, numSample);  // :181
    v->tot_est_tck[i] = v->transmitTime[i];
    VtOrbit here;
    const VtOrbit* o = ahead;
    if (!o || o->t != v->tot_est_tck[i]) {  // (bitwise: the same t is the same orbit)
        vt_orbit(*v, i, v->tot_est_tck[i], &here);
        o = &here;
    }
    if (o->st) return o->st;
    const double* sv = o->sv;
    const double* estPos = v->total_state;
    v->counter_corr[i] = v->counter_corr[i] + 1;  // :189-204
    if (v->counter_corr[i] == 0.1 / T) {
        double enu[3], llh[3];
        xyz2enu(sv, estPos, enu);
        const double el_rad = std::atan(enu[2] / std::sqrt(enu[0] * enu[0] + enu[1] * enu[1]));
        const double az_rad = std::atan2(enu[0], enu[1]);
        v->az[i] = az_rad * 180 / kPi;
        v->el[i] = el_rad * 180 / kPi;
        xyz2llh(estPos, llh);
        v->ionodel[i] = ionocorr(v->tot_est_tck[i], sv, v->cnslxyz, v->cfg.ALPHA, v->cfg.BETA);
        double trop;
        const int st = trop_unb3(v->cfg.doy, llh[0] * 180 / kPi, llh[2], v->el[i], &trop);
        if (st) return st;
        v->tropodel[i] = std::fabs(trop);
        v->counter_corr[i] = 0;
    }
    double svr[3];
    const double pr = predicted_pr(*v, i, sv, o->clkm, o->grp, svr);  // :208-215
    double dpr = 0;
    if (v->msIndex > 1) {  // :218-223
        dpr = (pr - v->predictedPr_last[i]) / T;
        *codeFreq = v->codeFreqBasis * (1 - dpr / v->cfg.cSpeed);
    }
    v->predictedPr_last[i] = pr;
    if (deltaPr) *deltaPr = dpr;  // deltaPr(svindex) keeps 0 until step 2 (:141, :221)
    if (sv_vel)
        for (int k = 0; k < 3; k++) sv_vel[k] = o->vel[k];
    return GNSS_OK;
}

// :357-398 up to the measurements: every channel's geometry at the common epoch, then the
// covariance propagation, innovation covariance, its inverse and the gain (none of them read
// newZ: the error state before the update is 0)
void gnss::vt_nav_gain(const gnss_vt_nav& v, VtGain* g)
{
    const int n = v.n, N = 2 * n;
    g->st = GNSS_OK;
    double* H = g->H;
    std::memset(H, 0, sizeof(double) * N * 8);
    int64_t nmin = v.numSample[0];  // :357-383
    for (int i = 1; i < n; i++) nmin = std::min(nmin, v.numSample[i]);
    nmin = nmin - 1;
    const double* estPos = v.total_state;
    const double* estVel = v.total_state + 3;
    g->localTime = 0;
    for (int i = 0; i < n; i++) {
        const double tot = v.tot_est_tck[i] - (double)(v.numSample[i] - nmin) / v.Fs;  // :363
        g->localTime = i == 0 ? tot : std::min(g->localTime, tot);
        double sv[3], vel[3], clkm, clkv, grp, svr[3];
        const int st = sv_pos_vel(v.eph[i], tot, sv, vel, &clkm, &clkv, &grp);  // :366-367
        if (st) {
            g->st = st;
            return;
        }
        predicted_pr(v, i, sv, clkm, grp, svr);  // :369-372 (svxyzr_pos)
        const double r = dist3(svr, estPos);
        double a[3];
        for (int k = 0; k < 3; k++) a[k] = (svr[k] - estPos[k]) / r;  // :374
        for (int k = 0; k < 3; k++) {
            H[i * 8 + k] = -a[k];
            H[(n + i) * 8 + 3 + k] = -a[k];
        }
        H[i * 8 + 6] = 1;
        H[(n + i) * 8 + 7] = 1;
        for (int k = 0; k < 3; k++) {
            g->svr_last[k] = svr[k];
            g->vel_last[k] = vel[k];
            g->sv_unrot[i][k] = sv[k];
        }
        g->prr_pred[i] = (estVel[0] - vel[0]) * a[0] + (estVel[1] - vel[1]) * a[1] +
                         (estVel[2] - vel[2]) * a[2];  // :381
        g->clkv[i] = clkv;
    }
    // Kalman filter (:387-398): error_state = T * 0 = 0, so the innovation is newZ itself
    double* T = g->T;
    double Tt[64], TP[64], P[64];
    transition(v.pdi, v.ms, T);
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) Tt[r * 8 + c] = T[c * 8 + r];
    matmul(T, v.state_cov, TP, 8, 8, 8);
    matmul(TP, Tt, P, 8, 8, 8);
    const double q[8] = {1e0, 1e0, 1e0, 1e-1, 1e-1, 1e-1, 1e-1, 1e-2};  // process_noise (:51-54)
    for (int k = 0; k < 8; k++) P[k * 9] = P[k * 9] + q[k];
    double Ht[8 * 2 * GNSS_VT_MAX_CH], PHt[8 * 2 * GNSS_VT_MAX_CH], HP[2 * GNSS_VT_MAX_CH * 8];
    double S[4 * GNSS_VT_MAX_CH * GNSS_VT_MAX_CH], Si[4 * GNSS_VT_MAX_CH * GNSS_VT_MAX_CH];
    for (int r = 0; r < N; r++)
        for (int c = 0; c < 8; c++) Ht[c * N + r] = H[r * 8 + c];
    matmul(P, Ht, PHt, 8, 8, N);   // state_cov * H'
    matmul(H, P, HP, N, 8, 8);
    matmul(HP, Ht, S, N, 8, N);    // H * state_cov * H'
    for (int k = 0; k < N; k++) S[k * N + k] = S[k * N + k] + v.R[k];  // + mesurement_noise
    if (!inv_lu(S, N, Si)) {  // MATLAB: inv of a singular matrix -> Inf
        g->st = GNSS_EINDEX;
        return;
    }
    matmul(PHt, Si, g->K, 8, N, N);  // kalman_gain
    double KH[64], IKH[64];
    matmul(g->K, H, KH, 8, N, 8);
    for (int k = 0; k < 64; k++) IKH[k] = ((k % 9 == 0) ? 1.0 : 0.0) - KH[k];
    matmul(IKH, P, g->cov, 8, 8, 8);  // (:398)
}

// :321, :380-382, :397-467: the measurements into newZ, the state update, the navigation
// solution row, the next epoch's state and the measurement noise
int gnss::vt_nav_correct(gnss_vt_nav* v, const VtGain& g, const double* codeError, const double* codeFreq,
                         const double* carrFreq, gnss_vt_navsol* sol)
{
    if (g.st) return g.st;
    const int n = v->n, N = 2 * n;
    const double cS = v->cfg.cSpeed;
    const double* H = g.H;
    const double* K = g.K;
    double Z[2 * GNSS_VT_MAX_CH];
    for (int i = 0; i < n; i++) Z[i] = codeError[i] * cS / codeFreq[i];  // :321
    const double clkDrift = v->total_state[7];
    for (int i = 0; i < n; i++) {
        const double prr_meas = (carrFreq[i] + v->IF) * cS / v->cfg.Fc;  // :380
        Z[n + i] = g.prr_pred[i] - prr_meas - clkDrift + g.clkv[i];  // :382
    }
    double es[8];
    matmul(K, Z, es, 8, N, 1);     // error_state = 0 + K * (newZ' - H * 0) (:397)
    for (int k = 0; k < N; k++) v->recordR2[k] = v->recordR2[k] + Z[k] * Z[k];  // recordR (:395)
    v->counterUptR += 1;
    for (int k = 0; k < 64; k++) v->state_cov[k] = g.cov[k];  // (:398)
    for (int k = 0; k < 8; k++) v->total_state[k] = v->total_state[k] + es[k];  // (:400-404)
    if (sol) {  // navSolutionsVT row (:406-436), at the updated state
        std::memset(sol, 0, sizeof *sol);
        const double* x = v->total_state;
        double llh[3];
        xyz2llh(v->cnslxyz, llh);
        const double Lb = llh[0], lb = llh[1];
        const double Cen[3][3] = {{-std::sin(lb), std::cos(lb), 0},
                                  {-std::sin(Lb) * std::cos(lb), -std::sin(Lb) * std::sin(lb), std::cos(Lb)},
                                  {-std::cos(Lb) * std::cos(lb), -std::cos(Lb) * std::sin(lb), -std::sin(Lb)}};
        mat3_vec(Cen, x + 3, sol->usrVelENU);
        xyz2enu(x, v->cnslxyz, sol->usrPosENU);
        xyz2llh(x, sol->usrPosLLH);
        sol->usrPosLLH[0] = sol->usrPosLLH[0] * 180 / kPi;
        sol->usrPosLLH[1] = sol->usrPosLLH[1] * 180 / kPi;
        sol->localTime = g.localTime;
        for (int k = 0; k < 3; k++) {
            sol->usrPos[k] = x[k];
            sol->usrVel[k] = x[3 + k];
        }
        sol->clkBias = x[6];
        sol->clkDrift = x[7];
        for (int k = 0; k < 8; k++) {
            sol->state[k] = es[k];
            sol->state_cov[k] = v->state_cov[k * 9];
        }
        double Hes[2 * GNSS_VT_MAX_CH];
        matmul(H, es, Hes, N, 8, 1);
        for (int k = 0; k < N; k++) {
            sol->newZ[k] = Z[k];
            sol->meas_inno[k] = Z[k] - Hes[k];  // (:432: with the UPDATED error_state)
            sol->predicted_z[k] = Hes[k];       // (:434)
        }
        for (int i = 0; i < n; i++) {
            sol->satEA[i] = v->el[i];
            sol->satAZ[i] = v->az[i];
            for (int k = 0; k < 3; k++) sol->svxyz_pos[i][k] = g.sv_unrot[i][k];
        }
        for (int k = 0; k < 3; k++) {
            sol->satePos[k] = g.svr_last[k];
            sol->sateVel[k] = g.vel_last[k];
        }
        for (int r = 0; r < 8; r++)
            for (int c = 0; c < N; c++) sol->kalman_gain[r][c] = K[r * N + c];
    }
    // predict the state of the next epoch (:440-442)
    double xn[8];
    matmul(g.T, v->total_state, xn, 8, 8, 1);
    for (int k = 0; k < 8; k++) v->total_state[k] = xn[k];
    // measurement noise from the innovations of the last 200 / pdi steps (:445-467); MATLAB
    // compares the integer counter with the real thresUptR = 200/track.pdi (:63), so a pdi that
    // does not divide 200 never updates R
    if (200 % v->pdi == 0 && v->counterUptR == 200 / v->pdi) {
        const double w = 1.0 / v->counterUptR;
        for (int i = 0; i < n; i++) {
            double rc = w * v->recordR2[i] * 10, rr = w * v->recordR2[n + i] * 1;
            rc = rc >= 12000 ? 12000 : (rc <= 0.01 ? 0.01 : rc);
            rr = rr >= 400 ? 400 : (rr <= 0.01 ? 0.01 : rr);
            v->R[i] = rc;
            v->R[n + i] = rr;
        }
        for (int k = 0; k < N; k++) v->recordR2[k] = 0;
        v->counterUptR = 0;
        v->counter_r += 1;
        if (sol) {
            sol->r_row = v->counter_r;
            for (int k = 0; k < N; k++) sol->R[k] = v->R[k];
        }
    }
    v->msIndex += 1;
    return GNSS_OK;
}


extern "C" {

int gnss_sv_pos_vel(const gnss_eph_sv* eph, double t, double pos[3], double vel[3], double* clkcorr_m,
                    double* clkcorr_m_vel, double* grpdel)
{
    if (!eph) return GNSS_EARG;
    return sv_pos_vel(*eph, t, pos, vel, clkcorr_m, clkcorr_m_vel, grpdel);
}

int gnss_geo(int fn, const double* in, double* out)
{
    if (!in || !out) return GNSS_EARG;
    switch (fn) {
    case GNSS_GEO_XYZ2LLH: xyz2llh(in, out); return GNSS_OK;
    case GNSS_GEO_LLH2XYZ: llh2xyz(in, out); return GNSS_OK;
    case GNSS_GEO_XYZ2ENU: xyz2enu(in, in + 3, out); return GNSS_OK;
    case GNSS_GEO_EROTCORR: erotcorr(in, in[3], out); return GNSS_OK;
    case GNSS_GEO_IONO: out[0] = ionocorr(in[0], in + 1, in + 4, in + 7, in + 11); return GNSS_OK;
    case GNSS_GEO_TROP: return trop_unb3(in[0], in[1], in[2], in[3], out);
    default: return GNSS_EARG;
    }
}

int gnss_vt_nav_init(const gnss_vt_nav_cfg* cfg, const gnss_signal* sg, int32_t pdi, int32_t n, const int32_t* prn,
                     const gnss_eph_sv* eph, const double usrPos[3], const double usrVel[3], double clkBias,
                     double clkDrift, const double* timeTransmit, gnss_vt_nav* v)
{
    if (!cfg || !sg || !prn || !eph || !usrPos || !usrVel || !timeTransmit || !v || n < 1 || n > GNSS_VT_MAX_CH ||
        pdi < 1 || !(sg->Fs > 0) || !(sg->ms > 0) || !(cfg->cSpeed > 0) || !(cfg->Fc > 0))
        return GNSS_EARG;
    std::memset(v, 0, sizeof *v);
    v->n = n;
    v->pdi = pdi;
    v->msIndex = 1;
    v->cfg = *cfg;
    v->Fs = sg->Fs;
    v->IF = sg->IF;
    v->codeFreqBasis = sg->codeFreqBasis;
    v->ms = sg->ms;
    for (int k = 0; k < 3; k++) v->cnslxyz[k] = cfg->cnslxyz[k];  // the caller's (SDR_main.m:66)
    for (int k = 0; k < 3; k++) {      // total_state = [estPos, estVel, clkBias, clkDrift]' (:66-70)
        v->total_state[k] = usrPos[k];
        v->total_state[3 + k] = usrVel[k];
    }
    v->total_state[6] = clkBias;
    v->total_state[7] = clkDrift;
    const double d[8] = {1e-1, 1e-1, 1e-1, 1e-1, 1e-1, 1e-1, 1e0, 1e0};  // :49
    for (int k = 0; k < 8; k++) v->state_cov[k * 9] = 1e5 * d[k];
    for (int i = 0; i < n; i++) {  // :55-56
        v->R[i] = 3e-1;
        v->R[n + i] = 1e-1;
    }
    const double corrUpt = 0.1 / (pdi * sg->ms);  // corrUpdateSec / (pdi * ms) (:84-86)
    for (int i = 0; i < n; i++) {
        if (prn[i] < 1 || prn[i] > 32) return GNSS_EARG;
        v->prn[i] = prn[i];
        v->eph[i] = eph[i];
        v->transmitTime[i] = timeTransmit[i];
        v->counter_corr[i] = corrUpt - 1;
    }
    return GNSS_OK;
}

int gnss_vt_nav_predict(gnss_vt_nav* v, int32_t i, int64_t numSample, double* codeFreq, double* deltaPr,
                        double sv_vel[3])
{
    if (!v || !codeFreq || i < 0 || i >= v->n || numSample < 1) return GNSS_EARG;
    return gnss::vt_nav_predict_at(v, i, numSample, nullptr, codeFreq, deltaPr, sv_vel);
}

int gnss_vt_nav_update(gnss_vt_nav* v, const double* codeError, const double* codeFreq, const double* carrFreq,
                       gnss_vt_navsol* sol)
{
    if (!v || !codeError || !codeFreq || !carrFreq) return GNSS_EARG;
    gnss::VtGain g;
    gnss::vt_nav_gain(*v, &g);
    return gnss::vt_nav_correct(v, g, codeError, codeFreq, carrFreq, sol);
}

}  // extern "C"
