// navdecode.cpp — naviDecode_updated.m: bit synchronisation, preamble
// search, parity and subframe 1-3 decoding on the tracking loop's prompt series P_i.
//
// Host C++ by design: per channel it is one sign scan over ~90 000 values and a few
// thousand 30-bit words, serial by construction (every channel's bit arrays carry over
// into the next, see below) — microseconds of host work, less than one kernel launch.
//
// Reproduced as the reference runs it (naviDecode_updated.m, paritychk_James.m,
// bin2dec_GPSSDR.m, comp2dec.m), quirks included:
//   * NaviData / NaviDataXOR are never cleared between channels (:95-110): a channel's
//     bits overwrite the previous channel's from index 1, unassigned bits (|tempx| <= 17
//     at a 20-ms boundary, tempx then carried on) keep older values, the length is the
//     longest so far;
//   * the parity routine transforms the whole bit array and its result replaces it even
//     when the check fails (:142); its word loop ends at the absolute index equal to the
//     word-aligned LENGTH from idx_sf1 (paritychk_James.m:22,32); `if (p ~= bits)` fails
//     the check only when all six parity bits differ (MATLAB `if` on a vector);
//   * after the first pass, every later preamble match (i and i + 300) re-decodes every
//     subframe from there on and appends (the ephemeris arrays hold repeats).
#include <cmath>
#include <cstring>
#include <vector>

#include "gnss_internal.h"

namespace gnss {
namespace {

constexpr double kPi = 3.14159265358979323846;  // MATLAB pi

struct EphArrays {
    std::vector<double> f[GNSS_EPH_NFIELDS];
    int updateflag = 0;
};

inline int sgn(double x) { return (x > 0) - (x < 0); }

// bin2dec_GPSSDR(b): polyval(fliplr(b), 2): b(end) is the most significant bit.
double bin2dec(const std::vector<int>& b)
{
    double v = 0;
    for (size_t i = b.size(); i-- > 0;) v = v * 2 + b[i];
    return v;
}

// comp2dec(bi, LSB) (comp2dec.m): two's complement with bi(end) the sign bit.
double comp2dec(const std::vector<int>& bi, int lsb)
{
    std::vector<int> m(bi.begin(), bi.end() - 1);
    if (bi.back() == 0) return bin2dec(m) * std::ldexp(1.0, lsb);
    for (int& x : m) x = x == 1 ? 0 : 1;
    return -1 * (1 + bin2dec(m)) * std::ldexp(1.0, lsb);
}

// subframe(hi:-1:lo) of a 1-based subframe row
std::vector<int> rng(const int* sf, int hi, int lo)
{
    std::vector<int> r;
    for (int k = hi; k >= lo; k--) r.push_back(sf[k]);
    return r;
}
std::vector<int> cat(std::vector<int> a, const std::vector<int>& b)
{
    a.insert(a.end(), b.begin(), b.end());
    return a;
}

// paritychk_James.m on the 1-based 0/1 array x (x[0] unused); returns pass.
int parity_check(std::vector<double>& x, int64_t idx_sf1)
{
    static const int H[6][24] = {
        {1, 1, 1, 0, 1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0, 0, 1, 0},
        {0, 1, 1, 1, 0, 1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0, 0, 1},
        {1, 0, 1, 1, 1, 0, 1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0, 0},
        {0, 1, 0, 1, 1, 1, 0, 1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0},
        {1, 0, 1, 0, 1, 1, 1, 0, 1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0, 1, 1, 0, 1},
        {0, 0, 1, 0, 1, 1, 0, 1, 1, 1, 1, 0, 1, 0, 1, 0, 0, 0, 1, 0, 0, 1, 1, 1}};
    const int64_t n = (int64_t)x.size() - 1;
    int pass = 1;
    for (int64_t i = 1; i <= n; i++) x[i] = x[i] == 1 ? -1 : (x[i] == 0 ? 1 : x[i]);  // (:19-20)
    const int64_t datalength = (n - idx_sf1 + 1) / 30 * 30;                             // (:22)
    for (int64_t idx = idx_sf1; idx <= datalength; idx += 30) {
        if (idx < 3 || idx + 29 > n) return -1;  // MATLAB: index out of bounds
        const double D30 = x[idx - 1], D29 = x[idx - 2];
        for (int k = 0; k < 24; k++) x[idx + k] = D30 * x[idx + k];
        const double Df[6] = {D29, D30, D29, D30, D30, D29};
        int all_differ = 1;
        for (int r = 0; r < 6; r++) {
            double p = Df[r];
            for (int k = 0; k < 24; k++)
                if (H[r][k]) p *= x[idx + k];  // prod over the nonzero H .* d
            if (p == x[idx + 24 + r]) all_differ = 0;
        }
        if (all_differ) pass = 0;
    }
    for (int64_t i = 1; i <= n; i++) x[i] = (-x[i] + 1) / 2;  // (:48-49)
    return pass;
}

void append(EphArrays& e, int f, double v) { e.f[f].push_back(v); }

}  // namespace
}  // namespace gnss

using namespace gnss;

int gnss_navi_decode(const gnss_acquired* acq, const double* P_i, const int64_t* len, int64_t stride,
                     gnss_nav_out* out)
{
    if (!acq || !P_i || !len || !out || acq->n <= 0 || acq->n > GNSS_MAX_SV || out->eph_cap <= 0)
        return GNSS_EARG;
    const int nsv = acq->n;
    const int startOffset = 3000;  // (:34)
    const int preamble[8] = {-1, 1, 1, 1, -1, 1, -1, -1};
    std::vector<EphArrays> eph((size_t)nsv);
    // persist across channels (never cleared in the reference)
    std::vector<double> NaviData(1, 0.0), NaviDataXOR(1, 0.0);  // 1-based
    std::vector<double> NaviDatams(1, 0.0);                      // (cleared before reuse)
    int status = GNSS_OK;
    for (int c = 0; c < nsv && status == GNSS_OK; c++) {
        const double* P = P_i + (int64_t)c * stride;
        const int64_t L = len[c];
        if (L <= startOffset + 2) { status = GNSS_EINDEX; break; }
        EphArrays& e = eph[(size_t)c];
        int case1_index = 0, flag_sfb1 = 0;
        (void)case1_index;
        int flag_sf[5] = {0, 0, 0, 0, 0};
        // RawNavigationData = P_i(1+startOffset:end) with outlier flips (:43-50)
        std::vector<double> R(P + startOffset, P + L);
        const int64_t nR = (int64_t)R.size();
        for (int64_t i = 1; i < nR - 1; i++)
            if (sgn(R[i - 1]) == sgn(R[i + 1]) && sgn(R[i]) != sgn(R[i - 1])) R[i] = -R[i];
        // NaviDatams over the previous channel's array (its tail beyond nR persists)
        if ((int64_t)NaviDatams.size() < nR + 1) NaviDatams.resize((size_t)nR + 1, 0.0);
        for (int64_t i = 0; i < nR; i++) NaviDatams[(size_t)i + 1] = R[i] >= 0 ? 1 : -1;
        const int64_t msl = (int64_t)NaviDatams.size() - 1;
        for (int64_t i = 2; i <= msl - 1; i++)
            if (sgn(NaviDatams[i - 1]) == sgn(NaviDatams[i + 1]) && sgn(NaviDatams[i]) != sgn(NaviDatams[i - 1]))
                NaviDatams[i] = -NaviDatams[i];
        int64_t startms = 2;
        for (; startms <= msl; startms++)
            if (NaviDatams[startms] != NaviDatams[startms - 1]) break;
        if (startms > msl) startms = msl;  // (a MATLAB for-loop variable keeps its last value)
        // second pass from the first transition (:67-77), no outlier flips
        const int64_t startOffset_2 = startms + startOffset;
        if (startOffset_2 - 1 > L) { status = GNSS_EINDEX; break; }
        NaviDatams.assign(1, 0.0);
        for (int64_t k = startOffset_2; k <= L; k++) NaviDatams.push_back(P[k - 1] >= 0 ? 1 : -1);  // P_i(startOffset_2:end)
        const int64_t msdatalength = (int64_t)NaviDatams.size() - 1;
        const int64_t nav1 = 1 + startOffset_2 - 1;  // startms = 1 (:78-80)
        if (out->nav1) out->nav1[c] = nav1;
        if (out->sfb1) out->sfb1[c] = 0;
        // bit synchronisation (:85-118)
        int64_t idx = 0, idx2 = 0;
        double tempx = 0;
        for (int64_t index = 1; index <= msdatalength; index++) {
            idx++;
            if (msdatalength - index > 100) {
                tempx += NaviDatams[index];
                if (idx % 20 == 0) {
                    idx2++;
                    auto put = [&](double xr, double d) {
                        if ((int64_t)NaviDataXOR.size() < idx2 + 1) {
                            NaviDataXOR.resize((size_t)idx2 + 1, 0.0);
                            NaviData.resize((size_t)idx2 + 1, 0.0);
                        }
                        NaviDataXOR[idx2] = xr;
                        NaviData[idx2] = d;
                    };
                    if (tempx > 17) { put(0, 1); tempx = 0; }
                    if (tempx < -17) { put(1, -1); tempx = 0; }
                }
            } else {
                break;
            }
        }
        // preamble, parity, subframes (:121-246)
        const int64_t ndl = (int64_t)NaviDataXOR.size() - 1;
        int flag = 0;
        std::vector<int> sf(301);
        for (int64_t index = 8; index <= ndl; index++) {
            if (!(ndl - index + 1 > 360)) continue;
            double s0 = 0, s1 = 0;
            for (int k = 0; k < 8; k++) {
                s0 += NaviData[index - 7 + k] * preamble[k];
                s1 += NaviData[index - 7 + 300 + k] * preamble[k];
            }
            if (!(std::fabs(s0) > 7.99 && std::fabs(s1) > 7.99)) continue;
            const double end_HOW = NaviData[index - 7 + 59] + NaviData[index - 7 + 58];
            const double end_HOW2 = NaviData[index - 7 + 359] + NaviData[index - 7 + 358];
            if (end_HOW == 0 || end_HOW2 == 0) continue;
            if (flag == 0) {
                const int pass = parity_check(NaviDataXOR, index - 7);
                if (pass < 0) { status = GNSS_EINDEX; break; }
                if (pass == 1) flag = 1;
            }
            if (flag != 1) continue;
            const int64_t num_sf = (ndl - (index - 7) + 1) / 300;
            for (int64_t j = 1; j <= num_sf; j++) {
                const int64_t b0 = index - 7 + 300 * (j - 1);
                for (int k = 1; k <= 300; k++) sf[k] = (int)NaviDataXOR[b0 + k - 1];
                const int* s = sf.data();
                append(e, GNSS_E_sfb, (double)b0);
                const double TOW = (bin2dec(rng(s, 47, 31)) - 1) * 6;
                append(e, GNSS_E_TOW, TOW);
                const int sid = (int)bin2dec(rng(s, 52, 50));
                switch (sid) {
                case 1:
                    case1_index++;
                    if (flag_sfb1 == 0) {
                        if (out->sfb1) out->sfb1[c] = b0;
                        flag_sfb1 = 1;
                    }
                    append(e, GNSS_E_sfb1, (double)b0);
                    append(e, GNSS_E_weeknum, bin2dec(rng(s, 70, 61)) + 1024 + 1024);
                    append(e, GNSS_E_TOW1, (bin2dec(rng(s, 47, 31)) - 1) * 6);
                    append(e, GNSS_E_N, bin2dec(rng(s, 76, 73)));
                    append(e, GNSS_E_health, bin2dec(rng(s, 82, 78)));
                    append(e, GNSS_E_IODC, bin2dec(rng(s, 218, 211)));
                    append(e, GNSS_E_TGD, comp2dec(rng(s, 204, 197), -31));
                    append(e, GNSS_E_toc, bin2dec(rng(s, 234, 219)) * 16);
                    append(e, GNSS_E_af2, comp2dec(rng(s, 248, 241), -55));
                    append(e, GNSS_E_af1, comp2dec(rng(s, 264, 249), -43));
                    append(e, GNSS_E_af0, comp2dec(rng(s, 292, 271), -31));
                    flag_sf[0] = 1;
                    break;
                case 2:
                    append(e, GNSS_E_IODE2, bin2dec(rng(s, 68, 61)));
                    append(e, GNSS_E_Crs, comp2dec(rng(s, 84, 69), -5));
                    append(e, GNSS_E_deltan, comp2dec(rng(s, 106, 91), -43) * kPi);
                    append(e, GNSS_E_M0, comp2dec(cat(rng(s, 144, 121), rng(s, 114, 107)), -31) * kPi);
                    append(e, GNSS_E_Cuc, comp2dec(rng(s, 166, 151), -29));
                    append(e, GNSS_E_ecc, bin2dec(cat(rng(s, 204, 181), rng(s, 174, 167))) * std::ldexp(1.0, -33));
                    append(e, GNSS_E_Cus, comp2dec(rng(s, 226, 211), -29));
                    append(e, GNSS_E_sqrta, bin2dec(cat(rng(s, 264, 241), rng(s, 234, 227))) * std::ldexp(1.0, -19));
                    append(e, GNSS_E_toe, bin2dec(rng(s, 286, 271)) * 16);
                    flag_sf[1] = 1;
                    break;
                case 3:
                    append(e, GNSS_E_Cic, comp2dec(rng(s, 76, 61), -29));
                    append(e, GNSS_E_omegae, comp2dec(cat(rng(s, 114, 91), rng(s, 84, 77)), -31) * kPi);
                    append(e, GNSS_E_Cis, comp2dec(rng(s, 136, 121), -29));
                    append(e, GNSS_E_i0, comp2dec(cat(rng(s, 174, 151), rng(s, 144, 137)), -31) * kPi);
                    append(e, GNSS_E_Crc, comp2dec(rng(s, 196, 181), -5));
                    append(e, GNSS_E_w, comp2dec(cat(rng(s, 234, 211), rng(s, 204, 197)), -31) * kPi);
                    append(e, GNSS_E_omegadot, comp2dec(rng(s, 264, 241), -43) * kPi);
                    append(e, GNSS_E_IODE3, bin2dec(rng(s, 278, 271)));
                    append(e, GNSS_E_idot, comp2dec(rng(s, 292, 279), -43) * kPi);
                    flag_sf[2] = 1;
                    break;
                case 4: flag_sf[3] = 1; break;
                case 5: flag_sf[4] = 1; break;
                default: break;
                }
                const std::vector<double>& h = e.f[GNSS_E_health];
                if (flag_sf[0] && flag_sf[1] && flag_sf[2] && flag_sf[3] && flag_sf[4] && !h.empty() &&
                    h.back() == 0) {
                    e.updateflag = 1;
                    append(e, GNSS_E_updatetime, (double)((index + j * 300) * 20 + (1 - 1)));
                    append(e, GNSS_E_updatetime_tow, e.f[GNSS_E_TOW].back() + 6);
                    for (int& v : flag_sf) v = 0;
                }
            }
        }
    }
    // outputs
    for (int c = 0; c < nsv; c++) {
        const EphArrays& e = eph[(size_t)c];
        if (out->updateflag) out->updateflag[c] = e.updateflag;
        for (int f = 0; f < GNSS_EPH_NFIELDS; f++) {
            const size_t n = e.f[f].size();
            if ((int64_t)n > out->eph_cap && status == GNSS_OK) status = GNSS_EARG;
            const size_t m = std::min<size_t>(n, (size_t)out->eph_cap);
            if (out->eph_len) out->eph_len[(int64_t)c * GNSS_EPH_NFIELDS + f] = (int32_t)m;
            if (out->eph)
                for (size_t k = 0; k < m; k++)
                    out->eph[((int64_t)c * GNSS_EPH_NFIELDS + f) * out->eph_cap + (int64_t)k] = e.f[f][k];
        }
    }
    return status;
}
