"""Pin the CPU oracle to known answers before trusting it as the parity checker.

* IS-GPS-200 first-10-chip octal table (generateCAcode.m:16-64)
* calcLoopCoef.m:41-45 values for the initParameters.m:58-66 loop settings
* bit-exact replay of the reference's own tracking output
  (SDR_MATLAB-main/tckRstCT_10ms_Opensky.mat, written by trackingCT_POS_updated.m
  on the real Opensky IF): NCO numSample/remChip/remCarrPhase/file offset and the
  DLL/PLL loop-filter recursion (same arithmetic as trackingCT.m:79-150)
* structure of the committed Acquired / countinx results
* MATLAB colon / fft / bit-edge semantics
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

# IS-GPS-200, Table 3-Ia: first 10 C/A chips in octal (bit 1 = chip value +1 in
# generateCAcode.m's -(g1.*g2) convention)
ICD_FIRST10 = {1: 0o1440, 2: 0o1620, 3: 0o1710, 4: 0o1744, 5: 0o1133, 6: 0o1455, 7: 0o1131,
               8: 0o1454, 9: 0o1626, 10: 0o1504, 11: 0o1642, 12: 0o1750, 13: 0o1764, 14: 0o1772,
               15: 0o1775, 16: 0o1776, 17: 0o1156, 18: 0o1467, 19: 0o1633, 20: 0o1715, 21: 0o1746,
               22: 0o1763, 23: 0o1063, 24: 0o1706, 25: 0o1743, 26: 0o1761, 27: 0o1770, 28: 0o1774,
               29: 0o1127, 30: 0o1453, 31: 0o1625, 32: 0o1712}


@pytest.mark.parametrize("prn", range(1, 33))
def test_ca_code_icd_first_chips(po, prn):
    ca = po.generate_ca(prn)
    assert set(np.unique(ca)) == {-1, 1}
    v = 0
    for c in ca[:10]:
        v = (v << 1) | (1 if c == 1 else 0)
    assert v == ICD_FIRST10[prn]
    # balanced Gold code: 512 of one sign, 511 of the other
    assert abs(int(ca.sum())) == 1


def test_ca_code_sbas_prns_exist(po):
    for prn in range(33, 52):
        assert len(po.generate_ca(prn)) == 1023


def test_calc_loop_coef(po):
    # SURVEY §8 a3 (DLL 2/0.707/0.1, PLL 15/0.707/0.25)
    assert po.calc_loop_coef(2, 0.707, 0.1) == (0.00703054225877465, 0.3749245)
    assert po.calc_loop_coef(15, 0.707, 0.25) == (0.00031246854483442903, 0.04998993333333334)


@pytest.fixture(scope="module")
def ref_trk():
    return np.load(os.path.join(GOLDEN, "ref_tckRstCT_10ms_Opensky.npz"))


@pytest.fixture(scope="module")
def ref_acq():
    with open(os.path.join(GOLDEN, "ref_acquired.json")) as f:
        return json.load(f)


def test_nco_replay_bit_exact(po, ref_trk, ref_acq):
    """numSample = ceil((1023*pdi - remChip)/(codeFreq/Fs)); remChip / remCarrPhase /
    file offset of the next step, replayed from the recorded previous state."""
    import ctypes as C
    lib = po.load()
    z = ref_trk
    nacq = ref_acq["nAcquired_Opensky_5000.mat"]
    cx = ref_acq["countinx.mat"]
    steps = z["steps"]
    checked = 0
    for ip, prn in enumerate(z["prns"]):
        switch = 1000 + cx[ip]  # countinx indexed by the nAcquired position (quirk A.17)
        ns, rc, ph = C.c_int64(), C.c_double(), C.c_double()
        lib.or_nco_replay(0.0, 1.023e6, float(nacq["fineFreq"][ip]), 0.0, 58e6, 1023.0, 1, 1,
                          C.byref(ns), C.byref(rc), C.byref(ph))
        assert (ns.value, rc.value, ph.value) == (z["numSample"][ip, 0], z["remChip"][ip, 0],
                                                  z["remCarrPhase"][ip, 0])
        for j in range(1, len(steps)):
            if steps[j - 1] != steps[j] - 1:
                continue
            pdi = 1 if steps[j] + 1 <= switch else 10
            lib.or_nco_replay(z["remChip"][ip, j - 1], z["codeFreq"][ip, j - 1],
                              z["carrFreq"][ip, j - 1], z["remCarrPhase"][ip, j - 1], 58e6, 1023.0,
                              pdi, 1, C.byref(ns), C.byref(rc), C.byref(ph))
            assert ns.value == z["numSample"][ip, j]
            assert rc.value == z["remChip"][ip, j]
            assert ph.value == z["remCarrPhase"][ip, j]
            assert z["absoluteSample"][ip, j - 1] + 2 * ns.value == z["absoluteSample"][ip, j]
            checked += 1
    assert checked > 800


def test_loop_filter_replay_bit_exact(po, ref_trk, ref_acq):
    """carrFreq/codeFreq recursions (trackingCT.m:140,147 arithmetic) from the recorded
    discriminator series reproduce the recorded NCO frequencies bit for bit."""
    lib = po.load()
    z = ref_trk
    nacq = ref_acq["nAcquired_Opensky_5000.mat"]
    t1c, t2c = po.calc_loop_coef(2, 0.707, 0.1)
    t1p, t2p = po.calc_loop_coef(15, 0.707, 0.25)
    for ip in range(len(z["prns"])):
        cn = cl = pn = pl = 0.0
        carr, code = [], []
        for k in range(1100):
            e = z["codeError"][ip, k]
            cn = lib.or_loop_filter(cn, e, cl, t1c, t2c, 0.001)
            cl = e
            pe = z["carrError"][ip, k]
            pn = lib.or_loop_filter(pn, pe, pl, t1p, t2p, 0.001)
            pl = pe
            code.append(1.023e6 + cn)  # sibling's sign convention (trackingCT_POS_updated.m:262)
            carr.append(nacq["fineFreq"][ip] + pn)
        s = z["steps"]
        assert np.array_equal(np.array(carr)[s], z["carrFreq"][ip])
        assert np.array_equal(np.array(code)[s], z["codeFreq"][ip])


def test_dll_discriminator_from_recorded_correlators(ref_trk):
    z = ref_trk
    E = np.sqrt(z["E_i"] ** 2 + z["E_q"] ** 2)
    L = np.sqrt(z["L_i"] ** 2 + z["L_q"] ** 2)
    d = 0.5 * (E - L) / (E + L)
    assert np.array_equal(d, z["codeError"][:, z["steps"]])


def test_reference_acquired_structure(ref_acq):
    a = ref_acq["Acquired_Opensky_5000.mat"]
    assert a["sv"] == [3, 4, 16, 22, 26, 27, 31, 32]
    # Doppler on the 500 Hz grid; fineFreq - IF on the Fs/fftlength = 5 Hz grid
    # (fftlength = L*S*datalen = 10*58000*20, acquisition.m:108,119)
    assert all(dop % 500 == 0 for dop in a["Doppler"])
    assert all(round(f - 4.58e6) % 5 == 0 for f in a["fineFreq"])
    assert all(0 <= cd < 58000 for cd in a["codedelay"])
    assert min(a["SNR"]) >= 12
    cx = ref_acq["countinx.mat"]
    assert len(cx) == 8 and all(-1 <= c <= 18 for c in cx)


def test_colon_semantics(po):
    v = po.colon(-0.6, 0.05, 0.6)
    assert len(v) == 25 and v[0] == -0.6 and v[-1] == 0.6 and v[12] == 0.0
    w = po.colon(-0.5, 0.1, 0.5)
    assert len(w) == 11 and (w[0], w[5], w[10]) == (-0.5, 0.0, 0.5)
    # integer ranges are exact; empty ranges are empty
    assert np.array_equal(po.colon(0, 1, 5), np.arange(6))
    assert len(po.colon(1, 1, 0)) == 0
    # first half built as a + k*d, second half as b - (n-k)*d
    a, d = 0.3, 0.0176379
    b = 57999 * d + a
    x = po.colon(a, d, b)
    assert len(x) == 58000
    assert x[100] == a + 100 * d
    assert x[-101] == b - 100 * d


@pytest.mark.parametrize("n", [1, 2, 29, 1000, 26000, 58000, 2 ** 7 * 5 ** 2 * 29])
def test_fft_matches_numpy(po, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    ref = np.fft.fft(x)
    got = po.fft(x)
    assert np.max(np.abs(got - ref)) <= 1e-13 * max(1.0, np.max(np.abs(ref)))
    back = po.fft(got, inverse=True)
    assert np.max(np.abs(back - x)) < 1e-12


def _pattern(n, edge):
    """P_i series whose sign flips at every 1-based i = edge (mod 20) (20-ms bits)."""
    i = np.arange(1, n + 1)
    sign = np.where(((i - edge) // 20) % 2 == 0, 1.0, -1.0)
    return sign * (100 + (i % 7))


def test_bit_edge_search(po):
    # transitions at i = 613, 633, ...: first i >= 600 with the 6-before / 17-after pattern
    P = _pattern(1000, 613)
    cx, st = po.bit_edge(P)
    assert st == 0 and cx == (613 % 20) - 1 == 12
    # mod(i,20) - 1 can be -1 (i = 620)
    cx, st = po.bit_edge(_pattern(1000, 620))
    assert st == 0 and cx == -1
    # no transition at all -> countinx stays 0
    cx, st = po.bit_edge(np.ones(1000))
    assert (cx, st) == (0, 0)


def test_bit_edge_index_error(po):
    """A first qualifying edge at i >= 984 makes MATLAB index P_i(i+17) past the end."""
    P = np.ones(1000)
    P[990:] = -1.0  # single transition at i = 991 (1-based)
    cx, st = po.bit_edge(P)
    assert st == 5  # GNSS_EINDEX
