"""The oracle's trackingCT_multiCorr-GIVEN.m loop (or_tracking_ct_given): per-step relations,
the literal 25-tap replica, and the shared-delayValue codedelay quirk.

No output of this function is committed in the reference (it saves
TckResultCT_multiCorr_<file>.mat, :314), so its correlator values are "parity unpinned" like
trackingCT's; its NCO / loop-filter relations are trackingCT.m's (replayed bit-exactly
against SDR/tckRstCT_10ms_Opensky.mat in test_oracle_kat.py) with numSample by ceil (:60),
and the oracle must satisfy them to the last bit here.
"""
import ctypes as C
import math
import os

import numpy as np
import pytest

from conftest import acquired_of, params

SVS = [3, 16, 26]
CD = [3684, 26051, 57908]
FF = [4580975.0, 4579675.0, 4581800.0]
DATALEN = 80
SKIP = 2
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_given_small.npz")


def given_record(pkg, po):
    cfg = pkg.synth.opensky(skip_ms=SKIP)
    return po.synth_if(cfg, 0, (SKIP + 1 + DATALEN + 4) * 58000)


@pytest.fixture(scope="module")
def given_run(pkg, po):
    data = given_record(pkg, po)
    file, signal, acq, track = params(pkg, SKIP, data)
    A = acquired_of(SVS, CD, FF)
    buf = po.trackingCT_multiCorr(file, signal, track, A, DATALEN, raw=True)
    assert buf.status == 0
    return pkg, po, data, buf, A, (file, signal, acq, track)


def test_given_step_relations_bit_exact(given_run):
    pkg, po, data, buf, A, _ = given_run
    lib = po.load()
    f = {k: i for i, k in enumerate(pkg.abi.FIELDS)}
    t1c, t2c = po.calc_loop_coef(2, 0.707, 0.1)
    t1p, t2p = po.calc_loop_coef(15, 0.707, 0.25)
    for c in range(len(SVS)):
        r = buf.rec[c]
        assert buf.len[c] == DATALEN
        ns, rc, ph = C.c_int64(), C.c_double(), C.c_double()
        state = (0.0, 1.023e6, FF[c], 0.0)
        pos = (58000 - CD[c] - 1 + SKIP * 58000) * 2  # fseek (:57)
        cn = cl = pn = pl = 0.0
        for j in range(DATALEN):
            assert r[f["remSample"], j] == (1023.0 - state[0]) / (state[1] / 58e6)  # :58
            lib.or_nco_replay(*state, 58e6, 1023.0, 1, 1, C.byref(ns), C.byref(rc), C.byref(ph))
            assert r[f["numSample"], j] == ns.value  # ceil (:60)
            assert r[f["remChip"], j] == rc.value
            assert r[f["remPhase"], j] == ph.value
            pos += 2 * ns.value
            assert r[f["absoluteSample"], j] == pos  # continuous fread
            assert r[f["delayValue"], j] == ns.value - 58000
            for name, k in (("E", 2), ("P", 12), ("L", 22)):  # Spacing(3) = -0.5, (13), (23)
                assert r[f[name + "_i"], j] == buf.taps[c, 0, k, j]
                assert r[f[name + "_q"], j] == buf.taps[c, 1, k, j]
            E = math.sqrt(r[f["E_i"], j] * r[f["E_i"], j] + r[f["E_q"], j] * r[f["E_q"], j])
            L = math.sqrt(r[f["L_i"], j] * r[f["L_i"], j] + r[f["L_q"], j] * r[f["L_q"], j])
            e = 0.5 * (E - L) / (E + L)
            assert r[f["DLLdiscri"], j] == e
            cn = lib.or_loop_filter(cn, e, cl, t1c, t2c, 0.001)
            cl = e
            assert r[f["codeFreq"], j] == 1.023e6 - cn  # :242
            pe = r[f["PLLdiscri"], j]
            pn = lib.or_loop_filter(pn, pe, pl, t1p, t2p, 0.001)
            pl = pe
            assert r[f["carrierFreq"], j] == FF[c] + pn  # :247
            state = (rc.value, r[f["codeFreq"], j], r[f["carrierFreq"], j], ph.value)
        pw = np.mean(buf.taps[c, 0, :, :DATALEN] ** 2 + buf.taps[c, 1, :, :DATALEN] ** 2, axis=1)
        assert 10 <= np.argmax(pw) <= 14 and pw.max() > 2 * min(pw[0], pw[24])


def test_given_codedelay_shared_matrix(given_run):
    """codedelay(msIndex) = Codedelay + sum(delayValue(1:msIndex)) with delayValue one
    nsv x datalength matrix (:29) filled channel by channel: the literal MATLAB sum."""
    pkg, po, data, buf, A, _ = given_run
    f = {k: i for i, k in enumerate(pkg.abi.FIELDS)}
    nsv = len(SVS)
    D = np.zeros((nsv, DATALEN))
    for c in range(nsv):  # the channel loop of :31, the matrix as it stands during channel c
        D[c] = buf.rec[c, f["delayValue"], :DATALEN]
        lin = D.flatten(order="F")  # delayValue(1:msIndex): column-major linear indexing
        for m in range(1, DATALEN + 1):
            assert buf.rec[c, f["codedelay"], m - 1] == CD[c] + lin[:m].sum(), (c, m)


def test_given_taps_equal_literal_replica_sums(given_run):
    pkg, po, data, buf, A, _ = given_run
    f = {k: i for i, k in enumerate(pkg.abi.FIELDS)}
    c, j = 2, 11
    r = buf.rec[c]
    n = int(r[f["numSample"], j])
    start = int(r[f["absoluteSample"], j]) - 2 * n
    rc, cf = r[f["remChip"], j - 1], r[f["codeFreq"], j - 1]
    fc, ph = r[f["carrierFreq"], j - 1], r[f["remPhase"], j - 1]
    x = data[start:start + 2 * n].astype(np.float64)
    raw = x[0::2] + 1j * x[1::2]
    d = cf / 58e6
    ca = po.generate_ca(SVS[c]).astype(np.float64)
    code = np.r_[ca[-1], ca, ca[0]]  # :40
    sig = raw * np.exp(1j * (2 * np.pi * (fc * (np.arange(n) / 58e6)) + ph))
    spacing = po.colon(-0.6, 0.05, 0.6)
    for k, sp in enumerate(spacing):
        t = po.colon((0 + sp) + rc, d, ((n - 1) * d + sp) + rc)
        rep = code[(np.ceil(t) + 1).astype(np.int64) - 1]
        assert abs(np.dot(rep, sig.imag) - buf.taps[c, 0, k, j]) < 1e-8
        assert abs(np.dot(rep, sig.real) - buf.taps[c, 1, k, j]) < 1e-8


def test_given_errors_and_cn0(given_run):
    pkg, po, data, buf, A, (file, signal, acq, track) = given_run
    assert buf.c.cn0_rows == DATALEN // 20 and np.all(buf.CN0[: DATALEN // 20] > 0)
    f16 = type(file)(**vars(file))
    f16.dataPrecision = 2
    assert po.trackingCT_multiCorr(f16, signal, track, A, DATALEN, raw=True).status == pkg.abi.EARG
    short = type(file)(**vars(file))
    short.data = data[: 2 * 58000 * (SKIP + 30)]
    assert po.trackingCT_multiCorr(short, signal, track, A, DATALEN, raw=True).status == pkg.abi.EIO


def test_given_oracle_matches_golden(given_run):
    pkg, po, data, buf, A, _ = given_run
    check_given_against_golden(np.load(GOLDEN), buf.rec, buf.taps, buf.len, buf.CN0[: buf.c.cn0_rows], 0)


def check_given_against_golden(g, rec, taps, length, cn0, tol):
    """Integer fields bit-exact; sums (25 taps) within tol of the series RMS; the NCO / loop
    fields within 1e-7 relative (identical for tol 0); C/N0 within 1e-6 dB."""
    assert np.array_equal(length, g["len"])
    L = int(g["len"][0])
    grec, gtaps = g["rec"], g["taps"]
    for k in (8, 14, 15, 16, 17):  # codedelay, numSample, delayValue, absoluteSample, codedelay2
        assert np.array_equal(rec[:, k, :L], grec[:, k]), k
    for c in range(grec.shape[0]):
        scale = np.sqrt(np.mean(grec[c, 0] ** 2 + grec[c, 1] ** 2))
        assert np.max(np.abs(taps[c, :, :, :L] - gtaps[c])) <= tol * scale
        assert np.max(np.abs(rec[c, :6, :L] - grec[c, :6])) <= tol * scale
    for k in (6, 7, 9, 10, 11, 12, 13):
        if tol == 0:
            assert np.array_equal(rec[:, k, :L], grec[:, k]), k
        else:
            assert np.allclose(rec[:, k, :L], grec[:, k], rtol=1e-7, atol=1e-9), k
    assert np.allclose(cn0, g["cn0"], rtol=0, atol=0 if tol == 0 else 1e-6)
