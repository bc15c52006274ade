"""The oracle's trackingCT_POS_updated_multicorrelator.m tracking loop (or_tracking_ct_mc)
against the reference's per-step relations and a literal numpy restatement of its replica.

No artefact of the reference holds this function's output (SDR_main.m:110-112 loads a
tckRstCT_10ms_mltCorr_*.mat that is not committed), so its correlator values are "parity
unpinned" like trackingCT's. Its loop shares every NCO / loop-filter / bookkeeping
relation with trackingCT_POS_updated.m, whose committed output
(SDR/tckRstCT_10ms_Opensky.mat) test_oracle_kat.py replays bit-exactly; here the mc loop
must satisfy the same relations to the last bit, with T = pdi*t in the loop filters
(:352,361), and its 25 taps must equal direct sums with the reference's literal replica
Code = [CA(end) repmat(CA,1,pdi) CA(1) CA(2)] indexed by ceil(t) + 2 (:94,233-258).
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
MS = {1: 60, 10: 300}  # track.msPosCT per pdi
SKIP = 2
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden_mc_small.npz")


def mc_record(pkg, po):
    cfg = pkg.synth.opensky(skip_ms=SKIP)
    return po.synth_if(cfg, 0, (SKIP + 1 + max(MS.values()) + 12) * 58000)


@pytest.fixture(scope="module")
def mc_runs(pkg, po):
    data = mc_record(pkg, po)
    out = {}
    for pdi, ms in MS.items():
        file, signal, acq, track = params(pkg, SKIP, data)
        track.msPosCT, track.pdi = ms, pdi
        A = acquired_of(SVS, CD, FF)
        buf = po.trackingCT_mc(file, signal, track, A, raw=True)
        assert buf.status == 0
        out[pdi] = (buf, A, (file, signal, acq, track))
    return pkg, po, data, out


@pytest.mark.parametrize("pdi", [1, 10])
def test_mc_step_relations_bit_exact(mc_runs, pdi):
    pkg, po, data, runs = mc_runs
    buf, A, _ = runs[pdi]
    lib = po.load()
    F = pkg.abi.FIELDS_POS
    f = {k: i for i, k in enumerate(F)}
    t1c, t2c = po.calc_loop_coef(2, 0.707, 0.1)
    t1p, t2p = po.calc_loop_coef(15, 0.707, 0.25)
    steps = MS[pdi] // pdi
    T = pdi * 0.001  # (pdi*t), :352,361
    for c in range(len(SVS)):
        r = buf.rec[c]
        assert buf.len[c] == steps
        ns, rc, ph = C.c_int64(), C.c_double(), C.c_double()
        state = (0.0, 1.023e6, FF[c], 0.0)
        pos = (58000 - CD[c] + 1 + SKIP * 58000) * 2  # :101-103
        cn = cl = pn = pl = 0.0
        dvsum = 0
        for j in range(steps):
            lib.or_nco_replay(*state, 58e6, 1023.0, pdi, 1, C.byref(ns), C.byref(rc), C.byref(ph))
            assert r[f["numSample"], j] == ns.value  # ceil (:177)
            assert r[f["remChip"], j] == rc.value  # t_CodePrompt(numSample) + step - L*pdi (:262)
            assert r[f["remCarrPhase"], j] == ph.value
            pos += 2 * ns.value
            assert r[f["absoluteSample"], j] == pos
            dv = ns.value - 58000 * pdi
            dvsum += dv
            assert r[f["delayValue"], j] == dv
            assert r[f["codedelay"], j] == 58000 - CD[c] + 1 + dvsum  # :437
            assert r[f["codedelay2"], j] == (pos / 2) % 58000
            # E / P / L are taps Spacing(3), (13), (23)
            for name, k in (("E", 2), ("P", 12), ("L", 22)):
                assert r[f[name + "_i"], j] == buf.taps[c, 0, k, j]
                assert r[f[name + "_q"], j] == buf.taps[c, 1, k, j]
            E = math.sqrt(r[f["E_i"], j] * r[f["E_i"], j] + r[f["E_q"], j] * r[f["E_q"], j])
            L = math.sqrt(r[f["L_i"], j] * r[f["L_i"], j] + r[f["L_q"], j] * r[f["L_q"], j])
            e = 0.5 * (E - L) / (E + L)
            assert r[f["codeError"], j] == e
            cn = lib.or_loop_filter(cn, e, cl, t1c, t2c, T)
            cl = e
            assert r[f["codeFreq"], j] == 1.023e6 + cn  # :356
            pe = r[f["carrError"], j]
            pn = lib.or_loop_filter(pn, pe, pl, t1p, t2p, T)
            pl = pe
            assert r[f["carrFreq"], j] == FF[c] + pn  # :364
            state = (rc.value, r[f["codeFreq"], j], r[f["carrFreq"], j], ph.value)
        # the correlation triangle lies inside the 25 taps. Code(ceil(t) + 2) from the same
        # file_ptr as trackingCT_POS_updated.m (Code(ceil(t) + 1)) reads the replica one chip
        # ahead, so the peak starts near Spacing = -0.5 (60 x 1 ms: tap 22) and the DLL pulls
        # it back to the prompt (30 x 10 ms: tap 11-12); a quirk of the reference, reproduced
        pw = np.mean(buf.taps[c, 0, :, :steps] ** 2 + buf.taps[c, 1, :, :steps] ** 2, axis=1)
        assert pw.max() > 2 * min(pw[0], pw[24]) and 10 <= np.argmax(pw) <= 24


@pytest.mark.parametrize("pdi,j", [(1, 9), (10, 5)])
def test_mc_taps_equal_literal_replica_sums(mc_runs, pdi, j):
    """All 25 taps of one step against the reference's literal construction:
    Code = [CA(end) repmat(CA,1,pdi) CA(1) CA(2)], Code(ceil(t_Spacing(k)) + 2)."""
    pkg, po, data, runs = mc_runs
    buf, A, _ = runs[pdi]
    F = pkg.abi.FIELDS_POS
    f = {k: i for i, k in enumerate(F)}
    c = 1
    r = buf.rec[c]
    n = int(r[f["numSample"], j])
    start = int(r[f["absoluteSample"], j]) - 2 * n
    rc = r[f["remChip"], j - 1]
    cf, fc, ph = r[f["codeFreq"], j - 1], r[f["carrFreq"], j - 1], r[f["remCarrPhase"], j - 1]
    x = data[start:start + 2 * n].astype(np.float64)
    raw = x[0::2] + 1j * x[1::2]
    d = cf / 58e6
    ca = po.generate_ca(SVS[c]).astype(np.float64)
    code = np.r_[ca[-1], np.tile(ca, pdi), ca[0], ca[1]]
    W = 2 * np.pi * (fc * (np.arange(n) / 58e6)) + ph
    sig = raw * np.exp(1j * W)
    I, Q = sig.imag, sig.real
    spacing = po.colon(0.6, -0.05, -0.6)
    assert len(spacing) == 25 and spacing[2] == 0.5 and spacing[12] == 0 and spacing[22] == -0.5
    for k, sp in enumerate(spacing):
        t = po.colon((0 + sp) + rc, d, (n - 1) * d + sp + rc)
        assert len(t) == n
        rep = code[(np.ceil(t) + 2).astype(np.int64) - 1]
        assert abs(np.dot(rep, I) - buf.taps[c, 0, k, j]) < 1e-9 * np.sqrt(n) * 10
        assert abs(np.dot(rep, Q) - buf.taps[c, 1, k, j]) < 1e-9 * np.sqrt(n) * 10


def test_mc_cn0_and_errors(mc_runs):
    pkg, po, data, runs = mc_runs
    buf, A, (file, signal, acq, track) = runs[10]
    assert buf.c.cn0_rows == (MS[10] // 10) // 20
    assert np.all(buf.CN0[: buf.c.cn0_rows] > 0)
    t2 = type(track)(**vars(track))
    t2.pdi = 5
    assert po.trackingCT_mc(file, signal, t2, A, raw=True).status == pkg.abi.EARG
    f16 = type(file)(**vars(file))
    f16.dataPrecision = 2
    assert po.trackingCT_mc(f16, signal, track, A, raw=True).status == pkg.abi.EARG


def test_mc_oracle_matches_golden(mc_runs):
    pkg, po, data, runs = mc_runs
    g = np.load(GOLDEN)
    for pdi in (1, 10):
        buf, A, _ = runs[pdi]
        check_mc_against_golden(g, pdi, buf.rec, buf.taps, buf.len, buf.CN0[: buf.c.cn0_rows], tol=0)


INT_K = (8, 13, 14, 15, 16, 17)  # codedelay, absoluteSampleCodedelay, numSample, delayValue,
#                                  absoluteSample, codedelay2 (FIELDS_POS slots)
SUM_K = range(6)


def check_mc_against_golden(g, pdi, rec, taps, length, cn0, tol):
    """Integer fields bit-exact; correlator sums within tol of the series RMS (0: identical);
    NCO / loop fields within 1e-7 relative (identical for tol 0); C/N0 within 1e-6 dB."""
    L = int(g[f"len{pdi}"][0])
    assert np.array_equal(length, g[f"len{pdi}"])
    grec, gtaps = g[f"rec{pdi}"], g[f"taps{pdi}"]
    for k in INT_K:
        assert np.array_equal(rec[:, k, :L], grec[:, k, :L]), k
    for c in range(grec.shape[0]):
        scale = np.sqrt(np.mean(grec[c, 0] ** 2 + grec[c, 1] ** 2))
        assert np.max(np.abs(taps[c, :, :, :L] - gtaps[c])) <= tol * scale, c
        for k in SUM_K:
            assert np.max(np.abs(rec[c, k, :L] - grec[c, k])) <= tol * scale, (c, k)
    for k in range(6, 18):
        if k in INT_K:
            continue
        if tol == 0:
            assert np.array_equal(rec[:, k, :L], grec[:, k]), k
        else:
            assert np.allclose(rec[:, k, :L], grec[:, k], rtol=1e-7, atol=1e-9), k
    assert np.allclose(cn0, g[f"cn0{pdi}"], rtol=0, atol=0 if tol == 0 else 1e-6)
