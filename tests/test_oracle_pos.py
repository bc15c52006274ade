"""The oracle's trackingCT_POS_updated.m tracking loop (or_tracking_ct_pos) against the
relations the reference's own output satisfies.

`SDR/tckRstCT_10ms_Opensky.mat` is a trackingCT_POS_updated.m run (test_oracle_kat.py
replays it bit-exactly: numSample by ceil, remChip / remCarrPhase / file offsets from the
previous state, codeFreq = f0 + loop output, carrFreq = fineFreq + loop output, T = 1e-3,
the 1 -> 10 ms switch at 1000 + countinx(position)). Here the oracle's closed loop on a
synthetic record must satisfy the same per-step relations on its own outputs, to the last
bit, so the full loop is pinned by the same reference artefact (its correlator values need
the absent IF file: parity unpinned there, as for trackingCT).
"""
import ctypes as C
import math

import numpy as np
import pytest

from conftest import acquired_of, params

SVS = [3, 16, 26]
CD = [3684, 26051, 57908]
FF = [4580975.0, 4579675.0, 4581800.0]
N1, CX, CTPOS = 40, [3, -1, 12], 75


@pytest.fixture(scope="module")
def pos_run(pkg, po):
    skip = 2
    cfg = pkg.synth.opensky(skip_ms=skip)
    n_ms = skip + 1 + N1 + max(CX) + 10 * (CTPOS - N1 + 1) + 4
    data = po.synth_if(cfg, 0, n_ms * 58000)
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.ctPOS = N1, CTPOS
    A = acquired_of(SVS, CD, FF)
    buf = po.trackingCT_POS(file, signal, track, A, CX, raw=True)
    assert buf.status == 0
    return pkg, po, buf, A, skip, data, (file, signal, acq, track)


def test_pos_step_relations_bit_exact(pos_run):
    pkg, po, buf, A, skip, data, _ = pos_run
    lib = po.load()
    F = pkg.abi.FIELDS_POS
    f = {k: i for i, k in enumerate(F)}
    t1c, t2c = po.calc_loop_coef(2, 0.707, 0.1)
    t1p, t2p = po.calc_loop_coef(15, 0.707, 0.25)
    for c in range(len(SVS)):
        r = buf.rec[c]
        assert buf.len[c] == CTPOS and buf.countinx[c] == CX[c]
        switch = N1 + CX[c]
        ns, rc, ph = C.c_int64(), C.c_double(), C.c_double()
        state = (0.0, 1.023e6, FF[c], 0.0)
        pos = (58000 - CD[c] + 1 + skip * 58000) * 2  # :108-110
        cn = cl = pn = pl = 0.0
        dvsum = 0
        for j in range(CTPOS):
            pdi = 1 if j + 1 <= switch else 10  # msIndex <= 1000 + countinx (:183)
            lib.or_nco_replay(*state, 58e6, 1023.0, pdi, 1, C.byref(ns), C.byref(rc), C.byref(ph))
            assert r[f["numSample"], j] == ns.value
            assert r[f["remChip"], j] == rc.value
            assert r[f["remCarrPhase"], j] == ph.value
            pos += 2 * ns.value  # one continuous read, no re-seek
            assert r[f["absoluteSample"], j] == pos
            dv = ns.value - 58000 * pdi
            dvsum += dv
            assert r[f["delayValue"], j] == dv
            assert r[f["codedelay"], j] == 58000 - CD[c] + 1 + dvsum  # :290
            assert r[f["codedelay2"], j] == (pos / 2) % 58000
            assert r[f["absoluteSampleCodedelay"], j] == r[f["codedelay2"], j]
            E = math.sqrt(r[f["E_i"], j] * r[f["E_i"], j] + r[f["E_q"], j] * r[f["E_q"], j])
            L = math.sqrt(r[f["L_i"], j] * r[f["L_i"], j] + r[f["L_q"], j] * r[f["L_q"], j])
            e = 0.5 * (E - L) / (E + L)
            assert r[f["codeError"], j] == e
            cn = lib.or_loop_filter(cn, e, cl, t1c, t2c, 0.001)
            cl = e
            assert r[f["codeFreq"], j] == 1.023e6 + cn  # :262 sign
            pe = r[f["carrError"], j]
            pn = lib.or_loop_filter(pn, pe, pl, t1p, t2p, 0.001)  # T = signal.ms at pdi 10 too
            pl = pe
            assert r[f["carrFreq"], j] == FF[c] + pn
            state = (rc.value, r[f["codeFreq"], j], r[f["carrFreq"], j], ph.value)
        # code lock: the prompt power exceeds the early and late powers (+-0.5 chip)
        pw = {k: np.mean(r[f[k + "_i"]] ** 2 + r[f[k + "_q"]] ** 2) for k in "EPL"}
        assert pw["P"] > pw["E"] and pw["P"] > pw["L"]


def test_pos_prompt_replica_offset(pos_run):
    """P_i / E_i / L_i of one step equal the direct sums with the reference's replica
    indices: Early Code(ceil(t+0.5)...), Prompt Code(ceil(t_P + 0.05) + 1), Late -0.5."""
    pkg, po, buf, A, skip, data, _ = pos_run
    F = pkg.abi.FIELDS_POS
    f = {k: i for i, k in enumerate(F)}
    c, j = 1, 7  # a 1-ms step of PRN 16
    r = buf.rec[c]
    n = int(r[f["numSample"], j])
    start = int(r[f["absoluteSample"], j]) - 2 * n
    rc = r[f["remChip"], j - 1]
    cf, fc, ph = r[f["codeFreq"], j - 1], r[f["carrFreq"], j - 1], r[f["remCarrPhase"], j - 1]
    x = data[start:start + 2 * n].astype(np.float64)
    raw = x[0::2] + 1j * x[1::2]
    d = cf / 58e6
    ca = po.generate_ca(SVS[c]).astype(np.float64)
    code = np.r_[ca[-1], ca, ca[0]]
    W = 2 * np.pi * (fc * (np.arange(n) / 58e6)) + ph
    sig = raw * np.exp(1j * W)
    I, Q = sig.imag, sig.real
    for name, sp, post in (("E", 0.5, 0.0), ("P", 0.0, 0.05), ("L", -0.5, 0.0)):
        t = po.colon((0 + sp) + rc, d, ((n - 1) * d + sp) + rc)
        rep = code[(np.ceil(t + post) + 1).astype(np.int64) - 1]
        assert abs(np.dot(rep, I) - r[f[name + "_i"], j]) < 1e-6 * np.sqrt(n) * 10
        assert abs(np.dot(rep, Q) - r[f[name + "_q"], j]) < 1e-6 * np.sqrt(n) * 10


def test_pos_cn0_rows_and_int16_rejected(pos_run):
    pkg, po, buf, A, skip, data, (file, signal, acq, track) = pos_run
    assert buf.c.cn0_rows == CTPOS // 20
    assert np.all(buf.CN0[: CTPOS // 20] > 0)
    f16 = type(file)(**vars(file))
    f16.dataPrecision = 2
    b = po.trackingCT_POS(f16, signal, track, A, CX, raw=True)
    assert b.status == pkg.abi.EARG
