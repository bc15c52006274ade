"""Vector tracking, SURVEY §8f row 4: the tracking half of trackingVT_POS_updated.m pinned by
the reference's own output of it on the real Opensky IF (tckRstVT_Opensky_updated.mat, 5 PRNs,
the first 1200 1-ms steps: tests/golden/ref_tckRstVT_Opensky.npz, extracted by
tests/golden/extract_reference_fixtures.py).

The product library's host half of gnss_tracking_vt_step (gnss_vt_nco_step, no GPU) is
replayed from each recorded step's state with that step's recorded code frequency (the
reference's EKF prediction, an input here, :211-215) and the step's recorded prompt sums:
  * bit-exact: the read size (absoluteSample), remChip (the new code frequency's colon over
    a read sized with the old one, :161,220,284), remCarrPhase (:285), codedelay (:347), the
    DLL discriminator (:314-316) and E / P / L -- which the replica quirk makes one chip value
    times the SAME two sums for all three taps (:247-249; ceil_mx(1) linear-indexes one
    element, the 1025 clamp of :240-246 inspects only it);
  * the PLL (:305-311): carrError = atan(P_q/P_i)/(2*pi) within 2 ulp of MATLAB's atan (libm), and
    carrNco / carrFreq bit-exact wherever carrError is."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLDEN

PATH = os.path.join(GOLDEN, "ref_tckRstVT_Opensky.npz")


def _fixture():
    with np.load(PATH) as f:
        return {k: f[k] for k in f.files}  # (an NpzFile decompresses on every access)


def _signal_track(pkg):
    file, signal, acq, track, _, _ = pkg.initParameters()
    return pkg.sdr.to_c_signal(signal), pkg.sdr.to_c_track(track)[0]


def test_oracle_vt_step_replay_against_reference(po):
    """The oracle's own restatement (or_vt_step, sums given) under the same replay."""
    z = _fixture()
    exact = checked = 0
    for ip, prn in enumerate(z["prns"]):
        cb = z["carrFreq"][ip, 0] - z["carrNco"][ip, 0]
        for k in range(1, z["P_i"].shape[1]):
            st = po.vt_state(z["absoluteSample"][ip, k - 1], z["remChip"][ip, k - 1], z["remCarrPhase"][ip, k - 1],
                             z["codeFreq"][ip, k - 1], z["carrFreq"][ip, k - 1], cb, z["carrNco"][ip, k - 1],
                             z["carrError"][ip, k - 1])
            # the step's prompt chip: recover the sums from P (the chip is +-1)
            _, r0 = po.vt_step(st.copy(), z["codeFreq"][ip, k], int(prn), sums=(1.0, 1.0))
            cP = r0[2]
            status, rec = po.vt_step(st, z["codeFreq"][ip, k], int(prn),
                                     sums=(cP * z["P_i"][ip, k], cP * z["P_q"][ip, k]))
            assert status == 0
            R = dict(zip(po.VT_REC, rec))
            for f in ("E_i", "E_q", "P_i", "P_q", "L_i", "L_q", "codeError", "remChip", "remCarrPhase",
                      "absoluteSample", "codedelay"):
                assert R[f] == z[f][ip, k], (prn, k, f)
            assert abs(R["carrError"] - z["carrError"][ip, k]) <= 2 * np.spacing(abs(z["carrError"][ip, k]))
            exact += R["carrError"] == z["carrError"][ip, k]
            checked += 1
    assert exact >= 0.95 * checked


def test_vt_nco_replay_against_reference(pkg):
    abi = pkg.abi
    lib = abi.load()
    z = _fixture()
    sg, tr = _signal_track(pkg)
    checked = exact_carr = 0
    for ip, prn in enumerate(z["prns"]):
        cb = z["carrFreq"][ip, 0] - z["carrNco"][ip, 0]
        assert np.array_equal(cb + z["carrNco"][ip], z["carrFreq"][ip])  # carrFreq = basis + Nco (:310)
        for k in range(1, z["P_i"].shape[1]):
            ch = abi.GnssVtChan(prn=int(prn), pad=0, file_ptr=int(z["absoluteSample"][ip, k - 1]),
                                remChip=z["remChip"][ip, k - 1], remCarrPhase=z["remCarrPhase"][ip, k - 1],
                                codeFreq=z["codeFreq"][ip, k - 1], carrFreq=z["carrFreq"][ip, k - 1],
                                carrFreqBasis=cb, oldCarrNco=z["carrNco"][ip, k - 1],
                                oldCarrError=z["carrError"][ip, k - 1], index_int=0, snrIndex=1)
            code = (C.c_int32 * 3)()
            ns = C.c_int64()
            cf = float(z["codeFreq"][ip, k])
            assert lib.gnss_vt_prepare(C.byref(sg), 1, C.byref(ch), cf, code, C.byref(ns)) == abi.OK
            cP = code[1]
            out = abi.GnssVtOut()
            assert lib.gnss_vt_nco_step(C.byref(sg), C.byref(tr), 1, C.byref(ch), cf, cP * z["P_i"][ip, k],
                                        cP * z["P_q"][ip, k], C.byref(out)) == abi.OK
            assert out.absoluteSample == z["absoluteSample"][ip, k], (prn, k)
            assert out.absoluteSample - int(z["absoluteSample"][ip, k - 1]) == 2 * ns.value
            assert out.remChip == z["remChip"][ip, k], (prn, k)
            assert out.remCarrPhase == z["remCarrPhase"][ip, k], (prn, k)
            assert out.codedelay == z["codedelay"][ip, k], (prn, k)
            for f in ("E_i", "E_q", "P_i", "P_q", "L_i", "L_q"):
                assert getattr(out, f) == z[f][ip, k], (prn, k, f)
            assert out.codeError == z["codeError"][ip, k], (prn, k)
            ref = z["carrError"][ip, k]
            assert abs(out.carrError - ref) <= 2 * np.spacing(abs(ref)), (prn, k)
            if out.carrError == ref:
                exact_carr += 1
                assert out.carrNco == z["carrNco"][ip, k] and out.carrFreq == z["carrFreq"][ip, k], (prn, k)
            checked += 1
    assert checked == 5 * 1199
    print(f"carrError bit-exact in {exact_carr} of {checked} steps (else within 2 ulp: libm atan)")
    assert exact_carr >= 0.95 * checked


def _cn0_check(got, ref):
    """CN0_VT rows against the reference: within 3 ulp (libm log / log10 / atan2 / hypot against
    MATLAB's; the complex branch of quirk A.16 takes four of them), >= 80 % bit-exact."""
    ulp = np.abs(got - ref) / np.spacing(np.abs(ref))
    assert ulp.max() <= 3.0, ulp.max()
    assert np.mean(ulp == 0) >= 0.8, np.mean(ulp == 0)
    return float(np.mean(ulp == 0))


def test_vt_cn0_against_reference(pkg, po):
    """The C/N0 estimator of the VT loop (trackingVT_POS_updated.m:292-304; the same estimator
    as trackingCT.m:120-134) pinned by the reference's own CN0_VT: the recorded P_i / P_q of
    every step fed through the product's host half (gnss_vt_nco_step, the C/N0 state carried
    from step to step from index_int 0 / snrIndex 1, :78-81) and through the oracle; every K =
    20 steps a row (CN0_VT(snrIndex, svindex)) -- 60 rows x 5 PRNs."""
    abi = pkg.abi
    lib = abi.load()
    z = _fixture()
    sg, tr = _signal_track(pkg)
    ref = z["CN0_VT"]
    nrow = ref.shape[0]
    got = np.zeros_like(ref)
    got_o = np.zeros_like(ref)
    for ip, prn in enumerate(z["prns"]):
        cb = z["carrFreq"][ip, 0] - z["carrNco"][ip, 0]
        cn = abi.GnssVtChan(index_int=0, snrIndex=1)
        so = po.vt_state(0, 0, 0, 1.023e6, 0, 0)
        for k in range(nrow * 20):
            kk = max(k - 1, 0)
            ch = abi.GnssVtChan(prn=int(prn), pad=0, file_ptr=int(z["absoluteSample"][ip, kk]),
                                remChip=z["remChip"][ip, kk], remCarrPhase=z["remCarrPhase"][ip, kk],
                                codeFreq=z["codeFreq"][ip, kk], carrFreq=z["carrFreq"][ip, kk],
                                carrFreqBasis=cb, oldCarrNco=z["carrNco"][ip, kk],
                                oldCarrError=z["carrError"][ip, kk], index_int=cn.index_int,
                                snrIndex=cn.snrIndex)
            ch.Zk[:] = cn.Zk[:]
            code = (C.c_int32 * 3)()
            ns = C.c_int64()
            cf = float(z["codeFreq"][ip, k])
            assert lib.gnss_vt_prepare(C.byref(sg), 1, C.byref(ch), cf, code, C.byref(ns)) == abi.OK
            cP = code[1]
            out = abi.GnssVtOut()
            assert lib.gnss_vt_nco_step(C.byref(sg), C.byref(tr), 1, C.byref(ch), cf, cP * z["P_i"][ip, k],
                                        cP * z["P_q"][ip, k], C.byref(out)) == abi.OK
            cn.index_int, cn.snrIndex = ch.index_int, ch.snrIndex
            cn.Zk[:] = ch.Zk[:]
            if out.cn0_row:
                got[out.cn0_row - 1, ip] = out.CN0
            # the oracle: its own state vector, the same NCO state and sums
            so[:8] = [z["absoluteSample"][ip, kk], z["remChip"][ip, kk], z["remCarrPhase"][ip, kk],
                      z["codeFreq"][ip, kk], z["carrFreq"][ip, kk], cb, z["carrNco"][ip, kk], z["carrError"][ip, kk]]
            st, rec = po.vt_step(so, cf, int(prn), sums=(cP * z["P_i"][ip, k], cP * z["P_q"][ip, k]))
            assert st == 0
            R = dict(zip(po.VT_REC, rec))
            if R["cn0_row"]:
                got_o[int(R["cn0_row"]) - 1, ip] = R["CN0"]
        assert cn.snrIndex == nrow + 1 and cn.index_int == 0
    print("CN0_VT bit-exact: product", _cn0_check(got, ref), "oracle", _cn0_check(got_o, ref))
