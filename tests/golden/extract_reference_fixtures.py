"""Extract small golden fixtures from the reference's committed result files.

Run in the build container only (reads /root/reference, read-only). The outputs
are data (inputs + expected outputs), committed under tests/golden/:

  ref_acquired.json            Acquired_Opensky_5000.mat, nAcquired_*_5000.mat, countinx.mat
  ref_tckRstCT_10ms_Opensky.npz  subset of SDR_MATLAB-main/tckRstCT_10ms_Opensky.mat
                               (output of trackingCT_POS_updated.m on the real Opensky IF):
                               NCO state for steps 1..60 and 989..1100, discriminator
                               inputs, and carrError/codeError for steps 1..1100.
  ref_navdecode_Opensky_90.npz the naviDecode_updated.m case: INPUT = the signs of the
                               eight TckResult_Eph(prn).P_i series of the 90-s trackingCT
                               run embedded in SDR/task3.fig (the decode uses P_i only
                               through sign and >= 0, naviDecode_updated.m:43-74), and its
                               OUTPUT from the same run, eph_Opensky_90.mat (ephemeris
                               arrays) and sbf_Opensky_90.mat (nav1, sfb1); and the 40-s
                               run's eph/sbf_Opensky_40.mat (its P_i = the first 1000 +
                               countinx + 40000 values of the same series).
  ref_tckRstVT_Opensky.npz     subset of SDR_MATLAB-main/tckRstVT_Opensky_updated.mat (output of
                               trackingVT_POS_updated.m on the real Opensky IF, 5 PRNs x 5000
                               1-ms steps): the correlator outputs and the NCO / loop state of
                               steps 1..1200 (the vector-tracking NCO replay, tests/test_vt_kat.py).
  ref_vt_nav_Opensky.npz       (--vtnav) the vector half of trackingVT_POS_updated.m: its inputs
                               (nAcquired sv, eph_Opensky_40 / sbf_Opensky_40, navSolCT_10ms_Opensky,
                               the TckResultCT_pos state at msStartTckVT) and its outputs over all
                               5000 steps (codeFreq, deltaPr, prRate, sv_vel; tests/test_vt_nav_kat.py).

Only scipy.io.loadmat (a MAT-v5 parser that executes nothing) is used.
"""
import json
import os
import sys

import numpy as np
import scipy.io as sio

REF = "/root/reference/SDR_MATLAB-main"
HERE = os.path.dirname(os.path.abspath(__file__))


def _struct(v):
    return {fn: np.atleast_1d(getattr(v, fn)).tolist() for fn in v._fieldnames}


def main():
    out = {}
    for name, key in [("Acquired_Opensky_5000.mat", "Acquired"),
                      ("nAcquired_Opensky_5000.mat", "nAcquired"),
                      ("nAcquired_Urban_5000.mat", "nAcquired")]:
        d = sio.loadmat(os.path.join(REF, name), squeeze_me=True, struct_as_record=False)
        out[name] = _struct(d[key])
    d = sio.loadmat(os.path.join(REF, "countinx.mat"), squeeze_me=True)
    out["countinx.mat"] = np.atleast_1d(d["countinx"]).astype(int).tolist()
    with open(os.path.join(HERE, "ref_acquired.json"), "w") as f:
        json.dump(out, f, indent=1)

    d = sio.loadmat(os.path.join(REF, "tckRstCT_10ms_Opensky.mat"), squeeze_me=True,
                    struct_as_record=False)
    T = d["TckResultCT_pos"]
    prns = [i + 1 for i, t in enumerate(T) if getattr(t, "P_i", np.array([])).size > 0]
    steps = np.r_[np.arange(0, 60), np.arange(988, 1100)]  # 0-based step indices
    state_fields = ["numSample", "remChip", "remCarrPhase", "codeFreq", "carrFreq",
                    "absoluteSample", "E_i", "E_q", "P_i", "P_q", "L_i", "L_q"]
    arrs = {"prns": np.array(prns), "steps": steps}
    for fld in state_fields:
        arrs[fld] = np.stack([np.asarray(getattr(T[p - 1], fld), dtype=np.float64)[steps]
                              for p in prns])
    for fld in ["carrError", "codeError"]:
        arrs[fld] = np.stack([np.asarray(getattr(T[p - 1], fld), dtype=np.float64)[:1100]
                              for p in prns])
    np.savez_compressed(os.path.join(HERE, "ref_tckRstCT_10ms_Opensky.npz"), **arrs)
    print("prns", prns, "wrote fixtures")
    vt_fixture()


def vt_fixture(nsteps=1200):
    d = sio.loadmat(os.path.join(REF, "tckRstVT_Opensky_updated.mat"), squeeze_me=True,
                    struct_as_record=False)
    T = d["TckResultVT"]
    prns = [i + 1 for i, t in enumerate(T) if np.asarray(getattr(t, "P_i", np.array([]))).size > 0]
    fields = ["E_i", "E_q", "P_i", "P_q", "L_i", "L_q", "carrError", "codeError", "remChip",
              "remCarrPhase", "codeFreq", "carrFreq", "carrNco", "absoluteSample", "codedelay"]
    arrs = {"prns": np.array(prns)}
    for fld in fields:
        arrs[fld] = np.stack([np.asarray(getattr(T[p - 1], fld), dtype=np.float64)[:nsteps] for p in prns])
    # CN0_VT(snrIndex, svindex) (:292-305): one row per K = 20 steps, columns in Acquired.sv order
    arrs["CN0_VT"] = np.asarray(d["CN0_VT"], dtype=np.float64)[: nsteps // 20]
    np.savez_compressed(os.path.join(HERE, "ref_tckRstVT_Opensky.npz"), **arrs)
    print("VT prns", prns)


EPH_SV_FIELDS = ["sqrta", "deltan", "toe", "M0", "ecc", "w", "Cus", "Cuc", "Crs", "Crc", "Cis", "Cic", "i0",
                 "idot", "omegae", "omegadot", "toc", "af0", "af1", "af2", "TGD"]


def vt_nav_fixture():
    """ref_vt_nav_Opensky.npz: the INPUTS SDR_main.m:69-93 hands trackingVT_POS_updated.m
    (nAcquired_Opensky_5000.mat's sv; eph_Opensky_40.mat, loaded for msToProcessCT_10ms = 40000,
    at eph_idx 1; sbf_Opensky_40.mat's nav1; navSolCT_10ms_Opensky.mat; the TckResultCT_pos
    state of tckRstCT_10ms_Opensky.mat at msStartTckVT) and its OUTPUT for all 5000 steps
    (tckRstVT_Opensky_updated.mat: codeFreq, deltaPr, prRate, sv_vel, and the correlator side's
    codeError / carrFreq / remChip / absoluteSample the EKF consumes)."""
    ld = lambda f, k: sio.loadmat(os.path.join(REF, f), squeeze_me=True, struct_as_record=False)[k]
    na = ld("nAcquired_Opensky_5000.mat", "nAcquired")
    sv = [int(p) for p in np.atleast_1d(na.sv)]
    eph = ld("eph_Opensky_40.mat", "eph")
    sbf = ld("sbf_Opensky_40.mat", "sbf")
    ns = ld("navSolCT_10ms_Opensky.mat", "navSolutionsCT")
    ct = ld("tckRstCT_10ms_Opensky.mat", "TckResultCT_pos")
    vt = ld("tckRstVT_Opensky_updated.mat", "TckResultVT")
    out = {"prns": np.array(sv)}
    out["eph"] = np.array([[float(np.atleast_1d(getattr(eph[p - 1], f))[0]) for f in EPH_SV_FIELDS] for p in sv])
    out["eph_sfb1"] = np.array([float(np.atleast_1d(eph[p - 1].sfb)[0]) for p in sv])  # eph(prn).sfb(1)
    out["nav1"] = np.array([float(np.atleast_1d(sbf.nav1)[p - 1]) for p in sv])
    for f in ("usrPos", "usrVel"):
        out["navSolCT_" + f] = np.asarray(getattr(ns, f), dtype=np.float64)[:10]
    for f in ("clkBias", "clkDrift"):
        out["navSolCT_" + f] = np.asarray(getattr(ns, f), dtype=np.float64).ravel()[:10]
    out["navSolCT_timeTransmit"] = np.asarray(ns.timeTransmit, dtype=np.float64)[:2]
    # TckResultCT_pos fields around msStartTckVT (min(.., 3000) = 3000 here): the last 3 steps
    out["ct_len"] = np.array([np.asarray(ct[p - 1].codeFreq).size for p in sv])
    for f in ("codeFreq", "remChip", "carrFreq", "remCarrPhase", "absoluteSample", "codedelay", "carrError"):
        out["ct_" + f] = np.stack([np.asarray(getattr(ct[p - 1], f), dtype=np.float64)[-3:] for p in sv])
    for f in ("codeFreq", "deltaPr", "prRate", "codeError", "carrFreq", "remChip", "absoluteSample"):
        out["vt_" + f] = np.stack([np.asarray(getattr(vt[p - 1], f), dtype=np.float64).ravel() for p in sv])
    out["vt_sv_vel"] = np.stack([np.asarray(vt[p - 1].sv_vel, dtype=np.float64) for p in sv])
    np.savez_compressed(os.path.join(HERE, "ref_vt_nav_Opensky.npz"), **out)
    print("VT nav fixture", sv, out["vt_codeFreq"].shape)


def fig_series(path):
    """YData/XData float arrays of a MATLAB .fig (SURVEY App. B recipe: the figure's
    __function_workspace__ re-framed as a MAT-file and read with scipy's MAT-v5 reader)."""
    import io
    from scipy.io.matlab._mio5 import MatFile5Reader
    m = sio.loadmat(path, squeeze_me=False)
    ws = m["__function_workspace__"].tobytes()
    buf = b"MATLAB 5.0 MAT-file".ljust(116) + b"\0" * 8 + ws[:4] + ws[8:]
    r = MatFile5Reader(io.BytesIO(buf), squeeze_me=False)
    r.mat_stream.seek(128)
    r.initialize_read()
    found = []

    def walk(x):
        if isinstance(x, np.ndarray):
            if x.dtype == object:
                for e in x.ravel():
                    walk(e)
            elif x.dtype.names:
                for nm in x.dtype.names:
                    for e in x[nm].ravel():
                        walk(e)
            elif 90000 < x.size < 92000 and x.dtype.kind == "f":
                found.append(x.ravel())
    while True:
        try:
            hdr, nxt = r.read_var_header()
        except Exception:
            break
        try:
            walk(r.read_var_array(hdr, process=True))
        except Exception:
            pass
        r.mat_stream.seek(nxt)
    return found


def navdecode_fixture():
    prns = [3, 4, 16, 22, 26, 27, 31, 32]
    found = fig_series(os.path.join(REF, "task3.fig"))
    # children in reverse plot order (PRN 32 first), each as an (XData, YData) pair
    series = {}
    for i, p in enumerate(reversed(prns)):
        a, b = found[2 * i], found[2 * i + 1]
        series[p] = b if np.array_equal(a, np.arange(1, len(a) + 1)) else a
    lens = np.array([len(series[p]) for p in prns])
    signs = np.zeros((len(prns), lens.max()), dtype=np.int8)
    for i, p in enumerate(prns):
        signs[i, : lens[i]] = np.sign(series[p]).astype(np.int8)
    eph = sio.loadmat(os.path.join(REF, "eph_Opensky_90.mat"), squeeze_me=True, struct_as_record=False)["eph"]
    sbf = sio.loadmat(os.path.join(REF, "sbf_Opensky_90.mat"), squeeze_me=True, struct_as_record=False)["sbf"]
    out = {"prns": np.array(prns), "P_i_sign": signs, "len": lens,
           "nav1": np.array([np.atleast_1d(sbf.nav1)[p - 1] for p in prns]),
           "sfb1": np.array([np.atleast_1d(sbf.sfb1)[p - 1] if p <= np.atleast_1d(sbf.sfb1).size else 0
                             for p in prns])}
    fields = eph[prns[0] - 1]._fieldnames
    for p in prns:
        e = eph[p - 1]
        for fn in fields:
            out[f"eph_{p}_{fn}"] = np.atleast_1d(np.asarray(getattr(e, fn), dtype=np.float64)).ravel()
    # the 40-s run (msToProcessCT_10ms = 40000) tracked the same IF with the same code: its
    # P_i are the first 1000 + countinx + 40000 values of the 90-s series; expected outputs
    # eph_Opensky_40.mat / sbf_Opensky_40.mat
    eph40 = sio.loadmat(os.path.join(REF, "eph_Opensky_40.mat"), squeeze_me=True, struct_as_record=False)["eph"]
    sbf40 = sio.loadmat(os.path.join(REF, "sbf_Opensky_40.mat"), squeeze_me=True, struct_as_record=False)["sbf"]
    cx = np.atleast_1d(sio.loadmat(os.path.join(REF, "countinx.mat"), squeeze_me=True)["countinx"]).astype(int)
    out["len40"] = np.array([1000 + cx[i] + 40000 for i in range(len(prns))])
    out["nav1_40"] = np.array([np.atleast_1d(sbf40.nav1)[p - 1] for p in prns])
    s40 = np.atleast_1d(sbf40.sfb1)
    out["sfb1_40"] = np.array([s40[p - 1] if p <= s40.size else 0 for p in prns])
    for p in prns:
        for fn in fields:
            out[f"eph40_{p}_{fn}"] = np.atleast_1d(np.asarray(getattr(eph40[p - 1], fn), dtype=np.float64)).ravel()
    np.savez_compressed(os.path.join(HERE, "ref_navdecode_Opensky_90.npz"), **out)


if __name__ == "__main__":
    if "--navdecode" in sys.argv:
        navdecode_fixture()
        sys.exit(0)
    if "--vtnav" in sys.argv:
        vt_nav_fixture()
        sys.exit(0)
    sys.exit(main())
