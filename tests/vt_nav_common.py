"""Shared set-up of the vector half of trackingVT_POS_updated.m for the CPU
known-answer tests (test_vt_nav_kat.py) and the GPU closed-loop tests (test_gpu_vtnav.py): the
reference's own inputs of its VT run (tests/golden/ref_vt_nav_Opensky.npz, extracted from the
reference's .mat files by tests/golden/extract_reference_fixtures.py --vtnav):

  * Acquired.sv = nAcquired_Opensky_5000.mat's 5 PRNs (3 16 22 26 31);
  * eph = eph_Opensky_40.mat at eph_idx 1 (SDR_main.m:80, trackingVT_POS_updated.m:36);
  * the EKF start = navSolCT_10ms_Opensky.mat row skiptimeVT / navSolPeriod = 100 / 20 = 5
    (:66-69) and transmitTimeVT = its timeTransmit(1, :) (:131);
  * cnslxyz = llh2xyz(solu.iniPos) (SDR_main.m:66), ALPHA / BETA / doy / cSpeed / Fc of
    initParameters.m:23-32,43.
"""
import ctypes as C
import os

import numpy as np

from conftest import GOLDEN

PATH = os.path.join(GOLDEN, "ref_vt_nav_Opensky.npz")
ROW = 100 // 20  # file.skiptimeVT / solu.navSolPeriod (:66)


def fixture():
    with np.load(PATH) as f:
        return {k: f[k] for k in f.files}


def cnslxyz(pkg):
    lib = pkg.abi.load()
    solu = pkg.initParameters()[4]
    out = (C.c_double * 3)()
    assert lib.gnss_geo(pkg.abi.GEO_LLH2XYZ, (C.c_double * 3)(*solu.iniPos), out) == 0
    return np.array(out[:])


def nav_cfg(pkg):
    abi = pkg.abi
    _, signal, _, _, _, cmn = pkg.initParameters()
    cfg = abi.GnssVtNavCfg()
    cfg.cnslxyz[:] = list(cnslxyz(pkg))
    cfg.ALPHA[:] = pkg.sdr.ALPHA
    cfg.BETA[:] = pkg.sdr.BETA
    cfg.doy, cfg.cSpeed, cfg.Fc = cmn.doy, cmn.cSpeed, signal.Fc
    return cfg


def product_nav(pkg, z, prns=None, pdi=1):
    """gnss_vt_nav_init from the reference's inputs -> GnssVtNav."""
    abi = pkg.abi
    lib = abi.load()
    _, signal, _, _, _, _ = pkg.initParameters()
    sel = range(len(z["prns"])) if prns is None else [list(z["prns"]).index(p) for p in prns]
    n = len(sel)
    eph = (abi.GnssEphSv * n)()
    for q, i in enumerate(sel):
        for j, f in enumerate(abi.EPH_SV_FIELDS):
            setattr(eph[q], f, z["eph"][i, j])
    nav = abi.GnssVtNav()
    st = lib.gnss_vt_nav_init(C.byref(nav_cfg(pkg)), C.byref(pkg.sdr.to_c_signal(signal)), pdi, n,
                              (C.c_int32 * n)(*[int(z["prns"][i]) for i in sel]), eph,
                              (C.c_double * 3)(*z["navSolCT_usrPos"][ROW - 1]),
                              (C.c_double * 3)(*z["navSolCT_usrVel"][ROW - 1]), z["navSolCT_clkBias"][ROW - 1],
                              z["navSolCT_clkDrift"][ROW - 1],
                              (C.c_double * n)(*[z["navSolCT_timeTransmit"][0, i] for i in sel]), C.byref(nav))
    assert st == abi.OK, st
    return nav


def oracle_nav(pkg, po, z, prns=None, pdi=1):
    _, signal, _, _, _, cmn = pkg.initParameters()
    sel = list(range(len(z["prns"]))) if prns is None else [list(z["prns"]).index(p) for p in prns]
    return po.VtNav([int(z["prns"][i]) for i in sel], z["eph"][sel], cnslxyz(pkg), pkg.sdr.ALPHA, pkg.sdr.BETA,
                    cmn.doy, cmn.cSpeed, signal.Fc, signal, z["navSolCT_usrPos"][ROW - 1],
                    z["navSolCT_usrVel"][ROW - 1], z["navSolCT_clkBias"][ROW - 1], z["navSolCT_clkDrift"][ROW - 1],
                    z["navSolCT_timeTransmit"][0, sel], pdi=pdi)
