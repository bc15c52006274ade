"""Vector tracking, the vector half: the code-frequency prediction
(trackingVT_POS_updated.m:180-227) and the 8-state EKF (:357-467) of the product's host code
(csrc/vtnav.cpp, gnss_vt_nav_*) and of the oracle's restatement (oracle/gnss_oracle.c,
or_vtnav_*), pinned by the reference's own VT run (tckRstVT_Opensky_updated.mat, 5 PRNs x 5 000
1-ms steps, tests/golden/ref_vt_nav_Opensky.npz).

The replay: from the reference's inputs (tests/vt_nav_common.py), every step feeds the
prediction the step's recorded read size (absoluteSample differences, :164-165) and the EKF the
step's recorded codeError / codeFreq / carrFreq (:318-321, :380); the prediction's codeFreq,
deltaPr and sv_vel must reproduce the recorded ones. navSolutionsVT (the EKF state) was not
shipped with the reference, so the state is pinned only through these outputs.

Bounds, and why they are not 0: MATLAB's libm (sin / cos / atan2 / sqrt / pow of svPosVel,
erotcorr, ionocorr, trop_UNB3) and its BLAS / LAPACK matrix products and inv() round in other
places than glibc and this fixed-order restatement. sv_vel (one svPosVel call) is within a few
ulp; the predicted pseudorange carries about one ulp of a 2e7-m range (2^-28 m), and deltaPr /
codeFreq are a DIFFERENCE of two such ranges over 1 ms, so their error is counted in ulps of
the range: <= 64 at the EKF's first two updates (its large initial innovation: the CT state at
row 5 is 1 743 m of range off), <= 8 from step 3 on, bit-exact in >= 35 % of steps. Product and
oracle agree bit for bit at every step.
"""
import ctypes as C

import numpy as np
import pytest

import vt_nav_common as V

PR_ULP = 2.0 ** -28  # spacing of a pseudorange in [2^24, 2^25) m
T = 1e-3             # track.pdi * signal.ms


def _geo(lib, fn, *vals, n_out=3):
    arr = np.concatenate([np.atleast_1d(np.asarray(v, dtype=np.float64)) for v in vals])
    out = (C.c_double * n_out)()
    st = lib.gnss_geo(fn, (C.c_double * len(arr))(*arr), out)
    return st, np.array(out[:])


def test_geo_helpers_product_equals_oracle(pkg, po):
    """xyz2llh / llh2xyz / xyz2enu / erotcorr / ionocorr / trop_UNB3 (SDR_MATLAB-main/geo) of
    the product and of the oracle, bit for bit, over receiver positions around the Opensky site
    and the 5 satellites along their orbits."""
    abi = pkg.abi
    lib = abi.load()
    z = V.fixture()
    rng = np.random.default_rng(7)
    org = V.cnslxyz(pkg)
    users = [org + rng.normal(0, 3e3, 3) for _ in range(8)] + [z["navSolCT_usrPos"][k] for k in range(10)]
    sats = [po.svposvel(z["eph"][i], t)[0] for i in range(5) for t in (390114.0, 390600.5, 391000.25)]
    for u in users:
        st, g = _geo(lib, abi.GEO_XYZ2LLH, u)
        assert st == 0 and np.array_equal(g, po.geo("xyz2llh", u))
        st, back = _geo(lib, abi.GEO_LLH2XYZ, g)
        assert np.array_equal(back, po.geo("llh2xyz", g))
        # the closed form and its inverse: within 0.1 mm (xyz2llh.m's b = 6356752.3142 is WGS-84's
        # rounded semi-minor axis, llh2xyz.m derives it from 1/298.257223563)
        assert np.max(np.abs(back - u)) < 1e-4
        for s in sats:
            st, e = _geo(lib, abi.GEO_XYZ2ENU, s, u)
            assert np.array_equal(e, po.geo("xyz2enu", s, u))
            pr = float(np.linalg.norm(s - u))
            st, r = _geo(lib, abi.GEO_EROTCORR, s, [pr])
            assert np.array_equal(r, po.geo("erotcorr", s, pr))
            assert abs(np.linalg.norm(r) - np.linalg.norm(s)) < 1e-6 and r[2] == s[2]  # a z-rotation
            st, io = _geo(lib, abi.GEO_IONO, [390114.0], s, u, pkg.sdr.ALPHA, pkg.sdr.BETA, n_out=1)
            assert st == 0 and io[0] == po.geo("ionocorr", 390114.0, s, u, pkg.sdr.ALPHA, pkg.sdr.BETA)
    for lat in (15.5, 22.3, 30.0, 44.9, 60.0, 74.9, 75.0, 80.0, -22.3, -50.0):
        for el in (5.0, 30.0, 45.0, 89.9, 90.0, -3.0):
            st, tr = _geo(lib, abi.GEO_TROP, [171, lat, 4.0, el], n_out=1)
            assert st == 0 and tr[0] == po.geo("trop_UNB3", 171, lat, 4.0, el)
    # Get_UNB3_Model.m:44-47: |lat| <= 15 indexes avg(0, :) -- MATLAB raises
    assert _geo(lib, abi.GEO_TROP, [171, 10.0, 4.0, 30.0], n_out=1)[0] == abi.EINDEX
    with pytest.raises(abi.GnssError):
        po.geo("trop_UNB3", 171, -15.0, 4.0, 30.0)
    assert lib.gnss_geo(99, (C.c_double * 3)(), (C.c_double * 3)()) == abi.EARG


def test_geo_known_answers(pkg):
    """Values fixed by their definitions: the Opensky site (initParameters.m:23) round-trips
    through llh2xyz / xyz2llh; the zenith Saastamoinen delay of UNB3 at sea level is 2.3-2.6 m
    and grows as 1/sin(el); the Klobuchar delay is at least its 5-ns night floor (ionocorr.m:58)."""
    abi = pkg.abi
    lib = abi.load()
    solu = pkg.initParameters()[4]
    st, xyz = _geo(lib, abi.GEO_LLH2XYZ, solu.iniPos)
    assert 6.37e6 < np.linalg.norm(xyz) < 6.38e6
    st, llh = _geo(lib, abi.GEO_XYZ2LLH, xyz)
    assert np.max(np.abs(llh[:2] - solu.iniPos[:2])) < 1e-11 and abs(llh[2] - solu.iniPos[2]) < 1e-4
    st, zen = _geo(lib, abi.GEO_TROP, [171, 22.3, 0.0, 90.0], n_out=1)
    assert 2.3 < zen[0] < 2.6
    st, low = _geo(lib, abi.GEO_TROP, [171, 22.3, 0.0, 10.0], n_out=1)
    assert 4.5 < low[0] / zen[0] < 6.0
    z = V.fixture()
    s = np.array([1.5e7, 1.5e7, 1.5e7])
    st, io = _geo(lib, abi.GEO_IONO, [390114.0], s, xyz, pkg.sdr.ALPHA, pkg.sdr.BETA, n_out=1)
    assert io[0] >= 5e-9 * 299792458 * 0.99 and io[0] < 60


def test_svposvel_product_equals_oracle(pkg, po):
    """svPosVel.m (Kepler orbit, clock correction) of product and oracle bit for bit over the
    fixture's 5 ephemerides and a week-crossing time; the orbit radius of a GPS satellite."""
    abi = pkg.abi
    lib = abi.load()
    z = V.fixture()
    for i in range(5):
        e = abi.GnssEphSv(*z["eph"][i])
        for t in (390114.0, 390114.5 + i, 395000.0, 390114.0 + 604800.0):
            pos, vel = (C.c_double * 3)(), (C.c_double * 3)()
            c1, c2, g = C.c_double(), C.c_double(), C.c_double()
            assert lib.gnss_sv_pos_vel(C.byref(e), t, pos, vel, C.byref(c1), C.byref(c2), C.byref(g)) == 0
            op, ov, oc1, oc2, og = po.svposvel(z["eph"][i], t)
            assert np.array_equal(pos[:], op) and np.array_equal(vel[:], ov)
            assert (c1.value, c2.value, g.value) == (oc1, oc2, og)
            assert 2.55e7 < np.linalg.norm(op) < 2.72e7 and 1.5e3 < np.linalg.norm(ov) < 4.5e3  # ECEF (rotating frame)
    # "Input time should be time of week in seconds" (svPosVel.m:48-60): more than 3 weeks off
    e = abi.GnssEphSv(*z["eph"][0])
    assert lib.gnss_sv_pos_vel(C.byref(e), 390114.0 + 5 * 604800.0, None, None, None, None, None) == abi.EARG


def _replay(pkg, po, z, nsteps):
    """The replay of the module docstring through the product and the oracle side by side."""
    abi = pkg.abi
    lib = abi.load()
    nav = V.product_nav(pkg, z)
    onav = V.oracle_nav(pkg, po, z)
    n = len(z["prns"])
    last_abs = z["ct_absoluteSample"][:, -1].copy()
    cf_last = z["ct_codeFreq"][:, -1].copy()
    got = {k: np.zeros((n, nsteps)) for k in ("codeFreq", "deltaPr")}
    got["sv_vel"] = np.zeros((n, nsteps, 3))
    sols = []
    mism = []
    for k in range(nsteps):
        for i in range(n):
            ns = int(z["vt_absoluteSample"][i, k] - last_abs[i]) // 2  # int8 I/Q: 2 bytes a sample
            cf, dpr, sv = C.c_double(cf_last[i]), C.c_double(), (C.c_double * 3)()
            assert lib.gnss_vt_nav_predict(C.byref(nav), i, ns, C.byref(cf), C.byref(dpr), sv) == abi.OK
            ocf, odp, ov = onav.predict(i, ns, cf_last[i])
            if (ocf, odp, list(ov)) != (cf.value, dpr.value, sv[:]):
                mism.append(("predict", k, i))
            got["codeFreq"][i, k], got["deltaPr"][i, k], got["sv_vel"][i, k] = cf.value, dpr.value, sv[:]
            last_abs[i], cf_last[i] = z["vt_absoluteSample"][i, k], z["vt_codeFreq"][i, k]
        args = [(C.c_double * n)(*z[f][:, k]) for f in ("vt_codeError", "vt_codeFreq", "vt_carrFreq")]
        sol = abi.GnssVtNavSol()
        assert lib.gnss_vt_nav_update(C.byref(nav), *args, C.byref(sol)) == abi.OK
        x, es = onav.update(z["vt_codeError"][:, k], z["vt_codeFreq"][:, k], z["vt_carrFreq"][:, k])
        if list(x) != sol.usrPos[:] + sol.usrVel[:] + [sol.clkBias, sol.clkDrift] or list(es) != sol.state[:]:
            mism.append(("update", k))
        sols.append(sol)
    assert nav.msIndex == nsteps + 1
    return got, sols, mism


def test_vt_nav_replay_against_reference(pkg, po):
    z = V.fixture()
    nsteps = z["vt_codeFreq"].shape[1]
    assert nsteps == 5000 and list(z["prns"]) == [3, 16, 22, 26, 31]
    got, sols, mism = _replay(pkg, po, z, nsteps)
    assert mism == [], mism[:5]  # product == oracle, every step
    # msIndex 1: codeFreq is TckResultCT's at msStartTckVT (:218-219), deltaPr its initial 0 (:141)
    assert np.array_equal(got["codeFreq"][:, 0], z["ct_codeFreq"][:, -1])
    assert np.array_equal(got["codeFreq"][:, 0], z["vt_codeFreq"][:, 0])
    assert np.all(got["deltaPr"][:, 0] == 0) and np.all(z["vt_deltaPr"][:, 0] == 0)
    # the prediction (:221-222) in ulps of the predicted pseudorange
    basis, c = 1.023e6, 299792458.0
    e_dpr = np.abs(got["deltaPr"] - z["vt_deltaPr"]) * T / PR_ULP
    e_cf = np.abs(got["codeFreq"] - z["vt_codeFreq"]) / (basis * PR_ULP / T / c)
    print(f"deltaPr: max {e_dpr.max():.1f} range-ulp (steps >= 3: {e_dpr[:, 3:].max():.1f}), "
          f"bit-exact {np.mean(e_dpr == 0):.3f}; codeFreq max {e_cf.max():.1f} range-ulp")
    assert e_dpr.max() <= 64 and e_cf.max() <= 64.5
    assert e_dpr[:, 3:].max() <= 8 and e_cf[:, 3:].max() <= 8.5
    assert np.mean(e_dpr == 0) >= 0.35
    # sv_vel: svPosVel at transmitTimeVT (:181-186; the transmit time itself is exact)
    d = np.abs(got["sv_vel"] - z["vt_sv_vel"])
    ulp = d / np.spacing(np.maximum(np.abs(z["vt_sv_vel"]), 1.0))
    assert d.max() < 1e-11 and np.mean(ulp == 0) >= 0.7, (d.max(), np.mean(ulp == 0))
    # prRate: never assigned in the loop (:142, :352)
    assert np.all(z["vt_prRate"] == 0)
    # navSolutionsVT: the R updates every 200 / pdi steps (:445-467) from the innovations
    R = np.array([s.R[:10] for s in sols if s.r_row])
    assert len(R) == nsteps // 200 and [s.r_row for s in sols if s.r_row] == list(range(1, 26))
    Z = np.array([s.newZ[:10] for s in sols])
    for r in range(len(R)):
        w = Z[200 * r:200 * (r + 1)]
        # error_state is 0 before the update, so recordR = newZ (:388-395); diag(1/N * sum(.^2))
        ref = np.concatenate([np.clip((1.0 / 200 * np.sum(w[:, :5] ** 2, axis=0)) * 10, 0.01, 12000),
                              np.clip(1.0 / 200 * np.sum(w[:, 5:] ** 2, axis=0) * 1, 0.01, 400)])
        assert np.allclose(R[r], ref, rtol=1e-13, atol=0)
    # DLL measurements: codeError * c / codeFreq (:321) -- the reference's E and L share one
    # chip (quirk: tests/test_vt_kat.py) so every code measurement is 0
    assert np.all(Z[:, :5] == 0)
    # meas_inno = newZ - predicted_z (:432-434)
    s = sols[-1]
    assert np.array_equal(np.array(s.meas_inno[:10]), np.array(s.newZ[:10]) - np.array(s.predicted_z[:10]))


def test_vt_nav_argument_errors(pkg):
    """gnss_vt_nav_init / predict / update refuse what the reference cannot run: no channel or
    more than GNSS_VT_MAX_CH, a PRN outside 1..32 (svPosVel indexes eph(prn)), a channel
    index outside 0..n-1, a read size < 1; and a receiver within 15 degrees of the equator
    makes trop_UNB3's table lookup fail as MATLAB's does (EINDEX)."""
    abi = pkg.abi
    lib = abi.load()
    z = V.fixture()
    _, signal, _, _, _, _ = pkg.initParameters()
    sg = pkg.sdr.to_c_signal(signal)
    cfg = V.nav_cfg(pkg)
    eph = (abi.GnssEphSv * 40)(*[abi.GnssEphSv(*z["eph"][0])] * 40)
    nav = abi.GnssVtNav()
    args = lambda n, prn: (C.byref(cfg), C.byref(sg), 1, n, (C.c_int32 * max(n, 1))(*([prn] * max(n, 1))), eph,
                           (C.c_double * 3)(*z["navSolCT_usrPos"][4]), (C.c_double * 3)(*z["navSolCT_usrVel"][4]),
                           0.0, 0.0, (C.c_double * max(n, 1))(*([390114.0] * max(n, 1))), C.byref(nav))
    assert lib.gnss_vt_nav_init(*args(0, 3)) == abi.EARG
    assert lib.gnss_vt_nav_init(*args(33, 3)) == abi.EARG
    assert lib.gnss_vt_nav_init(*args(2, 33)) == abi.EARG
    assert lib.gnss_vt_nav_init(*args(2, 3)) == abi.OK
    cf, d, v = C.c_double(1.023e6), C.c_double(), (C.c_double * 3)()
    assert lib.gnss_vt_nav_predict(C.byref(nav), 2, 58000, C.byref(cf), C.byref(d), v) == abi.EARG
    assert lib.gnss_vt_nav_predict(C.byref(nav), 0, 0, C.byref(cf), C.byref(d), v) == abi.EARG
    # a receiver on the equator: trop_UNB3 at step 1 (counter_corr reaches corrUpt, :190)
    on_eq = (C.c_double * 3)(6378137.0, 0.0, 0.0)
    a = list(args(2, 3))
    a[6] = on_eq
    assert lib.gnss_vt_nav_init(*a) == abi.OK
    assert lib.gnss_vt_nav_predict(C.byref(nav), 0, 58000, C.byref(cf), C.byref(d), v) == abi.EINDEX
