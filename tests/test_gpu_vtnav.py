"""GPU closed loop of vector tracking (trackingVT_POS_updated.m:157-476 through
sdr.trackingVT_POS_updated -> gnss_tracking_vt): the EKF-predicted code frequencies drive the VT
correlator kernel step by step and the correlator outputs drive the EKF, against the oracle's
closed loop (or_tracking_vt: or_vt_step's correlator, long-double sums, and the or_vtnav EKF,
itself pinned by the reference's recorded run in tests/test_vt_nav_kat.py).

Inputs: the reference's own VT inputs (tests/vt_nav_common.py: 5 PRNs, eph_Opensky_40,
navSolCT_10ms_Opensky row 5, TckResultCT at msStartTckVT) on the synthetic Opensky record (the
reference ships no IF), the channels' file pointers placed on the synthetic scene's code phases.

Tolerances: read sizes, file offsets, codedelay, sv_vel and the C/N0 row positions bit-exact; the
carrier-wiped sums within 1e-9 of |P| (fp64 fixed-order workgroup sums against long double, as
tests/test_gpu_vt.py); what the sums feed (carrier NCO, the EKF's Doppler measurements, its state
and the next code frequency) within the bounds written at each assert.
"""
from types import SimpleNamespace

import numpy as np
import pytest

import vt_nav_common as V
from conftest import params

pytestmark = pytest.mark.gpu

S = 58000


def _inputs(pkg, z, skip, bps=2):
    """The reference-shaped arguments of trackingVT_POS_updated (SDR_main.m:99) for the
    synthetic record: Acquired, eph, sbf, TckResultCT (3000 rows; row msStartTckVT = 3000 holds
    the reference's state, absoluteSample moved onto the scene), navSolutionsCT."""
    prns = [int(p) for p in z["prns"]]
    scene = dict(zip(pkg.synth.OPENSKY_SV, pkg.synth.OPENSKY_CODEDELAY))
    Acquired = SimpleNamespace(sv=np.array(prns))
    eph = {}
    for i, p in enumerate(prns):
        e = SimpleNamespace(**{f: np.array([z["eph"][i, j]]) for j, f in enumerate(pkg.abi.EPH_SV_FIELDS)})
        e.sfb = np.array([z["eph_sfb1"][i]])
        eph[p] = e
    nav1 = np.zeros(32)
    for i, p in enumerate(prns):
        nav1[p - 1] = z["nav1"][i]
    sbf = SimpleNamespace(nav1=nav1)
    ct = {}
    for i, p in enumerate(prns):
        e = SimpleNamespace()
        for f in ("codeFreq", "remChip", "carrFreq", "remCarrPhase", "codedelay", "carrError"):
            a = np.zeros(3000)
            a[-3:] = z["ct_" + f][i]
            setattr(e, f, a)
        e.absoluteSample = np.zeros(3000)
        e.absoluteSample[-1] = (S - scene[p] + 1 + skip * S) * bps
        ct[p] = e
    ns = SimpleNamespace(**{k: z["navSolCT_" + k] for k in ("usrPos", "usrVel", "clkBias", "clkDrift",
                                                          "timeTransmit")})
    return Acquired, eph, sbf, ct, ns


def _oracle_loop(pkg, po, z, ct, data, nsteps, prec=1, dtype=2):
    prns = [int(p) for p in z["prns"]]
    st = np.stack([po.vt_state(ct[p].absoluteSample[-1], ct[p].remChip[-1], ct[p].remCarrPhase[-1],
                               ct[p].codeFreq[-1], ct[p].carrFreq[-1], ct[p].carrFreq[-1], 0.0,
                               ct[p].carrError[-1]) for p in prns])
    onav = V.oracle_nav(pkg, po, z)
    status, rec, nav = onav.tracking(np.ascontiguousarray(data).view(np.int8), st, prns, nsteps, prec=prec,
                                     dtype=dtype)
    return status, rec, nav


def _compare(pkg, po, z, tck, nsol, rec, onav, tol_sum=1e-9):
    """The closed loops side by side: read sizes / offsets / codedelay / sv_vel exact, sums within
    tol_sum of |P|, code frequency within 1e-12 relative, the EKF state within 10 um."""
    R = {k: rec[:, :, j] for j, k in enumerate(po.VT_REC + ["deltaPr", "prRate"])}
    worst = 0.0
    for i, p in enumerate(int(x) for x in z["prns"]):
        g = tck(p)
        assert np.array_equal(g.absoluteSample, R["absoluteSample"][:, i]), p
        assert np.array_equal(g.codedelay, R["codedelay"][:, i]), p
        assert np.array_equal(g.sv_vel, rec[:, i, 20:23]), p
        scale = np.maximum(np.maximum(np.abs(R["P_i"][:, i]), np.abs(R["P_q"][:, i])), 1.0)
        for f in ("P_i", "P_q"):
            worst = max(worst, float(np.max(np.abs(getattr(g, f) - R[f][:, i]) / scale)))
        assert np.allclose(g.codeFreq, R["codeFreq"][:, i], rtol=1e-12, atol=0), p
        assert np.allclose(g.deltaPr, R["deltaPr"][:, i], rtol=0, atol=1e-4), p
    assert worst < tol_sum, worst
    assert np.allclose(nsol.usrPos, onav[:, :3], rtol=0, atol=1e-5)
    assert np.allclose(nsol.clkBias, onav[:, 6], rtol=0, atol=1e-5)
    return worst


def test_vector_tracking_closed_loop_against_oracle(pkg, po, ctx, opensky_short):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    _, _, _, _, solu, cmn = pkg.initParameters()
    z = V.fixture()
    Acquired, eph, sbf, ct, ns = _inputs(pkg, z, skip)
    nsteps = 1200
    ctx.set_profiling(True)
    tck, nsol, cn0 = pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, V.cnslxyz(pkg), eph,
                                                sbf, None, ct, ns, ctx=ctx, nsteps=nsteps, return_cn0=True)
    t = ctx.timing()
    ctx.set_profiling(False)
    assert t["track_launches"] == nsteps
    print(f"gnss_tracking_vt: {nsteps} steps x 5 channels, loop {t['track_ms']:.1f} ms, kernel "
          f"{t['track_kernel_ms']:.1f} ms")
    status, rec, onav = _oracle_loop(pkg, po, z, ct, data, nsteps)
    assert status == 0
    R = {k: rec[:, :, j] for j, k in enumerate(po.VT_REC + ["deltaPr", "prRate"])}
    prns = [int(p) for p in z["prns"]]
    worst = dict(sum=0.0, cf=0.0, dpr=0.0, carr=0.0)
    for i, p in enumerate(prns):
        g = tck(p)
        # integer / exact: the read sizes and offsets the code frequencies produced
        assert np.array_equal(g.absoluteSample, R["absoluteSample"][:, i]), p
        assert np.array_equal(g.codedelay, R["codedelay"][:, i]), p
        assert np.array_equal(g.sv_vel, rec[:, i, 20:23]), p  # svPosVel at the (exact) transmit time
        assert np.all(g.prRate == 0) and np.all(g.amplitude == 0)
        scale = np.maximum(np.maximum(np.abs(R["P_i"][:, i]), np.abs(R["P_q"][:, i])), 1.0)
        for f in ("E_i", "E_q", "P_i", "P_q", "L_i", "L_q"):
            worst["sum"] = max(worst["sum"], float(np.max(np.abs(getattr(g, f) - R[f][:, i]) / scale)))
        worst["cf"] = max(worst["cf"], float(np.max(np.abs(g.codeFreq - R["codeFreq"][:, i]) / g.codeFreq)))
        worst["dpr"] = max(worst["dpr"], float(np.max(np.abs(g.deltaPr - R["deltaPr"][:, i]))))
        worst["carr"] = max(worst["carr"], float(np.max(np.abs(g.carrFreq - R["carrFreq"][:, i]))))
        for f in ("remChip", "remCarrPhase", "carrNco", "carrError"):
            assert np.allclose(getattr(g, f), R[f][:, i], rtol=1e-9, atol=1e-9), (p, f)
        assert g.codeFreq[0] == ct[p].codeFreq[-1]  # msIndex 1 keeps TckResultCT's (:218-219)
    print({k: f"{v:.3g}" for k, v in worst.items()})
    assert worst["sum"] < 1e-9
    assert worst["carr"] < 1e-6          # Hz: the PLL's carrError differs by the sums' rounding
    assert worst["cf"] < 1e-12           # relative: the Doppler measurements move the state by < 1 um
    assert worst["dpr"] < 1e-4           # m/s: a few ulps of a 2e7-m range over 1 ms
    # the EKF state after each update (navSolutionsVT.usrPos / usrVel / clkBias / clkDrift)
    assert np.allclose(nsol.usrPos, onav[:, :3], rtol=0, atol=1e-5)
    assert np.allclose(nsol.usrVel, onav[:, 3:6], rtol=0, atol=1e-5)
    assert np.allclose(nsol.clkBias, onav[:, 6], rtol=0, atol=1e-5)
    assert np.allclose(nsol.clkDrift, onav[:, 7], rtol=0, atol=1e-6)
    # navSolutionsVT's shapes (:418-436, :466) and the R updates every 200 steps
    n = len(prns)
    assert nsol.usrPosENU.shape == (nsteps, 3) and nsol.state.shape == (nsteps, 8)
    assert nsol.newZ.shape == (nsteps, 2 * n) and nsol.satEA.shape == (nsteps, n)
    assert nsol.svxyz_pos.shape == (n, 3, nsteps) and nsol.kalman_gain.shape == (8, 2 * n, nsteps)
    assert nsol.R.shape == (nsteps // 200, 2 * n)
    assert np.all(nsol.R[:, :n] >= 0.01) and np.all(nsol.R[:, :n] <= 12000)
    assert np.all(nsol.R[:, n:] >= 0.01) and np.all(nsol.R[:, n:] <= 400)
    # CN0_VT: one row per 20 steps and channel (:296-304)
    assert cn0.shape == (nsteps // 20, n)
    c_ref = np.zeros_like(cn0)
    for i in range(n):
        m = R["cn0_row"][:, i] > 0
        c_ref[R["cn0_row"][:, i][m].astype(int) - 1, i] = R["CN0"][:, i][m]
    assert np.allclose(cn0, c_ref, rtol=1e-9, atol=0)


def test_vector_tracking_stops_past_eof(pkg, ctx, opensky_short):
    """A read past the end of the record stops the loop with EIO, as MATLAB's fread of a short
    block feeds a size-mismatched product and raises (:165-181)."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    _, _, _, _, solu, cmn = pkg.initParameters()
    z = V.fixture()
    Acquired, eph, sbf, ct, ns = _inputs(pkg, z, skip)
    steps_left = (len(data) - int(max(ct[p].absoluteSample[-1] for p in ct))) // (2 * S)
    with pytest.raises(pkg.abi.GnssError) as ei:
        pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, V.cnslxyz(pkg), eph, sbf, None, ct,
                                   ns, ctx=ctx, nsteps=steps_left + 20)
    assert ei.value.status == pkg.abi.EIO
    # the context stays usable
    tck, nsol = pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, V.cnslxyz(pkg), eph, sbf,
                                           None, ct, ns, ctx=ctx, nsteps=10)
    assert nsol.usrPos.shape == (10, 3)


@pytest.mark.parametrize("prec,dtyp", [(2, 2), (1, 1)], ids=["int16-iq", "int8-real"])
def test_vector_tracking_formats(pkg, po, ctx, opensky_short, prec, dtyp):
    """The EKF-driven loop on the other record formats of :163-176 (int16 I/Q with each read's
    means removed: the one-block-per-channel step; int8 real: the multi-block step), 300 steps
    against the oracle's closed loop on the same bytes."""
    skip, cfg, data = opensky_short
    rec8 = pkg.synth.convert_record(data, prec, dtyp)
    file = SimpleNamespace(skip=skip, dataType=dtyp, dataPrecision=prec, data=rec8, fileRoute=None, dev=None,
                           skiptimeVT=100)
    _, signal, _, track, solu, cmn = pkg.initParameters()
    z = V.fixture()
    Acquired, eph, sbf, ct, ns = _inputs(pkg, z, skip, bps=prec * dtyp)
    nsteps = 300
    tck, nsol = pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, V.cnslxyz(pkg), eph, sbf,
                                           None, ct, ns, ctx=ctx, nsteps=nsteps)
    status, rec, onav = _oracle_loop(pkg, po, z, ct, rec8, nsteps, prec=prec, dtype=dtyp)
    assert status == 0
    print(prec, dtyp, "worst sum / |P|", _compare(pkg, po, z, tck, nsol, rec, onav))


@pytest.mark.parametrize("nb", [1, 7, 64, 300, 1024])
def test_vector_tracking_step_blocks(pkg, po, ctx, opensky_short, opts, nb):
    """The multi-block step (vt_step_kernel) at other block counts per channel
    (GNSS_OPT_VT_BLOCKS; the engine's is 29): another fixed association of the same per-sample
    terms, the same loop against the oracle. The host adds a channel's nb partials in block
    order whatever nb is (up to GNSS_VT_MAX_BLOCKS, 1 024 x 5 partials)."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    _, _, _, _, solu, cmn = pkg.initParameters()
    z = V.fixture()
    Acquired, eph, sbf, ct, ns = _inputs(pkg, z, skip)
    opts(pkg.abi.OPT_VT_BLOCKS, nb)
    nsteps = 300
    tck, nsol = pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, V.cnslxyz(pkg), eph, sbf,
                                           None, ct, ns, ctx=ctx, nsteps=nsteps)
    status, rec, onav = _oracle_loop(pkg, po, z, ct, data, nsteps)
    assert status == 0
    print(nb, "worst sum / |P|", _compare(pkg, po, z, tck, nsol, rec, onav))


def _vt_run(pkg, ctx, opts, data, skip, nsteps, **opt):
    for k, v in opt.items():
        opts(getattr(pkg.abi, k), v)
    file, signal, acq, track = params(pkg, skip, data)
    _, _, _, _, solu, cmn = pkg.initParameters()
    z = V.fixture()
    Acquired, eph, sbf, ct, ns = _inputs(pkg, z, skip)
    tck, nsol = pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, V.cnslxyz(pkg), eph, sbf,
                                           None, ct, ns, ctx=ctx, nsteps=nsteps)
    return z, ct, tck, nsol, ctx.timing()


def test_vector_tracking_loop_mode_equals_step_launches(pkg, po, ctx, opensky_short, opts):
    """Loop mode (one vt_loop_kernel launch serves the steps through the host mailbox) against
    one vt_step_kernel launch per step (GNSS_OPT_NO_PERSIST): the same block sums in the same
    order, so every output is bit-identical. GNSS_OPT_VT_SPAN = 40 re-stages the host record's
    IF window every ~40 steps, so the loop launch is stopped and relaunched mid-call; the loop
    run is also held against the oracle's closed loop."""
    skip, cfg, data = opensky_short
    nsteps = 300
    # (the same blocks per channel on both paths: the engine's choice differs between them)
    z, ct, tck_l, nsol_l, t_l = _vt_run(pkg, ctx, opts, data, skip, nsteps, OPT_VT_SPAN=40, OPT_VT_BLOCKS=76)
    _, _, tck_s, nsol_s, t_s = _vt_run(pkg, ctx, opts, data, skip, nsteps, OPT_VT_SPAN=40, OPT_VT_BLOCKS=76,
                                       OPT_NO_PERSIST=1)
    assert t_l["track_launches"] == t_s["track_launches"] == nsteps
    assert t_l["h2d_bytes"] > 0 and t_l["h2d_bytes"] == t_s["h2d_bytes"]  # (the same windows staged)
    for p in (int(x) for x in z["prns"]):
        a, b = tck_l(p), tck_s(p)
        for f in ("P_i", "P_q", "E_i", "L_q", "carrFreq", "codeFreq", "remChip", "remCarrPhase", "absoluteSample",
                  "codeError", "deltaPr", "sv_vel"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), (p, f)
    for f in ("usrPos", "usrVel", "clkBias", "clkDrift", "state"):
        assert np.array_equal(getattr(nsol_l, f), getattr(nsol_s, f)), f
    status, rec, onav = _oracle_loop(pkg, po, z, ct, data, nsteps)
    assert status == 0
    _compare(pkg, po, z, tck_l, nsol_l, rec, onav)


def test_vector_tracking_loop_mode_at_max_channels(pkg, ctx, opensky_short, opts):
    """The largest loop-mode grid: GNSS_VT_MAX_CH = 32 channels (the fixture's 5 repeated) at
    the engine's 32 blocks per channel, 1 024 blocks, the loop kernel's bound: the lead relays
    160 mailbox granules and gathers 2 048 partial granules per step. Held bit for bit against
    one vt_step_kernel launch per step at the same blocks per channel (GNSS_OPT_NO_PERSIST):
    every channel record and every EKF row over 60 steps."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    _, _, _, _, solu, cmn = pkg.initParameters()
    z = V.fixture()
    Acquired, eph, sbf, ct, ns = _inputs(pkg, z, skip)
    n = pkg.abi.VT_MAX_CH
    reps = [int(p) for p in z["prns"]]
    sv = [reps[i % len(reps)] for i in range(n)]
    Acq = SimpleNamespace(sv=np.array(sv))
    ns32 = SimpleNamespace(usrPos=ns.usrPos, usrVel=ns.usrVel, clkBias=ns.clkBias, clkDrift=ns.clkDrift,
                           timeTransmit=np.array([[ns.timeTransmit[0][i % len(reps)] for i in range(n)]]))
    nsteps = 60

    def run(**opt):
        for k, v in opt.items():
            opts(getattr(pkg.abi, k), v)
        tck, nsol = pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acq, V.cnslxyz(pkg), eph, sbf,
                                               None, ct, ns32, ctx=ctx, nsteps=nsteps)
        return tck, nsol, ctx.timing()

    tck_l, nsol_l, t_l = run()
    tck_s, nsol_s, t_s = run(OPT_VT_BLOCKS=1024 // n, OPT_NO_PERSIST=1)
    assert t_l["track_launches"] == t_s["track_launches"] == nsteps
    for p in reps:
        for f in ("P_i", "P_q", "E_q", "L_i", "carrFreq", "codeFreq", "remChip", "absoluteSample", "deltaPr"):
            assert np.array_equal(getattr(tck_l(p), f), getattr(tck_s(p), f)), (p, f)
    for f in ("usrPos", "usrVel", "clkBias", "clkDrift", "state", "newZ", "kalman_gain"):
        assert np.array_equal(getattr(nsol_l, f), getattr(nsol_s, f)), f
    assert np.all(np.isfinite(nsol_l.usrPos))


def test_vector_tracking_span_option_bound(pkg, ctx):
    abi = pkg.abi
    for bad in (-1, 2001):
        assert ctx.lib.gnss_ctx_set_option(ctx.h, abi.OPT_VT_SPAN, bad) == abi.EARG
    assert ctx.lib.gnss_ctx_set_option(ctx.h, abi.OPT_VT_SPAN, 2000) == 0
    assert ctx.lib.gnss_ctx_set_option(ctx.h, abi.OPT_VT_SPAN, 0) == 0


def test_vector_tracking_block_option_bound(pkg, ctx):
    """GNSS_OPT_VT_BLOCKS takes 0 (the engine's choice) .. GNSS_VT_MAX_BLOCKS and refuses
    anything else with GNSS_EARG."""
    abi = pkg.abi
    for bad in (-1, 1025, 1 << 20):
        assert ctx.lib.gnss_ctx_set_option(ctx.h, abi.OPT_VT_BLOCKS, bad) == abi.EARG
    assert ctx.lib.gnss_ctx_set_option(ctx.h, abi.OPT_VT_BLOCKS, 1024) == 0
    assert ctx.lib.gnss_ctx_set_option(ctx.h, abi.OPT_VT_BLOCKS, 0) == 0


def test_vector_tracking_channel_bound(pkg, ctx):
    """gnss_tracking_vt refuses more than GNSS_VT_MAX_CH channels (its per-step kernel arguments
    hold that many code frequencies) before touching anything, and the context stays usable."""
    import ctypes as C
    abi = pkg.abi
    file, signal, _, track, _, _ = pkg.initParameters()
    file.data = np.zeros(4096, dtype=np.int8)  # (never read: the call fails on n first)
    f, keep = pkg.sdr.to_c_file(file)
    s = pkg.sdr.to_c_signal(signal)
    t, keep2 = pkg.sdr.to_c_track(track)
    n = 33
    chans = (abi.GnssVtChan * n)()
    nav = abi.GnssVtNav()
    nav.n = n
    outs = (abi.GnssVtOut * n)()
    st = ctx.lib.gnss_tracking_vt(ctx.h, C.byref(f), C.byref(s), C.byref(t), n, 1, chans, C.byref(nav), outs, None)
    assert st == abi.EARG
    assert ctx.lib.gnss_tracking_vt(ctx.h, C.byref(f), C.byref(s), C.byref(t), 0, 1, chans, C.byref(nav), outs,
                                    None) == abi.EARG
    ctx.timing()  # (the context still answers)
