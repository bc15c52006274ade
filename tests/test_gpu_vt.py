"""GPU parity of vector tracking (gnss_tracking_vt_run / _step, the tracking
half of trackingVT_POS_updated.m:157-349) against the oracle's restatement (or_vt_step, itself
pinned by the reference's tckRstVT output and CN0_VT in tests/test_vt_kat.py), on the synthetic
Opensky record. The code frequency of every step is given (the caller's EKF prediction,
trackingVT_POS_updated.m:211-215). Read sizes, file offsets, codedelay and the C/N0 rows'
positions bit-exact; the carrier-wiped sums (exact per-sample Wave on both sides, fp64
fixed-order workgroup sums on the GPU, long-double sums in the oracle), the NCO / PLL state
and C/N0 within 1e-9 relative."""
import numpy as np
import pytest

from conftest import params

pytestmark = pytest.mark.gpu

S = 58000
PRNS, CDS, FFS = [3, 16, 26], [3684, 26051, 57908], [4580975.0, 4579675.0, 4581800.0]
SUMS = ("E_i", "E_q", "P_i", "P_q", "L_i", "L_q")
NCO = ("remChip", "remCarrPhase", "codeFreq", "carrFreq", "carrNco", "carrError", "codeError")


def _chans(pkg, po, prns, cds, ffs, skip, bps=2):
    chans = [pkg.vt_channel(p, (S - cd + 1 + skip * S) * bps, 0.0, 0.0, 1.023e6, f, f)
             for p, cd, f in zip(prns, cds, ffs)]
    st = [po.vt_state(c.file_ptr, 0.0, 0.0, 1.023e6, c.carrFreq, c.carrFreqBasis) for c in chans]
    return chans, st


def _check(g, R, k, prn, worst):
    for f in ("numSample", "absoluteSample", "codedelay", "cn0_row"):
        assert g[f] == R[f], (k, prn, f, g[f], R[f])
    scale = max(abs(R["P_i"]), abs(R["P_q"]), 1.0)
    for f in SUMS:
        worst[0] = max(worst[0], abs(g[f] - R[f]) / scale)
    for f in NCO:
        assert np.isclose(g[f], R[f], rtol=1e-9, atol=1e-9), (k, prn, f, g[f], R[f])
    if R["cn0_row"]:
        assert np.isclose(g["CN0"], R["CN0"], rtol=1e-9, atol=0), (k, prn, g["CN0"], R["CN0"])


def test_vt_steps_against_oracle(pkg, po, ctx, opensky_short):
    """One launch per step (gnss_tracking_vt_step): 3 channels x 300 closed-loop 1-ms steps,
    a constant code frequency."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    chans, st = _chans(pkg, po, PRNS, CDS, FFS, skip)
    cf = [1.023e6] * 3
    iq = np.ascontiguousarray(data, dtype=np.int8)
    worst = [0.0]
    for k in range(300):
        g = pkg.trackingVT_step(file, signal, track, chans, cf, ctx=ctx)
        for i, prn in enumerate(PRNS):
            status, rec = po.vt_step(st[i], cf[i], prn, iq=iq)
            assert status == 0
            _check(g[i], dict(zip(po.VT_REC, rec)), k, prn, worst)
    print("worst sum error / |P|", worst[0])
    assert worst[0] < 1e-9


def test_vt_run_1200_steps_recorded_code_frequency(pkg, po, ctx, opensky_short):
    """1 200 steps of the 5 channels of the reference's VT run in ONE launch
    (gnss_tracking_vt_run), each step's code frequency the reference's own recorded series
    (tckRstVT_Opensky_updated.mat codeFreq, tests/golden/ref_tckRstVT_Opensky.npz, the EKF's
    predictions), against the oracle replaying the same series step by step: every record
    field, and the 60 CN0_VT rows of each channel."""
    import os
    from conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "ref_tckRstVT_Opensky.npz"))
    prns = [int(p) for p in z["prns"]]  # 3 16 22 26 31: all in the synthetic Opensky scene
    scene = dict(zip(pkg.synth.OPENSKY_SV, zip(pkg.synth.OPENSKY_CODEDELAY, pkg.synth.OPENSKY_FINEFREQ)))
    cds = [scene[p][0] for p in prns]
    ffs = [scene[p][1] for p in prns]
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    nsteps = 1200
    series = np.ascontiguousarray(z["codeFreq"][:, :nsteps].T)  # [step][channel]
    chans, st = _chans(pkg, po, prns, cds, ffs, skip)
    out = pkg.trackingVT_run(file, signal, track, chans, series, ctx=ctx)
    t = ctx.timing()
    assert t["track_launches"] == 1
    assert (out["status"] == 0).all()
    iq = np.ascontiguousarray(data, dtype=np.int8)
    worst = [0.0]
    rows = 0
    for k in range(nsteps):
        for i, prn in enumerate(prns):
            status, rec = po.vt_step(st[i], series[k, i], prn, iq=iq)
            assert status == 0
            R = dict(zip(po.VT_REC, rec))
            _check({f: out[f][k, i] for f in out}, R, k, prn, worst)
            rows += R["cn0_row"] > 0
    assert rows == 5 * nsteps // 20
    for i in range(len(prns)):  # the channel state after the run = the oracle's
        assert chans[i].file_ptr == int(st[i][0]) and chans[i].snrIndex == int(st[i][9])
    print(f"worst sum error / |P| {worst[0]:.2e}; {nsteps} steps x {len(prns)} channels in "
          f"{t['track_ms']:.1f} ms (one launch)")
    assert worst[0] < 1e-9


@pytest.mark.parametrize("prec,dtyp", [(2, 2), (1, 1)], ids=["int16-iq", "int8-real"])
def test_vt_run_formats(pkg, po, ctx, opensky_short, prec, dtyp):
    """The record formats of trackingVT_POS_updated.m:163-176: int16 I/Q with each
    read's means removed and int8 real, 200 steps of 3 channels in one launch vs the oracle."""
    from types import SimpleNamespace
    skip, cfg, data = opensky_short
    rec8 = pkg.synth.convert_record(data, prec, dtyp)
    file = SimpleNamespace(skip=skip, dataType=dtyp, dataPrecision=prec, data=rec8, fileRoute=None, dev=None)
    _, signal, acq, track, _, _ = pkg.initParameters()
    bps = prec * dtyp
    chans, st = _chans(pkg, po, PRNS, CDS, FFS, skip, bps)
    nsteps = 200
    series = np.full((nsteps, 3), 1.023e6)
    out = pkg.trackingVT_run(file, signal, track, chans, series, ctx=ctx)
    worst = [0.0]
    for k in range(nsteps):
        for i, prn in enumerate(PRNS):
            status, r = po.vt_step(st[i], series[k, i], prn, iq=rec8, prec=prec, dtype=dtyp)
            assert status == 0
            _check({f: out[f][k, i] for f in out}, dict(zip(po.VT_REC, r)), k, prn, worst)
    print(prec, dtyp, "worst sum error / |P|", worst[0])
    assert worst[0] < 1e-9


def test_vt_run_stops_past_eof(pkg, ctx, opensky_short):
    """A read past the end of the record stops that channel with GNSS_EIO (MATLAB's short
    fread makes `rawsignal .* carrsig` raise, :172, :279); the call reports it."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * S * (skip + 40)])
    import importlib
    po = importlib.import_module("pyoracle")
    chans, _ = _chans(pkg, po, PRNS[:1], CDS[:1], FFS[:1], skip)
    with pytest.raises(pkg.abi.GnssError) as e:
        pkg.trackingVT_run(file, signal, track, chans, np.full((100, 1), 1.023e6), ctx=ctx)
    assert e.value.status == pkg.abi.EIO
