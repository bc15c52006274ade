"""GPU parity for the tracking loop of trackingCT_POS_updated_multicorrelator.m
(gnss_tracking_ct_mc, SURVEY §8f row 1: the 25-tap sibling) against the CPU oracle and the
committed golden vectors, through the C-ABI.

The step kernel with 25 taps (4 lanes per value in the channel sum), Code(ceil(t) + 2),
T = pdi*t, every step at track.pdi. Tolerances as test_gpu_pos.py: integer fields
bit-exact, correlator sums (all 25 taps) within 1e-5 of the series RMS (north-star) and
1e-8 (fp64 guard), NCO state 1e-7 relative, C/N0 1e-6 dB.
"""
import numpy as np
import pytest

from conftest import acquired_of, params
from test_gpu_pos import OPENSKY, compare_pos

pytestmark = pytest.mark.gpu


def compare_mc(pkg, g, r, tol=1e-8):
    compare_pos(pkg, g, r, tol)
    for c in range(len(g.len)):
        n = int(r.len[c])
        scale = np.sqrt(np.mean(r.rec[c, 0, :n] ** 2 + r.rec[c, 1, :n] ** 2))
        err = np.max(np.abs(g.taps[c, :, :, :n] - r.taps[c, :, :, :n])) / scale
        assert err < 1e-5 and err < tol, (c, err)


@pytest.mark.parametrize("pdi,ms", [(1, 400), (10, 800)])
def test_mc_parity_opensky_8ch(pkg, po, ctx, opensky_short, pdi, ms):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msPosCT, track.pdi = ms, pdi
    A = acquired_of(OPENSKY["svs"], OPENSKY["cd"], OPENSKY["ff"])
    g = pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=ctx, raw=True)
    r = po.trackingCT_mc(file, signal, track, A, raw=True)
    assert r.status == 0
    compare_mc(pkg, g, r)
    T, cn0 = pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=ctx)
    assert T.prns() == sorted(OPENSKY["svs"]) and len(T(16).E_i_060) == ms // pdi
    assert np.array_equal(T(16).L_q060, g.taps[2, 1, 24, : ms // pdi])
    assert np.array_equal(T(16).P_i, T(16).taps_i[12]) and np.array_equal(T(16).L_i, T(16).taps_i[22])
    assert cn0.shape == (ms // pdi // 20, 8)


def test_mc_matches_golden_vectors(pkg, po, ctx):
    import test_oracle_mc as tm
    g = np.load(tm.GOLDEN)
    data = tm.mc_record(pkg, po)
    for pdi, ms in tm.MS.items():
        file, signal, acq, track = params(pkg, tm.SKIP, data)
        track.msPosCT, track.pdi = ms, pdi
        A = acquired_of(tm.SVS, tm.CD, tm.FF)
        b = pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=ctx, raw=True)
        tm.check_mc_against_golden(g, pdi, b.rec, b.taps, b.len, b.CN0[: b.c.cn0_rows], tol=1e-8)


def test_mc_errors(pkg, ctx, opensky_short):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 400])
    A = acquired_of([16], [26051], [4579675.0])
    track.msPosCT, track.pdi = 600, 10  # 60 x 10 ms > 400 ms of record
    with pytest.raises(pkg.abi.GnssError) as e:
        pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=ctx)
    assert e.value.status == pkg.abi.EIO
    track.pdi = 20
    with pytest.raises(pkg.abi.GnssError) as e:
        pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=ctx)
    assert e.value.status == pkg.abi.EARG


# ---- trackingCT_multiCorr-GIVEN.m (gnss_tracking_ct_multicorr) --------
def compare_given(pkg, g, r, tol=1e-8):
    from test_gpu_tracking import compare
    compare(pkg, g, r)
    for c in range(len(g.len)):
        n = int(r.len[c])
        scale = np.sqrt(np.mean(r.rec[c, 0, :n] ** 2 + r.rec[c, 1, :n] ** 2))
        err = np.max(np.abs(g.taps[c, :, :, :n] - r.taps[c, :, :, :n])) / scale
        assert err < 1e-5 and err < tol, (c, err)


def test_given_parity_opensky_8ch(pkg, po, ctx, opensky_short):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    A = acquired_of(OPENSKY["svs"], OPENSKY["cd"], OPENSKY["ff"])
    g = pkg.trackingCT_multiCorr(file, signal, track, A, datalength=600, ctx=ctx, raw=True)
    r = po.trackingCT_multiCorr(file, signal, track, A, 600, raw=True)
    assert r.status == 0
    compare_given(pkg, g, r)
    T, cn0 = pkg.trackingCT_multiCorr(file, signal, track, A, datalength=600, ctx=ctx)
    assert len(T(3).E_i_060) == 600 and np.array_equal(T(3).E_i, T(3).taps_i[2])
    assert cn0.shape == (30, 8)


def test_given_matches_golden_vectors(pkg, po, ctx):
    import test_oracle_given as tg
    g = np.load(tg.GOLDEN)
    data = tg.given_record(pkg, po)
    file, signal, acq, track = params(pkg, tg.SKIP, data)
    A = acquired_of(tg.SVS, tg.CD, tg.FF)
    b = pkg.trackingCT_multiCorr(file, signal, track, A, datalength=tg.DATALEN, ctx=ctx, raw=True)
    tg.check_given_against_golden(g, b.rec, b.taps, b.len, b.CN0[: b.c.cn0_rows], 1e-8)


def test_given_errors(pkg, ctx, opensky_short):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 300])
    A = acquired_of([16], [26051], [4579675.0])
    with pytest.raises(pkg.abi.GnssError) as e:  # short read: MATLAB raises
        pkg.trackingCT_multiCorr(file, signal, track, A, datalength=400, ctx=ctx)
    assert e.value.status == pkg.abi.EIO
    file.dataPrecision = 2
    with pytest.raises(pkg.abi.GnssError) as e:
        pkg.trackingCT_multiCorr(file, signal, track, A, datalength=100, ctx=ctx)
    assert e.value.status == pkg.abi.EARG


def test_mc_channel_shards_equal_full_run(pkg, ctx, opensky_short):
    """Channel shards (the multi-GPU split) of the 25-tap loop reproduce the full run's rows
    bit for bit (lane geometry and reductions do not depend on the channel set)."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msPosCT, track.pdi = 300, 10
    A = acquired_of(OPENSKY["svs"], OPENSKY["cd"], OPENSKY["ff"])
    full = pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=ctx, raw=True)
    for shard in ([0, 2, 4, 6], [1, 3, 5, 7]):
        part = pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=ctx,
                                                          channels=shard, raw=True)
        for c in shard:
            assert np.array_equal(part.rec[c], full.rec[c]) and np.array_equal(part.taps[c], full.taps[c])
