"""GPU parity for the tracking loop of trackingCT_POS_updated.m (gnss_tracking_ct_pos,
SURVEY §8f row 1) against the CPU oracle, through the C-ABI.

Same kernels as trackingCT with the sibling's conventions (ceil numSample, prompt
Code(ceil(t + 0.05) + 1), E at +0.5 / L at -0.5, codeFreq = f0 + codeNco, T = 1 ms at
every pdi, no negation, no re-seek, per-channel 1 -> 10 ms switch at 1000 + countinx).
Tolerances as test_gpu_tracking.py: integer fields bit-exact, P/E/L within 1e-5 of the
series RMS (north-star) and 1e-8 (fp64 guard), NCO state 1e-7 relative, C/N0 1e-6 dB.
"""
import numpy as np
import pytest

from conftest import acquired_of, params

pytestmark = pytest.mark.gpu

INT_FIELDS = ["codedelay", "numSample", "delayValue", "absoluteSample", "codedelay2",
              "absoluteSampleCodedelay"]
NCO_FIELDS = ["remChip", "codeFreq", "carrFreq", "remCarrPhase", "carrError", "codeError"]

OPENSKY = dict(svs=[3, 4, 16, 22, 26, 27, 31, 32],
               cd=[3684, 12700, 26051, 2611, 57908, 49777, 39064, 20170],
               ff=[4580975.0, 4576875.0, 4579675.0, 4581525.0, 4581800.0, 4576750.0, 4581025.0,
                   4583325.0],
               cx=[12, 12, 3, 13, 5, 9, 9, 12])  # SDR/countinx.mat


def compare_pos(pkg, g, r, tol=1e-8):
    F = pkg.abi.FIELDS_POS
    assert np.array_equal(g.len, r.len)
    assert np.array_equal(g.countinx, r.countinx)
    for c in range(len(g.len)):
        n = int(r.len[c])
        for k, f in enumerate(F):
            if f in INT_FIELDS:
                assert np.array_equal(g.rec[c, k, :n], r.rec[c, k, :n]), (c, f)
        scale = np.sqrt(np.mean(r.rec[c, 0, :n] ** 2 + r.rec[c, 1, :n] ** 2))
        for k in range(6):
            err = np.max(np.abs(g.rec[c, k, :n] - r.rec[c, k, :n])) / scale
            assert err < 1e-5 and err < tol, (c, F[k], err)
        for f in NCO_FIELDS:
            k = F.index(f)
            assert np.allclose(g.rec[c, k, :n], r.rec[c, k, :n], rtol=1e-7, atol=1e-9), (c, f)
    rows = r.c.cn0_rows
    assert g.c.cn0_rows == rows
    assert np.allclose(g.CN0[:rows], r.CN0[:rows], rtol=0, atol=1e-6)


def test_pos_parity_opensky_8ch(pkg, po, ctx, opensky_short):
    """8 channels, countinx.mat's switch points, 1000 + countinx steps at 1 ms then 10 ms."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.ctPOS = 1000, 1000 + 12 + 80
    A = acquired_of(OPENSKY["svs"], OPENSKY["cd"], OPENSKY["ff"])
    g = pkg.trackingCT_POS(file, signal, track, A, OPENSKY["cx"], ctx=ctx, raw=True)
    r = po.trackingCT_POS(file, signal, track, A, OPENSKY["cx"], raw=True)
    assert r.status == 0
    compare_pos(pkg, g, r)
    T, cn0 = pkg.trackingCT_POS(file, signal, track, A, OPENSKY["cx"], ctx=ctx)
    assert T.prns() == sorted(OPENSKY["svs"]) and len(T(16).carrFreq) == track.ctPOS
    assert cn0.shape == (track.ctPOS // 20, 8)


@pytest.mark.parametrize("persist", [True, False], ids=["persistent", "step"])
@pytest.mark.parametrize("sub", ["1", "3"])
def test_pos_parity_kernel_variants(pkg, po, ctx, opensky_short, opts, sub, persist):
    opts(pkg.abi.OPT_FORCE_SUB, int(sub))
    if not persist:
        opts(pkg.abi.OPT_NO_PERSIST, 1)
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.ctPOS = 300, 360
    A = acquired_of([16, 26, 31], [26051, 57908, 39064], [4579675.0, 4581800.0, 4581025.0])
    cx = [-1, 18, 7]
    g = pkg.trackingCT_POS(file, signal, track, A, cx, ctx=ctx, raw=True)
    r = po.trackingCT_POS(file, signal, track, A, cx, raw=True)
    compare_pos(pkg, g, r)


def test_pos_persistent_and_step_paths_bit_identical(pkg, ctx, opensky_short, opts):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.ctPOS = 300, 400
    A = acquired_of([3, 16, 22], [3684, 26051, 2611], [4580975.0, 4579675.0, 4581525.0])
    cx = [12, 3, 13]
    p = pkg.trackingCT_POS(file, signal, track, A, cx, ctx=ctx, raw=True)
    assert ctx.timing()["track_launches"] <= 4
    opts(pkg.abi.OPT_NO_PERSIST, 1)
    q = pkg.trackingCT_POS(file, signal, track, A, cx, ctx=ctx, raw=True)
    assert ctx.timing()["track_launches"] > 100
    assert np.array_equal(p.rec, q.rec) and np.array_equal(p.CN0, q.CN0)


def test_pos_matches_golden_vectors(pkg, po, ctx):
    from test_golden_oracle import check_pos_against_golden, pos_inputs
    g, file, signal, track, A = pos_inputs(pkg, po)
    b = pkg.trackingCT_POS(file, signal, track, A, g["countinx"], ctx=ctx, raw=True)
    check_pos_against_golden(pkg, g, b.rec, b.len, b.CN0[: b.c.cn0_rows], tol=1e-8)


def test_pos_errors(pkg, ctx, opensky_short):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 400])
    track.msToProcessCT_1ms, track.ctPOS = 300, 400  # 300 ms + 100 x 10 ms > 400 ms
    A = acquired_of([16], [26051], [4579675.0])
    with pytest.raises(pkg.abi.GnssError) as e:  # short read: MATLAB raises
        pkg.trackingCT_POS(file, signal, track, A, [3], ctx=ctx)
    assert e.value.status == pkg.abi.EIO
    file.dataPrecision = 2
    with pytest.raises(pkg.abi.GnssError) as e:
        pkg.trackingCT_POS(file, signal, track, A, [3], ctx=ctx)
    assert e.value.status == pkg.abi.EARG
