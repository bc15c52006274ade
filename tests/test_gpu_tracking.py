"""GPU parity for trackingCT (through the C-ABI) against the CPU oracle.

Tolerances: integer / index fields (numSample, delayValue, absoluteSample,
codedelay, codedelay2, countinx) bit-exact; P/E/L I/Q series within 1e-5 of the
series RMS (north-star tolerance) — and, as a regression guard on the fp64
design, within 1e-8; NCO state (remChip, codeFreq, carrierFreq, remPhase, ...)
within 1e-7 relative / 1e-9 absolute; CN0 within 1e-6 dB. (Closed-loop: the
discriminators feed 1-ulp libm differences (atan) back into the NCOs, so late
steps of a weak channel drift apart at the 1e-10 level.)
"""
import os
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import GOLDEN, acquired_of, params

pytestmark = pytest.mark.gpu

INT_FIELDS = ["codedelay", "numSample", "delayValue", "absoluteSample", "codedelay2"]
NCO_FIELDS = ["remChip", "codeFreq", "carrierFreq", "remPhase", "remSample", "PLLdiscri", "DLLdiscri"]


def compare(pkg, g, r, tol=1e-8):
    F = pkg.abi.FIELDS
    assert np.array_equal(g.len, r.len)
    assert np.array_equal(g.countinx, r.countinx)
    for c in range(len(g.len)):
        n = int(r.len[c])
        if n == 0:
            continue
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


OPENSKY_A = dict(svs=[3, 4, 16, 22, 26, 27, 31, 32],
                 cd=[3684, 12700, 26051, 2611, 57908, 49777, 39064, 20170],
                 ff=[4580975.0, 4576875.0, 4579675.0, 4581525.0, 4581800.0, 4576750.0, 4581025.0,
                     4583325.0])


def test_tracking_parity_opensky_8ch(pkg, po, ctx, opensky_short):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, 1000
    A = acquired_of(OPENSKY_A["svs"], OPENSKY_A["cd"], OPENSKY_A["ff"])
    g = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    r = po.trackingCT(file, signal, track, A, raw=True)
    assert r.status == 0
    compare(pkg, g, r)
    # the mirror's struct view (TckResultCT(prn).P_i) over the same buffers
    T, cn0, cx = pkg.trackingCT(file, signal, track, A, ctx=ctx)
    assert T.prns() == sorted(OPENSKY_A["svs"])
    assert len(T(16).P_i) == 1000 + cx[2] + 1000


@pytest.mark.parametrize("persist", [True, False], ids=["persistent", "step"])
@pytest.mark.parametrize("sub", ["1", "2", "3", "4"])
def test_tracking_parity_every_kernel_variant(pkg, po, ctx, opensky_short, opts, sub, persist):
    """Every lane span, through the persistent step loop and through one launch per step."""
    opts(pkg.abi.OPT_FORCE_SUB, int(sub))
    if not persist:
        opts(pkg.abi.OPT_NO_PERSIST, 1)
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 300
    A = acquired_of([16, 26, 31], [26051, 57908, 39064], [4579675.0, 4581800.0, 4581025.0])
    g = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    r = po.trackingCT(file, signal, track, A, raw=True)
    compare(pkg, g, r)


def test_persistent_loop_runs_the_bench_shape(pkg, po, ctx, opensky_short):
    """8 channels (the bench's trackingCT shape): each phase run is one persistent launch
    (the step kernel would take one launch per step), with the same outputs."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 1000
    A = acquired_of(OPENSKY_A["svs"], OPENSKY_A["cd"], OPENSKY_A["ff"])
    g = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    assert ctx.timing()["track_launches"] <= 4
    r = po.trackingCT(file, signal, track, A, raw=True)
    compare(pkg, g, r)


def test_tracking_parity_11_taps(pkg, po, ctx, opensky_short):
    """Config-5 ACF taps -0.5:0.1:0.5 (E = tap 0, P = tap 5, L = tap 10)."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 300
    taps = po.colon(-0.5, 0.1, 0.5)
    A = acquired_of([3, 26], [3684, 57908], [4580975.0, 4581800.0])
    g = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
    r = po.trackingCT(file, signal, track, A, taps=taps, raw=True)
    compare(pkg, g, r)
    for c in range(2):
        n = int(r.len[c])
        scale = np.sqrt(np.mean(r.taps[c, :, :, :n] ** 2))
        assert np.max(np.abs(g.taps[c, :, :, :n] - r.taps[c, :, :, :n])) / scale < 1e-10
        # E/P/L rows of the record are taps 0 / 5 / 10
        assert np.array_equal(g.rec[c, 0, :n], g.taps[c, 0, 5, :n])
        assert np.array_equal(g.rec[c, 2, :n], g.taps[c, 0, 0, :n])
        assert np.array_equal(g.rec[c, 5, :n], g.taps[c, 1, 10, :n])


def test_tracking_parity_25_taps(pkg, po, ctx, opensky_short):
    """The 25 taps of trackingCT_multiCorr-GIVEN.m:25 (Spacing = -0.6:0.05:0.6; E = Spacing(3)
    = -0.5, P = (13), L = (23) = +0.5) on trackingCT's loop, both phases (step kernel)."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 300
    taps = po.colon(-0.6, 0.05, 0.6)
    assert len(taps) == 25 and (taps[2], taps[12], taps[22]) == (-0.5, 0.0, 0.5)
    A = acquired_of([3, 26], [3684, 57908], [4580975.0, 4581800.0])  # (bit edges within 700 ms)
    g = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
    r = po.trackingCT(file, signal, track, A, taps=taps, raw=True)
    assert r.status == 0
    compare(pkg, g, r)
    for c in range(2):
        n = int(r.len[c])
        scale = np.sqrt(np.mean(r.taps[c, :, :, :n] ** 2))
        assert np.max(np.abs(g.taps[c, :, :, :n] - r.taps[c, :, :, :n])) / scale < 1e-10
        assert np.array_equal(g.rec[c, 0, :n], g.taps[c, 0, 12, :n])
        assert np.array_equal(g.rec[c, 2, :n], g.taps[c, 0, 2, :n])
        assert np.array_equal(g.rec[c, 5, :n], g.taps[c, 1, 22, :n])


def test_correlate_step_random_states(pkg, po, ctx, opensky_short):
    import importlib
    sdr = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd.sdr")
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    rng = np.random.default_rng(11)
    for trial in range(30):
        prn = int(rng.choice([3, 4, 16, 22, 26, 27, 31, 32]))
        pdi = 10 if trial % 3 == 0 else 1
        rc = float(rng.uniform(-0.009, 0.009))
        cf = 1.023e6 + float(rng.normal(0, 5))
        f = 4.58e6 + float(rng.uniform(-5000, 5000))
        ph = float(rng.uniform(0, 2 * np.pi))
        pos = 2 * int(rng.integers(0, 2000 * 58000))
        taps = po.colon(-0.5, 0.1, 0.5) if trial % 2 else np.array([-0.5, 0.0, 0.5])
        g, ns = sdr.correlate_step(file, signal, prn, pdi, rc, cf, f, ph, pos, taps, ctx=ctx)
        n = int(np.round((1023.0 * pdi - rc) / (cf / 58e6)))
        assert ns == n
        r = po.correlate_step(data[pos:pos + 2 * n], n, rc, cf, 58e6, f, ph, po.generate_ca(prn),
                              pdi, taps)
        assert np.max(np.abs(g - r)) / np.sqrt(np.mean(r ** 2)) < 1e-12


def test_tracking_matches_golden_vectors(pkg, po, ctx):
    from test_golden_oracle import check_track_against_golden, golden_record
    g, data = golden_record(pkg, po)
    file, signal, acq, track = params(pkg, int(g["skip"]), data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = int(g["N1"]), int(g["N10"])
    A = SimpleNamespace(sv=g["sv"], SNR=np.zeros(2), Doppler=np.zeros(2), codedelay=g["codedelay"],
                        fineFreq=g["fineFreq"])
    b = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    check_track_against_golden(pkg, g, b.rec, b.len, b.countinx, b.CN0[: b.c.cn0_rows])


def test_channel_shards_equal_full_run(pkg, ctx, opensky_short):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 200
    A = acquired_of([3, 16, 22], [3684, 26051, 2611], [4580975.0, 4579675.0, 4581525.0])
    full = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    a = pkg.trackingCT(file, signal, track, A, ctx=ctx, channels=[0, 2], raw=True)
    b = pkg.trackingCT(file, signal, track, A, ctx=ctx, channels=[1], raw=True)
    for c, part in ((0, a), (1, b), (2, a)):
        assert np.array_equal(full.rec[c], part.rec[c])
        assert full.len[c] == part.len[c] and full.countinx[c] == part.countinx[c]


def test_persistent_and_step_paths_bit_identical(pkg, ctx, opensky_short, opts):
    """The persistent loop and one launch per step share the lane geometry and both
    fixed-order reductions: the same records to the last bit."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 300
    A = acquired_of([3, 16, 22], [3684, 26051, 2611], [4580975.0, 4579675.0, 4581525.0])
    p = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    assert ctx.timing()["track_launches"] <= 4
    opts(pkg.abi.OPT_NO_PERSIST, 1)
    q = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    assert ctx.timing()["track_launches"] > 100
    for c in range(3):
        assert np.array_equal(p.rec[c], q.rec[c])
        assert p.len[c] == q.len[c] and p.countinx[c] == q.countinx[c]


def test_reused_output_buffers(pkg, ctx, opensky_short):
    """trackingCT(out=...) writes the same records into a buffer from an earlier call."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 200
    A1 = acquired_of([3, 16], [3684, 26051], [4580975.0, 4579675.0])
    A2 = acquired_of([22, 26], [2611, 57908], [4581525.0, 4581800.0])
    fresh = pkg.trackingCT(file, signal, track, A2, ctx=ctx, raw=True)
    buf = pkg.trackingCT(file, signal, track, A1, ctx=ctx, raw=True)
    again = pkg.trackingCT(file, signal, track, A2, ctx=ctx, raw=True, out=buf)
    assert again is buf
    assert np.array_equal(fresh.rec, again.rec) and np.array_equal(fresh.CN0, again.CN0)
    assert np.array_equal(fresh.len, again.len) and np.array_equal(fresh.countinx, again.countinx)


def test_not_enough_raw_data_in_1ms_phase(pkg, ctx, opensky_short):
    """trackingCT.m:108-112: short record in the 1-ms phases -> TckResultCT = []."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 600])
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, 100
    A = acquired_of([16], [26051], [4579675.0])
    T, cn0, cx = pkg.trackingCT(file, signal, track, A, ctx=ctx)
    assert not T and len(T.prns()) == 0


def test_read_past_eof_in_10ms_phase_raises(pkg, ctx, opensky_short):
    """trackingCT.m:442 has no length check: MATLAB errors -> GNSS_EIO."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 1200])
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, 1000
    A = acquired_of([16], [26051], [4579675.0])
    with pytest.raises(pkg.abi.GnssError) as e:
        pkg.trackingCT(file, signal, track, A, ctx=ctx)
    assert e.value.status == pkg.abi.EIO


def test_argument_errors_raise(pkg, ctx, opensky_short):
    """Nothing acquired: trackingCT.m:20-22 tracks no channel and never assigns TckResultCT,
    so MATLAB stops with an unassigned-output error -> GNSS_EARG. So do a channel index past
    Acquired.sv (the shard list) and tap sets the loops cannot run on: a count other than
    3 / 11 / 25, and three taps without -spacing, 0, +spacing (no E / P / L,
    trackingCT.m:24)."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 1400])
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 200
    A = acquired_of([26], [57908], [4581800.0])
    sp = float(track.CorrelatorSpacing)
    for kw, Aq in [({}, acquired_of([], [], [])), (dict(channels=[1]), A), (dict(channels=[-1]), A),
                   (dict(taps=[-sp, 0.0, sp, 2 * sp]), A), (dict(taps=[-sp / 2, 0.0, sp / 2]), A)]:
        with pytest.raises(pkg.abi.GnssError) as e:
            pkg.trackingCT(file, signal, track, Aq, ctx=ctx, **kw)
        assert e.value.status == pkg.abi.EARG, kw
    # and the context is still usable afterwards
    T, cn0, cx = pkg.trackingCT(file, signal, track, A, ctx=ctx)
    assert T.prns() == [26]


def test_wide_tap_set_is_an_index_error(pkg, ctx, opensky_short):
    """11 taps spanning more than the persistent loop's 30-chip tap window (kTapSpan) are no
    argument error: they take the per-step path, where a tap 16 chips early indexes
    Code(ceil(t) + 1) below 1 on the first step, MATLAB's index error (trackingCT.m:96-100) ->
    GNSS_EINDEX. The context stays usable."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 1400])
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 200
    A = acquired_of([26], [57908], [4581800.0])
    taps = list(pkg.colon(-0.5, 0.1, 0.5))
    taps[1], taps[-2] = -16.0, 16.0  # (E, P, L at -0.5, 0, 0.5 stay)
    with pytest.raises(pkg.abi.GnssError) as e:
        pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps)
    assert e.value.status == pkg.abi.EINDEX
    T, cn0, cx = pkg.trackingCT(file, signal, track, A, ctx=ctx)
    assert T.prns() == [26]


def test_file_route_positioned_reads(pkg, ctx, opensky_short, tmp_path):
    """file.fileRoute path (positioned reads) == in-memory record."""
    skip, cfg, data = opensky_short
    p = tmp_path / "Opensky.bin"
    data[: 2 * 58000 * 1400].tofile(p)
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 1400])
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 200
    A = acquired_of([26], [57908], [4581800.0])
    a = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    file.data, file.fileRoute = None, str(p)
    b = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    assert np.array_equal(a.rec, b.rec)


def test_config5_shape_32_channels_11_taps(pkg, po, ctx):
    """BASELINE config 5's shape at reduced length: 32 channels (every PRN present), the 11
    ACF taps -0.5:0.1:0.5, one GPU (the persistent loop with several of the step's blocks
    per resident block: 32 x 96 blocks would not all be resident), against the oracle."""
    from types import SimpleNamespace
    skip, N1, N10 = 0, 1000, 20  # (the bit-edge search window of trackingCT.m:179-204: the channels
    # are locked, the first data-bit edge after 600 ms can lie well past it)
    cfg = pkg.synth.all_prn(32, skip_ms=skip)
    data = po.synth_if(cfg, 0, (skip + N1 + 19 + N10 + 4) * 58000)
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = N1, N10
    cds = pkg.synth.codedelays(cfg, skip)
    A = SimpleNamespace(sv=np.array([cfg.sv[i].prn for i in range(32)]), SNR=np.zeros(32),
                        Doppler=np.zeros(32), codedelay=np.array(cds),
                        fineFreq=np.array([4.58e6 + cfg.sv[i].doppler_hz for i in range(32)]))
    taps = pkg.colon(-0.5, 0.1, 0.5)
    assert np.array_equal(taps, po.colon(-0.5, 0.1, 0.5))
    g = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
    assert ctx.timing()["track_launches"] <= 4  # persistent, not one launch per step
    r = po.trackingCT(file, signal, track, A, taps=taps, raw=True)
    assert r.status == 0
    compare(pkg, g, r)


@pytest.mark.parametrize("route", ["host", "path"])
def test_streamed_windows_equal_resident(pkg, ctx, opensky_short, tmp_path, route):
    """Streaming (gnss_ctx_set_window): a 100 MB HBM window over a ~200 MB read range -- the
    1-ms phases' range staged first, the 10-ms phase in segments staged through the pinned
    double buffer -- gives the same bits as the whole range resident, from host memory and
    from the file (trackingCT.m:84-93,416-426 read every step from the file)."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 1000
    A = acquired_of([16, 26, 31], [26051, 57908, 39064], [4579675.0, 4581800.0, 4581025.0])
    g0 = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    if route == "path":
        p = tmp_path / "if.bin"
        p.write_bytes(np.asarray(data, dtype=np.int8).tobytes())
        file.data, file.fileRoute = None, str(p)
    ctx.set_window(100 * 1000 * 1000)
    try:
        g1 = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
        t = ctx.timing()
    finally:
        ctx.set_window(0)
    assert t["track_segments"] >= 2 and t["h2d_bytes"] > 0
    assert np.array_equal(g0.len, g1.len) and np.array_equal(g0.countinx, g1.countinx)
    for c in range(3):
        n = int(g0.len[c])
        assert np.array_equal(g0.rec[c, :, :n], g1.rec[c, :, :n]), c
    assert np.array_equal(g0.CN0, g1.CN0)


@pytest.mark.parametrize("ntaps,vpb", [(3, 4), (11, 3)])
def test_virtual_blocks_bit_identical(pkg, ctx, opensky_short, opts, ntaps, vpb):
    """The persistent loop with several of the step's blocks per resident block (how 32
    channels x 11 taps stay persistent on one GPU) gives the same records as one block each
    and as the per-step path."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 300
    taps = pkg.colon(-0.5, 0.1, 0.5) if ntaps == 11 else None
    A = acquired_of([3, 16, 22], [3684, 26051, 2611], [4580975.0, 4579675.0, 4581525.0])
    p = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
    opts(pkg.abi.OPT_FORCE_VPB, vpb)
    v = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
    assert ctx.timing()["track_launches"] <= 4
    opts(pkg.abi.OPT_FORCE_VPB, 0)
    opts(pkg.abi.OPT_NO_PERSIST, 1)
    q = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
    for c in range(3):
        assert np.array_equal(p.rec[c], v.rec[c]) and np.array_equal(q.rec[c], v.rec[c]), c
        assert p.len[c] == v.len[c] and p.countinx[c] == v.countinx[c]
        if ntaps == 11:  # (the persistent loop writes the non-E/P/L taps one step late: same bits)
            assert np.array_equal(p.taps[c], v.taps[c]) and np.array_equal(q.taps[c], v.taps[c]), c
    assert np.array_equal(p.CN0, v.CN0)
