"""The multi-device C-ABI context (gnss_ctx_create_multi): a MEX caller of SDR_main.m:22,38 that
hands the library several devices gets the PRN loop of acquisition.m:47-80 and the channel loop
of trackingCT.m:22-528 dealt over one member context per device, with results bit-identical to
one context. The GPU box has one device, so the members here are {0, 0} / {0, 0, 0} (members
of one device run one after the other), and GNSS_OPT_FORCE_PEER routes the dev_data record and
GNSS_OUT_DEVICE rows through the peer-copy path a member on another device takes."""
import numpy as np
import pytest

from conftest import acquired_of, params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mctx(pkg, ctx):
    c = pkg.Context(devices=[0, 0, 0])
    assert c.members == 3
    yield c
    c.close()


def _same_acq(a, b):
    for f in ("sv", "SNR", "Doppler", "codedelay", "fineFreq"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_multi_context_acquisition_equals_one(pkg, ctx, mctx, opensky_short):
    """32 PRNs dealt over three members (11 / 11 / 10): Acquired and every diag row equal the
    one-context call bit for bit, in PRN-list order; an explicit PRN list too."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    acq.freqMin, acq.freqNum, acq.freqStep, acq.datalen, acq.L = -7000, 29, 500, 8, 10
    g1, d1 = pkg.acquisition(file, signal, acq, ctx=ctx, diag=True)
    g3, d3 = pkg.acquisition(file, signal, acq, ctx=mctx, diag=True)
    _same_acq(g1, g3)
    for f in ("prn", "SNR", "fbin", "codePhase", "peak", "peak2"):
        assert np.array_equal(getattr(d1, f), getattr(d3, f)), f
    assert len(g1.sv) >= 6
    t = mctx.timing()
    assert t["acq_hypothesis_samples"] == 32 * 29 * 8 * 58000  # (summed over the members)
    lst = [26, 3, 31, 16, 22]
    _same_acq(pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=lst),
              pkg.acquisition(file, signal, acq, ctx=mctx, prn_list=lst))


def test_multi_context_tracking_equals_one(pkg, ctx, mctx, opensky_short):
    """Five channels over three members, 11 ACF taps: records, taps, C/N0, countinx and lengths
    equal the one-context call bit for bit; a channel subset as well."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 300
    A = acquired_of([3, 16, 22, 26, 31], [3684, 26051, 2611, 57908, 39064],
                    [4580975.0, 4579675.0, 4581525.0, 4581800.0, 4581025.0])
    taps = pkg.colon(-0.5, 0.1, 0.5)
    one = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
    grp = pkg.trackingCT(file, signal, track, A, ctx=mctx, taps=taps, raw=True)
    assert np.array_equal(one.rec, grp.rec) and np.array_equal(one.taps, grp.taps)
    assert np.array_equal(one.CN0, grp.CN0) and one.c.cn0_rows == grp.c.cn0_rows
    assert np.array_equal(one.len, grp.len) and np.array_equal(one.countinx, grp.countinx)
    sub = pkg.trackingCT(file, signal, track, A, ctx=mctx, taps=taps, raw=True, channels=[4, 1])
    for c in (1, 4):
        assert np.array_equal(one.rec[c], sub.rec[c]) and np.array_equal(one.taps[c], sub.taps[c])


def test_multi_context_device_io_peer_path(pkg, ctx, mctx, opensky_short, tmp_path):
    """The record resident in HBM (dev_data) and GNSS_OUT_DEVICE rows, through the peer-copy
    path (GNSS_OPT_FORCE_PEER: each member copies its read range in and its rows out as a member
    on another device does over xGMI): bit-identical to one context."""
    import torch
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 300
    A = acquired_of([3, 16, 22, 26], [3684, 26051, 2611, 57908], [4580975.0, 4579675.0, 4581525.0, 4581800.0])
    one = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    dev = pkg.DeviceRecord.from_host(mctx, data)
    file.data, file.dev = None, dev
    out = pkg.sdr.DeviceTrackOutBuffers(len(A.sv), track, 0)
    mctx.set_option(pkg.abi.OPT_FORCE_PEER, 1)
    try:
        pkg.trackingCT(file, signal, track, A, ctx=mctx, raw=True, out=out)
        t = mctx.timing()
    finally:
        mctx.set_option(pkg.abi.OPT_FORCE_PEER, 0)
        dev_keep = dev
    h = out.host()
    assert np.array_equal(one.rec, h.rec)
    assert np.array_equal(one.len, h.len) and np.array_equal(one.CN0, h.CN0)
    assert t["h2d_bytes"] > 0  # (the members' range copies)
    torch.cuda.synchronize()
    dev_keep.free()


def test_multi_context_record_stays_resident(pkg, ctx, mctx, opensky_short):
    """a member copies a dev_data record on another device (here: the
    FORCE_PEER path on one GPU) ONCE and keeps it -- the second call moves no bytes
    (h2d_bytes == 0) and gives the same bits; a write into the record through the library
    (gnss_dev_upload) drops the stale copies, the next call copies again and sees the new bytes;
    gnss_ctx_drop_record drops them explicitly (SDR_main.m:22,38 through INTEGRATION.md's MEX)."""
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 200
    A = acquired_of([3, 16, 22, 26], [3684, 26051, 2611, 57908], [4580975.0, 4579675.0, 4581525.0, 4581800.0])
    one = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    dev = pkg.DeviceRecord.from_host(mctx, data)
    file.data, file.dev = None, dev
    mctx.set_option(pkg.abi.OPT_FORCE_PEER, 1)
    try:
        assert mctx.resident_records == 0
        a = pkg.trackingCT(file, signal, track, A, ctx=mctx, raw=True)
        t1 = mctx.timing()
        assert mctx.resident_records == 3  # (one copy per member: every member read the record)
        b = pkg.trackingCT(file, signal, track, A, ctx=mctx, raw=True)
        t2 = mctx.timing()
        assert t1["h2d_bytes"] == 3 * data.nbytes and t2["h2d_bytes"] == 0
        assert np.array_equal(a.rec, one.rec) and np.array_equal(b.rec, one.rec)
        # the acquisition reads the same resident copies
        acq.freqMin, acq.freqNum, acq.freqStep, acq.datalen, acq.L = -7000, 29, 500, 4, 10
        g1 = pkg.acquisition(file, signal, acq, ctx=mctx, prn_list=[3, 16, 22, 26])
        assert mctx.timing()["h2d_bytes"] == 0
        # rewrite the record through the library (every byte negated): the copies are dropped and
        # the next call tracks the new bytes
        z = np.clip(-data.astype(np.int16), -128, 127).astype(np.int8)
        dev.upload(z)
        assert mctx.resident_records == 0
        c = pkg.trackingCT(file, signal, track, A, ctx=mctx, raw=True)
        assert mctx.timing()["h2d_bytes"] == 3 * data.nbytes
        ref = pkg.trackingCT(params(pkg, skip, z)[0], signal, track, A, ctx=ctx, raw=True)
        assert np.array_equal(c.rec, ref.rec) and not np.array_equal(c.rec, one.rec)
        mctx.drop_record(dev)
        assert mctx.resident_records == 0
        pkg.acquisition(file, signal, acq, ctx=mctx, prn_list=[3, 16, 22, 26])
        assert mctx.resident_records == 3 and mctx.timing()["h2d_bytes"] == 3 * data.nbytes
        mctx.drop_record(None)
        assert mctx.resident_records == 0
        del g1
    finally:
        mctx.set_option(pkg.abi.OPT_FORCE_PEER, 0)
        dev.free()


def test_multi_context_errors_match_one(pkg, ctx, mctx, opensky_short):
    """A short record: the sharded call returns the one-context status (GNSS_EIO for the 10-ms
    phase's read past EOF, trackingCT.m:442) and the group stays usable; bad device lists are
    GNSS_EARG."""
    import ctypes as C
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data[: 2 * 58000 * 1200])
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, 1000
    A = acquired_of([16, 26], [26051, 57908], [4579675.0, 4581800.0])
    codes = []
    for c in (ctx, mctx):
        with pytest.raises(pkg.abi.GnssError) as e:
            pkg.trackingCT(file, signal, track, A, ctx=c)
        codes.append(e.value.status)
    assert codes[0] == codes[1] == pkg.abi.EIO
    lib = pkg.abi.load()
    h = C.c_void_p()
    import torch
    for devs in ([], [0] * 17, [torch.cuda.device_count()], [-1]):
        arr = (C.c_int * max(1, len(devs)))(*(devs or [0]))
        assert lib.gnss_ctx_create_multi(arr, len(devs), C.byref(h)) != 0, devs
    file, signal, acq, track = params(pkg, skip, data)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 700, 100
    T, cn0, cx = pkg.trackingCT(file, signal, track, A, ctx=mctx)
    assert T.prns() == [16, 26]


def test_multi_context_pos_and_mc_equal_one(pkg, ctx, mctx, opensky_short):
    """The sibling loops through the group context: trackingCT_POS_updated (per-channel
    1 000 + countinx 1-ms steps, then 10-ms to ctPOS) and the 25-tap
    trackingCT_POS_updated_multicorrelator (pdi 10) with the 8 Opensky channels dealt over three
    members: every record, tap, C/N0 row and length equal the one-context call bit for bit
    (trackingCT_POS_updated.m:179-413; trackingCT_POS_updated_multicorrelator.m)."""
    from test_gpu_pos import OPENSKY
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    A = acquired_of(OPENSKY["svs"], OPENSKY["cd"], OPENSKY["ff"])
    track.msToProcessCT_1ms, track.ctPOS = 1000, 1000 + 12 + 80
    one = pkg.trackingCT_POS(file, signal, track, A, OPENSKY["cx"], ctx=ctx, raw=True)
    grp = pkg.trackingCT_POS(file, signal, track, A, OPENSKY["cx"], ctx=mctx, raw=True)
    assert np.array_equal(one.rec, grp.rec) and np.array_equal(one.CN0, grp.CN0)
    assert np.array_equal(one.len, grp.len)
    track.msPosCT, track.pdi = 800, 10
    one = pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=ctx, raw=True)
    grp = pkg.trackingCT_POS_updated_multicorrelator(file, signal, track, A, ctx=mctx, raw=True)
    assert np.array_equal(one.rec, grp.rec) and np.array_equal(one.taps, grp.taps)
    assert np.array_equal(one.CN0, grp.CN0) and np.array_equal(one.len, grp.len)


def test_multi_context_vector_tracking_equals_one(pkg, ctx, mctx, opensky_short):
    """trackingVT_POS_updated on the multi-device context (the VT loop is one host-driven chain:
    it runs on devices[0]) equals the one-context call bit for bit over 200 steps, in
    loop mode (the persistent VT launch) on both."""
    import vt_nav_common as V
    from test_gpu_vtnav import _inputs
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    _, _, _, _, solu, cmn = pkg.initParameters()
    z = V.fixture()
    Acquired, eph, sbf, ct, ns = _inputs(pkg, z, skip)
    runs = [pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, V.cnslxyz(pkg), eph, sbf, None, ct,
                                       ns, ctx=c, nsteps=200) for c in (ctx, mctx)]
    (t1, n1), (t3, n3) = runs
    for p in (int(x) for x in z["prns"]):
        for f in ("P_i", "P_q", "carrFreq", "codeFreq", "absoluteSample", "deltaPr"):
            assert np.array_equal(getattr(t1(p), f), getattr(t3(p), f)), (p, f)
    for f in ("usrPos", "usrVel", "clkBias", "clkDrift", "state"):
        assert np.array_equal(getattr(n1, f), getattr(n3, f)), f
