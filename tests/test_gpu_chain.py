"""The whole in-scope chain of SDR_main.m (acquisition -> trackingCT -> naviDecode_updated,
SDR_main.m:20-56) on the GPU, on a synthetic Opensky record whose SVs carry the synthetic
LNAV message (gnss_synth_sv.lnav; csrc/lnav.cpp): the decoded ephemeris must be the one the
message encodes. The decoder itself is pinned by the reference's eph/sbf files
(tests/test_navdecode.py); this checks the GPU tracking output feeds it correctly.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_acquire_track_decode_synthetic_lnav(pkg, ctx):
    file, signal, acq, track, _, _ = pkg.initParameters()
    skip, N10 = 100, 45000  # (5 subframes after the first preamble need ~40 s of P_i)
    cfg = pkg.synth.opensky(skip_ms=skip)
    for i in range(cfg.n_sv):
        cfg.sv[i].lnav = 1
    dev = pkg.DeviceRecord(ctx, (skip + 1000 + 19 + N10 + 3) * signal.Sample * 2)
    pkg.synth.generate_device(ctx, cfg, dev)
    file.skip, file.dev = skip, dev
    acq.freqMin, acq.freqNum = -7000, 29
    A = pkg.acquisition(file, signal, acq, ctx=ctx)
    assert list(A.sv) == [3, 4, 16, 22, 26, 27, 31, 32]
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, N10
    T, cn0, cx = pkg.trackingCT(file, signal, track, A, ctx=ctx)
    eph, _, for_prest = pkg.naviDecode_updated(A, T)
    decoded = [int(p) for p in A.sv if eph(int(p)).updateflag == 1]
    # (a channel whose loops do not settle on this record decodes nothing — the same
    # happens in the reference's own run, PRN 32 of eph_Opensky_90.mat; here PRNs 4 and 27,
    # which the CPU oracle loses too on the same record: profiles/r02_lnav_lock_oracle.txt)
    assert len(decoded) >= 5, decoded
    for prn in decoded:
        e = eph(prn)
        for f in pkg.synth.LNAV_FIELDS:
            vals = getattr(e, f)
            want = pkg.synth.lnav_expected(f)
            assert len(vals) > 0 and vals[0] == want, (prn, f, vals[:3], want)
            assert np.mean(vals == want) > 0.8, (prn, f)
        assert (e.TOW[0] - pkg.synth.LNAV_TOW0) % 6 == 0
