"""GPU parity of the vector-tracking step (gnss_tracking_vt_step) against the
oracle's restatement (or_vt_step, itself pinned by the reference's tckRstVT output in
tests/test_vt_kat.py): 3 channels x 300 closed-loop 1-ms steps on the synthetic Opensky
record, the code frequency of every step given (a constant stand-in for the caller's EKF
prediction, trackingVT_POS_updated.m:211-215). Read sizes, file offsets and codedelay
bit-exact; the carrier-wiped sums (exact per-sample Wave on both sides, fp64 block sums on
the GPU, long-double sums in the oracle) and the NCO / PLL state within 1e-9."""
import numpy as np
import pytest

from conftest import params

pytestmark = pytest.mark.gpu


def test_vt_steps_against_oracle(pkg, po, ctx, opensky_short):
    skip, cfg, data = opensky_short
    file, signal, acq, track = params(pkg, skip, data)
    S = 58000
    prns, cds, ffs = [3, 16, 26], [3684, 26051, 57908], [4580975.0, 4579675.0, 4581800.0]
    chans = [pkg.vt_channel(p, (S - cd + 1 + skip * S) * 2, 0.0, 0.0, 1.023e6, f, f)
             for p, cd, f in zip(prns, cds, ffs)]
    st = [np.array([c.file_ptr, 0.0, 0.0, 1.023e6, c.carrFreq, c.carrFreqBasis, 0.0, 0.0]) for c in chans]
    cf = [1.023e6] * 3
    iq = np.ascontiguousarray(data, dtype=np.int8)
    worst = 0.0
    for k in range(300):
        g = pkg.trackingVT_step(file, signal, track, chans, cf, ctx=ctx)
        for i, prn in enumerate(prns):
            status, rec = po.vt_step(st[i], cf[i], prn, iq=iq)
            assert status == 0
            R = dict(zip(po.VT_REC, rec))
            for f in ("numSample", "absoluteSample", "codedelay"):
                assert g[i][f] == R[f], (k, prn, f)
            scale = max(abs(R["P_i"]), abs(R["P_q"]), 1.0)
            for f in ("E_i", "E_q", "P_i", "P_q", "L_i", "L_q"):
                worst = max(worst, abs(g[i][f] - R[f]) / scale)
            for f in ("remChip", "remCarrPhase", "codeFreq", "carrFreq", "carrNco", "carrError", "codeError"):
                assert np.isclose(g[i][f], R[f], rtol=1e-9, atol=1e-9), (k, prn, f, g[i][f], R[f])
    print("worst sum error / |P|", worst)
    assert worst < 1e-9
