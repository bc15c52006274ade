"""GPU parity for the IF record formats (initParameters.m:35-38,
acquisition.m:28-37 / :90-99, trackingCT.m:84-93): int16 I/Q (per-read mean removal) and
int8 real records, against the CPU oracle, through the C-ABI. Same tolerances as
test_gpu_acquisition / test_gpu_tracking (decisions and integer fields bit-exact)."""
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import acquired_of
from test_gpu_acquisition import compare as compare_acq
from test_gpu_tracking import compare as compare_trk

pytestmark = pytest.mark.gpu

FORMATS = [(2, 2), (1, 1)]
FMT_IDS = ["int16-iq", "int8-real"]


def _file(pkg, rec, skip, prec, dtyp):
    return SimpleNamespace(skip=skip, dataType=dtyp, dataPrecision=prec, data=rec, fileRoute=None, dev=None)


@pytest.fixture(scope="module")
def opensky_acq(pkg, po):
    skip = 4
    cfg = pkg.synth.opensky(skip_ms=skip)
    return skip, po.synth_if(cfg, 0, (skip + 12) * 58000)


@pytest.mark.parametrize("prec,dtyp", FORMATS, ids=FMT_IDS)
@pytest.mark.parametrize("path", ["own-fft", "rocfft"])
def test_acquisition_formats(pkg, po, ctx, opensky_acq, opts, prec, dtyp, path):
    if path == "rocfft":
        opts(pkg.abi.OPT_ACQ_ROCFFT, 1)
        opts(pkg.abi.OPT_FINE_ROCFFT, 1)
    skip, iq8 = opensky_acq
    rec = pkg.synth.convert_record(iq8, prec, dtyp)
    file = _file(pkg, rec, skip, prec, dtyp)
    _, signal, acq, _, _, _ = pkg.initParameters()
    acq.freqMin, acq.freqNum, acq.freqStep, acq.datalen, acq.L = -5000, 21, 500, 4, 10
    prns = [3, 16, 26, 5]
    g, gd = pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=prns, diag=True)
    r, rd = po.acquisition(file, signal, acq, prn_list=prns, diag=True)
    compare_acq(g, gd, r, rd)
    assert {3, 16, 26} <= set(g.sv)


def test_acquisition_int16_real_status(pkg, ctx, opensky_acq):
    skip, iq8 = opensky_acq
    rec = pkg.synth.convert_record(iq8, 2, 1)
    _, signal, acq, _, _, _ = pkg.initParameters()
    acq.datalen = 4
    with pytest.raises(pkg.abi.GnssError) as e:
        pkg.acquisition(_file(pkg, rec, skip, 2, 1), signal, acq, ctx=ctx, prn_list=[3])
    assert e.value.status == pkg.abi.EINDEX


@pytest.fixture(scope="module")
def opensky_trk(pkg, po):
    skip = 5
    cfg = pkg.synth.opensky(skip_ms=skip)
    n_ms = skip + 300 + 19 + 200 + 4
    return skip, po.synth_if(cfg, 0, n_ms * 58000)


@pytest.mark.parametrize("prec,dtyp", FORMATS, ids=FMT_IDS)
@pytest.mark.parametrize("sub", ["default", "1"])
def test_tracking_formats(pkg, po, ctx, opensky_trk, opts, prec, dtyp, sub):
    """300 ms @1 ms + 200 ms @10 ms, 3 channels; int16 runs the per-step kernel with the
    mean of every read from prefix sums, int8 real the int8 kernels on (x, 0) pairs."""
    if sub != "default":
        opts(pkg.abi.OPT_FORCE_SUB, int(sub))
    skip, iq8 = opensky_trk
    rec = pkg.synth.convert_record(iq8, prec, dtyp)
    file = _file(pkg, rec, skip, prec, dtyp)
    _, signal, _, track, _, _ = pkg.initParameters()
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 300, 200
    A = acquired_of([16, 26, 31], [26051, 57908, 39064], [4579675.0, 4581800.0, 4581025.0])
    g = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
    r = po.trackingCT(file, signal, track, A, raw=True)
    assert r.status == 0
    compare_trk(pkg, g, r)
    # absoluteSample advances by numSample * bytes per sample (ftell)
    F = pkg.abi.FIELDS
    n = int(r.len[0])
    pos = g.rec[0, F.index("absoluteSample"), :n]
    ns = g.rec[0, F.index("numSample"), :n]
    assert np.array_equal(np.diff(pos[:300]), ns[1:300] * prec * dtyp)


def test_tracking_int16_real_status(pkg, ctx, opensky_trk):
    skip, iq8 = opensky_trk
    rec = pkg.synth.convert_record(iq8[: 2 * 58000 * 60], 2, 1)
    _, signal, _, track, _, _ = pkg.initParameters()
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 30, 0
    A = acquired_of([16], [26051], [4579675.0])
    # numSample = 58000 (even): fewer samples than carrier values -> TckResultCT = []
    T, cn0, cx = pkg.trackingCT(_file(pkg, rec, 0, 2, 1), signal, track, A, ctx=ctx)
    assert not T
