"""IF record formats (initParameters.m:35-38; acquisition.m:28-37, :90-99;
trackingCT.m:84-93): int8 real, int16 I/Q with per-read mean removal, and the reference's
int16 + dataType 1 behaviour, on the CPU oracle against the numpy twin."""
from types import SimpleNamespace

import numpy as np
import pytest

import numpy_twin as tw

Fs, IF, S = 5.115e6, 1.25e6, 5115


def _scene(pkg, po, n_ms):
    cfg = pkg.synth.scenario([3, 16], [1200, 4000], [1500, -2500], [48, 47], Fs=Fs, IF=IF, skip_ms=0)
    return po.synth_if(cfg, 0, n_ms * S)


def _signal():
    return SimpleNamespace(IF=IF, Fs=Fs, codeFreqBasis=1.023e6, ms=1e-3, Sample=S, codelength=1023.0)


def test_read_samples_matlab_forming(pkg, po):
    iq8 = _scene(pkg, po, 1)
    b16 = pkg.synth.convert_record(iq8, 2, 2)
    x = tw.read_samples(b16, 2, 2, S)
    i16 = b16.view("<i2")[0::2].astype(float)
    assert np.array_equal(x.real, i16 - i16.mean())
    assert abs(np.mean(x.real)) < 1e-9 and abs(np.mean(x.imag)) < 1e-9
    r = tw.read_samples(pkg.synth.convert_record(iq8, 1, 1), 1, 1, S)
    assert np.array_equal(r.real, iq8[0::2].astype(float)) and not r.imag.any()
    # int16 real values are still de-interleaved: half as many samples
    assert len(tw.read_samples(pkg.synth.convert_record(iq8, 2, 1), 2, 1, 2 * (S // 2))) == S // 2


@pytest.mark.parametrize("prec,dtype", [(2, 2), (1, 1)])
def test_acquisition_formats_twin(pkg, po, prec, dtype):
    """Same peaks / SNR as the twin on the converted record (the SVs stay acquired)."""
    iq8 = _scene(pkg, po, 12)
    rec = pkg.synth.convert_record(iq8, prec, dtype)
    file = SimpleNamespace(skip=0, dataType=dtype, dataPrecision=prec, data=rec, fileRoute=None, dev=None)
    acq = SimpleNamespace(freqNum=13, freqMin=-3000, freqStep=500, datalen=3, L=2)
    A, d = po.acquisition(file, _signal(), acq, prn_list=[3, 7, 16], diag=True)
    x = tw.read_samples(rec, prec, dtype, 3 * S)
    tw_res = tw.acquisition(x, S, Fs, IF, 1.023e6, -3000, 500, 13, 3, [3, 7, 16])
    for k, (prn, fbin, cp, snr) in enumerate(tw_res):
        assert d.prn[k] == prn and d.fbin[k] == fbin and d.codePhase[k] == cp
        assert abs(d.SNR[k] - snr) < 1e-9
    assert {3, 16} <= set(A.sv)
    if dtype == 1:
        # real record: unshifted fft, FreqPeakIndex * Fs/N (acquisition.m:108-119); the
        # lower of the two mirror bins -> +(IF + Doppler), one bin high (1-based index)
        binw = Fs / (acq.L * S * acq.datalen)
        for sv, ff in zip(A.sv, A.fineFreq):
            fd = {3: 1500, 16: -2500}.get(int(sv))
            if fd is not None:
                assert abs(ff - binw - (IF + fd)) <= binw / 2 + 1e-6


def test_acquisition_int16_real_is_matlab_index_error(pkg, po):
    iq8 = _scene(pkg, po, 4)
    rec = pkg.synth.convert_record(iq8, 2, 1)
    file = SimpleNamespace(skip=0, dataType=1, dataPrecision=2, data=rec, fileRoute=None, dev=None)
    acq = SimpleNamespace(freqNum=3, freqMin=-500, freqStep=500, datalen=2, L=1)
    with pytest.raises(pkg.abi.GnssError) as e:
        po.acquisition(file, _signal(), acq, prn_list=[3])
    assert e.value.status == pkg.abi.EINDEX


def _track_args(pkg, n1=30, n10=20):
    file, signal, acq, track, _, _ = pkg.initParameters()
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = n1, n10
    A = SimpleNamespace(sv=np.array([3]), SNR=np.zeros(1), Doppler=np.zeros(1),
                        codedelay=np.array([1200]), fineFreq=np.array([IF + 1500.0]))
    return track, A


@pytest.mark.parametrize("prec,dtype", [(2, 2), (1, 1)])
def test_tracking_first_step_formats_twin(pkg, po, prec, dtype):
    """The first trackingCT step on a converted record = the twin's correlator on the
    samples the twin reads (mean removed per read for int16)."""
    iq8 = _scene(pkg, po, 60)
    rec = pkg.synth.convert_record(iq8, prec, dtype)
    file = SimpleNamespace(skip=0, dataType=dtype, dataPrecision=prec, data=rec, fileRoute=None, dev=None)
    track, A = _track_args(pkg)
    T, cn0, cx = po.trackingCT(file, _signal(), track, A)
    r = T(3)
    n = int(r.numSample[0])
    bps = prec * dtype
    pos0 = (S - 1200 + 1) * bps  # trackingCT.m:63 (skip 0)
    assert r.absoluteSample[0] == pos0 + n * bps
    x = tw.read_samples(rec[pos0:], prec, dtype, n)
    ca = tw.ca_code(3)
    Code = np.concatenate([[ca[-1]], ca, [ca[0]]])
    d = 1.023e6 / Fs
    W = (2 * np.pi * (float(IF + 1500.0) * (np.arange(n + 1) / Fs))) + 0.0
    prod = x * np.exp(1j * W[:n])
    t = tw.colon(0.0, d, (n - 1) * d)
    code = Code[np.ceil(t).astype(int)]
    import math
    Pi, Pq = math.fsum(code * prod.imag), math.fsum(code * prod.real)
    scale = max(abs(Pi), abs(Pq))
    assert abs(r.P_i[0] - Pi) / scale < 1e-12 and abs(r.P_q[0] - Pq) / scale < 1e-12


def test_tracking_int16_real_reference_behaviour(pkg, po):
    """int16 + dataType 1: fread(numSample, 'int16') gives numSample/2 I/Q samples. Odd
    numSample: I and Q halves of unequal length, MATLAB raises (EINDEX); even: the size
    check fails -> 'Not enough raw data', TckResultCT = [] (trackingCT.m:108-112)."""
    iq8 = _scene(pkg, po, 40)
    rec = pkg.synth.convert_record(iq8, 2, 1)
    file = SimpleNamespace(skip=0, dataType=1, dataPrecision=2, data=rec, fileRoute=None, dev=None)
    track, A = _track_args(pkg)
    buf = po.trackingCT(file, _signal(), track, A, raw=True)
    assert buf.status == pkg.abi.EINDEX  # numSample = 5115 here
    # an even numSample (5116: codeFreq a little below nominal) -> ENODATA
    sig = _signal()
    sig.codeFreqBasis = 1.023e6 * 5115 / 5116
    assert po.trackingCT(file, sig, track, A, raw=True).status == pkg.abi.ENODATA
