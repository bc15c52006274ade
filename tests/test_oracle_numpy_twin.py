"""Cross-check the C oracle against an independent numpy restatement (small sizes)."""
import numpy as np
import pytest

import numpy_twin as tw


def test_ca_code_twin(po):
    for prn in range(1, 33):
        assert np.array_equal(po.generate_ca(prn), tw.ca_code(prn).astype(np.int8))


@pytest.mark.parametrize("a,d,b", [(-0.6, 0.05, 0.6), (-0.5, 0.1, 0.5), (0.013, 0.0176379, 1022.9),
                                   (-0.5 + 0.00731, 1.0229e6 / 58e6, 57999 * 1.0229e6 / 58e6 - 0.5 + 0.00731)])
def test_colon_twin(po, a, d, b):
    assert np.array_equal(po.colon(a, d, b), tw.colon(a, d, b))


@pytest.mark.parametrize("pdi,taps", [(1, [-0.5, 0.0, 0.5]), (10, [-0.5, 0.0, 0.5]),
                                      (1, list(np.round(np.arange(-0.5, 0.51, 0.1), 12)))])
def test_correlate_step_twin(po, pkg, pdi, taps):
    rng = np.random.default_rng(pdi * 31 + len(taps))
    cfg = pkg.synth.opensky(skip_ms=0)
    n = int(round((1023.0 * pdi - 0.004) / (1.0230031e6 / 58e6)))
    iq = po.synth_if(cfg, 12345, n + 16)
    ca = po.generate_ca(16)
    taps = po.colon(-0.5, 0.1, 0.5) if len(taps) == 11 else np.array(taps)
    args = (n, 0.004, 1.0230031e6, 58e6, 4.58e6 - 305.25, float(rng.uniform(0, 6.28)))
    got = po.correlate_step(iq, *args, ca, pdi, taps)
    ref = tw.correlate_step(iq, *args, ca, taps)
    scale = np.sqrt(np.mean(ref ** 2))
    assert np.max(np.abs(got - ref)) / scale < 1e-12


def test_acquisition_twin(po, pkg):
    """Reduced acquisition (Fs 5.115 MHz, 3 PRNs) — same peaks and SNR as the twin."""
    from types import SimpleNamespace
    Fs, IF, S = 5.115e6, 1.25e6, 5115
    cfg = pkg.synth.scenario([3, 16], [1200, 4000], [1500, -2500], [48, 47], Fs=Fs, IF=IF,
                             skip_ms=0)
    data = po.synth_if(cfg, 0, 12 * S)
    file = SimpleNamespace(skip=0, dataType=2, dataPrecision=1, data=data, fileRoute=None, dev=None)
    signal = SimpleNamespace(IF=IF, Fs=Fs, codeFreqBasis=1.023e6, ms=1e-3, Sample=S,
                             codelength=1023.0)
    acq = SimpleNamespace(freqNum=13, freqMin=-3000, freqStep=500, datalen=3, L=2)
    A, d = po.acquisition(file, signal, acq, prn_list=[3, 7, 16], diag=True)
    tw_res = tw.acquisition(data, S, Fs, IF, 1.023e6, -3000, 500, 13, 3, [3, 7, 16])
    for k, (prn, fbin, cp, snr) in enumerate(tw_res):
        assert d.prn[k] == prn and d.fbin[k] == fbin and d.codePhase[k] == cp
        assert abs(d.SNR[k] - snr) < 1e-9
    # with 3 ms non-coherent the 12 dB threshold also passes noise (it is tuned for 20 ms)
    assert list(A.sv) == [prn for prn, _, _, snr in tw_res if snr >= 12]
    assert {3, 16} <= set(A.sv)
