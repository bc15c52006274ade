"""Experiment (test tooling): does the closed trackingCT loop depend on reproducing
MATLAB's per-sample rounding of Wave? Runs the oracle twice on the same synthetic
record -- carrier mode 0 (the reference's rounded Wave) and mode 1 (unrounded phase) --
and reports the first step where any integer field differs, per channel.
usage: python tools/eta_experiment.py [ms10=40000] [seed=6102] [nch=8]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po
import importlib
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")

ms10 = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 6102
nch = int(sys.argv[3]) if len(sys.argv) > 3 else 8
file, signal, acq, track, _, _ = pkg.initParameters()
skip = 2
cfg = pkg.synth.opensky(skip_ms=skip, seed=seed)
n_ms = skip + 1000 + 20 + ms10 + 12
t0 = time.time()
data = po.synth_if(cfg, 0, n_ms * signal.Sample)
print("synth", time.time() - t0, flush=True)
file.skip, file.data = skip, data
S = pkg.synth
Acq = pkg.sdr.from_c_acquired(pkg.sdr.to_c_acquired(type("A", (), dict(
    sv=S.OPENSKY_SV[:nch], SNR=S.OPENSKY_SNR[:nch], Doppler=[0.0] * nch,
    codedelay=S.OPENSKY_CODEDELAY[:nch], fineFreq=[float(f) for f in S.OPENSKY_FINEFREQ[:nch]]))))
track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, ms10
res = []
for mode in [int(m) for m in os.environ.get("MODES", "0,1").split(",")]:
    po.load().or_set_carrier_mode(mode)
    t0 = time.time()
    res.append(po.trackingCT(file, signal, track, Acq, nthreads=8))
    print("mode", mode, "oracle s", time.time() - t0, flush=True)
modes = [int(m) for m in os.environ.get("MODES", "0,1").split(",")]
T0, c0, x0 = res[0]
for mode, (T1, c1, x1) in zip(modes[1:], res[1:]):
    print("== mode", modes[0], "vs", mode, "countinx", list(x0), list(x1))
    for prn in Acq.sv:
        a, b = T0(prn), T1(prn)
        first = None
        for f in ("numSample", "absoluteSample", "delayValue"):
            d = np.nonzero(np.asarray(getattr(a, f)) != np.asarray(getattr(b, f)))[0]
            if len(d):
                first = d[0] if first is None else min(first, d[0])
        scale = np.sqrt(np.mean(a.P_i ** 2 + a.P_q ** 2))
        err = max(np.max(np.abs(a.P_i - b.P_i)), np.max(np.abs(a.P_q - b.P_q))) / scale
        dll = np.max(np.abs(a.DLLdiscri - b.DLLdiscri))
        print(f"PRN {prn}: len {len(a.P_i)} first int diff {first} P err/rms {err:.3e} "
              f"max dDLL {dll:.3e} max dremChip {np.max(np.abs(a.remChip - b.remChip)):.3e}", flush=True)
