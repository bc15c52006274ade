"""Per-step diagnostics: GPU correlate step vs oracle at random NCO states, and
first divergence of the closed-loop trackers."""
import importlib, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
sdr = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd.sdr")
ctx = pkg.Context(0)
file, signal, acq, track, _, _ = pkg.initParameters()
skip = 5
cfg = pkg.synth.opensky(skip_ms=skip)
data = po.synth_if(cfg, 0, 80 * 58000)
file.skip, file.data = skip, data
rng = np.random.default_rng(1)
taps3 = np.array([-0.5, 0, 0.5]); taps11 = po.colon(-0.5, 0.1, 0.5)
worst = 0
for trial in range(40):
    prn = int(rng.choice(pkg.synth.OPENSKY_SV))
    pdi = 1 if trial % 4 else 10
    rc = float(rng.uniform(-0.009, 0.009)); cf = 1.023e6 + float(rng.normal(0, 3)); f = 4.58e6 + float(rng.uniform(-4000, 4000))
    ph = float(rng.uniform(0, 2 * np.pi)); pos = 2 * int(rng.integers(0, 50 * 58000))
    taps = taps11 if trial % 3 == 0 else taps3
    g, ns = sdr.correlate_step(file, signal, prn, pdi, rc, cf, f, ph, pos, taps, ctx=ctx)
    n = int(np.round((1023.0 * pdi - rc) / (cf / 58e6)))
    r = po.correlate_step(data[pos: pos + 2 * n], n, rc, cf, 58e6, f, ph, po.generate_ca(prn), pdi, taps)
    sc = np.sqrt(np.mean(r ** 2))
    e = np.max(np.abs(g - r)) / sc
    worst = max(worst, e)
    if e > 1e-6 or trial < 4:
        print(trial, prn, pdi, len(taps), "ns", ns, n, "rel", e, "absmax", np.max(np.abs(g - r)), "scale", sc)
print("worst single-step rel err", worst)
