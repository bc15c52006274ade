"""Where the bench step's wall time goes outside the GPU: times acquisition and trackingCT
calls (wall vs device) on the bench workload, with GNSS_HOSTPROF phases on stderr."""
import importlib, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
ctx = pkg.Context(0)
file, signal, acq, track, _, _ = pkg.initParameters()
S = signal.Sample
file.skip = 5000
acq.freqMin, acq.freqStep, acq.datalen, acq.L = -7000, 500, 20, 10
acq.freqNum = 29
track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, 40000
cfg = pkg.synth.opensky(skip_ms=5000)
dev = pkg.DeviceRecord(ctx, (5000 + 1000 + 19 + 40000 + 3) * S * 2)
pkg.synth.generate_device(ctx, cfg, dev)
file.dev = dev
out = None
for it in range(4):
    t0 = time.perf_counter()
    A = pkg.acquisition(file, signal, acq, ctx=ctx)
    t1 = time.perf_counter()
    ta = ctx.timing()
    out = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True, out=out)
    t2 = time.perf_counter()
    tt = ctx.timing()
    print(f"acq wall {1e3*(t1-t0):.2f} dev {ta['acq_ms']:.2f} | track wall {1e3*(t2-t1):.2f} dev {tt['track_ms']:.2f}", flush=True)
