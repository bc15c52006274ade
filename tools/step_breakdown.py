"""Wall-clock breakdown of one bench step (acquisition + trackingCT) against the
library's own timers: what the Python mirror and the host side add."""
import importlib, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
ctx = pkg.Context(0)
file, signal, acq, track, _, _ = pkg.initParameters()
S = signal.Sample
acq.freqMin, acq.freqStep, acq.datalen, acq.L = -7000, 500, 20, 10
acq.freqNum = int(2 * abs(acq.freqMin) / acq.freqStep + 1)
n10 = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, n10
cfg = pkg.synth.opensky(skip_ms=0, seed=6102)
dev = pkg.DeviceRecord(ctx, (1000 + 19 + n10 + 3) * S * 2)
pkg.synth.generate_device(ctx, cfg, dev)
file.skip, file.dev = 0, dev
for it in range(4):
    t0 = time.perf_counter()
    A = pkg.acquisition(file, signal, acq, ctx=ctx)
    t1 = time.perf_counter()
    ta = ctx.timing()
    buf = pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True, out=buf if it else None)
    t2 = time.perf_counter()
    tb = time.perf_counter()
    _ = pkg.sdr.TrackOutBuffers(len(A.sv), track, 0)
    print(f"   (TrackOutBuffers alloc alone {1e3*(time.perf_counter()-tb):.2f} ms)")
    tt = ctx.timing()
    print(f"iter {it}: acq wall {1e3*(t1-t0):7.2f} lib {ta['acq_ms']:7.2f} | track wall {1e3*(t2-t1):7.2f} "
          f"lib {tt['track_ms']:7.2f} | step {1e3*(t2-t0):7.2f}", flush=True)
