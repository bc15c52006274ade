"""Staging throughput of an IF record read from disk (file.fileRoute) into HBM: writes a
synthetic Opensky record of ~N seconds to a temp file, runs trackingCT from the file route
(the library stages the whole needed window through its pinned double buffers) and prints
the staged bytes / time. usage: python tools/stage_probe.py [seconds=20]"""
import importlib, os, sys, tempfile, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
sec = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = pkg.Context(0)
file, signal, acq, track, _, _ = pkg.initParameters()
S = signal.Sample
n_ms = 5 + 1000 + 19 + (sec - 1) * 1000 + 5
dev = pkg.DeviceRecord(ctx, n_ms * S * 2)
pkg.synth.generate_device(ctx, pkg.synth.opensky(skip_ms=5), dev)
data = dev.download()
with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp"), suffix=".bin", delete=False) as f:
    f.write(np.asarray(data, dtype=np.int8).tobytes())
    path = f.name
try:
    os.sync() if hasattr(os, "sync") else None
    file.skip, file.fileRoute, file.data, file.dev = 5, path, None, None
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, (sec - 1) * 1000
    A = pkg.sdr.from_c_acquired(pkg.sdr.to_c_acquired(type("A", (), dict(
        sv=pkg.synth.OPENSKY_SV[:4], SNR=[20.0] * 4, Doppler=[0.0] * 4, codedelay=pkg.synth.OPENSKY_CODEDELAY[:4],
        fineFreq=[float(x) for x in pkg.synth.OPENSKY_FINEFREQ[:4]]))))
    for it in range(2):
        t0 = time.perf_counter()
        pkg.trackingCT(file, signal, track, A, ctx=ctx, raw=True)
        wall = time.perf_counter() - t0
        t = ctx.timing()
        print(f"iter {it}: wall {wall:.3f} s, staged {t['h2d_bytes'] / 1e9:.3f} GB in {t['h2d_ms']:.1f} ms "
              f"= {t['h2d_bytes'] / (t['h2d_ms'] * 1e-3) / 1e9:.2f} GB/s (disk/page cache -> pinned -> HBM), "
              f"tracking {t['track_ms']:.1f} ms", flush=True)
finally:
    os.unlink(path)
