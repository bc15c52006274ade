import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
ctx = pkg.Context(0)
file, signal, acq, track, _, _ = pkg.initParameters()
skip, N10 = 100, 21000
cfg = pkg.synth.opensky(skip_ms=skip)
for i in range(cfg.n_sv):
    cfg.sv[i].lnav = 1
dev = pkg.DeviceRecord(ctx, (skip + 1000 + 19 + N10 + 3) * signal.Sample * 2)
pkg.synth.generate_device(ctx, cfg, dev)
file.skip, file.dev = skip, dev
acq.freqMin, acq.freqNum = -7000, 29
A = pkg.acquisition(file, signal, acq, ctx=ctx)
print("sv", list(A.sv), "cd", list(A.codedelay))
track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, N10
T, cn0, cx = pkg.trackingCT(file, signal, track, A, ctx=ctx)
print("countinx", list(cx))
for prn in A.sv[:3]:
    P = T(int(prn)).P_i
    s = np.sign(P[3000:])
    tr = np.flatnonzero(np.diff(s) != 0)
    print(prn, "len", len(P), "transitions", len(tr), "first", tr[:6], "gaps mod 20", np.unique(np.diff(tr) % 20)[:10])
    print("  P_i sample", np.round(P[3000:3060:10]).tolist())
np.save("gpurun_out/chain_pi.npy", np.stack([T(int(p)).P_i[:22000] for p in A.sv]))
eph, _, fp = pkg.naviDecode_updated(A, T)
for prn in A.sv:
    e = eph(int(prn))
    print(prn, "nav1", fp.nav1[prn - 1], "TOW", e.TOW[:4], "sfb", e.sfb[:4], "upd", e.updateflag)
