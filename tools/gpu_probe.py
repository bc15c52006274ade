"""Diagnostic probe (not a test): GPU vs oracle on a small synthetic Opensky case,
printing per-field errors and timings."""
import importlib, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
ctx = pkg.Context(0)
file, signal, acq, track, _, _ = pkg.initParameters()
skip = 5
cfg = pkg.synth.opensky(skip_ms=skip)
N10 = int(os.environ.get("N10", "500"))
n_ms = skip + 1000 + 19 + N10 + 4
t = time.time(); data = po.synth_if(cfg, 0, n_ms * 58000); print("gen", time.time() - t, flush=True)
# GPU generator agreement
dev = pkg.DeviceRecord(ctx, 2 * 58000 * 50)
pkg.synth.generate_device(ctx, cfg, dev)
gd = dev.download()
print("synth gpu==cpu bytes:", np.mean(gd == data[: gd.size]), "max diff", np.abs(gd.astype(int) - data[: gd.size]).max(), flush=True)
file.skip, file.data = skip, data
acq.freqMin, acq.freqNum, acq.datalen = -7000, 29, int(os.environ.get("DL", "4"))
t = time.time(); ga, gd_ = pkg.acquisition(file, signal, acq, ctx=ctx, diag=True); tg = time.time() - t
print("gpu acq wall", tg, ctx.timing(), flush=True)
t = time.time(); ra, rd = po.acquisition(file, signal, acq, diag=True); print("cpu acq", time.time() - t, flush=True)
print("sv eq", np.array_equal(ga.sv, ra.sv), "cd eq", np.array_equal(ga.codedelay, ra.codedelay),
      "dop eq", np.array_equal(ga.Doppler, ra.Doppler), "fine eq", np.array_equal(ga.fineFreq, ra.fineFreq))
print("snr diff max", np.max(np.abs(gd_.SNR - rd.SNR)), "fbin eq", np.array_equal(gd_.fbin, rd.fbin), "cp eq", np.array_equal(gd_.codePhase, rd.codePhase))
bad = np.where((gd_.fbin != rd.fbin) | (gd_.codePhase != rd.codePhase))[0]
for i in bad: print("  mismatch prn", rd.prn[i], gd_.fbin[i], rd.fbin[i], gd_.codePhase[i], rd.codePhase[i], rd.SNR[i], rd.peak[i], rd.peak2[i])
print("gpu fine", ga.fineFreq - 4.58e6)
print("cpu fine", ra.fineFreq - 4.58e6)
# tracking on the true SVs
sel = [i for i, p in enumerate(ra.sv) if p in pkg.synth.OPENSKY_SV]
A = type("A", (), {})()
for f in ["sv", "SNR", "Doppler", "codedelay", "fineFreq"]: setattr(A, f, getattr(ra, f)[sel])
track.msToProcessCT_10ms = N10
t = time.time(); gT, gcn, gcx = pkg.trackingCT(file, signal, track, A, ctx=ctx); print("gpu track wall", time.time() - t, ctx.timing(), flush=True)
t = time.time(); rT, rcn, rcx = po.trackingCT(file, signal, track, A); print("cpu track", time.time() - t, flush=True)
print("countinx", gcx, rcx)
for prn in rT.prns():
    g, r = gT(prn), rT(prn)
    sc = np.sqrt(np.mean(r.P_i**2 + r.P_q**2))
    errs = {f: float(np.max(np.abs(getattr(g, f) - getattr(r, f)))) for f in pkg.abi.FIELDS}
    print(prn, "len", len(g.P_i), len(r.P_i), "P rel", max(errs["P_i"], errs["P_q"]) / sc,
          "E rel", max(errs["E_i"], errs["L_q"]) / sc, "ns", errs["numSample"], "abs", errs["absoluteSample"],
          "cd", errs["codedelay"], "remChip", errs["remChip"], "carrF", errs["carrierFreq"], "codeF", errs["codeFreq"], "remPhase", errs["remPhase"])
print("cn0 max diff", np.max(np.abs(gcn - rcn)) if gcn.shape == rcn.shape else (gcn.shape, rcn.shape))
# 11 taps
print("---- first divergence per channel")
for prn in rT.prns():
    g, r = gT(prn), rT(prn)
    sc = np.sqrt(np.mean(r.P_i[:1000]**2 + r.P_q[:1000]**2))
    e = np.maximum(np.abs(g.P_i - r.P_i), np.abs(g.P_q - r.P_q)) / sc
    i5 = int(np.argmax(e > 1e-5)) if np.any(e > 1e-5) else -1
    i3 = int(np.argmax(e > 1e-3)) if np.any(e > 1e-3) else -1
    ins = int(np.argmax(g.numSample != r.numSample)) if np.any(g.numSample != r.numSample) else -1
    print(prn, "first>1e-5", i5, "first>1e-3", i3, "first ns diff", ins, "phaseC start", 1000 + int(rcx[list(rT.prns()).index(prn)]),
          "max err in 1ms phase", float(e[:1000].max()), "PLLdiscri@i5", r.PLLdiscri[max(i5,0)], "P_i@i5", r.P_i[max(i5,0)])
taps = po.colon(-0.5, 0.1, 0.5)
track.msToProcessCT_10ms = 100
A2 = type("A", (), {})()
for f in ["sv", "SNR", "Doppler", "codedelay", "fineFreq"]: setattr(A2, f, getattr(A, f)[:2])
gb = pkg.trackingCT(file, signal, track, A2, ctx=ctx, taps=taps, raw=True)
rb = po.trackingCT(file, signal, track, A2, taps=taps, raw=True)
sc = np.sqrt(np.mean(rb.taps ** 2))
print("11-tap rel err", np.max(np.abs(gb.taps - rb.taps)) / sc, "rec eq ns", np.array_equal(gb.rec[:, 14], rb.rec[:, 14]), ctx.timing())
