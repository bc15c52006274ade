"""Diagnostic: config 5 at full length (as tests/test_gpu_longrun.py::test_config5_full_length_against_oracle)
and, for the golden's channels, every (step, tap) whose tap sum differs from the oracle golden by more than
1e-8 of the series RMS, with the step's NCO state. Args: [channel ...] (default: every golden channel)."""
import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle")]
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
import make_golden_cfg5 as mg  # noqa: E402
import make_golden_long as mgl  # noqa: E402
z = np.load(os.path.join(ROOT, "tests", "golden", "golden_cfg5_long.npz"))
want = [int(a) for a in sys.argv[1:]] or [int(c) for c in z["channels"]]
ctx = pkg.Context(0)
file, signal, acq, track, _, _ = pkg.initParameters()
N1, N10, skip = int(z["N1"]), int(z["N10"]), int(z["skip"])
cfg = pkg.synth.all_prn(int(z["nsv"]), skip_ms=skip)
dev = pkg.DeviceRecord(ctx, mg.record_bytes(signal.Sample))
pkg.synth.generate_device(ctx, cfg, dev)
file.skip, file.dev = skip, dev
track.msToProcessCT_1ms, track.msToProcessCT_10ms = N1, N10
A = mg.acquired(cfg, signal)
taps = pkg.colon(-0.5, 0.1, 0.5)
F = pkg.abi.FIELDS
variants = [v for v in os.environ.get("TD_VARIANTS", "default").split(";")]
for var in variants:
  opts = {} if var == "default" else dict(kv.split("=") for kv in var.split(","))
  for k in ("NO_PERSIST", "FORCE_VPB"):
    ctx.set_option(getattr(pkg.abi, "OPT_" + k), int(opts.get(k, 0)))
  b = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
  print(f"=== variant {var}: launches {ctx.timing()['track_launches']}", flush=True)
  for j, c in enumerate(z["channels"]):
      if int(c) not in want:
          continue
      n1 = N1 + int(z["countinx"][j])
      L = int(b.len[c])
      got = mg.distinct_steps(b.rec[c, :, :L], n1)
      gt = mg.distinct_steps(b.taps[c, :, :, :L], n1)
      iv, rtaps, rnco, rms = mg.expand(z, j)
      d = np.abs(gt - rtaps) / rms  # [2][11][steps]
      bad = np.argwhere(d > 1e-8)
      print(f"channel {int(c)} (PRN {int(A.sv[c])}): n1 {n1}, steps {got.shape[1]}, rms {rms:.6g}, {len(bad)} tap values off, int fields off from step "
                f"{min([int(np.nonzero(got[i] != iv[k])[0][0]) for k, i in enumerate(mg.field_rows(F)[0]) if (got[i] != iv[k]).any()] or [-1])}")
      for fname in ("remChip", "codeFreq", "carrierFreq", "remPhase"):
          k = F.index(fname)
          ref = rnco[mg.field_rows(F)[1].index(k)]
          dd = got[k] - ref
          nz = np.nonzero(dd != 0)[0]
          print(f"    {fname}: first bitwise difference at step {int(nz[0]) if len(nz) else -1} (n1 {n1}), "
                f"{len(nz)} steps differ, max |diff| {np.max(np.abs(dd)):.3e}, at steps n1-1/n1/n1+10/+1000: "
                f"{[float(dd[i]) for i in (n1 - 1, n1, n1 + 10, n1 + 1000) if i < len(dd)]}")
      for (iq, t, st) in sorted(bad.tolist(), key=lambda r: r[2])[:int(os.environ.get('TD_SHOW', '6'))]:
          print(f"  step {st} ({'1ms' if st < n1 else '10ms #%d' % (st - n1)}) tap {t} ({taps[t]:+.1f}) {'IQ'[iq]}: "
                f"got {gt[iq, t, st]:.10g} ref {rtaps[iq, t, st]:.10g} diff/rms {d[iq, t, st]:.3e}; "
                f"remChip {got[F.index('remChip'), st - 1] if st else float('nan'):.17g} codeFreq "
                f"{got[F.index('codeFreq'), st - 1] if st else float('nan'):.17g} numSample {got[F.index('numSample'), st]:.0f}")
