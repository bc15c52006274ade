"""Acquisition-only driver for profiling: BASELINE config 2 (32 PRNs, +-7 kHz / 500 Hz,
20 ms) on a device-resident synthetic Opensky record, fp64 correlation (ACQ_FP32=1: the
fp32 fast mode; ACQ_FUSED=<ring slots>: the fused correlator; ACQ_CFG=4: BASELINE config 4
instead, the bench's Urban record: Fs 26 MHz, IF 0, 32 PRNs, +-10 kHz / 250 Hz, 10 ms;
ACQ_PIPE=1|2: the split correlator's batches on one stream / pipelined over two; ACQ_BATCH=n:
n (bin, PRN) pairs per batch).
Args: [datalen] [freqNum] (config 2 only). Three calls."""
import importlib, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
dl = int(sys.argv[1]) if len(sys.argv) > 1 else 20
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 29
ctx = pkg.Context(0)
ctx.set_acq_precision(not os.environ.get("ACQ_FP32"))  # ACQ_FP32=1: the fp32 fast mode
if os.environ.get("ACQ_FUSED"):
    ctx.set_option(pkg.abi.OPT_ACQ_FUSED, 1)
    ctx.set_option(pkg.abi.OPT_ACQ_RING, int(os.environ["ACQ_FUSED"]))
if os.environ.get("ACQ_BATCH"):  # (bin, PRN) pairs per correlator batch (GNSS_OPT_ACQ_BATCH)
    ctx.set_option(pkg.abi.OPT_ACQ_BATCH, int(os.environ["ACQ_BATCH"]))
if os.environ.get("ACQ_PIPE"):
    ctx.set_option(pkg.abi.OPT_ACQ_PIPE, int(os.environ["ACQ_PIPE"]))
file, signal, acq, track, _, _ = pkg.initParameters()
if os.environ.get("ACQ_CFG") == "4":  # bench.py run_cfg4's record and parameters
    skip, S = 1000, 26000
    cfg = pkg.synth.urban(skip_ms=skip, Fs=26e6)
    signal.IF, signal.Fs, signal.Sample = 0.0, 26e6, S
    acq.freqNum, acq.freqMin, acq.freqStep, acq.datalen, acq.L = 81, -10000, 250, 10, 10
else:
    skip, S = 5000, 58000
    cfg = pkg.synth.opensky(skip_ms=skip)
    acq.freqMin, acq.freqNum, acq.datalen = -(nb // 2) * 500, nb, dl
dev = pkg.DeviceRecord(ctx, (skip + 40) * S * 2)
pkg.synth.generate_device(ctx, cfg, dev)
file.skip, file.dev = skip, dev
for it in range(3):
    t = time.perf_counter()
    A, d = pkg.acquisition(file, signal, acq, ctx=ctx, diag=True)
    print("acq wall", time.perf_counter() - t, ctx.timing(), flush=True)
print("sv", list(A.sv), "cd", list(A.codedelay), "ff", list(A.fineFreq))
print("fbin", list(d.fbin), "cp", list(d.codePhase))
print("snr", [round(x, 4) for x in d.SNR])
print("snrhex", [float(x).hex() for x in d.SNR])  # (bit-identity across library builds)
