"""does the CPU oracle (the reference's algorithm restated) also lose
lock on PRNs 4 and 27 of the 45-s synthetic LNAV scenario of tests/test_gpu_chain.py? Runs the
same chain on the CPU -- oracle acquisition, oracle trackingCT (8 channels, 1000 ms @1 ms +
45 000 ms @10 ms), the library's host naviDecode_updated -- and prints, per PRN, whether it
decoded and a lock indicator (share of 10-ms steps with |P_i| > |P_q|, last 10 s).
Usage: python3 tools/oracle_lock_check.py [nthreads]"""
import importlib, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
import pyoracle as po

nt = int(sys.argv[1]) if len(sys.argv) > 1 else 8
file, signal, acq, track, _, _ = pkg.initParameters()
skip, N10 = 100, 45000
cfg = pkg.synth.opensky(skip_ms=skip)
for i in range(cfg.n_sv):
    cfg.sv[i].lnav = 1
t = time.perf_counter()
data = po.synth_if(cfg, 0, (skip + 1000 + 19 + N10 + 3) * signal.Sample, nthreads=nt)
print("synth s", round(time.perf_counter() - t, 1), flush=True)
file.skip, file.data = skip, data
acq.freqMin, acq.freqNum = -7000, 29
t = time.perf_counter()
A = po.acquisition(file, signal, acq, nthreads=nt)
print("acquired", list(A.sv), "s", round(time.perf_counter() - t, 1), flush=True)
track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, N10
t = time.perf_counter()
T, cn0, cx = po.trackingCT(file, signal, track, A, nthreads=nt)
print("tracked s", round(time.perf_counter() - t, 1), "countinx", list(cx), flush=True)
eph, _, fp = pkg.naviDecode_updated(A, T)
for p in A.sv:
    p = int(p)
    Pi, Pq = np.asarray(T(p).P_i), np.asarray(T(p).P_q)
    tail = slice(len(Pi) - 10000, len(Pi), 10)
    lock = float(np.mean(np.abs(Pi[tail]) > np.abs(Pq[tail])))
    print(f"PRN {p:2d}: decoded {int(eph(p).updateflag == 1)}  lock(|P_i|>|P_q|, last 10 s) {lock:.2f}", flush=True)
