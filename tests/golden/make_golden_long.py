"""Long-run golden of the headline tracking shape: the oracle's
trackingCT over the FULL config-3 length (1000 ms @1 ms + countinx + 40 000 ms @10 ms) on
the bench's own record, for every acquired channel (round 4; rounds 1-3: two), plus the
bench acquisition of that record. The channels run in parallel threads (one oracle thread
each; ctypes releases the GIL).

Runs ON THE GPU BOX (the record is the HIP synthetic generator's, resident in HBM: it is
downloaded here and fed to the CPU oracle), e.g.
    gpurun -- python tests/golden/make_golden_long.py
and writes gpurun_out/golden_track_long.npz, which is committed as
tests/golden/golden_track_long.npz. The record's xxh64 digest is stored with it, so the
GPU test (tests/test_gpu_longrun.py) proves it regenerated the same bytes.
Test infrastructure only."""
import importlib
import os
import sys
import threading
import time

import numpy as np
import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import pyoracle as po  # noqa: E402

pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")

SKIP, N1, N10, SEED = 5000, 1000, 40000, 6102
CHANNELS = tuple(range(8))  # all 8 acquired SVs (channel index = svindex - 1)


def record_bytes(S=58000):
    return (SKIP + N1 + 19 + N10 + 3) * S * 2


def digest(a: np.ndarray) -> str:
    h = xxhash.xxh64()
    step = 1 << 28
    for i in range(0, len(a), step):
        h.update(memoryview(a[i:i + step]))
    return h.hexdigest()


def beat(stop):
    t0 = time.time()
    while not stop.wait(20):
        print(f"  ... {time.time() - t0:.0f} s", flush=True)


def main(out):
    ctx = pkg.Context(0)
    file, signal, acq, track, _, _ = pkg.initParameters()
    cfg = pkg.synth.opensky(skip_ms=SKIP, seed=SEED)
    dev = pkg.DeviceRecord(ctx, record_bytes(signal.Sample))
    pkg.synth.generate_device(ctx, cfg, dev)
    data = dev.download()
    dg = digest(data)
    print("record", len(data), "bytes, xxh64", dg, flush=True)
    file.skip, file.data = SKIP, data
    acq.freqMin, acq.freqStep, acq.datalen, acq.L = -7000, 500, 20, 10
    acq.freqNum = int(2 * abs(acq.freqMin) / acq.freqStep + 1)
    stop = threading.Event()
    threading.Thread(target=beat, args=(stop,), daemon=True).start()
    t = time.time()
    A = po.acquisition(file, signal, acq, nthreads=16)
    print("oracle acquisition", list(A.sv), f"{time.time() - t:.1f} s", flush=True)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = N1, N10
    res = {}

    def one(c):
        t = time.time()
        b = po.trackingCT(file, signal, track, A, channels=[c], nthreads=1, raw=True)
        assert b.status == 0, b.status
        n1 = N1 + int(b.countinx[c])
        L = int(b.len[c])
        assert L == n1 + N10
        rec = b.rec[c, :, :L]
        assert np.array_equal(rec[:, n1::10], rec[:, n1 + 9::10])  # 10x replication
        res[c] = (np.concatenate([rec[:, :n1], rec[:, n1::10]], axis=1), int(b.countinx[c]),
                  b.CN0[: b.c.cn0_rows, c].copy())
        print(f"oracle channel {c} (PRN {int(A.sv[c])}): countinx {int(b.countinx[c])}, "
              f"{time.time() - t:.1f} s", flush=True)

    workers = [threading.Thread(target=one, args=(c,)) for c in CHANNELS]
    for w in workers:
        w.start()
    for w in workers:
        w.join()
    assert sorted(res) == sorted(CHANNELS)
    stop.set()
    np.savez_compressed(out, digest=dg, skip=SKIP, N1=N1, N10=N10, seed=SEED,
                        sv=A.sv, SNR=A.SNR, Doppler=A.Doppler, codedelay=A.codedelay, fineFreq=A.fineFreq,
                        channels=np.array(CHANNELS),
                        countinx=np.array([res[c][1] for c in CHANNELS]),
                        **{f"rec_{j}": res[c][0] for j, c in enumerate(CHANNELS)},
                        **{f"CN0_{j}": res[c][2] for j, c in enumerate(CHANNELS)})
    print("wrote", out, flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "golden_track_long.npz"))
