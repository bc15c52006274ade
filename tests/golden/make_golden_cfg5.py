"""Long-run golden of BASELINE config 5: the oracle's 11-tap trackingCT
(taps -0.5:0.1:0.5, trackingCT_multiCorr-GIVEN.m:25 tap semantics on trackingCT.m's loop)
over the FULL benchmarked length -- 1000 ms @1 ms + countinx + 90 000 ms @10 ms
(trackingCT.m:73-171, :178-213, :377-525) -- on the bench's own 32-SV record, for eight of
the 32 channels (round 4; rounds 2-3: three), and from round 5 the other 24 in two sets
(--set b / c, compact_lite: integer fields, E / P / L and the NCO fields).

Runs ON THE GPU BOX (the record is the HIP synthetic generator's, resident in HBM: it is
downloaded there and fed to the CPU oracle, one OpenMP thread per channel, ~13-15 min), e.g.
    gpurun --timeout 1200 -- python -u tests/golden/make_golden_cfg5.py
and writes gpurun_out/golden_cfg5_long.npz, committed as tests/golden/golden_cfg5_long.npz.
The record's xxh64 digest is stored with it, so tests/test_gpu_longrun.py proves it
regenerated the same bytes. Storage (compact(), ~1.3 MB per channel): the integer fields exact, as their
first value and int32 step differences; the 22 tap sums (E / P / L are taps 0 / 5 / 10) as
int32 multiples of q = 2e-9 x the channel's P RMS (the test's tolerance is 1e-8 of the RMS,
5 quanta); the NCO fields as float64. Test infrastructure only."""
import importlib
import os
import sys
import threading
import time
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), HERE]
import make_golden_long as mgl  # noqa: E402  (digest, beat)
import pyoracle as po  # noqa: E402

pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")

SKIP, N1, N10, NSV = 0, 1000, 90000, 32
# PRN 3 (the weakest, 40.8 dB-Hz), PRN 18 (-3.9 kHz), PRN 32 (the grid's last) -- rounds 2-3 --
# and every fifth channel besides
CHANNELS = (2, 17, 31, 0, 7, 12, 22, 27)
QREL = 2e-9


def record_bytes(S=58000):
    return (SKIP + N1 + 19 + N10 + 3) * S * 2


def acquired(cfg, signal):
    S = signal.Sample
    cds = pkg.synth.codedelays(cfg, SKIP)  # where the scenario put each SV
    return SimpleNamespace(sv=np.array([cfg.sv[i].prn for i in range(NSV)]), SNR=np.zeros(NSV),
                           Doppler=np.zeros(NSV), codedelay=np.array(cds),
                           fineFreq=np.array([signal.IF + cfg.sv[i].doppler_hz for i in range(NSV)]))


def distinct_steps(a, n1):
    """The record's distinct steps: the 1-ms ones and one of each 10-fold 10-ms row."""
    return np.concatenate([a[..., :n1], a[..., n1::10]], axis=-1)


INT_FIELDS = ("codedelay", "numSample", "delayValue", "absoluteSample", "codedelay2")


def field_rows(F):
    ints = [F.index(f) for f in INT_FIELDS]
    return ints, [i for i in range(6, len(F)) if i not in ints]


def compact(j, r, tp, cn0, F):
    """Channel j's arrays in the committed form: r = distinct-step record [18][steps],
    tp = taps [2][11][steps]; E / P / L (r[:6]) must be taps 0 / 5 / 10."""
    ints, nco = field_rows(F)
    assert all(np.array_equal(r[k], tp[k % 2, (5, 5, 0, 0, 10, 10)[k]]) for k in range(6))
    rms = float(np.sqrt(np.mean(r[0] ** 2 + r[1] ** 2)))
    qt = np.rint(tp / (QREL * rms))
    assert np.abs(qt).max() < 2 ** 31
    iv = r[ints].astype(np.int64)
    d = np.diff(iv, axis=1)
    assert np.abs(d).max() < 2 ** 31
    return {f"rms_{j}": rms, f"int0_{j}": iv[:, 0], f"intd_{j}": d.astype(np.int32),
            f"taps_{j}": qt.astype(np.int32), f"nco_{j}": r[nco], f"CN0_{j}": cn0}


def compact_lite(j, r, cn0, F):
    """The other 24 channels (round 5) in a smaller form: the integer fields
    exact as above, E / P / L (r[:6]) as int32 quanta of QREL x RMS, the NCO fields as float32
    (their test tolerance, 1e-7 relative, is above float32's 6e-8) and remChip / codeFreq again as
    float64 -- no non-loop taps."""
    ints, nco = field_rows(F)
    rms = float(np.sqrt(np.mean(r[0] ** 2 + r[1] ** 2)))
    qe = np.rint(r[:6] / (QREL * rms))
    assert np.abs(qe).max() < 2 ** 31
    iv = r[ints].astype(np.int64)
    d = np.diff(iv, axis=1)
    assert np.abs(d).max() < 2 ** 31
    # remChip and codeFreq also at full precision: the test's tie-flip check rebuilds the replica
    # coordinates from the oracle's state to 1e-9 chip (float32 would give ~1e-3 chip)
    tie = [F.index("remChip"), F.index("codeFreq")]
    return {f"rms_{j}": rms, f"int0_{j}": iv[:, 0], f"intd_{j}": d.astype(np.int32),
            f"epl_{j}": qe.astype(np.int32), f"nco32_{j}": r[nco].astype(np.float32),
            f"ncotie_{j}": r[tie], f"CN0_{j}": cn0}


def expand(z, j):
    """(integer fields [5][steps], taps [2][11][steps] as floats, nco [7][steps], rms)."""
    iv = np.concatenate([z[f"int0_{j}"][:, None], z[f"intd_{j}"].astype(np.int64)], axis=1).cumsum(axis=1)
    rms = float(z[f"rms_{j}"])
    if f"taps_{j}" not in z:  # (compact_lite: E / P / L only, as the [2][11] tap array's rows 0 / 5 / 10)
        e = z[f"epl_{j}"] * (float(z["qrel"]) * rms)
        taps = np.full((2, 11, e.shape[1]), np.nan)
        for k in range(6):
            taps[k % 2, (5, 5, 0, 0, 10, 10)[k]] = e[k]
        nv = z[f"nco32_{j}"].astype(np.float64)
        if f"ncotie_{j}" in z:  # (remChip, codeFreq at full precision)
            F = pkg.abi.FIELDS
            nco = field_rows(F)[1]
            for k, f in enumerate(("remChip", "codeFreq")):
                nv[nco.index(F.index(f))] = z[f"ncotie_{j}"][k]
        return iv, taps, nv, rms
    return iv, z[f"taps_{j}"] * (float(z["qrel"]) * rms), z[f"nco_{j}"], rms


# round 5: the other 24 channels in two sets (one GPU-box call each: 12 oracle threads, ~15 min)
CHANNEL_SETS = {"b": (1, 3, 4, 5, 6, 8, 9, 10, 11, 13, 14, 15),
                "c": (16, 18, 19, 20, 21, 23, 24, 25, 26, 28, 29, 30)}


def main(out, channels=CHANNELS, lite=False, cpu=False):
    file, signal, acq, track = pkg.initParameters()[:4]
    cfg = pkg.synth.all_prn(NSV, skip_ms=SKIP)
    if cpu:  # (tools/synth_cmp.py showed or_synth_if == gnss_synth_if_device for this scenario)
        data = po.synth_if(cfg, 0, record_bytes(signal.Sample) // 2)
    else:
        ctx = pkg.Context(0)
        dev = pkg.DeviceRecord(ctx, record_bytes(signal.Sample))
        pkg.synth.generate_device(ctx, cfg, dev)
        data = dev.download()
    dg = mgl.digest(data)
    print("record", len(data), "bytes, xxh64", dg, flush=True)
    file.skip, file.data = SKIP, data
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = N1, N10
    A = acquired(cfg, signal)
    taps = pkg.colon(-0.5, 0.1, 0.5)
    stop = threading.Event()
    threading.Thread(target=mgl.beat, args=(stop,), daemon=True).start()
    t = time.time()
    b = po.trackingCT(file, signal, track, A, taps=taps, channels=list(channels), nthreads=len(channels),
                      raw=True)
    stop.set()
    assert b.status == 0, b.status
    print(f"oracle channels {channels}: {time.time() - t:.1f} s", flush=True)
    save = dict(digest=dg, skip=SKIP, N1=N1, N10=N10, nsv=NSV, channels=np.array(channels), qrel=QREL,
                taps=taps, countinx=np.array([int(b.countinx[c]) for c in channels]),
                len=np.array([int(b.len[c]) for c in channels]))
    for j, c in enumerate(channels):
        n1 = N1 + int(b.countinx[c])
        L = int(b.len[c])
        assert L == n1 + N10
        rec = b.rec[c, :, :L]
        assert np.array_equal(rec[:, n1::10], rec[:, n1 + 9::10])  # 10x replication
        r = distinct_steps(rec, n1)
        tp = distinct_steps(b.taps[c, :, :, :L], n1)  # [2][11][steps]
        if lite:
            save.update(compact_lite(j, r, b.CN0[: b.c.cn0_rows, c], pkg.abi.FIELDS))
        else:
            save.update(compact(j, r, tp, b.CN0[: b.c.cn0_rows, c], pkg.abi.FIELDS))
        lock = float(np.mean(np.abs(r[0, n1:]) > np.abs(r[1, n1:])))  # |P_i| > |P_q| in the 10-ms phase
        save[f"lock_{j}"] = lock
        print(f"channel {c} (PRN {int(A.sv[c])}): countinx {int(b.countinx[c])}, 10-ms lock {lock:.3f}", flush=True)
    np.savez_compressed(out, **save)
    print("wrote", out, os.path.getsize(out), "bytes", flush=True)


if __name__ == "__main__":
    # make_golden_cfg5.py [OUT]                -> the eight channels of CHANNELS, full taps
    # make_golden_cfg5.py --set b|c [--cpu]    -> CHANNEL_SETS[b|c], compact_lite, golden_cfg5_long_<set>.npz
    args = sys.argv[1:]
    if args and args[0] == "--set":
        st = args[1]
        main(os.path.join(ROOT, "gpurun_out", f"golden_cfg5_long_{st}.npz"), CHANNEL_SETS[st], lite=True,
             cpu="--cpu" in args)
    else:
        main(args[0] if args else os.path.join(ROOT, "gpurun_out", "golden_cfg5_long.npz"))
