"""Why do config 5's channels 19 and 29 (PRN 20, PRN 30) never lock, in the oracle as on the GPU
? The CPU oracle (test infrastructure) tracks a few channels of the
config-5 scenario (synth.all_prn, the CPU generator's record = the GPU generator's bytes) over the
1-ms phase and the first N10 ms of the 10-ms phase, and prints per channel the loop's carrier and
code frequency against the scenario's truth (IF + Doppler; 1.023 MHz x (1 + Doppler / L1)) at the
end of the 1-ms phase and through the 10-ms phase, the |P_i| > |P_q| share per window, countinx
against the scenario's bit phase, and the PLL discriminator's spread.
    python tools/cfg5_lockdiag.py [N10_ms] [channels ...]   (defaults 3000; 17 18 19 29)"""
import importlib
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")]
import pyoracle as po  # noqa: E402
import make_golden_cfg5 as mg  # noqa: E402

pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
FL1, FC = 1575.42e6, 1.023e6


def main():
    n10 = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    chans = [int(x) for x in sys.argv[2:]] or [17, 18, 19, 29]
    file, signal, acq, track, _, _ = pkg.initParameters()
    S = signal.Sample
    cfg = pkg.synth.all_prn(32, skip_ms=0)
    t = time.time()
    data = po.synth_if(cfg, 0, (1000 + 19 + n10 + 3) * S)
    print(f"record {data.nbytes / 1e6:.0f} MB in {time.time() - t:.1f} s", flush=True)
    file.skip, file.data = 0, data
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, n10
    A = mg.acquired(cfg, signal)
    b = po.trackingCT(file, signal, track, A, taps=np.asarray(pkg.colon(-0.5, 0.1, 0.5)), channels=chans,
                      nthreads=len(chans), raw=True)
    F = pkg.abi.FIELDS
    fi = {f: F.index(f) for f in F}
    for c in chans:
        v = cfg.sv[c]
        n1 = 1000 + int(b.countinx[c])
        rec = b.rec[c, :, : int(b.len[c])]
        r = np.concatenate([rec[:, :n1], rec[:, n1::10]], axis=1)
        fcar, fcode = signal.IF + v.doppler_hz, FC * (1 + v.doppler_hz / FL1)
        cf, kf = r[fi["carrierFreq"]], r[fi["codeFreq"]]
        pi, pq = r[fi["P_i"]], r[fi["P_q"]]
        pll = r[fi["PLLdiscri"]]
        # bit edges of the scenario: bit_phase_chips (chips into a 20460-chip bit at sample 0)
        print(f"\n== channel {c} PRN {v.prn}: Doppler {v.doppler_hz:.1f} Hz, C/N0 {v.cn0_dbhz:.2f} dB-Hz, "
              f"bit phase {v.bit_phase_chips:.1f} chips, countinx {int(b.countinx[c])}")
        for lab, k in (("end of 1-ms phase", n1 - 1), ("10-ms step 1", n1), ("10-ms step 10", n1 + 9),
                       ("10-ms step 50", n1 + 49), ("10-ms step 100", n1 + 99), ("last", r.shape[1] - 1)):
            if k < r.shape[1]:
                print(f"  {lab:18s} carrier err {cf[k] - fcar:+9.3f} Hz  code err {kf[k] - fcode:+8.4f} Hz  "
                      f"PLLdiscri {pll[k]:+.3f}")
        for lo, hi in ((500, 1000), (n1, n1 + 50), (n1 + 50, n1 + 150), (n1 + 150, r.shape[1])):
            if hi > lo:
                s = slice(lo, min(hi, r.shape[1]))
                print(f"  steps {lo}-{hi}: |P_i|>|P_q| {np.mean(np.abs(pi[s]) > np.abs(pq[s])):.3f}, "
                      f"PLLdiscri std {np.std(pll[s]):.3f}, carrier err mean {np.mean(cf[s] - fcar):+.2f} "
                      f"std {np.std(cf[s]):.2f} Hz")
        np.savez(f"/tmp/diag/lock_{c}.npz", r=r, n1=n1)


if __name__ == "__main__":
    main()
