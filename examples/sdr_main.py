"""SDR_main.m (SDR_MATLAB-main/SDR_main.m:16-56) on the MI355X engine: parameter
initialisation, acquisition, conventional tracking and navigation-data decoding, with the
reference's result files (Acquired_<file>_<skip>.mat, TckResult_Eph<file>_<s>.mat,
eph_<file>_<s>.mat, sbf_<file>_<s>.mat) written and re-used the same way. Positioning
(SDR_main.m:59-) is outside this engine.

    python examples/sdr_main.py --file Opensky.bin          # a recorded IF file
    python examples/sdr_main.py --synthetic --n10 45000     # the synthetic Opensky scenario
                                                            # (LNAV message on every SV)
"""
import argparse
import importlib
import os
import sys

import numpy as np
import scipy.io as sio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sdr = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")


def struct_of(T, prns, fields):
    """TckResultCT(prn) entries as a MATLAB struct array indexed by PRN."""
    n = max(prns)
    arr = np.empty((1, n), dtype=object)
    empty = {f: np.zeros((1, 0)) for f in fields}
    for p in range(1, n + 1):
        src = T(p) if p in prns else None
        arr[0, p - 1] = {f: (np.atleast_2d(getattr(src, f)) if src is not None else empty[f]) for f in fields}
    return arr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--file", help="IF record (int8 I/Q, Opensky parameters)")
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--skip", type=int, default=None)
    ap.add_argument("--n10", type=int, default=None, help="track.msToProcessCT_10ms")
    ap.add_argument("--out", default=".")
    args = ap.parse_args()

    # [file, signal, acq, track, solu, cmn] = initParameters()  (SDR_main.m:17)
    file, signal, acq, track, solu, cmn = sdr.initParameters(args.file)
    if args.skip is not None:
        file.skip = args.skip
    if args.n10 is not None:
        track.msToProcessCT_10ms = args.n10
    ctx = sdr.Context(0)
    if args.synthetic or not args.file:
        file.fileName = "Synthetic"
        cfg = sdr.synth.opensky(skip_ms=file.skip)
        for i in range(cfg.n_sv):
            cfg.sv[i].lnav = 1
        ms = file.skip + track.msToProcessCT_1ms + 19 + track.msToProcessCT_10ms + 3
        dev = sdr.DeviceRecord(ctx, ms * signal.Sample * 2)
        sdr.synth.generate_device(ctx, cfg, dev)
        file.dev = dev
    os.makedirs(args.out, exist_ok=True)
    path = lambda name: os.path.join(args.out, name + ".mat")
    tag10 = str(track.msToProcessCT_10ms // 1000)

    # Acquisition (SDR_main.m:20-30)
    f_acq = path(f"Acquired_{file.fileName}_{file.skip}")
    if not os.path.exists(f_acq):
        Acquired = sdr.acquisition(file, signal, acq, ctx=ctx)
        sio.savemat(f_acq, {"Acquired": {k: np.atleast_2d(getattr(Acquired, k)) for k in
                                         ("sv", "SNR", "Doppler", "codedelay", "fineFreq")}})
    else:
        m = sio.loadmat(f_acq, squeeze_me=True, struct_as_record=False)["Acquired"]
        from types import SimpleNamespace
        Acquired = SimpleNamespace(**{k: np.atleast_1d(getattr(m, k)) for k in
                                      ("sv", "SNR", "Doppler", "codedelay", "fineFreq")})
    if len(Acquired.sv) == 0:
        print("No satellites acquired. Check parameter settings. \n ")
        return
    print("Acquired", list(Acquired.sv))

    # Conventional tracking and navigation-data decoding (SDR_main.m:33-56)
    f_eph = path(f"eph_{file.fileName}_{tag10}")
    if os.path.exists(f_eph):
        print("eph file exists:", f_eph)
        return
    print("Tracking for navigation data decoding ... \n")
    TckResultCT, CN0_Eph, countinx = sdr.trackingCT(file, signal, track, Acquired, ctx=ctx,
                                                     save_countinx=os.path.join(args.out, "countinx.mat"))
    if not TckResultCT:
        print("Not enough raw data for navigation data decoding.  \n\n ")
        return
    prns = [int(p) for p in Acquired.sv]
    sio.savemat(path(f"TckResult_Eph{file.fileName}_{tag10}"),
                {"TckResult_Eph": struct_of(TckResultCT, prns, sdr.abi.FIELDS), "CN0_Eph": CN0_Eph,
                 "countinx": countinx.reshape(1, -1)})
    print("Navigation data decoding ... \n")
    eph, _, sbf = sdr.naviDecode_updated(Acquired, TckResultCT)
    fields = sdr.abi.EPH_FIELDS + ["updateflag"]
    sio.savemat(f_eph, {"eph": struct_of(eph, prns, fields)})
    sio.savemat(path(f"sbf_{file.fileName}_{tag10}"), {"sbf": {"nav1": sbf.nav1.reshape(1, -1),
                                                               "sfb1": sbf.sfb1.reshape(1, -1)}})
    for p in prns:
        e = eph(p)
        print(f"PRN {p:2d}: nav1 {sbf.nav1[p - 1]}, subframes decoded {len(e.sfb)}, "
              f"updateflag {e.updateflag}" + (f", sqrta {e.sqrta[0]:.6f}" if len(e.sqrta) else ""))


if __name__ == "__main__":
    main()
