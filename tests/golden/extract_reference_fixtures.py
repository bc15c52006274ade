"""Extract small golden fixtures from the reference's committed result files.

Run in the build container only (reads /root/reference, read-only). The outputs
are data (inputs + expected outputs), committed under tests/golden/:

  ref_acquired.json            Acquired_Opensky_5000.mat, nAcquired_*_5000.mat, countinx.mat
  ref_tckRstCT_10ms_Opensky.npz  subset of SDR_MATLAB-main/tckRstCT_10ms_Opensky.mat
                               (output of trackingCT_POS_updated.m on the real Opensky IF):
                               NCO state for steps 1..60 and 989..1100, discriminator
                               inputs, and carrError/codeError for steps 1..1100.

Only scipy.io.loadmat (a MAT-v5 parser that executes nothing) is used.
"""
import json
import os
import sys

import numpy as np
import scipy.io as sio

REF = "/root/reference/SDR_MATLAB-main"
HERE = os.path.dirname(os.path.abspath(__file__))


def _struct(v):
    return {fn: np.atleast_1d(getattr(v, fn)).tolist() for fn in v._fieldnames}


def main():
    out = {}
    for name, key in [("Acquired_Opensky_5000.mat", "Acquired"),
                      ("nAcquired_Opensky_5000.mat", "nAcquired"),
                      ("nAcquired_Urban_5000.mat", "nAcquired")]:
        d = sio.loadmat(os.path.join(REF, name), squeeze_me=True, struct_as_record=False)
        out[name] = _struct(d[key])
    d = sio.loadmat(os.path.join(REF, "countinx.mat"), squeeze_me=True)
    out["countinx.mat"] = np.atleast_1d(d["countinx"]).astype(int).tolist()
    with open(os.path.join(HERE, "ref_acquired.json"), "w") as f:
        json.dump(out, f, indent=1)

    d = sio.loadmat(os.path.join(REF, "tckRstCT_10ms_Opensky.mat"), squeeze_me=True,
                    struct_as_record=False)
    T = d["TckResultCT_pos"]
    prns = [i + 1 for i, t in enumerate(T) if getattr(t, "P_i", np.array([])).size > 0]
    steps = np.r_[np.arange(0, 60), np.arange(988, 1100)]  # 0-based step indices
    state_fields = ["numSample", "remChip", "remCarrPhase", "codeFreq", "carrFreq",
                    "absoluteSample", "E_i", "E_q", "P_i", "P_q", "L_i", "L_q"]
    arrs = {"prns": np.array(prns), "steps": steps}
    for fld in state_fields:
        arrs[fld] = np.stack([np.asarray(getattr(T[p - 1], fld), dtype=np.float64)[steps]
                              for p in prns])
    for fld in ["carrError", "codeError"]:
        arrs[fld] = np.stack([np.asarray(getattr(T[p - 1], fld), dtype=np.float64)[:1100]
                              for p in prns])
    np.savez_compressed(os.path.join(HERE, "ref_tckRstCT_10ms_Opensky.npz"), **arrs)
    print("prns", prns, "wrote fixtures")


if __name__ == "__main__":
    sys.exit(main())
