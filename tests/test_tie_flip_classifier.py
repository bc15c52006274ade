"""The config-5 parity test's tie-flip rule on constructed states (CPU): two runs whose replica
coordinates t = tap + remChip + k*codeFreq/Fs straddle an integer for one sample because their
remChip differ by a few 1e-9 chip are a tie flip; a 1e-6-chip difference that moves samples
across a chip boundary is not, nor are two equal states (tests/test_gpu_longrun.py::_tie_flip;
trackingCT.m:96-98)."""
import math

import numpy as np

import test_gpu_longrun as tl


def _states(pkg, r_gpu, r_oracle, cf=1.023e6, n=58000):
    import importlib
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    mg = importlib.import_module("make_golden_cfg5")
    F = pkg.abi.FIELDS
    nco = mg.field_rows(F)[1]
    got = np.zeros((len(F), 2))
    rnco = np.zeros((len(nco), 2))
    got[F.index("remChip"), 0], got[F.index("codeFreq"), 0], got[F.index("numSample"), 1] = r_gpu, cf, n
    rnco[nco.index(F.index("remChip")), 0], rnco[nco.index(F.index("codeFreq")), 0] = r_oracle, cf
    return got, rnco, F, nco


def test_tie_flip_rule(pkg):
    Fs, cf, k0 = 58e6, 1.023e6, 31337
    d = cf / Fs
    frac = math.ceil(k0 * d) - k0 * d          # remChip putting sample k0 on an integer
    r_o = frac + 2e-9                           # the oracle's t just above it ...
    for r_g, want in ((r_o - 4e-9, True),       # ... the GPU's just below: one sample, 4e-9 apart
                      (r_o - 1e-6, False),      # 1e-6 chip apart: not a rounding-level difference
                      (r_o, False)):            # equal states: no sample differs
        got, rnco, F, nco = _states(pkg, r_g, r_o, cf)
        assert tl._tie_flip(got, rnco, F, nco, 1, 0.0, Fs) is want, (r_g - r_o, want)
    # the bounds the config-5 test applies (TIE_TOL): a locked channel's tie must sit within 3e-9
    # chip, an unlocked one's within 6e-8 -- a 4e-8 difference is a tie only for an unlocked loop
    got, rnco, F, nco = _states(pkg, r_o - 4e-8, r_o, cf)
    m = tl._tie_flip_margin(got, rnco, F, nco, 1, 0.0, Fs)
    assert m is not None and tl.TIE_TOL[False] > m > tl.TIE_TOL[True]
    assert not tl._tie_flip(got, rnco, F, nco, 1, 0.0, Fs, tol=tl.TIE_TOL[True])
    assert tl._tie_flip(got, rnco, F, nco, 1, 0.0, Fs, tol=tl.TIE_TOL[False])
