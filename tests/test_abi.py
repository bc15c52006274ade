"""The C-ABI boundary: the library loads, exports every entry point the header
declares, and the ctypes mirror has the header's exact struct layout. No GPU."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gnss_mi355x.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gnss_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg.abi.load()
    names = header_functions()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(pkg.abi.PROTOTYPES), set(names) ^ set(pkg.abi.PROTOTYPES)


def test_abi_version_and_strerror(pkg):
    lib = pkg.abi.load()
    assert lib.gnss_abi_version() == 13
    for code in range(6):
        assert lib.gnss_strerror(code)


STRUCTS = {
    "gnss_file": "GnssFile", "gnss_signal": "GnssSignal", "gnss_acq": "GnssAcq",
    "gnss_acquired": "GnssAcquired", "gnss_acq_diag": "GnssAcqDiag", "gnss_track": "GnssTrack",
    "gnss_track_out": "GnssTrackOut", "gnss_timing": "GnssTiming", "gnss_synth_sv": "GnssSynthSv",
    "gnss_synth": "GnssSynth", "gnss_vt_chan": "GnssVtChan", "gnss_vt_out": "GnssVtOut",
    "gnss_eph_sv": "GnssEphSv", "gnss_vt_nav_cfg": "GnssVtNavCfg", "gnss_vt_nav": "GnssVtNav",
    "gnss_vt_navsol": "GnssVtNavSol",
}


def test_struct_layout_matches_header(pkg):
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(){"]
    for cname, pyname in STRUCTS.items():
        st = getattr(pkg.abi, pyname)
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in st._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-o", exe, c], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    got = dict(l.rsplit(" ", 1) for l in out.strip().splitlines())
    for cname, pyname in STRUCTS.items():
        st = getattr(pkg.abi, pyname)
        assert int(got[cname]) == C.sizeof(st), cname
        for fname, _ in st._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(st, fname).offset, (cname, fname)


def test_ca_code_export_matches_oracle(pkg, po):
    import numpy as np
    for prn in (1, 3, 16, 32, 51):
        assert np.array_equal(pkg.ca_code(prn), po.generate_ca(prn))


def test_context_fails_loudly_without_device(pkg):
    """No HIP device here: creating a context must return an error, not fall back."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = C.c_void_p()
    st = pkg.abi.load().gnss_ctx_create(0, C.byref(h))
    assert st == pkg.abi.EDEVICE and not h.value


def test_missing_library_raises(pkg, tmp_path):
    with pytest.raises(ImportError):
        pkg.abi.load(str(tmp_path / "nope.so"))
