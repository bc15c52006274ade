"""Host-side checks of helpers the kernels share with the host (compiled with hipcc,
host code only; no GPU needed)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_colon_make_hint_equals_colonop(tmp_path):
    src = os.path.join(ROOT, "tests", "native", "colon_hint.cpp")
    exe = tmp_path / "colon_hint"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), src],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_fmod_pos_equals_c_fmod(tmp_path):
    src = os.path.join(ROOT, "tests", "native", "fmod_pos.cpp")
    exe = tmp_path / "fmod_pos"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), src],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_div_const_equals_ieee_division(tmp_path):
    """The tracking tail's divisions by Fs and 2*pi (div_const, Markstein's correction)
    return the IEEE quotient the reference's `/` computes (trackingCT.m:80,102,106,146)."""
    src = os.path.join(ROOT, "tests", "native", "markstein.cpp")
    exe = tmp_path / "markstein"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), src],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_multi_device_bookkeeping(tmp_path):
    """gnss_ctx_create_multi's dealing and merging (csrc/group.h): the PRN / channel deal, the
    Acquired / diag rows merged back into PRN-list order, and a sharded call's status equal the
    one-context results (acquisition.m:47-80,84-85; trackingCT.m:22-528 and the channel loop's
    status rule in gnss_api.cpp). Host C++ only."""
    cxx = shutil.which("g++") or HIPCC
    src = os.path.join(ROOT, "tests", "native", "group_test.cpp")
    exe = tmp_path / "group_test"
    subprocess.run([cxx, "-O2", "-std=c++17", "-pthread", "-o", str(exe), src], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
    # the same under ThreadSanitizer: the member threads' shared host state (the reciprocal
    # cache) has no data race
    tsan = tmp_path / "group_test_tsan"
    b = subprocess.run([cxx, "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=thread", "-o", str(tsan), src],
                       capture_output=True, text=True)
    if b.returncode == 0:
        r = subprocess.run([str(tsan)], capture_output=True, text=True)
        if "FATAL: ThreadSanitizer: unexpected memory mapping" not in r.stderr:  # (TSan vs this kernel's ASLR)
            assert r.returncode == 0 and "WARNING: ThreadSanitizer" not in r.stderr, r.stdout + r.stderr[-3000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_acq_fft_contraction_is_fixed_by_source():
    """acq_fft.hip lets the compiler fuse products into sums (`fp contract(fast)`), but no sum
    of two products is left to it: the backend would fuse either one by the schedule, so the
    fused and two-launch correlators (or one kernel after a refactor) could round differently
    and their bit-identity tests fail for no arithmetic reason (round 5: 2 482 such sums, the
    fused-vs-split test failed after a no-op refactor). tools/contract_scan.py over the device
    LLVM IR (acquisition.m:47-61, 103-116 arithmetic)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("contract_scan", os.path.join(ROOT, "tools", "contract_scan.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    n = mod.main(os.path.join(ROOT, "assignment-for-aae6102_gnss-sdr_amd", "csrc", "acq_fft.hip"))
    assert n == 0


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_vt_loop_granules_and_next_read(tmp_path):
    """The VT loop mode's host helpers (gnss_internal.h): a 16-B granule returns its value with
    its tag, one whose halves carry different tags (read mid-rewrite) is rejected, every read
    accepted under a concurrent writer is one it wrote; vt_remchip_next equals vt_finish's
    remChip (trackingVT_POS_updated.m:284), which sizes the next read a step ahead."""
    src = os.path.join(ROOT, "tests", "native", "vt_gran.cpp")
    exe = tmp_path / "vt_gran"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-o", str(exe), src],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
