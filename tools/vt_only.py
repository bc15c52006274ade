"""Vector-tracking driver for timing (trackingVT_POS_updated through gnss_tracking_vt): the
reference's 5 channels and EKF start (tests/vt_nav_common.py) on a device-resident synthetic
Opensky record, NSTEPS 1-ms steps (default 5000 = track.msToProcessVT). Prints the wall time,
the VT kernel's time (hipEvents) and the per-step host share. Args: [NSTEPS] [ITERS]."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: F401,E402  (PyTorch's runtime first)

pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
import vt_nav_common as V  # noqa: E402
from test_gpu_vtnav import _inputs  # noqa: E402

NSTEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = pkg.Context(0)
if os.environ.get("VT_NB"):  # blocks per channel of the step kernel (A/B)
    ctx.set_option(pkg.abi.OPT_VT_BLOCKS, int(os.environ["VT_NB"]))
file, signal, acq, track, solu, cmn = pkg.initParameters()
skip = 5
cfg = pkg.synth.opensky(skip_ms=skip)
dev = pkg.DeviceRecord(ctx, (skip + NSTEPS + 60) * 58000 * 2)
pkg.synth.generate_device(ctx, cfg, dev)
file.skip, file.dev, file.data = skip, dev, None
z = V.fixture()
Acquired, eph, sbf, ct, ns = _inputs(pkg, z, skip)
for it in range(ITERS):
    ctx.set_profiling(it == 0)  # per-step kernel events in the first iteration only
    t = time.perf_counter()
    tck, nsol = pkg.trackingVT_POS_updated(file, signal, track, cmn, solu, Acquired, V.cnslxyz(pkg), eph, sbf,
                                           None, ct, ns, ctx=ctx, nsteps=NSTEPS)
    wall = time.perf_counter() - t
    tm = ctx.timing()
    print(f"vt {NSTEPS} steps x {len(Acquired.sv)} ch: wall {wall * 1e3:.1f} ms ({wall / NSTEPS * 1e6:.1f} us/step), "
          f"loop {tm['track_ms']:.1f} ms, kernel {tm['track_kernel_ms']:.1f} ms "
          f"({tm['track_kernel_ms'] / NSTEPS * 1e3:.1f} us/step{', events' if it == 0 else ', not timed'}), "
          f"launches {tm['track_launches']}, final ENU {nsol.usrPosENU[-1].round(2).tolist()}", flush=True)
