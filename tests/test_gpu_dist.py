"""The sharded HIP path with its collectives, on one MI355X: two ranks (gloo, both on
device 0, spawned before any GPU call) each run the C-ABI library on their PRN / channel
shard through dist.py -- acquisition PRNs round-robin + the per-PRN all-gather, then
trackingCT channels round-robin into HBM-resident TckResultCT rows
(DeviceTrackOutBuffers, gnss_track_out.flags = GNSS_OUT_DEVICE) + the row-packed
device all-gather. The gathered result must equal the single-process HIP result bit for
bit (trackingCT.m:22-528: channels share no state; acquisition.m:47-80: PRNs neither).
On the 8-GPU node the same code runs over RCCL (bench.py --gpus N)."""
import importlib
import os
import socket
import sys
from types import SimpleNamespace

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

PRNS = [3, 4, 7, 16, 22]
SKIP, N1, N10 = 2, 1000, 60  # (N1 = 1000: the bit-edge search window of trackingCT.m:179-204)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(pkg, po):
    data = po.synth_if(pkg.synth.opensky(skip_ms=SKIP), 0, (SKIP + N1 + 19 + N10 + 4) * 58000)
    file, signal, acq, track, _, _ = pkg.initParameters()
    file.skip, file.data = SKIP, data
    acq.freqMin, acq.freqNum, acq.datalen, acq.L = -5000, 21, 4, 4
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = N1, N10
    return file, signal, acq, track


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
    D = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd.dist")
    import pyoracle as po
    ctx = pkg.Context(0)
    file, signal, acq, track = _setup(pkg, po)
    mine = [PRNS[i] for i in D.shard(len(PRNS), world, rank)]
    A = D.gather_acquired(pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=mine), mine, PRNS)
    nsv = len(A.sv)
    shards = [D.shard(nsv, world, r) for r in range(world)]
    out = {"sv": A.sv, "codedelay": A.codedelay, "fineFreq": A.fineFreq, "SNR": A.SNR}
    for name, taps in (("ept", None), ("acf", pkg.colon(-0.5, 0.1, 0.5))):
        nt = 0 if taps is None else len(taps)
        buf = pkg.DeviceTrackOutBuffers(nsv, track, nt, device="cuda:0")
        pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, channels=shards[rank], raw=True, out=buf)
        D.gather_tracking_rows_device(buf, shards)
        torch.cuda.synchronize()
        out[name + "_rec"] = buf.rec.cpu().numpy()
        if nt:
            out[name + "_taps"] = buf.taps.cpu().numpy()
        out[name + "_len"], out[name + "_cx"] = buf.len.copy(), buf.countinx.copy()
        out[name + "_CN0"] = buf.CN0[: buf.c.cn0_rows].copy()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_hip_equals_single_process(tmp_path, pkg, po, ctx):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    file, signal, acq, track = _setup(pkg, po)
    A = pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=PRNS)
    assert len(A.sv) >= 3
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["sv"], A.sv) and np.array_equal(z["codedelay"], A.codedelay)
        assert np.array_equal(z["fineFreq"], A.fineFreq) and np.array_equal(z["SNR"], A.SNR)
        for name, taps in (("ept", None), ("acf", pkg.colon(-0.5, 0.1, 0.5))):
            full = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
            assert np.array_equal(z[name + "_rec"], full.rec), (r, name)
            if taps is not None:
                assert np.array_equal(z[name + "_taps"], full.taps), (r, name)
            assert np.array_equal(z[name + "_len"], full.len)
            assert np.array_equal(z[name + "_cx"], full.countinx)
            assert np.array_equal(z[name + "_CN0"], full.CN0[: full.c.cn0_rows])


def test_device_output_equals_host_output(pkg, po, ctx):
    """GNSS_OUT_DEVICE: the GPU-expanded TckResultCT (HBM) equals the host-expanded one,
    including a reused buffer's zeroed tail."""
    file, signal, acq, track = _setup(pkg, po)
    A = SimpleNamespace(sv=np.array([3, 16, 22]), SNR=np.zeros(3), Doppler=np.zeros(3),
                        codedelay=np.array([3683, 26051, 2610]),
                        fineFreq=np.array([4580990.0, 4579695.0, 4581565.0]))
    taps = pkg.colon(-0.5, 0.1, 0.5)
    host = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True)
    dev = pkg.DeviceTrackOutBuffers(3, track, len(taps), device="cuda:0")
    dev.rec.fill_(7.0)
    dev.taps.fill_(7.0)
    pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, raw=True, out=dev)
    assert np.array_equal(dev.rec.cpu().numpy(), host.rec)
    assert np.array_equal(dev.taps.cpu().numpy(), host.taps)
    assert np.array_equal(dev.len, host.len) and np.array_equal(dev.countinx, host.countinx)
    # the struct view of a device result (host copy) reads like the host one
    T, cn0, cx = pkg.trackingCT(file, signal, track, A, ctx=ctx, out=dev)
    Th, cn0h, cxh = pkg.trackingCT(file, signal, track, A, ctx=ctx)
    assert np.array_equal(T(16).P_i, Th(16).P_i) and np.array_equal(cn0, cn0h)
