"""Benchmark: correlator throughput (acquisition + trackingCT) on MI355X.

One bench step = one pass of the hot path over one synthetic Opensky-shape IF
record resident in HBM, exactly as SDR_main.m:17-45 runs it:
  * acquisition (BASELINE config 2): 32 PRNs, +-7 kHz / 500 Hz (29 bins),
    datalen 20 ms non-coherent, fine frequency over L = 10 ms;
  * trackingCT (BASELINE config 3): the acquired channels (8 SVs present),
    msToProcessCT_1ms 1000, msToProcessCT_10ms 40000, E/P/L spacing 0.5.
Units: acquisition hypothesis-samples (PRN x bin x ms x Sample) + tracking
channel-samples (one IF sample correlated by one channel, all taps).

Multi-GPU (torchrun, one process per GPU): strong scaling of ONE job -- every rank
holds the same record in its HBM, the 32 PRNs of the acquisition and then the
acquired channels are sharded round-robin over the ranks, and every step ends with
the result gathers (RCCL over xGMI; the TckResultCT rows never leave HBM), so every
rank holds the full outputs. Timing is bracketed by barriers, the max over ranks
is reported, `value` = all ranks' units / that time.
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# the package (and with it the HIP library) is imported in main(), after the N-rank launcher
# has decided whether this process is a parent that only spawns ranks (it never touches the GPU)
pkg = None

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X vector fp64 (half the 157.3 TF fp32 vector rate: 4-cycle wave64 fp64 ops)
N_SIMD = 1024  # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4
SAMPLES_PER_MS = 58000  # Opensky Fs 58 MHz
# counter evidence read by the bench, newest first; each file carries the source digest it was
# measured at (tools/srcdigest.py) and the line says whether it matches the running tree
TRAFFIC_FILES = ("traffic_r06.json", "traffic_r05.json", "traffic_r04.json", "traffic_r03.json", "traffic_r02.json")          # PMC bytes per 10-ms launch
TRACK_SQ_FILES = ("r06_track_sq.json", "r05_track_sq.json", "r04_track_sq.json", "r03_track_sq.json")                            # SQ counters of the tracking launches
ACQ_BOUND_FILES = ("acq_bound_r06.json", "acq_bound_r05.json", "acq_bound_r04.json", "acq_bound_r03.json", "acq_bound_r02.json")     # fp64 acquisition kernels (tools/acq_bound.py)
TRAFFIC_FILES_CFG5 = ("traffic_cfg5_r06.json", "traffic_cfg5_r05.json", "traffic_cfg5_r04.json", "traffic_cfg5_r03.json", "traffic_cfg5_r02.json")  # the 11-tap 10-ms launch
CFG5_SQ_FILES = ("r06_cfg5_sq.json", "r05_cfg5_sq.json", "r04_cfg5_sq.json", "r03_cfg5_sq.json")
TRAFFIC_FILES_CFG4 = ("traffic_cfg4_r06.json", "traffic_cfg4_r05.json", "traffic_cfg4_r04.json", "traffic_cfg4_r03.json")  # the config-4 correlator's kernels, bytes per call
sys.path.insert(0, os.path.join(ROOT, "tools"))
import srcdigest  # noqa: E402

SRC_DIGEST = srcdigest.src_digest()


def evidence(names):
    """The first profiles/<name> that exists, and its provenance: the source digest / commit
    it was measured at and whether that digest is the running tree's."""
    for n in names:
        try:
            with open(os.path.join(ROOT, "profiles", n)) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        meta = d.get("_meta", d) if isinstance(d, dict) else {}
        dig = meta.get("src_digest")
        return d, {"file": f"profiles/{n}", "src_digest": dig, "git_commit": meta.get("git_commit"),
                   "matches_code": dig == SRC_DIGEST}
    return None, None


def valu_roofline(sq, kernel, steps_per_dispatch=None):
    """fp64 VALU line of a kernel from its SQ counter passes (chip totals per dispatch,
    tools/pmc_sq.py): achieved fp64 TFLOP/s (FMA = 2) against the 78.6 TF vector peak, and the
    VALU issue fraction (fp64 ops 4 cycles, other VALU 2 cycles per wave64 instruction on a
    SIMD-32, over 1024 SIMDs x the dispatch duration at 2.4 GHz)."""
    if not sq:
        return None
    k = next((x for x in sq if x != "_meta" and kernel in x), None)
    if k is None:
        return None
    c = {n: v["median_per_dispatch"] for n, v in sq[k].items()}
    need = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU", "duration_us")
    if not all(n in c for n in need):
        return None
    dur = c["duration_us"] * 1e-6
    f64 = c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"]
    flops = 64 * (2 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"])
    cycles = 4 * (f64 + c.get("SQ_INSTS_VALU_TRANS_F64", 0)) + 2 * (c["SQ_INSTS_VALU"] - f64)
    tf = flops / dur / 1e12
    out = {"bound": "valu", "unit": "TFLOP/s", "achieved": round(tf, 3), "peak": FP64_VALU_PEAK_TFLOPS,
           "frac": round(tf / FP64_VALU_PEAK_TFLOPS, 4),
           "valu_issue_frac": round(cycles / (N_SIMD * dur * CLOCK_GHZ * 1e9), 4),
           "fp64_share_of_valu_cycles": round(4 * f64 / cycles, 4),
           "counter_dispatch_us": round(c["duration_us"], 1), "kernel": k}
    if steps_per_dispatch:
        out["valu_instr_per_step"] = round(c["SQ_INSTS_VALU"] / steps_per_dispatch)
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n10", type=int, default=40000, help="msToProcessCT_10ms")
    ap.add_argument("--skip", type=int, default=5000, help="file.skip (ms)")
    ap.add_argument("--datalen", type=int, default=20)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--no-profile-pass", action="store_true")
    ap.add_argument("--workload", choices=["cfg2+3", "cfg4", "cfg5", "dist-selftest"], default="cfg2+3",
                    help="cfg2+3: the headline step (default); cfg4: BASELINE config 4, 32-PRN Urban "
                         "acquisition, PRNs sharded over the ranks; cfg5: BASELINE config 5, 32-channel "
                         "11-tap trackingCT, channels sharded over the ranks; dist-selftest: the launcher, "
                         "shards and result gathers on host arrays only (no GPU, no library: a CPU check "
                         "of the N-rank path, never a bench line)")
    ap.add_argument("--n10-cfg5", type=int, default=90000, help="cfg5 msToProcessCT_10ms")
    ap.add_argument("--multi-ctx", type=int, default=0,
                    help="N > 0: the headline step in ONE process through the C-ABI's multi-device context "
                         "(gnss_ctx_create_multi over devices 0..N-1, the path INTEGRATION.md's MEX takes for "
                         "SDR_main.m:22,38) instead of torch.distributed ranks; BENCH_MULTI_DEVICES=0,0 lists "
                         "the devices explicitly (a one-GPU rehearsal)")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`python3 bench.py --gpus N` without a launcher (RANK unset): start N child processes of
    this same command, one rank per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR 127.0.0.1 /
    MASTER_PORT in their environment), and return the job's exit status. This parent runs before
    anything imports the HIP library or torch, so it never touches a GPU; the children are new
    processes (no fork of GPU state, no exec). Rank 0 prints the one JSON line. If a child fails,
    the others are terminated and the parent exits with that child's status."""
    import ctypes
    import signal
    import subprocess
    port = _free_port()
    procs = []

    def die_with_parent():  # (in the child, before exec: SIGTERM when this parent dies, even by SIGKILL)
        try:
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except OSError:
            pass

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      preexec_fn=die_with_parent))

    def forward(signum, _frame):  # a launcher's SIGTERM / SIGINT reaches every rank
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"bench.py: rank {procs.index(p)} exited with status {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return status


def setup_dist(args):
    rank, world, local = 0, 1, 0
    dist = None
    # (BENCH_FORCE_DIST: a rehearsal hook, never set by the driver -- a one-rank torchrun job takes
    # the distributed path, process group and gathers included, so the RCCL calls run on a 1-GPU box)
    if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("BENCH_FORCE_DIST"):
        import torch
        import torch.distributed as dist
        rank = int(os.environ["RANK"])
        world = int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", rank))
        # rehearsal hooks for a one-GPU box (never set by the driver): every rank on one
        # device, collectives over gloo
        if os.environ.get("BENCH_FORCE_DEVICE"):
            local = int(os.environ["BENCH_FORCE_DEVICE"])
        torch.cuda.set_device(local)
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local, dist


def barrier(dist, local):
    if dist is not None:
        import torch
        torch.cuda.synchronize(local)
        dist.barrier()


def max_over_ranks(dist, local, x):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, local, x):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def run_cfg5(args, rank, world, local, dist, ctx):
    """BASELINE config 5: trackingCT of 32 channels (every PRN present) with the 11 ACF taps
    -0.5:0.1:0.5 (trackingCT_multiCorr-GIVEN.m:25 tap semantics), 1000 ms @1 ms + n10 ms
    @10 ms on a synthetic record at Opensky rates; the 32 channels are sharded round-robin
    over the ranks (strong scaling: the total work is fixed), each rank tracking its
    channels of the same record; the step ends with an all-gather of every rank's rows
    (RCCL), so every rank holds the full TckResultCT."""
    import importlib as _il
    D = _il.import_module("assignment-for-aae6102_gnss-sdr_amd.dist")
    from types import SimpleNamespace
    file, signal, acq, track, _, _ = pkg.initParameters()
    S = signal.Sample
    skip, nsv = 0, 32
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, args.n10_cfg5
    cfg = pkg.synth.all_prn(nsv, skip_ms=skip)
    dev = pkg.DeviceRecord(ctx, (skip + 1000 + 19 + args.n10_cfg5 + 3) * S * 2)
    pkg.synth.generate_device(ctx, cfg, dev)
    file.skip, file.dev = skip, dev
    cds = pkg.synth.codedelays(cfg, skip)  # where the scenario put each SV (acquisition.m convention)
    A = SimpleNamespace(sv=np.array([cfg.sv[i].prn for i in range(nsv)]), SNR=np.zeros(nsv),
                        Doppler=np.zeros(nsv), codedelay=np.array(cds),
                        fineFreq=np.array([signal.IF + cfg.sv[i].doppler_hz for i in range(nsv)]))
    taps = pkg.colon(-0.5, 0.1, 0.5)
    mine = D.shard(nsv, world, rank)
    shards = [D.shard(nsv, world, r) for r in range(world)]
    outs = [None]

    def one_step():
        # TckResultCT rows (and the 11 taps) stay in HBM; N > 1: every rank ends with all 32
        # channels by one RCCL all-gather of the ranks' own rows, without a host round trip
        if outs[0] is None:
            outs[0] = pkg.DeviceTrackOutBuffers(nsv, track, len(taps), device=f"cuda:{local}")
        buf = pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, channels=mine, raw=True,
                             out=outs[0])
        tt = ctx.timing()
        if dist is not None:
            D.gather_tracking_rows_device(buf, shards)
        return tt

    for _ in range(args.warmup):
        one_step()
    barrier(dist, local)
    t0 = time.perf_counter()
    units = 0
    for _ in range(args.steps):
        units += one_step()["track_channel_samples"]
    barrier(dist, local)
    elapsed = max_over_ranks(dist, local, time.perf_counter() - t0)
    total = sum_over_ranks(dist, local, float(units))
    roof = None
    if not args.no_profile_pass:
        ctx.set_profiling(True)
        pkg.trackingCT(file, signal, track, A, ctx=ctx, taps=taps, channels=mine, raw=True, out=outs[0])
        tp = ctx.timing()
        ctx.set_profiling(False)
        launches = max(1, tp["track10_launches"])
        avg_ms = tp["track10_kernel_ms"] / launches
        bpl = 2.0 * tp["track10_channel_samples"] / launches
        achieved = bpl / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": "10-ms phase correlator, 11 taps (persistent or per-step launches)",
                "launches": int(launches), "avg_launch_us": round(avg_ms * 1e3, 3),
                "algorithmic_bytes_per_launch": bpl}
        tj, prov = evidence(TRAFFIC_FILES_CFG5)
        if world == 1 and tj:
            roof["traffic"] = tj.get("bytes_per_launch")
            roof["traffic_source"] = prov
        # what binds it: fp64 VALU (the 32 channels share record lines in L2 / MALL, so the HBM
        # fraction overstates the memory work), from the SQ passes of the same launch shape
        sq, sq_prov = evidence(CFG5_SQ_FILES)
        v = valu_roofline(sq, "track_run_kernel<11, 3", steps_per_dispatch=40)
        if v:
            v["source"] = sq_prov
            v["counter_workload"] = "tools/track_only.py 1000 400 11 32 (32 channels x 11 taps, 40 10-ms steps)"
            roof["valu"] = v
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline_cfg5(file, signal, track, A, taps, dev)
    line = {"metric": "correlator Msamples/s (trackingCT cfg5), whole job", "value": round(total / elapsed / 1e6, 2),
            "unit": "Msamples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "int8 in, f64 compute",
            "data": "synthetic 32-SV IF at Opensky rates (int8 I/Q), resident in HBM",
            "config": {"workload": f"trackingCT cfg5 (32 ch, 11 taps -0.5:0.1:0.5, 1000 ms @1ms + "
                                   f"{args.n10_cfg5} ms @10ms)", "parallelism": f"channels x{world}",
                       "channels_per_rank": len(mine),
                       "channels_by_rank": [len(x) for x in shards]},
            **dist_world(dist),
            "code": code_stamp(),
            "roofline": roof, "cpu_baseline": cpu}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def run_cfg4(args, rank, world, local, dist, ctx):
    """BASELINE config 4: acquisition of PRNs 1..32 with the Urban parameters (IF = 0,
    Fs = 26 MHz assumed, +-10 kHz / 250 Hz = 81 bins, datalen 10, L = 10) on a
    synthetic Urban record; the PRNs are sharded round-robin over the ranks (strong
    scaling) and the step ends with the all-gather of the per-PRN results (RCCL), so
    every rank holds the full Acquired."""
    import importlib as _il
    D = _il.import_module("assignment-for-aae6102_gnss-sdr_amd.dist")
    from types import SimpleNamespace
    Fs, skip = 26e6, 1000
    S = 26000
    file = SimpleNamespace(skip=skip, dataType=2, dataPrecision=1, data=None, fileRoute=None, dev=None)
    signal = SimpleNamespace(IF=0.0, Fs=Fs, codeFreqBasis=1.023e6, ms=1e-3, Sample=S, codelength=1023.0)
    acq = SimpleNamespace(freqNum=81, freqMin=-10000, freqStep=250, datalen=10, L=10)
    cfg = pkg.synth.urban(skip_ms=skip, Fs=Fs)
    dev = pkg.DeviceRecord(ctx, (skip + 30) * S * 2)
    pkg.synth.generate_device(ctx, cfg, dev)
    file.dev = dev
    prns = list(range(1, 33))
    mine = [prns[i] for i in D.shard(len(prns), world, rank)]

    def one_step():
        A = pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=mine)
        ta = ctx.timing()
        if dist is not None:
            A = D.gather_acquired(A, mine, prns, device=f"cuda:{local}")
        return A, ta

    for _ in range(args.warmup):
        one_step()
    barrier(dist, local)
    t0 = time.perf_counter()
    units = 0
    corr_ms = 0.0
    for _ in range(args.steps):
        A, ta = one_step()
        units += ta["acq_hypothesis_samples"]
        corr_ms += ta["acq_corr_ms"]
    barrier(dist, local)
    elapsed = max_over_ranks(dist, local, time.perf_counter() - t0)
    total = sum_over_ranks(dist, local, float(units))
    # the acquisition model (16 B per hypothesis-sample) over this rank's correlation
    # time (the fine-frequency FFTs excluded, timed in acq_ms)
    roof = None
    if corr_ms > 0:
        ach = 16.0 * units / (corr_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": "acquisition correlator (fwd/inv P x 2000 FFT passes, fp64), rank 0",
                "corr_ms_per_step": round(corr_ms / args.steps, 3),
                "algorithmic_bytes_per_step": 16.0 * units / args.steps}
        tj, prov = evidence(TRAFFIC_FILES_CFG4)
        if tj and world == 1:  # (bytes of one full 32-PRN call: the N=1 step)
            roof["traffic"] = tj.get("bytes_per_call")
            roof["traffic_kernels"] = {k: v["bytes_per_call"] for k, v in tj.get("kernels", {}).items()}
            roof["traffic_source"] = prov
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline_cfg4(file, signal, acq, dev, prns, S)
    line = {"metric": "correlator Msamples/s (acquisition cfg4), whole job",
            "value": round(total / elapsed / 1e6, 2), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "int8 in, f64 correlation / f64 fine search",
            "data": "synthetic Urban-shape IF (int8 I/Q, Fs 26 MHz, IF 0), resident in HBM",
            "config": {"workload": "acquisition cfg4 (32 PRN, +-10kHz/250Hz, 10 ms, L 10)",
                       "parallelism": f"PRNs x{world}", "prns_per_rank": len(mine),
                       "prns_by_rank": [len(D.shard(len(prns), world, r)) for r in range(world)]},
            **dist_world(dist),
            "acquired": [int(x) for x in A.sv], "acq_ms_rank0": round(ta["acq_ms"], 3),
            "code": code_stamp(),
            "roofline": roof, "cpu_baseline": cpu}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def dist_world(dist):
    """What the line says about the process group: its size and backend (RCCL = "nccl")."""
    if dist is None:
        return {"rccl_world": 1, "backend": None}
    return {"rccl_world": dist.get_world_size(), "backend": dist.get_backend()}


def run_dist_selftest(args):
    """The N-rank path without a GPU (CPU test of the launcher): each rank takes its round-robin
    shard of 32 PRNs and of 8 channels, fills its rows of host result tables with a seeded
    function of the unit index (the same values whatever rank computes them), and runs the bench's
    result gathers (dist.gather_acquired, dist.gather_tracking_rows) over the process group; rank 0
    prints a digest of the gathered tables, which must equal the N = 1 run's."""
    import hashlib
    import torch.distributed as tdist
    from types import SimpleNamespace
    D = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd.dist")
    dist = None
    rank, world = 0, 1
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        tdist.init_process_group("gloo")
        dist, rank, world = tdist, tdist.get_rank(), tdist.get_world_size()
    if os.environ.get("BENCH_SELFTEST_FAIL_RANK") == str(rank):  # (test hook: a failing rank)
        sys.exit(3)
    if os.environ.get("BENCH_SELFTEST_SLEEP"):  # (test hook: a busy rank, its pid recorded)
        with open(os.environ["BENCH_SELFTEST_PIDFILE"], "a") as fh:
            fh.write(f"{os.getpid()}\n")
        time.sleep(float(os.environ["BENCH_SELFTEST_SLEEP"]))
    t0 = time.perf_counter()
    prns = list(range(1, 33))
    mine = [prns[i] for i in D.shard(32, world, rank)]
    acq_prns = [p for p in mine if p % 3]  # "acquired": a rank-independent rule per PRN
    A = SimpleNamespace(sv=np.array(acq_prns, dtype=np.int64), SNR=np.array([17.0 + p / 7 for p in acq_prns]),
                        Doppler=np.array([500.0 * (p % 29 - 14) for p in acq_prns]),
                        codedelay=np.array([1000 * p + 7 for p in acq_prns], dtype=np.int64),
                        fineFreq=np.array([4.58e6 + 13.0 * p for p in acq_prns]))
    if dist is not None:
        A = D.gather_acquired(A, mine, prns)
    nch, nrow, nlen = 8, 18, 50
    rec = np.zeros((nch, nrow, nlen))
    buf = SimpleNamespace(rec=rec, len=np.zeros(nch, dtype=np.int64), countinx=np.zeros(nch, dtype=np.int64),
                          CN0=np.zeros((4, nch)), taps=None, c=SimpleNamespace(cn0_rows=0))
    shards = [D.shard(nch, world, r) for r in range(world)]
    for c in shards[rank]:
        buf.rec[c] = np.random.default_rng(c).standard_normal((nrow, nlen))
        buf.len[c], buf.countinx[c] = 1000 + c, c % 20
        buf.CN0[:, c] = 40.0 + c + np.arange(4)
    buf.c.cn0_rows = 4
    if dist is not None:
        D.gather_tracking_rows(buf, shards)
    h = hashlib.sha256()
    for a in (A.sv, A.SNR, A.Doppler, A.codedelay, A.fineFreq, buf.rec, buf.len, buf.countinx, buf.CN0):
        h.update(np.ascontiguousarray(a).tobytes())
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = __import__("torch").tensor([elapsed], dtype=__import__("torch").float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    line = {"metric": "dist-selftest (not a bench line)", "n_gpus": world, "digest": h.hexdigest(),
            "acquired": [int(x) for x in A.sv], "ms": round(elapsed * 1e3, 3),
            "spawned": bool(os.environ.get("BENCH_SPAWNED")),
            "config": {"prns_per_rank": [len(D.shard(32, world, r)) for r in range(world)],
                       "channels_per_rank": [len(s) for s in shards]}, **dist_world(dist)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    global pkg
    args = parse()
    # N ranks with no launcher: this process only spawns them (before any GPU or library import)
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
    if args.workload == "dist-selftest":
        return run_dist_selftest(args)
    if args.multi_ctx > 0:
        if args.gpus > 1 or args.workload != "cfg2+3":
            sys.exit("bench.py: --multi-ctx runs the cfg2+3 step in one process (no --gpus)")
        import torch  # noqa: F401
        devs = [int(x) for x in os.environ.get("BENCH_MULTI_DEVICES", "").split(",") if x.strip()] or \
            list(range(args.multi_ctx))
        ctx = pkg.Context(devices=devs)
        return run_headline(args, 0, 1, devs[0], None, ctx, multi=devs)
    rank, world, local, dist = setup_dist(args)
    import torch  # noqa: F401  (before the library: device-resident outputs are torch tensors)
    ctx = pkg.Context(local)
    if args.workload == "cfg5":
        return run_cfg5(args, rank, world, local, dist, ctx)
    if args.workload == "cfg4":
        return run_cfg4(args, rank, world, local, dist, ctx)
    return run_headline(args, rank, world, local, dist, ctx)


def run_headline(args, rank, world, local, dist, ctx, multi=None):
    """The headline step (acquisition cfg2 + trackingCT cfg3), on torch.distributed ranks
    (world > 1), on one GPU, or (multi = the device list) in one process through the C-ABI's
    multi-device context, whose members deal the PRNs and channels among themselves."""
    import importlib as _il
    D = _il.import_module("assignment-for-aae6102_gnss-sdr_amd.dist")
    file, signal, acq, track, _, _ = pkg.initParameters()
    S = signal.Sample
    file.skip = args.skip
    acq.freqMin, acq.freqStep, acq.datalen, acq.L = -7000, 500, args.datalen, 10
    acq.freqNum = int(2 * abs(acq.freqMin) / acq.freqStep + 1)
    track.msToProcessCT_1ms, track.msToProcessCT_10ms = 1000, args.n10

    # ONE record (the same bytes on every rank: each rank's HBM holds its own copy, made by
    # the HIP generator outside the timed region): byte 0 .. skip + 1000 + 19 + n10 (+ margin) ms
    rec_ms = args.skip + 1000 + 19 + args.n10 + 3
    cfg = pkg.synth.opensky(skip_ms=args.skip, seed=6102)
    dev = pkg.DeviceRecord(ctx, rec_ms * S * 2)
    pkg.synth.generate_device(ctx, cfg, dev)
    file.dev = dev

    # strong scaling of one job: acquisition PRNs 1..32 and then the acquired
    # channels round-robin over the ranks; every step ends with the result gathers (RCCL
    # over xGMI on the node, device-resident TckResultCT rows), so every rank holds the
    # full Acquired and TckResultCT. N = 1: the same step without the gathers.
    prns = list(range(1, 33))
    my_prns = [prns[i] for i in D.shard(len(prns), world, rank)]
    outs = [None]  # the trackingCT output buffers (HBM), reused from step to step
    gather_s = [0.0]  # host wall time inside the result gathers (distributed path only)
    # (distributed path) the previous step's tracking gather, enqueued on the GPU and completed
    # after this step's acquisition: its host round trip would otherwise leave the GPU idle right
    # before the acquisition, which then starts slower (profiles/r05_dist_overhead.txt); the last
    # step's is completed inside the timed region (finish_gather)
    pending = [None]

    def finish_gather():
        if pending[0] is not None:
            g0 = time.perf_counter()
            pending[0]()
            pending[0] = None
            gather_s[0] += time.perf_counter() - g0

    skip_gathers = bool(os.environ.get("BENCH_DIAG_NO_GATHER")) and world == 1  # (diagnostic hook)

    def one_step():
        A = pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=my_prns)
        ta = ctx.timing()
        finish_gather()
        if dist is not None and not skip_gathers:
            g0 = time.perf_counter()
            A = D.gather_acquired(A, my_prns, prns, device=f"cuda:{local}")
            gather_s[0] += time.perf_counter() - g0
        nsv = len(A.sv)
        shards = [D.shard(nsv, world, r) for r in range(world)]
        if outs[0] is None or not outs[0].fits(nsv, track, 0):
            outs[0] = pkg.DeviceTrackOutBuffers(nsv, track, 0, device=f"cuda:{local}")
        # the previous step's deferred gather still scatters into outs[0] until finish_gather()
        # has run; trackingCT must not write the buffers before that
        assert pending[0] is None, "tracking gather still pending on the output buffers"
        buf = pkg.trackingCT(file, signal, track, A, ctx=ctx, channels=shards[rank], raw=True, out=outs[0])
        tt = ctx.timing()
        if dist is not None and not skip_gathers:
            g0 = time.perf_counter()
            pending[0] = D.gather_tracking_rows_device(buf, shards, defer=True)
            gather_s[0] += time.perf_counter() - g0
        return A, ta, tt, buf, shards

    for _ in range(args.warmup):
        one_step()
    finish_gather()
    barrier(dist, local)
    gather_s[0] = 0.0
    t0 = time.perf_counter()
    acq_units = trk_units = 0
    acq_ms = trk_ms = acq_corr_ms = acq_fine_ms = 0.0
    h2d = 0  # record bytes copied in the timed steps (multi-device context: 0, the copies stay resident)
    for _ in range(args.steps):
        A, ta, tt, buf, shards = one_step()
        h2d += int(ta["h2d_bytes"]) + int(tt["h2d_bytes"])
        acq_units += ta["acq_hypothesis_samples"]
        trk_units += tt["track_channel_samples"]
        acq_ms += ta["acq_ms"]
        acq_corr_ms += ta["acq_corr_ms"]
        acq_fine_ms += ta["acq_fine_ms"]
        trk_ms += tt["track_ms"]
    finish_gather()  # (the last step's tracking gather, inside the timed region)
    barrier(dist, local)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(dist, local, elapsed)
    units = sum_over_ranks(dist, local, float(acq_units + trk_units))
    nch = len(A.sv)
    mine = shards[rank]
    # the step's outputs, checked (not timed): the scenario's 8 SVs acquired, every channel
    # tracked to full length, the gathered TckResultCT complete on this rank
    full_len = [1000 + int(c) + args.n10 for c in buf.countinx]
    outputs_ok = (sorted(int(x) for x in A.sv) == sorted(pkg.synth.OPENSKY_SV)
                  and [int(x) for x in buf.len] == full_len
                  and bool((buf.rec[:, abi_f("numSample"), 0] > 0).all().item()))

    # roofline of the dominant kernel: the tracking correlator of the 10-ms phase (most
    # of the time): the persistent track_run_kernel<3, 3, false> (one launch runs the
    # whole phase; 24-sample lanes) or, where its grid cannot be resident,
    # track_step_kernel<3, 3, false> (one launch per step). A profiling pass brackets every
    # launch with hipEvents on the ctx stream; algorithmic bytes = 2 B (int8 I + Q) per
    # channel-sample of the launch.
    roof = None
    if multi:  # (the group's timing combines its members': the per-launch roofline is the N = 1 line's)
        args.no_profile_pass, args.no_cpu = True, True
    if not args.no_profile_pass:
        ctx.set_profiling(True)
        pkg.trackingCT(file, signal, track, A, ctx=ctx, channels=mine, raw=True, out=outs[0])
        tp = ctx.timing()
        ctx.set_profiling(False)
        launches = tp["track10_launches"]
        avg_ms = tp["track10_kernel_ms"] / max(1, launches)
        bytes_per_launch = 2.0 * tp["track10_channel_samples"] / max(1, launches)
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": ("track_run_kernel<3, 3, false, false> (persistent: every step of the 10-ms phase, "
                           "all channels of the rank)" if launches <= 2 else
                           "track_step_kernel<3, 3, false> (10-ms phase step, all channels)"),
                "steps_per_launch": round(tp["track10_channel_samples"] / max(1, launches) /
                                          (len(mine) * 10 * SAMPLES_PER_MS), 1),
                "launches": int(launches), "avg_launch_us": round(avg_ms * 1e3, 3),
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "all_steps_avg_launch_us": round(tp["track_kernel_ms"] * 1e3 / max(1, tp["track_launches"]), 3),
                "track_wall_ms_profiling": round(tp["track_ms"], 3)}
        tj, prov = evidence(TRAFFIC_FILES)
        if world == 1 and tj:
            # PMC HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE) of the same kernel and its
            # rocprofv3 kernel-trace average, from the separate rocprofv3 passes (tools/gpu.sh
            # traffic; a PMC pass cannot run inside this process); prov says whether they were
            # measured on the code this bench runs
            roof["traffic"] = tj.get("bytes_per_launch")
            roof["traffic_source"] = prov
            roof["rocprof_avg_launch_us"] = tj.get("rocprof_avg_launch_us")
        sq, sq_prov = evidence(TRACK_SQ_FILES)
        v = valu_roofline(sq, "track_run_kernel<3, 3", steps_per_dispatch=40)
        if v:
            v["source"] = sq_prov
            v["counter_workload"] = "tools/track_only.py 1000 400 (8 channels, 40 10-ms steps per dispatch)"
            roof["valu"] = v

    # the acquisition's fp32 fast mode (gnss_ctx_set_acq_precision(ctx, 0)) on the same
    # record, after the timed region: its time and whether its decisions equal the fp64 ones
    fast = None
    if not args.no_profile_pass:
        ctx.set_acq_precision(False)
        try:
            pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=my_prns)
            f_ms = f_corr = 0.0
            for _ in range(2):
                Af = pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=my_prns)
                tf_ = ctx.timing()
                f_ms += tf_["acq_ms"] / 2
                f_corr += tf_["acq_corr_ms"] / 2
        finally:
            ctx.set_acq_precision(True)
        Ad = pkg.acquisition(file, signal, acq, ctx=ctx, prn_list=my_prns)
        same = all(np_equal(getattr(Af, f), getattr(Ad, f)) for f in ("sv", "codedelay", "Doppler", "fineFreq"))
        fast = {"dtype": "f32 correlation + f64 fine search", "acq_ms": round(f_ms, 3),
                "corr_ms": round(f_corr, 3),
                "acq_Msamples_s": round(ta["acq_hypothesis_samples"] / (f_ms * 1e-3) / 1e6, 2),
                "decisions_equal_fp64": bool(same)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(file, signal, acq, track, A, dev, args, ta, tt)

    value = units / elapsed / 1e6
    step_ms = elapsed / args.steps * 1e3
    line = {
        "metric": "correlator Msamples/s (acq+track), whole job",
        "value": round(value, 2),
        "unit": "Msamples/s",
        "n_gpus": world if not multi else len(set(multi)),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int8 in; acquisition: f64 correlation + f64 fine search; tracking: f64",
        "dtype_per_leg": {"acquisition_correlation": "f64", "acquisition_fine_frequency": "f64",
                          "tracking": "f64"},
        "data": "synthetic Opensky-shape IF (int8 I/Q, Fs 58 MHz, IF 4.58 MHz), resident in HBM",
        "config": {"workload": "acquisition cfg2 (32 PRN, +-7kHz/500Hz, 20 ms) + trackingCT cfg3 "
                               f"({nch} ch, 1000 ms @1ms + {args.n10} ms @10ms, E/P/L)",
                   "parallelism": (f"PRNs and channels x{world} (one record, strong scaling)" if not multi else
                                   f"C-ABI multi-device context, members on devices {multi} (one process; "
                                   "PRNs and channels dealt over the members, record resident per member)"),
                   "prns_per_rank": len(my_prns), "channels_per_rank": len(mine),
                   "prns_by_rank": [len(D.shard(len(prns), world, r)) for r in range(world)],
                   "channels_by_rank": [len(x) for x in shards]},
        **dist_world(dist),
        "outputs_ok": outputs_ok,
        **({"multi_ctx": {"devices": multi, "members": ctx.members, "resident_records": ctx.resident_records,
                          "record_bytes_copied_in_timed_steps": h2d}} if multi else {}),
        "acquired": [int(x) for x in A.sv],
        "per_gpu_Msamples_s": round(value / world, 2),
        "acq_Msamples_s": round(acq_units / (acq_ms * 1e-3) / 1e6, 2) if acq_ms else None,
        "track_Msamples_s": round(trk_units / (trk_ms * 1e-3) / 1e6, 2) if trk_ms else None,
        "acq_ms": round(acq_ms / args.steps, 3),
        "track_ms": round(trk_ms / args.steps, 3),
        # (distributed path) rank 0's host wall time inside the result gathers per timed step
        "gather_ms": round(gather_s[0] / args.steps * 1e3, 3) if dist is not None else None,
        # device-busy evidence of the timed steps: the ctx stream's event-timed acquisition +
        # tracking spans over the step's wall time (rank 0)
        "device_busy_frac": round((acq_ms + trk_ms) / args.steps / step_ms, 4),
        "roofline": roof,
        # the acquisition's own line (16 B per hypothesis-sample over the
        # correlation time, the fine-frequency FFTs timed separately); frac_fp64_model: the
        # same model restated at the precision the path computes in (32 B: a complex-fp64
        # spectrum read + an fp64 accumulator read and write)
        "acq_roofline": ({"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                          "achieved": round(16.0 * acq_units / (acq_corr_ms * 1e-3) / 1e9, 2),
                          "frac": round(16.0 * acq_units / (acq_corr_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                          "frac_fp64_model": round(32.0 * acq_units / (acq_corr_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                          "corr_ms": round(acq_corr_ms / args.steps, 3),
                          "fine_ms": round(acq_fine_ms / args.steps, 3)} if acq_corr_ms else None),
        # what bounds the acquisition kernels (PMC counters + rocprofv3 averages of this
        # round's separate passes, tools/acq_bound.py; a PMC pass cannot run in this process)
        "acq_kernel_bounds": acq_bounds(),
        "acq_fp32_fast_mode": fast,
        "code": code_stamp(),
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def acq_bounds():
    d, prov = evidence(ACQ_BOUND_FILES)
    return {"source": prov, "kernels": d.get("kernels", d)} if d else None


def np_equal(a, b):
    import numpy as np
    return bool(np.array_equal(np.asarray(a), np.asarray(b)))


def abi_f(name):
    return pkg.abi.FIELDS.index(name)


def host_cpu():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


def cpu_baseline_cfg4(file, signal, acq, dev, prns, S):
    """Config 4's CPU leg: the oracle's acquisition with the Urban grid (81 bins) on a bounded
    sample (2 of the 10 non-coherent ms, + the fine search): 1 PRN on one thread and the 32
    PRNs on a thread each, median of 3; hypothesis-samples per second."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    from types import SimpleNamespace
    win = dev.download()
    f2 = SimpleNamespace(**vars(file))
    f2.data, f2.dev = win, None
    a1 = SimpleNamespace(**vars(acq))
    a1.datalen = 2

    def leg(pl, nt):
        r = []
        for _ in range(3):
            t = time.perf_counter()
            po.acquisition(f2, signal, a1, prn_list=pl, nthreads=nt)
            r.append(len(pl) * a1.freqNum * a1.datalen * S / (time.perf_counter() - t))
        return float(np.median(r))

    one = leg([prns[0]], 1)
    nt = quota_threads(len(prns))
    many = leg(list(prns), nt)
    model, ncpu = host_cpu()
    return {"value": round(many / 1e6, 4), "unit": "Msamples/s", "cores": nt, "kind": "port",
            "sample": f"oracle/ C fp64 restatement, acquisition of the {len(prns)} PRNs on {nt} threads over "
                      f"{a1.freqNum} bins x {a1.datalen} ms + fine FFT (median of 3)",
            "one_thread": {"value": round(one / 1e6, 4), "sample": "1 PRN, same grid"},
            "cpu_quota": cpu_quota(), "host_cpu": model, "nproc": ncpu}


def cpu_baseline_cfg5(file, signal, track, A, taps, dev):
    """Config 5's CPU leg: the oracle's trackingCT with the same 11 taps on a bounded sample
    (1 000 ms @1 ms + 100 ms @10 ms; 1 channel on one thread, every channel of the step on a
    thread of its own, median of 3), channel-samples per second."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    from types import SimpleNamespace
    S = signal.Sample
    n10s = 100
    win = dev.download(0, (1000 + 19 + n10s + 3) * S * 2)
    f2 = SimpleNamespace(skip=0, dataType=2, dataPrecision=1, data=win, fileRoute=None, dev=None)
    tr = SimpleNamespace(**vars(track))
    tr.msToProcessCT_10ms = n10s

    def leg(nch, nt):
        A1 = SimpleNamespace(sv=A.sv[:nch], SNR=A.SNR[:nch], Doppler=A.Doppler[:nch],
                             codedelay=A.codedelay[:nch], fineFreq=A.fineFreq[:nch])
        r = []
        for _ in range(3):
            t = time.perf_counter()
            po.trackingCT(f2, signal, tr, A1, taps=np.asarray(taps), nthreads=nt)
            r.append(nch * (1000 + n10s) * S / (time.perf_counter() - t))
        return float(np.median(r))

    one = leg(1, 1)
    nall = len(A.sv)
    nt = quota_threads(nall)
    many = leg(nall, nt)
    model, ncpu = host_cpu()
    return {"value": round(many / 1e6, 4), "unit": "Msamples/s", "cores": nt, "kind": "port",
            "sample": f"oracle/ C fp64 restatement, trackingCT with 11 taps, {nall} channels x (1000 ms @1ms "
                      f"+ {n10s} ms @10ms) on {nt} threads (median of 3)",
            "one_thread": {"value": round(one / 1e6, 4), "sample": "1 channel, same length"},
            "cpu_quota": cpu_quota(), "host_cpu": model, "nproc": ncpu}


def cpu_baseline(file, signal, acq, track, A, dev, args, ta, tt):
    """The CPU fp64 restatement (oracle/, C, -O2) timed on a bounded sample of the same
    workload (SURVEY 8d / BASELINE.md 2): one thread, and every unit of the step on a thread of
    its own (the 32 PRNs of the acquisition, the acquired channels of trackingCT; OpenMP across
    PRNs / channels), median of 3 runs each, plus the numpy restatement (the "MATLAB-like
    vectorised" proxy, tests/numpy_twin.py) on one tracking step set. Per-unit rates are
    extrapolated to the GPU step's unit mix. Labelled "restatement", never "MATLAB"."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import pyoracle as po
    from types import SimpleNamespace
    S = signal.Sample
    # bounded sample: IF window [skip, skip + 1000 + 19 + n10s + 2] ms
    n10s = 200
    lo = file.skip * S * 2
    nbytes = (1000 + 19 + n10s + 4) * S * 2
    win = dev.download(lo, nbytes)
    f2 = SimpleNamespace(skip=0, dataType=2, dataPrecision=1, data=win, fileRoute=None, dev=None)
    a1 = SimpleNamespace(**vars(acq))
    a1.datalen = 4  # the same grid (29 bins x S) over 4 non-coherent ms
    tr = SimpleNamespace(**vars(track))
    tr.msToProcessCT_10ms = n10s
    U_acq, U_trk = ta["acq_hypothesis_samples"], tt["track_channel_samples"]

    def leg(nprn, nch, reps):
        # one PRN / channel per thread: acquisition of nprn PRNs, trackingCT of nch channels
        prn_list = [int(p) for p in (list(A.sv) + [p for p in range(1, 33) if p not in A.sv])[:nprn]]
        A1 = SimpleNamespace(sv=A.sv[:nch], SNR=A.SNR[:nch], Doppler=A.Doppler[:nch],
                             codedelay=A.codedelay[:nch], fineFreq=A.fineFreq[:nch])
        ra, rt = [], []
        for _ in range(reps):
            t = time.perf_counter()
            po.acquisition(f2, signal, a1, prn_list=prn_list, nthreads=quota_threads(nprn))
            ra.append(len(prn_list) * a1.freqNum * a1.datalen * S / (time.perf_counter() - t))
            t = time.perf_counter()
            po.trackingCT(f2, signal, tr, A1, nthreads=quota_threads(nch))
            rt.append(nch * (1000 + n10s) * S / (time.perf_counter() - t))
        r_acq, r_trk = float(np.median(ra)), float(np.median(rt))
        return r_acq, r_trk, (U_acq + U_trk) / (U_acq / r_acq + U_trk / r_trk)

    a_1, t_1, v_1 = leg(1, 1, 3)
    n_prn, n_ch = 32, len(A.sv)
    a_n, t_n, v_n = leg(n_prn, n_ch, 3)
    # numpy restatement (one thread, vectorised like the MATLAB code): 10 correlator steps
    # of 10 ms (trackingCT.m:96-118) and one PRN's 29-bin x 1 ms acquisition (:40-78)
    np_trk = np_acq = None
    try:
        import numpy_twin as tw
        ca = tw.ca_code(int(A.sv[0]))
        t = time.perf_counter()
        for k in range(10):
            tw.correlate_step(win[2 * 10 * S * k:], 10 * S, 0.0, 1.023e6, signal.Fs, float(A.fineFreq[0]),
                              0.0, ca, [-0.5, 0.0, 0.5])
        np_trk = 10 * 10 * S / (time.perf_counter() - t)
        t = time.perf_counter()
        tw.acquisition(win[: 2 * S], S, signal.Fs, signal.IF, signal.codeFreqBasis, acq.freqMin, acq.freqStep,
                       acq.freqNum, 1, [int(A.sv[0])])
        np_acq = acq.freqNum * S / (time.perf_counter() - t)
    except Exception:
        pass
    model, ncpu = host_cpu()
    th_a, th_t = quota_threads(n_prn), quota_threads(n_ch)
    return {"value": round(v_n / 1e6, 4), "unit": "Msamples/s", "cores": max(th_a, th_t), "kind": "port",
            "sample": f"oracle/ C fp64 restatement (median of 3): acquisition of the {n_prn} PRNs ({th_a} "
                      f"threads) over {a1.freqNum} bins x {a1.datalen} ms + fine FFT, trackingCT of the {n_ch} "
                      f"channels ({th_t} threads) 1000 ms @1ms (+phase-B rerun) + {n10s} ms @10ms; per-unit "
                      "rates extrapolated to the GPU step's unit mix",
            "threads": {"acquisition": th_a, "tracking": th_t}, "cpu_quota": cpu_quota(),
            "one_thread": {"value": round(v_1 / 1e6, 4), "acq_Msamples_s": round(a_1 / 1e6, 4),
                           "track_Msamples_s": round(t_1 / 1e6, 4), "sample": "1 PRN, 1 channel, same lengths"},
            "all_units": {"value": round(v_n / 1e6, 4), "acq_Msamples_s": round(a_n / 1e6, 4),
                          "track_Msamples_s": round(t_n / 1e6, 4)},
            "numpy_restatement": {"track_Msamples_s": round(np_trk / 1e6, 4) if np_trk else None,
                                  "acq_Msamples_s": round(np_acq / 1e6, 4) if np_acq else None,
                                  "threads": 1},
            "host_cpu": model, "nproc": ncpu,
            "label": "CPU restatement of acquisition.m / trackingCT.m (MATLAB itself is absent)"}


def code_stamp():
    """What the line was measured with: the sources' digest, the commit (git where the tree has
    .git, else .head_sha; its source named), and the sha256 of the library file this process
    actually loaded."""
    lib = pkg.abi.LOADED_PATH
    return {"src_digest": SRC_DIGEST, "git_commit": srcdigest.head_commit(),
            "git_commit_source": srcdigest.head_commit_source(),
            "lib": os.path.relpath(lib, ROOT) if lib else None,
            "lib_sha256": srcdigest.file_digest(lib) if lib else None}


def quota_threads(units):
    """Threads for a CPU leg of `units` independent units: one per unit, capped at the CPU
    quota (32 threads on a 16-CPU share ran oversubscribed under a 32-core label)."""
    return max(1, min(int(units), int(cpu_quota())))


def cpu_quota():
    """CPUs this process may use: the cgroup CPU quota (cpu.max) where one is set, else the
    affinity mask (the GPU box shows the whole machine's CPUs to nproc)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                return round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count()


if __name__ == "__main__":
    main()
