"""Config-2 acquisition timing (tools/acq_only.py's workload) after various amounts of torch /
torch.distributed initialisation in the same process, to find why the bench's one-rank
distributed run showed +1.2-1.4 ms of correlation. MODE: none | torch (set_device + one cuda
tensor before the library context) | torch_after (the same after the context) | gloo | nccl
(a one-rank process group initialised before the context; MASTER_ADDR/PORT set here)."""
import importlib, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mode = sys.argv[1] if len(sys.argv) > 1 else "none"
import torch
if mode in ("torch", "gloo", "nccl"):
    torch.cuda.set_device(0)
    x = torch.ones(16, device="cuda:0")
if mode in ("gloo", "nccl"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29541", RANK="0", WORLD_SIZE="1")
    if mode == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    if os.environ.get("PROBE_BARRIER") == "1":  # one collective before the context
        dist.barrier()
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
ctx = pkg.Context(0)
if os.environ.get("PROBE_BARRIER") == "after":  # the first collective after the context (bench.py's order)
    dist.barrier()
if mode == "torch_after":
    torch.cuda.set_device(0)
    x = torch.ones(16, device="cuda:0")
if os.environ.get("ACQ_PIPE"):
    ctx.set_option(pkg.abi.OPT_ACQ_PIPE, int(os.environ["ACQ_PIPE"]))
file, signal, acq, track, _, _ = pkg.initParameters()
skip, S = 5000, 58000
cfg = pkg.synth.opensky(skip_ms=skip)
acq.freqMin, acq.freqNum, acq.datalen = -7000, 29, 20
dev = pkg.DeviceRecord(ctx, (skip + 40) * S * 2)
pkg.synth.generate_device(ctx, cfg, dev)
file.skip, file.dev = skip, dev
c = []
between = os.environ.get("BETWEEN", "")  # between the calls: copy | gather | sleep<ms>
if between == "gather":
    D = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd.dist")
for it in range(4):
    A = pkg.acquisition(file, signal, acq, ctx=ctx)
    c.append(ctx.timing()["acq_corr_ms"])
    if between == "copy":
        y = torch.arange(160, dtype=torch.float64).to("cuda:0").cpu()
    elif between.startswith("sleep"):  # the GPU idle for that many ms before the next call
        time.sleep(float(between[5:]) * 1e-3)
    elif between == "gather":
        A = D.gather_acquired(A, list(range(1, 33)), list(range(1, 33)), device="cuda:0")
print(f"mode={mode} barrier={os.environ.get('PROBE_BARRIER', '')} between={between} pipe={os.environ.get('ACQ_PIPE', 'default')} corr_ms", " ".join(f"{v:.3f}" for v in c), "sv", list(A.sv), flush=True)
if mode in ("gloo", "nccl"):
    dist.destroy_process_group()
