# The bench's distributed path (process group, result gathers) on a one-GPU box: one torchrun
# rank with BENCH_FORCE_DIST=1, backend nccl (= RCCL) and then gloo, beside the plain N = 1 run;
# NCCL_DEBUG=INFO shows RCCL's own init lines. Writes gpurun_out/rccl_*.json / .err.
set -o pipefail
mkdir -p gpurun_out
ARGS="--gpus 1 --steps 2 --warmup 1 --no-cpu"
timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/rccl_plain.json 2> gpurun_out/rccl_plain.err || { tail -20 gpurun_out/rccl_plain.err; exit 1; }
for be in nccl gloo; do
  BENCH_FORCE_DIST=1 BENCH_DIST_BACKEND=$be NCCL_DEBUG=INFO timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py $ARGS > gpurun_out/rccl_$be.json 2> gpurun_out/rccl_$be.err || { tail -30 gpurun_out/rccl_$be.err; exit 1; }
done
python3 - <<'PY'
import json
for n in ("plain", "nccl", "gloo"):
    d = json.loads(open(f"gpurun_out/rccl_{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["value"], d.get("outputs_ok"), d.get("acquired"), d["config"].get("parallelism"))
PY
grep -h -m5 -E "RCCL version|NCCL INFO (Init|comm|Channel 00)" gpurun_out/rccl_nccl.err || true
