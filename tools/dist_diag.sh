# the bench's one-rank distributed path with and without the result gathers (BENCH_DIAG_NO_GATHER),
# beside the plain run: where the distributed step's extra acquisition time comes from
set -o pipefail
mkdir -p gpurun_out
ARGS="--gpus 1 --steps 4 --warmup 1 --no-cpu"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py $ARGS > gpurun_out/dd_$n.json 2> gpurun_out/dd_$n.err || { tail -20 gpurun_out/dd_$n.err; return 1; }
}
timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/dd_plain.json 2> gpurun_out/dd_plain.err || exit 1
run torchrun_plain A=1 || exit 1
run nccl_nogather BENCH_FORCE_DIST=1 BENCH_DIAG_NO_GATHER=1 || exit 1
run nccl BENCH_FORCE_DIST=1 || exit 1
python3 - <<'PY'
import json
for n in ("plain", "torchrun_plain", "nccl_nogather", "nccl"):
    d = json.loads([l for l in open(f"gpurun_out/dd_{n}.json") if l.startswith('{"metric"')][-1])
    print(f"{n:15s} step {d['ms_per_step']:7.3f} gather {d.get('gather_ms')} acq {d['acq_ms']:.3f} corr {d['acq_roofline']['corr_ms']:.3f} track {d['track_ms']:.3f} ok {d.get('outputs_ok')}")
PY
