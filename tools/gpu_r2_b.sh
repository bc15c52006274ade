# Round-2 GPU check B: the whole GPU suite (with the long-run golden test), then the
# 2-rank bench rehearsal on this one GPU (gloo, both ranks on device 0).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -s > gpurun_out/pt_b.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|max err" gpurun_out/pt_b.log | tail -80 | cut -c1-200; [ $rc -eq 0 ] || { tail -60 gpurun_out/pt_b.log | cut -c1-300; exit 1; }
BENCH_DIST_BACKEND=gloo BENCH_FORCE_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-profile-pass > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err && tail -1 gpurun_out/bench_2rank.json | cut -c1-1500 || { tail -30 gpurun_out/bench_2rank.err; exit 1; }
