# Virtual blocks (prefetch overlapped with the reduction): the tests that exercise them, cfg5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tracking.py -k "virtual or config5 or bench_shape or bit_identical" > gpurun_out/pt_vpb.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pt_vpb.log | tail -8; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pt_vpb.log | head -20; exit 1; }
timeout -k 10 300 python3 bench.py --workload cfg5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err && tail -1 gpurun_out/bench_cfg5.json | cut -c1-300 || { tail -20 gpurun_out/bench_cfg5.err; exit 1; }
