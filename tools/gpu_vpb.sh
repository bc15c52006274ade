# Virtual blocks of the persistent loop: tracking tests, then the config-5 bench (32 ch x 11 taps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tracking.py > gpurun_out/pt_vpb.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pt_vpb.log | tail -30; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pt_vpb.log | head -20; exit 1; }
timeout -k 10 300 python3 bench.py --workload cfg5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err && tail -1 gpurun_out/bench_cfg5.json | cut -c1-700 || { tail -20 gpurun_out/bench_cfg5.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench_vpb.json 2> gpurun_out/bench_vpb.err && tail -1 gpurun_out/bench_vpb.json | cut -c1-300 || { tail -20 gpurun_out/bench_vpb.err; exit 1; }
