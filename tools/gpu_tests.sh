# GPU test suite (+ optional bench) on one MI355X, from the repo root via gpurun
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $PYTEST_K > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK || { grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -30; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_gpu.log
if [ -n "$WITH_BENCH" ]; then
  timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err && tail -1 gpurun_out/bench.json | cut -c1-600 || { tail -20 gpurun_out/bench.err; exit 1; }
fi
