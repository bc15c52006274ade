# acquisition after a change: config-2 timing, acquisition GPU tests, bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/acq_only.py > gpurun_out/acq.log 2>&1 || exit 1
grep "acq wall" gpurun_out/acq.log | sed -E "s/.*'acq_ms': ([0-9.]+), 'acq_corr_ms': ([0-9.]+).*/acq_ms \1 corr_ms \2/"
timeout -k 10 600 python -u -m pytest tests/test_gpu_acquisition.py tests/test_gpu_formats.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.json | cut -c1-200
