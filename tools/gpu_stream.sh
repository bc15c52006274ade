# Streaming windows (GPU tests) and the staging-throughput probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tracking.py -k "streamed or file_route" > gpurun_out/pt_stream.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pt_stream.log | tail -5; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pt_stream.log | head -20; exit 1; }
TMPDIR=/tmp timeout -k 10 300 python3 tools/stage_probe.py 20 2>&1 | grep -v amdgpu.ids
