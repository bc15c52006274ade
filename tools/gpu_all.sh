# The whole GPU suite (one process), then the bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -s > gpurun_out/pt_all.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|worst|margins" gpurun_out/pt_all.log | tail -90 | cut -c1-160; [ $rc -eq 0 ] || { tail -40 gpurun_out/pt_all.log | cut -c1-300; exit 1; }
