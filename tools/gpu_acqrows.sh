# fp64 acquisition correlation time at config 2 and the acquisition parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/acq_only.py > gpurun_out/acqrows.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/acqrows.log; exit 1; }
echo "$(grep 'acq wall' gpurun_out/acqrows.log | tail -1 | grep -o "'acq_corr_ms': [0-9.]*")"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/acq64 -o acq64 -- python3 tools/acq_only.py > gpurun_out/acq64.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
python3 tools/prof_db.py gpurun_out/acq64/acq64_results.db | head -8
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_acquisition.py > gpurun_out/pt_acqrows.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pt_acqrows.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pt_acqrows.log | head -20; exit 1; }
