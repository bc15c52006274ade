# fp64 acquisition: kernel-trace stats of config 2, the acquisition tests
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/acq64 -o acq64 -- python3 tools/acq_only.py > gpurun_out/acq64.log 2>&1 || { echo "rocprof fp64 rc=$?"; tail -5 gpurun_out/acq64.log; exit 1; }
grep "acq wall" gpurun_out/acq64.log | tail -1 | cut -c1-200
python3 tools/prof_db.py gpurun_out/acq64/acq64_results.db | head -8
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_acquisition.py > gpurun_out/pt_acq.log 2>&1; rc=$?; tail -2 gpurun_out/pt_acq.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pt_acq.log | head -20; exit 1; }
