# fp64 acquisition correlation: GPU parity tests (both precisions), kernel-trace stats of
# config 2 at fp64 and fp32, then the bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_acquisition.py tests/test_gpu_formats.py > gpurun_out/pt_acq.log 2>&1; rc=$?; tail -3 gpurun_out/pt_acq.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pt_acq.log | head -20; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/acq64 -o acq64 -- python3 tools/acq_only.py > gpurun_out/acq64.log 2>&1 || { echo "rocprof fp64 rc=$?"; tail -5 gpurun_out/acq64.log; exit 1; }
ACQ_FP32=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/acq32 -o acq32 -- python3 tools/acq_only.py > gpurun_out/acq32.log 2>&1 || { echo "rocprof fp32 rc=$?"; tail -5 gpurun_out/acq32.log; exit 1; }
grep "acq wall" gpurun_out/acq64.log | tail -1 | cut -c1-200; grep "acq wall" gpurun_out/acq32.log | tail -1 | cut -c1-200
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err && tail -1 gpurun_out/bench_iter.json | cut -c1-2500 || { tail -20 gpurun_out/bench_iter.err; exit 1; }
