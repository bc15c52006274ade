# acquisition-only kernel times (rocprofv3 kernel trace) + the acquisition GPU tests
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python3 tools/acq_only.py > gpurun_out/acq.log 2>&1 || { tail -5 gpurun_out/acq.log; exit 1; }
grep -E "acq wall" gpurun_out/acq.log | tail -1 | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_acq -o run -- python3 $R/tools/acq_only.py > $R/gpurun_out/acq_prof.log 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py gpurun_out/prof_acq | head -12
if [ -n "$WITH_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_acquisition.py tests/test_gpu_formats.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pt.log
fi
