# fine-frequency kernels after a change: kernel trace + acquisition GPU tests
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_acq -o run -- python3 $R/tools/acq_only.py > $R/gpurun_out/acq_prof.log 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py gpurun_out/prof_acq | head -10
timeout -k 10 600 python -u -m pytest tests/test_gpu_acquisition.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pt.log
