# (rocprofv3 --kernel-trace segfaults in this image after ~20k graph-launched dispatches
#  in one process, e.g. 4 full trackingCT calls; the traced bench runs one step.)
# Round check on one MI355X: GPU tests, bench, rocprofv3 kernel-trace of the bench and
# PMC traffic of the dominant kernel (run from the repo root via gpurun).
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && tail -1 gpurun_out/bench.json || { tail -20 gpurun_out/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/bench_prof.json 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/tools/track_only.py 1000 40000 > $R/gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/tools/track_only.py 1000 40000 > $R/gpurun_out/pmc_write.log 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py gpurun_out/prof_bench > gpurun_out/prof_bench_summary.txt && head -12 gpurun_out/prof_bench_summary.txt
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write "track_run_kernel<3, 3, false>" gpurun_out/traffic.json
rm -f gpurun_out/pmc_*/**/*kernel_trace.csv
