# Final round check: smoke(), the GPU tests, the bench line and one traced bench step
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "TESTS_OK $(tail -1 gpurun_out/pytest_gpu.log)" || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && tail -1 gpurun_out/bench.json | cut -c1-300 || { tail -20 gpurun_out/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/bench_prof.json 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py gpurun_out/prof_bench > gpurun_out/prof_bench_summary.txt && head -8 gpurun_out/prof_bench_summary.txt
rm -f gpurun_out/prof_bench/*kernel_trace.csv
