# Config 5 on one MI355X: PMC traffic of the 11-tap persistent 10-ms launch, then the cfg5 bench line
# (with its CPU leg)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
TRK_ITERS=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/c5_fetch -o run -- python3 $R/tools/track_only.py 1000 90000 11 32 > $R/gpurun_out/c5_fetch.log 2>&1 || { tail -5 $R/gpurun_out/c5_fetch.log; exit 1; }
TRK_ITERS=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/c5_write -o run -- python3 $R/tools/track_only.py 1000 90000 11 32 > $R/gpurun_out/c5_write.log 2>&1 || { tail -5 $R/gpurun_out/c5_write.log; exit 1; }
cd $R && python3 tools/pmc_traffic.py gpurun_out/c5_fetch gpurun_out/c5_write "track_run_kernel<11, 3, false, true>" gpurun_out/traffic_cfg5.json || exit 1
rm -f gpurun_out/c5_*/**/*kernel_trace.csv
timeout -k 10 400 python3 bench.py --workload cfg5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err && tail -1 gpurun_out/bench_cfg5.json | cut -c1-300 || { tail -20 gpurun_out/bench_cfg5.err; exit 1; }
