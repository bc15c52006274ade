set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/bench_prof.json 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/tools/track_only.py 100 4000 > $R/gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/tools/track_only.py 100 4000 > $R/gpurun_out/pmc_write.log 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py gpurun_out/prof_bench > gpurun_out/prof_bench_summary.txt && head -12 gpurun_out/prof_bench_summary.txt
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write "track_step_kernel<3, 4, false>" gpurun_out/traffic.json
rm -f gpurun_out/pmc_*/**/*kernel_trace.csv
