# Round check on one MI355X: the GPU tests, the bench line, rocprofv3 kernel-trace of one
# bench step, PMC traffic of the dominant tracking kernel, PMC traffic + SQ counters of
# the fp64 acquisition kernels (one counter group per pass, each pass its own run).
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "TESTS_OK $(tail -1 gpurun_out/pytest_gpu.log)" || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && tail -1 gpurun_out/bench.json | cut -c1-400 || { tail -20 gpurun_out/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/bench_prof.json 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/tools/track_only.py 1000 40000 > $R/gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/tools/track_only.py 1000 40000 > $R/gpurun_out/pmc_write.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/acq_fetch -o run -- python3 $R/tools/acq_only.py > $R/gpurun_out/acq_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/acq_write -o run -- python3 $R/tools/acq_only.py > $R/gpurun_out/acq_write.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/acq_sq1 -o run -- python3 $R/tools/acq_only.py > $R/gpurun_out/acq_sq1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU --kernel-trace --output-format csv -d $R/gpurun_out/acq_sq2 -o run -- python3 $R/tools/acq_only.py > $R/gpurun_out/acq_sq2.log 2>&1 || exit 1
cd $R && python3 tools/prof_summary.py gpurun_out/prof_bench > gpurun_out/prof_bench_summary.txt && head -14 gpurun_out/prof_bench_summary.txt
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write "track_run_kernel<3, 3, false, false>" gpurun_out/traffic.json
python3 tools/pmc_sq.py gpurun_out/acq_counters.json gpurun_out/acq_fetch gpurun_out/acq_write gpurun_out/acq_sq1 gpurun_out/acq_sq2 -- "inv_cols_kernel<29, HIP_vector_type<double" "inv_rows_kernel_f64<29>" "fwd_rows_kernel<29" "fine_rows_kernel<29" "fine_cols_kernel<29>"
rm -f gpurun_out/pmc_*/**/*kernel_trace.csv gpurun_out/acq_*/**/*kernel_trace.csv
