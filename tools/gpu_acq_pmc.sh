# bench line (N=1) + HBM traffic (PMC) of the acquisition's inverse passes, one counter per pass
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && tail -1 gpurun_out/bench.json || { tail -20 gpurun_out/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/acq_fetch -o run -- python3 $R/tools/acq_only.py > $R/gpurun_out/acq_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/acq_write -o run -- python3 $R/tools/acq_only.py > $R/gpurun_out/acq_write.log 2>&1 || exit 1
cd $R
for k in "inv_cols_kernel<29>" "inv_rows_kernel<29>" "fine_rows_kernel<29" "fine_cols_kernel<29>"; do
  python3 tools/pmc_traffic.py gpurun_out/acq_fetch gpurun_out/acq_write "$k" "gpurun_out/acq_traffic_$(echo $k | tr -dc a-z_).json" || exit 1
done
rm -f gpurun_out/acq_*/**/*kernel_trace.csv
