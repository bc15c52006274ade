# Round-2 baseline on one MI355X: fp64 latency micro-probe, per-step stamps of the
# 10-ms persistent loop (8 ch), and the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/lat > gpurun_out/lat.txt 2>&1 && cat gpurun_out/lat.txt || exit 1
GNSS_STAMPS=gpurun_out/st.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 100 40000 3 8 > gpurun_out/t.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t.log; exit 1; }
python3 tools/stamps_run.py gpurun_out/st.bin > gpurun_out/stamps_r2_base.txt; cat gpurun_out/stamps_r2_base.txt; rm -f gpurun_out/st.bin
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench_r2_base.json 2> gpurun_out/bench.err && tail -1 gpurun_out/bench_r2_base.json | cut -c1-1500 || { tail -20 gpurun_out/bench.err; exit 1; }
