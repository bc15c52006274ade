# XCD-local channel placement (GNSS_PROBE 256 forces the blockIdx placement): stamps of the
# 10-ms persistent loop at 8 channels, then the tracking parity tests and the bench line.
set -o pipefail
mkdir -p gpurun_out
for pr in 256 0; do
  echo "== GNSS_PROBE=$pr"
  GNSS_PROBE=$pr GNSS_STAMPS=gpurun_out/st.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 100 20000 3 8 > gpurun_out/t.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t.log; exit 1; }
  python3 tools/stamps_run.py gpurun_out/st.bin | grep -v "^gpurun_out"; rm -f gpurun_out/st.bin
done
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_tracking.py tests/test_gpu_longrun.py tests/test_gpu_dist.py > gpurun_out/pt_trk.log 2>&1; rc=$?; tail -3 gpurun_out/pt_trk.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pt_trk.log | head -20; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err && tail -1 gpurun_out/bench_iter.json | cut -c1-400 || { tail -20 gpurun_out/bench_iter.err; exit 1; }
