# XCD-local placement in the 1-ms phase (one block per CU; GNSS_PROBE 256 forces blockIdx
# placement): stamps of the 1-ms persistent loop at 8 channels.
set -o pipefail
mkdir -p gpurun_out
for pr in 256 0; do
  echo "== GNSS_PROBE=$pr"
  GNSS_PROBE=$pr GNSS_STAMPS=gpurun_out/st.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 2000 0 3 8 > gpurun_out/t.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t.log; exit 1; }
  python3 tools/stamps_run.py gpurun_out/st.bin | grep -v "^gpurun_out"; rm -f gpurun_out/st.bin; tail -1 gpurun_out/t.log | cut -c1-200
done
