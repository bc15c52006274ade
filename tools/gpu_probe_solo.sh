# stamps of the persistent tracking loop: 1 channel alone (latency floor) vs 8 channels,
# and the 1-ms phase
set -o pipefail
mkdir -p gpurun_out
for cfg in "1000 4000 3 1" "1000 4000 3 2" "1000 4000 3 4" "3000 0 3 8"; do
  echo "== track_only $cfg"
  GNSS_STAMPS=gpurun_out/st.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py $cfg > gpurun_out/t.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t.log; exit 1; }
  python3 tools/stamps_run.py gpurun_out/st.bin; rm -f gpurun_out/st.bin
done
