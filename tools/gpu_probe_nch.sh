# Persistent 10-ms loop stamps by channel count (1 channel: one block per CU, no contention)
# and by correlator priority scheme (GNSS_PROBE 64: fixed ch % 3, 128: all 0).
set -o pipefail
mkdir -p gpurun_out
for cfg in "1 0" "2 0" "4 0" "8 0" "8 64" "8 128"; do
  set -- $cfg
  echo "== nch=$1 GNSS_PROBE=$2"
  GNSS_PROBE=$2 GNSS_STAMPS=gpurun_out/st.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 100 20000 3 $1 > gpurun_out/t.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t.log; exit 1; }
  python3 tools/stamps_run.py gpurun_out/st.bin | grep -v "^gpurun_out"; rm -f gpurun_out/st.bin
done
