# correlator wave-priority schemes of the persistent loop (GNSS_PROBE bits 64 / 128)
set -o pipefail
mkdir -p gpurun_out
for pr in 0 64 128 0; do
  echo "== GNSS_PROBE=$pr"
  GNSS_PROBE=$pr GNSS_STAMPS=gpurun_out/st.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 100 40000 > gpurun_out/t.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t.log; exit 1; }
  python3 tools/stamps_run.py gpurun_out/st.bin | grep -E "per-channel|period|computed  "; rm -f gpurun_out/st.bin
done
