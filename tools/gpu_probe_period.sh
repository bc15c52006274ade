# per-step periods of the persistent tracking loop: 10-ms (8 ch, 4000 steps) and 1-ms
# (8 ch, 3000 steps), stamps summary; then the tracking parity tests
set -o pipefail
mkdir -p gpurun_out
for cfg in "100 40000 3 8" "3000 0 3 8" "100 4000 3 1"; do
  echo "== track_only $cfg"
  GNSS_STAMPS=gpurun_out/st.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py $cfg > gpurun_out/t.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t.log; exit 1; }
  python3 tools/stamps_run.py gpurun_out/st.bin | grep -E "per-channel|period|computed  |partials in  |desc ready"; rm -f gpurun_out/st.bin
done
if [ -n "$WITH_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "track or Track" > gpurun_out/pt.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pt.log
fi
