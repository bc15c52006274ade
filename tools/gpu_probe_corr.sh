# correlator part timings of the persistent 10-ms loop (8 ch, 4000 steps) for the
# GNSS_CORR_PROBE builds of tools/build_probe.sh
set -o pipefail
mkdir -p gpurun_out
for n in 0 1 2 4 7; do
  echo "== probe $n"
  GNSS_LIB=tools/probe_lib/libgnss_probe$n.so GNSS_STAMPS=gpurun_out/st.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 100 4000 > gpurun_out/t.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t.log; exit 1; }
  python3 tools/stamps_run.py gpurun_out/st.bin | grep -E "per-channel|period|computed  |partials in  |desc ready"; rm -f gpurun_out/st.bin
done
