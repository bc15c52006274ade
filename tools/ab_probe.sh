#!/bin/bash
# A/B of probe-bit variants of one probe library (GPU box): LIB=name PROBES="0 256 512" ->
# per variant the 10-ms launch times (hipEvents) and full-length GNSS_STAMPS of channel 0.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for pb in $PROBES; do
  GNSS_PROBE=$pb GNSS_LIB=$R/tools/probe_lib/libgnss_$LIB.so TRK_PROFILE=1 TRK_ITERS=3 timeout -k 10 120 python3 tools/track_only.py 1000 40000 > gpurun_out/abp_$pb.log 2>&1 || { tail -5 gpurun_out/abp_$pb.log; exit 1; }
  GNSS_PROBE=$pb GNSS_LIB=$R/tools/probe_lib/libgnss_$LIB.so GNSS_STAMPS=gpurun_out/abpst_$pb.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 1000 40000 > /dev/null 2>&1 || exit 1
  echo "abp $LIB probe $pb: $(grep track10 gpurun_out/abp_$pb.log | tail -2 | tr '\n' ' ')"
  python3 tools/stamps_run.py gpurun_out/abpst_$pb.bin | grep -E "period \(|computed|all partials|next desc|turn" | sed "s/^/   /"
  rm -f gpurun_out/abpst_$pb.bin
done
