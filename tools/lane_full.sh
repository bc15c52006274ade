#!/bin/bash
# Full-length (4 000 x 10-ms) lane-phase stamps (probe bit 32) of probe libraries: RUNS="lib:probe ..."
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in $RUNS; do
  lib=${v%%:*}; pb=${v##*:}
  GNSS_PROBE=$pb GNSS_LIB=$R/tools/probe_lib/libgnss_$lib.so GNSS_STAMPS=gpurun_out/lf.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 1000 ${STEPS_MS:-40000} > /dev/null 2>&1 || exit 1
  echo "lane $lib probe $pb (${STEPS_MS:-40000} ms):"
  python3 tools/stamps_run.py gpurun_out/lf.bin | grep -E "period \(|computed|lane:|turn" | sed "s/^/   /"
  rm -f gpurun_out/lf.bin
done
