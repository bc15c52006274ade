set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${LIBS}; do
  GNSS_LIB=$PWD/tools/probe_lib/libgnss_$v.so GNSS_STAMPS=gpurun_out/s10_$v.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 1000 30000 ${TAPS} ${NCH} > gpurun_out/s10_$v.log 2>&1 || { tail -5 gpurun_out/s10_$v.log; exit 1; }
  echo "== $v taps=$TAPS nch=$NCH $(grep track10 gpurun_out/s10_$v.log | tail -1)"
  python3 tools/stamps_run.py gpurun_out/s10_$v.bin | grep -E "start ->|computed ->|partial out ->|all in ->|period \(|blk0 tail|lane:"
  rm -f gpurun_out/s10_$v.bin
done
