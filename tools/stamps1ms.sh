# 1-ms phase per-block stamps of probe libraries (LIBS="name ..." -> tools/probe_lib/libgnss_<name>.so):
# tools/track_only.py 1000 10 (channel 0, 29 blocks), tools/stamps_run.py + tools/stamps_blocks.py
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${LIBS}; do
  GNSS_LIB=$PWD/tools/probe_lib/libgnss_$v.so GNSS_STAMPS=gpurun_out/s1_$v.bin TRK_ITERS=1 timeout -k 10 120 python3 tools/track_only.py 1000 10 > gpurun_out/s1_$v.log 2>&1 || { tail -5 gpurun_out/s1_$v.log; exit 1; }
  echo "== $v (1-ms phase)"
  python3 tools/stamps_run.py gpurun_out/s1_$v.bin | grep -E "start ->|computed ->|partial out ->|all in ->|period \(|blk0 tail|flush"
  python3 tools/stamps_blocks.py gpurun_out/s1_$v.bin 29
  rm -f gpurun_out/s1_$v.bin
done
