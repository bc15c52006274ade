# A/B of the headline tracking launch: tmp_ab/libgnss_old.so = the library built from commit a2deb7b (before the virtual blocks; build it there and copy it in to re-run) vs now
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=tmp_ab/libgnss_old.so; else L=assignment-for-aae6102_gnss-sdr_amd/lib/libgnss_mi355x.so; fi
    GNSS_LIB=$L TRK_ITERS=3 timeout -k 10 200 python3 tools/track_only.py 1000 40000 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    echo "$v: $(grep 'track wall' gpurun_out/ab_$v.log | grep -o "'track_ms': [0-9.]*" | tr '\n' ' ')"
  done
done
