# A/B of the headline tracking launch (tmp_ab/libgnss_old.so = the library of commit a2deb7b, before the virtual blocks), the virtual-block
# tests, and the cfg5 bench
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=tmp_ab/libgnss_old.so; else L=assignment-for-aae6102_gnss-sdr_amd/lib/libgnss_mi355x.so; fi
    GNSS_LIB=$L TRK_ITERS=3 timeout -k 10 200 python3 tools/track_only.py 1000 40000 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    echo "$v: $(grep 'track wall' gpurun_out/ab_$v.log | grep -o "'track_ms': [0-9.]*" | tr '\n' ' ')"
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tracking.py -k "virtual or config5 or bench_shape or bit_identical" > gpurun_out/pt_vpb.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pt_vpb.log | tail -8; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pt_vpb.log | head -20; exit 1; }
timeout -k 10 400 python3 bench.py --workload cfg5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err && tail -1 gpurun_out/bench_cfg5.json | cut -c1-300 || { tail -20 gpurun_out/bench_cfg5.err; exit 1; }
