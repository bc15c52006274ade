# 10-ms lane span probe: SUB10 = 3 (default, 96 blocks per channel) vs 4 (72), 8 channels
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in 3 4; do
    GNSS_FORCE_SUB10=$v TRK_ITERS=3 timeout -k 10 200 python3 tools/track_only.py 1000 40000 > gpurun_out/sub10_$v.log 2>&1 || { tail -5 gpurun_out/sub10_$v.log; exit 1; }
    echo "sub10=$v: $(grep 'track wall' gpurun_out/sub10_$v.log | grep -o "'track_ms': [0-9.]*" | tr '\n' ' ')"
  done
done
