# 1-ms phase period vs lane span (GNSS_FORCE_SUB), 8 channels, 1000 1-ms steps
set -o pipefail
mkdir -p gpurun_out
for v in 1 2 3 4 1; do
  echo "== GNSS_FORCE_SUB=$v"
  GNSS_FORCE_SUB=$v TRK_ITERS=3 timeout -k 10 120 python3 tools/track_only.py 1000 10 || exit 1
done
