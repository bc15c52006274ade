# gpurun with retries ONLY when no box was obtained (exit 3: nothing ran, nothing charged).
# Usage: bash tools/gpurun_retry.sh TIMEOUT 'command'   (writes .head_sha first)
cd "$(dirname "$0")/.." || exit 1
(git rev-parse --short HEAD; git diff --quiet HEAD -- assignment-for-aae6102_gnss-sdr_amd include || echo dirty) | paste -sd+ > .head_sha
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry] no box (exit 3), attempt $i; waiting 60 s"
  sleep 60
done
exit 3
