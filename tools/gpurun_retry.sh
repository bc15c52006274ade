# gpurun with retries ONLY when no box was obtained (exit 3: nothing ran, nothing charged);
# waits as long as gpurun's back-off message asks (at least 60 s).
# Usage: bash tools/gpurun_retry.sh TIMEOUT 'command'   (writes .head_sha first)
cd "$(dirname "$0")/.." || exit 1
(git rev-parse --short HEAD; git diff --quiet HEAD -- assignment-for-aae6102_gnss-sdr_amd include || echo dirty) | paste -sd+ > .head_sha
for i in 1 2 3 4 5 6 7 8 9 10; do
  out=$(mktemp)
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" 2>&1 | tee "$out"
  rc=${PIPESTATUS[0]}
  [ $rc -ne 3 ] && { rm -f "$out"; exit $rc; }
  w=$(grep -o 'retry in [0-9]*s' "$out" | tail -1 | grep -o '[0-9]*')
  rm -f "$out"
  w=$(( ${w:-60} < 60 ? 60 : ${w:-60} + 5 ))
  echo "[retry] no box (exit 3), attempt $i; waiting $w s"
  sleep $w
done
exit 3
