# acquisition config 2 time vs the inverse-pass batch size (GNSS_ACQ_BATCH, (bin, PRN) pairs)
set -o pipefail
mkdir -p gpurun_out
for b in 28 14 56 112 232 28; do
  echo "== GNSS_ACQ_BATCH=$b"
  GNSS_ACQ_BATCH=$b timeout -k 10 120 python3 tools/acq_only.py > gpurun_out/acqb_$b.log 2>&1 || exit 1
  grep "acq wall" gpurun_out/acqb_$b.log | sed -E "s/.*'acq_ms': ([0-9.]+), 'acq_corr_ms': ([0-9.]+).*/acq_ms \1 corr_ms \2/"
  tail -3 gpurun_out/acqb_$b.log | head -1 | cut -c1-120
done
