# fp64 inverse-row kernel variants: 0 = full twiddle table (64 KB LDS), 1 = split table,
# 2 = split table + radix 10-10-20; acquisition time of config 2 and the parity tests
set -o pipefail
mkdir -p gpurun_out
for v in 0 2 3; do
  GNSS_ACQ_ROWS_VAR=$v timeout -k 10 300 python3 tools/acq_only.py > gpurun_out/acqrows_$v.log 2>&1 || { echo "var $v rc=$?"; tail -5 gpurun_out/acqrows_$v.log; exit 1; }
  echo "var $v: $(grep 'acq wall' gpurun_out/acqrows_$v.log | tail -1 | grep -o "'acq_corr_ms': [0-9.]*")"
done
for v in 3; do
  GNSS_ACQ_ROWS_VAR=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_acquisition.py > gpurun_out/pt_acqrows_$v.log 2>&1; rc=$?; echo "tests var $v: $(tail -1 gpurun_out/pt_acqrows_$v.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pt_acqrows_$v.log | head -20; exit 1; }
done
