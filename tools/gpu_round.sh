set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/acq_only.py > gpurun_out/acq_own.log 2>&1; tail -4 gpurun_out/acq_own.log | cut -c1-400
GNSS_FINE_ROCFFT=1 timeout -k 10 120 python3 tools/acq_only.py > gpurun_out/acq_roc.log 2>&1; tail -4 gpurun_out/acq_roc.log | cut -c1-300
timeout -k 10 600 python -m pytest tests/test_gpu_acquisition.py -x -q > gpurun_out/pytest_acq.log 2>&1 && echo TESTS_OK || { tail -30 gpurun_out/pytest_acq.log; exit 1; }
