set -o pipefail
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 120 python3 tools/track_only.py "$@" > gpurun_out/t_$tag.log 2>&1; echo "$tag $(grep 'track wall' gpurun_out/t_$tag.log | tail -1 | grep -o "'track_ms': [0-9.]*")"; }
timeout -k 10 600 python -m pytest tests/test_gpu_tracking.py -x -q > gpurun_out/pytest_trk.log 2>&1 && echo TESTS_OK || { tail -30 gpurun_out/pytest_trk.log; exit 1; }
GNSS_STAMPS=gpurun_out/st_a.bin run sta 1000 0 || exit 1
GNSS_STAMPS=gpurun_out/st_c.bin run stc 100 20000 || exit 1
run cfg3 1000 40000
python3 tools/stamps.py gpurun_out/st_a.bin gpurun_out/st_c.bin; rm -f gpurun_out/*.bin
