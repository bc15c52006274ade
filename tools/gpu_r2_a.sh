# Round-2 GPU check A: new GPU tests (2-rank sharded HIP path, device outputs, config-2
# datalen-20 parity), the sharded bench line with the CPU baseline legs, and the long-run
# golden made from the bench record on this box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py "tests/test_gpu_acquisition.py::test_config2_datalen20_against_oracle" -s > gpurun_out/pt_a.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|margins|assert" gpurun_out/pt_a.log | tail -20; [ $rc -eq 0 ] || { tail -40 gpurun_out/pt_a.log; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err && tail -1 gpurun_out/bench_a.json | cut -c1-3000 || { tail -20 gpurun_out/bench_a.err; exit 1; }
timeout -k 10 600 python3 -u tests/golden/make_golden_long.py gpurun_out/golden_track_long.npz
