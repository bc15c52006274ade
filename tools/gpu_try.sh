set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/step_breakdown.py || exit 1
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pt.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pt.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && tail -1 gpurun_out/bench.json | cut -c1-700
