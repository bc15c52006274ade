set -o pipefail
mkdir -p gpurun_out
GNSS_STAMPS=gpurun_out/st_c.bin timeout -k 10 120 python3 tools/track_only.py 1000 40000 > gpurun_out/t_c.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t_c.log; exit 1; }
python3 tools/stamps_run.py gpurun_out/st_c.bin; rm -f gpurun_out/*.bin
tail -n 1 gpurun_out/t_c.log | cut -c1-100
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -k "track or Track" > gpurun_out/pt.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pt.log
