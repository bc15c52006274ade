set -o pipefail
mkdir -p gpurun_out
GNSS_STAMPS=gpurun_out/st_c.bin timeout -k 10 120 python3 tools/track_only.py 1000 40000 > gpurun_out/t_c.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/t_c.log; exit 1; }
python3 tools/stamps_run.py gpurun_out/st_c.bin; rm -f gpurun_out/*.bin
GNSS_HOSTPROF=1 timeout -k 10 200 python3 bench.py --no-cpu --steps 3 > gpurun_out/bench_hp.json 2> gpurun_out/bench_hp.err || { tail -5 gpurun_out/bench_hp.err; exit 1; }
grep hostprof gpurun_out/bench_hp.err | tail -12; tail -1 gpurun_out/bench_hp.json | cut -c1-300
