set -o pipefail
mkdir -p gpurun_out
for v in "nccl:1:" "nccl:after:" "gloo:after:" "nccl:after:" "none::"; do
  IFS=: read m b w <<< "$v"
  PROBE_BARRIER=$b BETWEEN=$w timeout -k 10 120 python3 tools/acq_env_probe.py $m > gpurun_out/aep_${m}_$b.txt 2>&1 || { tail -5 gpurun_out/aep_${m}_$b.txt; exit 1; }
  grep "^mode=" gpurun_out/aep_${m}_$b.txt | cut -c1-100
done
