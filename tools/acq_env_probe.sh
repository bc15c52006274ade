set -o pipefail
mkdir -p gpurun_out
for v in "none:" "none:sleep1" "none:sleep5" "none:sleep50" "none:" "none:sleep1"; do
  m=${v%%:*}; b=${v#*:}
  BETWEEN=$b timeout -k 10 120 python3 tools/acq_env_probe.py $m > gpurun_out/aep_${m}_$b.txt 2>&1 || { tail -5 gpurun_out/aep_${m}_$b.txt; exit 1; }
  grep "^mode=" gpurun_out/aep_${m}_$b.txt | cut -c1-90
done
