set -e
for w in default 3000 4000 6000; do
  if [ $w = default ]; then unset SDSJ_WARM_BITS; else export SDSJ_WARM_BITS=$w; fi
  timeout -k 10 300 python -u bench.py --workload mixed512 --no-cpu-baseline --steps 10 > gpurun_out/mixed_$w.json 2> gpurun_out/mixed_$w.err
done
