#!/bin/bash
# r05: the loader shape at 2/4/8/16 workers -- service (defaults), Pillow, null -- twice, on one box.
export TMPDIR=/tmp
for pass in 1 2; do
  for w in 2 4 8 16; do
    for kind in service pil null; do
      n=${kind}_w${w}_p${pass}
      timeout -k 10 120 python -u tools/persample_bench.py 512 4 ${kind}_fork_workers${w}_pinned > gpurun_out/$n.log 2>&1 || exit $?
      echo "$n $(grep -h '^{' gpurun_out/$n.log)" >> gpurun_out/svc_sweep.log
    done
  done
done
