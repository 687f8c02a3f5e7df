#!/bin/bash
# configs[1] (batch 32,768) by lane count: 4 (product), 6 and 8 lanes with 8 hardware queues
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "l4|product|4|4" "l4q8|product|4|8" "l6q8|lanes8|6|8" "l8q8|lanes8|8|8"; do
    IFS='|' read name lib lanes q <<< "$cfg"
    if [ "$lib" = "product" ]; then unset SDSJ_LIBRARY; else export SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_$lib.so; fi
    SDSJ_LANES=$lanes GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/l_$name.json 2> gpurun_out/l_$name.err || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/l_$name.json') if l.startswith('{')][-1]); print('$name', d['value'])" >> gpurun_out/lanes.log
  done
done
unset SDSJ_LIBRARY
