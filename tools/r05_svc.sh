#!/bin/bash
# r05: decode service in the reference's loader shape -- stream waits sleeping (default) vs spinning
# (SDSJ_SERVICE_SPIN=1), 2 / 4 / 8 engines, 8 and 16 workers; plus Pillow / null at 8 and 16.
export TMPDIR=/tmp
run() {  # name env... -- mode
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u tools/persample_bench.py 512 4 "${@: -1}" > gpurun_out/$name.log 2>&1 || return $?
  echo "$name $(grep -h '^{' gpurun_out/$name.log)" >> gpurun_out/svc_sweep.log
}
for w in 16 8; do
  for e in 2 4 8; do
    run blk_e${e}_w${w} SDS_AMD_SERVICE_ENGINES=$e service_fork_workers${w}_pinned || exit $?
    run spin_e${e}_w${w} SDS_AMD_SERVICE_ENGINES=$e SDSJ_SERVICE_SPIN=1 service_fork_workers${w}_pinned || exit $?
  done
  run pil_w${w} X=1 pil_fork_workers${w}_pinned || exit $?
  run null_w${w} X=1 null_fork_workers${w}_pinned || exit $?
done
