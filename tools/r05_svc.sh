#!/bin/bash
# r05: decode service in the reference's loader shape -- stream waits sleeping (default) vs spinning
# (SDSJ_SERVICE_SPIN=1), 2 / 4 / 8 engines, 8 and 16 workers; plus Pillow / null at 8 and 16.
export TMPDIR=/tmp
run() {  # name mode [VAR=value ...]
  local name=$1 mode=$2; shift 2
  env "$@" timeout -k 10 120 python -u tools/persample_bench.py 512 4 $mode > gpurun_out/$name.log 2>&1 || return $?
  echo "$name $(grep -h '^{' gpurun_out/$name.log)" >> gpurun_out/svc_sweep.log
}
for w in 16 8; do
  for e in 2 4 8; do
    run blk_e${e}_w${w} service_fork_workers${w}_pinned SDS_AMD_SERVICE_ENGINES=$e || exit $?
    run spin_e${e}_w${w} service_fork_workers${w}_pinned SDS_AMD_SERVICE_ENGINES=$e SDSJ_SERVICE_SPIN=1 || exit $?
  done
  run pil_w${w} pil_fork_workers${w}_pinned || exit $?
  run null_w${w} null_fork_workers${w}_pinned || exit $?
done
# secondary rates at HEAD (verdict r04 item 7)
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload mixed512 > gpurun_out/mixed1024.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/prog_bench.py 4096 > gpurun_out/prog.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/sampling_bench.py > gpurun_out/sampling.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/batched_bench.py 2048 5 256 8 > gpurun_out/batched_w8.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/batched_bench.py 2048 5 256 16 > gpurun_out/batched_w16.log 2>&1 || exit $?
