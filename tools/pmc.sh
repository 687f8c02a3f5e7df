#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains) over a short bench run;
# tools/pmc_summary.py then folds the CSVs into gpurun_out/pmc.json (mean per dispatch per kernel).
# SDSJ_LANES (default 1 here) is the engine's lane count for the whole run: at 1, one dispatch of a
# kernel covers the whole batch, the unit bench.py's roofline prices.
# (--no-pixel-check: the check's reference and walk batches would enter the per-dispatch means)
# usage: tools/pmc.sh [extra bench args]
set -e
export TMPDIR=/tmp
export SDSJ_LANES=${SDSJ_LANES:-1}
BATCH=${BATCH:-65536}  # bench.py's default configs[1] batch (the PMC summary is per dispatch of one lane)
ROWS=$(( BATCH + 4096 ))
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pixel-check --roofline-steps 1 --rows $ROWS --batch $BATCH $*"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_$i
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$i -o p -- $B > gpurun_out/pmc_$i.log 2>&1
done
python3 tools/pmc_summary.py gpurun_out "$BATCH" "$SDSJ_LANES" > gpurun_out/${PMC_OUT:-pmc.json}
