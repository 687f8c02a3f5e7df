#!/bin/bash
# PMC passes over the progressive bench (tools/prog_bench.py, one dispatch of k_prog per call at
# SDSJ_LANES=1); tools/pmc_summary.py folds them into gpurun_out/pmc_prog.json (mean per dispatch).
# usage: tools/pmc_prog.sh [batch]
set -e
export TMPDIR=/tmp
export SDSJ_LANES=1
BATCH=${1:-4096}
B="python3 tools/prog_bench.py $BATCH nocpu"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  rm -rf gpurun_out/pmcp_$i
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcp_$i -o p -- $B > gpurun_out/pmcp_$i.log 2>&1
done
python3 tools/pmc_summary.py gpurun_out "$BATCH" 1 pmcp > gpurun_out/pmc_prog.json
