#!/bin/bash
# A/B of library variants on configs[1] (2 rounds) and configs[2] (1 round), no GPU suite (product unchanged).
# usage: tools/r05_ab5.sh name=lib ...
export TMPDIR=/tmp
tools/ab.sh 2 "" "$@" || exit $?
mv gpurun_out/ab.log gpurun_out/ab_vga.log
tools/ab.sh 1 "--workload mixed512" "$@" || exit $?
mv gpurun_out/ab.log gpurun_out/ab_mixed.log
