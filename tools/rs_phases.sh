#!/bin/bash
# Builds k_resample phase-ablation variants (SDSJ_RS_PHASES mask) into tools/_exp/ (CPU side).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_exp
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DSDSJ_RS_PHASES=$m \
    -I include -o tools/_exp/libsdsj_p$m.so sds_amd/csrc/*.hip &
done
wait
