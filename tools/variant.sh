#!/bin/bash
# Builds the working tree's sources (or those of a git revision: REV=...) into sds_amd/lib/exp/libsdsj_$1.so
# for tools/ab.sh (SDSJ_LIBRARY variants), with extra compiler flags from CFLAGS.  usage: [REV=..] [CFLAGS=..] tools/variant.sh name
set -e
name=$1
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root
if [ -n "$REV" ]; then
  src=$(mktemp -d)
  git -C "$root" archive "$REV" sds_amd/csrc include | tar -x -C "$src"
fi
mkdir -p "$root/sds_amd/lib/exp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wl,-z,defs \
  -Wno-unused-function -Wno-unused-variable -Wno-pass-failed -I "$src/include" \
  $CFLAGS -o "$root/sds_amd/lib/exp/libsdsj_$name.so" "$src"/sds_amd/csrc/*.hip
[ -n "$REV" ] && rm -rf "$src"
echo "$root/sds_amd/lib/exp/libsdsj_$name.so"
