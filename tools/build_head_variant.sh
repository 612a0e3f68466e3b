#!/bin/bash
# Build libneptune_hip.so from a git revision's sources (default HEAD) into
# neptune-core_amd/build/variants/libneptune_hip_<name>.so, for A/B runs against the working tree
# (select it with NHIP_LIB).  Usage: bash tools/build_head_variant.sh NAME [REV]
set -e
NAME=$1; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" neptune-core_amd/csrc include | tar -x -C "$TMP"
cd "$TMP/neptune-core_amd"
mkdir -p build "$ROOT/neptune-core_amd/build/variants"
SRCS=$(sed -n 's/^SRCS := //p' "$ROOT/neptune-core_amd/Makefile")
objs=""
for s in $SRCS; do
  o=build/$(basename ${s%.*}).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -c $s -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/neptune-core_amd/build/variants/libneptune_hip_$NAME.so" $objs
rm -rf "$TMP"
echo neptune-core_amd/build/variants/libneptune_hip_$NAME.so
