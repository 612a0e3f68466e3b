#!/bin/bash
# Build a complete variant of libneptune_hip.so with extra compile flags, for A/B runs:
#   bash tools/build_variant.sh NAME "-DFLAG=V ..."  ->  neptune-core_amd/build/variants/libneptune_hip_NAME.so
# (select it at run time with NHIP_LIB=...).  All objects are rebuilt with the same flags, as an A/B
# build (-DNHIP_AB_BUILD: the NHIP_* tuning switches are read, csrc/ab_env.hpp).
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../neptune-core_amd"
SRCS=$(sed -n 's/^SRCS := //p' Makefile)
OUT=build/v_$NAME; mkdir -p $OUT build/variants
objs=""
for s in $SRCS; do
  o=$OUT/$(basename ${s%.*}).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -DNHIP_AB_BUILD $FLAGS -c $s -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/libneptune_hip_$NAME.so $objs
echo build/variants/libneptune_hip_$NAME.so
