#!/bin/bash
# Build a variant of the library for same-box A/B runs (tools/ab.sh):
#   bash tools/build_variant.sh NAME [extra hipcc flags...]   ->  build_ab/NAME.so
# e.g. the phase-ablation build tools/ablate.py needs: bash tools/build_variant.sh ablation -DWH_ABLATION
cd "$(dirname "$0")/../rllib-warehouse_amd/csrc" || exit 2
NAME=$1; shift
mkdir -p ../../build_ab
if [ -n "$SCHED" ]; then   # another scheduler setting for the step object (abrun "sched")
  make -s -j2 OUT=../../build_ab/$NAME.so OBJDIR=../../build/obj_$NAME EXTRA="$*" SCHED_warehouse_amd="$SCHED" lib
else
  make -s -j2 OUT=../../build_ab/$NAME.so OBJDIR=../../build/obj_$NAME EXTRA="$*" lib
fi
