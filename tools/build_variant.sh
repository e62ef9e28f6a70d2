#!/bin/bash
# Build a variant of the library for same-box A/B runs (tools/ab.sh):
#   bash tools/build_variant.sh NAME [extra hipcc flags...]   ->  build_ab/NAME.so
cd "$(dirname "$0")/../rllib-warehouse_amd/csrc" || exit 2
NAME=$1; shift
mkdir -p ../../build_ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function -I../../include \
  "$@" warehouse_amd.hip policy_mlp.hip -o ../../build_ab/$NAME.so
