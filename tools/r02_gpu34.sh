#!/bin/bash
# SQ counters of the lazy-grid build vs the eager one (200-step Medium-8 launches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/sq_probe.sh lazy_k200 --steps 200 --launches 5 || exit $?
WAREHOUSE_AMD_LIB=build_ab/eager.so bash tools/sq_probe.sh eager_k200 --steps 200 --launches 5 || exit $?
