#!/bin/bash
# desynchronised episodes: SQ counters of the lazy-grid build vs the eager one (20-step launches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/sq_probe.sh lazy_desync --steps 20 --launches 20 --stagger || exit $?
WAREHOUSE_AMD_LIB=build_ab/eager.so bash tools/sq_probe.sh eager_desync --steps 20 --launches 20 --stagger || exit $?
