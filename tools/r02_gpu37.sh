#!/bin/bash
# lazy rebuild v3 (co-location found by returning ORs, grid check after moves): parity, suite,
# then A/B against v2 (build_ab/cm.so, pairwise co-location) and eager (build_ab/eager.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
P="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
S="python tools/step_probe.py"
args=()
for v in "" "WAREHOUSE_AMD_LIB=build_ab/cm.so " "WAREHOUSE_AMD_LIB=build_ab/eager.so "; do
  args+=("$v$S --steps 200 --launches 6" "$v$S --variant large --agents 16 --steps 200 --launches 6" "$v$S --steps 20 --launches 20 --stagger")
done
bash tools/gpu_round.sh "$P tests/test_gpu_parity.py -k co_located" "$P tests -m gpu" "${args[@]}" "${args[@]}"
