#!/bin/bash
# tools/pmc_summary.py over every launch shape of a tools/profile_r06.sh output directory (here or on
# the GPU box, so a bench run in the same call reads the same-sha profile):
#   bash tools/summarize_r06.sh gpurun_out/prof_TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=${1:?usage: summarize_r06.sh PROF_DIR}
for s in medium_n8_fused_k20:20 medium_n8_fused_k200:200 large_n16_fused_k20:20 large_n16_fused_k200:200 small_n4_random_b4096_fused_k20:20; do
  t=${s%%:*}; k=${s##*:}
  python3 tools/pmc_summary.py "$D/$t" "$t" --round r06 --steps-per-launch "$k" --probe 200,6 > /dev/null || exit 1
done
echo "summarized $D"
