# Step-kernel evidence after a kernel change: the default bench line, then rocprofv3
# kernel-trace/stats + FETCH/WRITE (+ SQ) passes for the fused and the 1-step graph launches.
# Summaries go to profiles/ via tools/pmc_summary.py (run here afterwards).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 && \
SQ=1 bash tools/profile_round.sh medium_n8_fused --no-alt --no-sampler --no-policy && \
bash tools/profile_round.sh medium_n8_graph --mode graph --no-alt --no-sampler --no-policy
