set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 && \
SQ=1 bash tools/profile_round.sh medium_n8_fused --no-alt --no-sampler && \
bash tools/profile_round.sh medium_n8_graph --mode graph --no-alt --no-sampler && \
bash tools/profile_round.sh medium_n8_observe --no-alt
