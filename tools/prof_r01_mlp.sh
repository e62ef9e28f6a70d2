set -o pipefail
bash tools/profile_round.sh medium_n8_mlp --no-alt --no-sampler --steps 400 --policy-steps 100
