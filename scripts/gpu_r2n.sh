# Fused Euler step check: the round-end script (every GPU test, smoke, both bench forms), then the profile of the
# bench command (kernel trace + PMC passes).  Stops at the first failure.
set -o pipefail
bash scripts/gpu_round_end.sh || exit $?
bash scripts/gpu_profile_round.sh r2n_prof
