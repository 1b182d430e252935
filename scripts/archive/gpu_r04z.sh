set -o pipefail
# the forward encode's scheduling group (levels between scheduling barriers:
# 1 / 2 (default) / 4) with the wave priority in place
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04z var_base var_g1 var_g4 || exit 1
