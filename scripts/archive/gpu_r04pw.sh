set -o pipefail
# forward priority region widened over the coarse-twin feature loads (var_wide) vs default
REPS=3 PROF=1 bash scripts/gpu_lib_ab.sh r04pw var_base var_wide || exit 1
