set -o pipefail
# forward wave priority while encoding (s_setprio 1 / 2) against the default
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04x var_base var_prio1 var_prio2 || exit 1
