set -o pipefail
# MLP backward: VALU per MFMA slot of the split pipelining (5/3 and 10/6 against 7/4)
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04sw var_base var_swpA var_swpB || exit 1
