set -o pipefail
# forward MLP: priority 1 while a chunk's weight fragments are issued (var_fprio) vs default
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04fp var_base var_fprio || exit 1
