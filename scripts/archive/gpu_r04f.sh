set -o pipefail
mkdir -p gpurun_out/r04f
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_stag4_prof.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r04f/prof.json 2> gpurun_out/r04f/prof.err || exit 1
grep hn_fwd_profile gpurun_out/r04f/prof.err | tail -2
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04f var_l0 var_ldsw var_stag2 var_stag4 var_stag8 || exit 1
