#!/bin/bash
# Forward phase timers (HN_PROFILE=1 variant library): shader-clock cycles per wave.
set -o pipefail
O=gpurun_out/fwdprof; mkdir -p $O
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_prof.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/bench.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
grep hn_fwd_profile $O/prof.err | tail -3
