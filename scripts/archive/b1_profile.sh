#!/bin/bash
# Diagnostic: per-phase shader-clock cycles of the backward MLP kernels
# (HN_PROFILE build; synchronises after every backward, so step times are not
# representative).   usage: scripts/b1_profile.sh [bench args...]
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
python - <<'PY' || exit 1
import sys; sys.path.insert(0, "hashnerf-pytorch_amd")
import build
import os
build.build_variant(["-DHN_PROFILE=1"] + os.environ.get("PROFILE_DEFS", "").split(), "/tmp/hn_profile.so")
PY
HN_LIB_PATH=/tmp/hn_profile.so timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline "$@" \
    > $OUT/b1_profile.json 2> $OUT/b1_profile.err || exit 1
grep "hn_b1_\|hn_fwd_" $OUT/b1_profile.err | tail -8
