#!/bin/bash
# Diagnostic: phase cycles of the binned-scatter owner pass (HN_BR_PROF build;
# synchronises after every backward).   usage: scripts/br_profile.sh [defines...]
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
python - "$@" <<'PY' || exit 1
import sys; sys.path.insert(0, "hashnerf-pytorch_amd")
import build
build.build_variant(["-DHN_BR_PROF=1"] + sys.argv[1:], "/tmp/hn_brprof.so")
PY
HN_LIB_PATH=/tmp/hn_brprof.so timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline \
    > $OUT/br_profile.json 2> $OUT/br_profile.err || { tail -3 $OUT/br_profile.err; exit 1; }
grep 'hn_br_profile' $OUT/br_profile.err | tail -3
