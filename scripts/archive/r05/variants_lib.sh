#!/bin/bash
# Diagnostic: bench prebuilt variant libraries (hashnerf-pytorch_amd/build/var_*.so,
# built on the CPU side with build.build_variant) one after the other.
#   usage: scripts/variants_lib.sh var_a var_b ...
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
for V in "$@"; do
  HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
      > $OUT/$V.json 2> $OUT/$V.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels'])"
done
