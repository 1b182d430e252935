#!/bin/bash
# Diagnostic: bench (library, environment) pairs.   usage: scripts/variants_env.sh "var_a ENV=1" "var_b" ...
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
i=0
for SPEC in "$@"; do
  i=$((i+1))
  V=${SPEC%% *}; E=""; [ "$SPEC" != "$V" ] && E=${SPEC#* }
  env $E HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
      > $OUT/venv$i.json 2> $OUT/venv$i.err || exit 1
  python -c "import json;d=json.load(open('$OUT/venv$i.json'));print('$SPEC', d['value'], d['ms_per_step'], d['kernels'], d['loss'])"
done
