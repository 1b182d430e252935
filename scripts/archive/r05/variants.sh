#!/bin/bash
# Diagnostic: bench the library built with different -D settings.
#   usage: scripts/variants.sh "-DFOO=1" "-DFOO=2" ...
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
i=0
for V in "$@"; do
  i=$((i+1))
  python - "$V" "$i" <<'PY' || exit 1
import sys; sys.path.insert(0, "hashnerf-pytorch_amd")
import build
defs = sys.argv[1].split()
build.build_variant(defs, f"/tmp/hn_variant{sys.argv[2]}.so")
PY
  HN_LIB_PATH=/tmp/hn_variant$i.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
      > $OUT/variant$i.json 2> $OUT/variant$i.err || exit 1
  python -c "import json;d=json.load(open('$OUT/variant$i.json'));print('$V', d['value'], d['ms_per_step'], d['kernels'])"
done
