#!/bin/bash
# Diagnostic: time the fused backward with parts removed (HN_ABLATE builds).
#   see HN_ABLATE in csrc/hn_common.h; usage: scripts/ablate.sh [variants...]
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
VARIANTS=${@:-1 2 3 4}
python - $VARIANTS <<'EOF' || exit 1
import sys; sys.path.insert(0, "hashnerf-pytorch_amd")
import build
for v in map(int, sys.argv[1:]):
    build.build_variant([f"-DHN_ABLATE={v}"], f"/tmp/hn_ablate{v}.so")
EOF
for v in $VARIANTS; do
  HN_LIB_PATH=/tmp/hn_ablate$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 \
      --no-cpu-baseline > $OUT/ablate$v.json 2> $OUT/ablate$v.err || exit 1
  python -c "import json;d=json.load(open('$OUT/ablate$v.json'));print('ablate$v', d['kernels'])"
done
