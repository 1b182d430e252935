#!/bin/bash
# Diagnostic: one pytest selection (-k EXPR) against each -D build variant of
# the library.   usage: K=EXPR scripts/variants_test.sh "-DFOO=1" "-DFOO=0" ...   ("-" = default)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
i=0
for V in "$@"; do
  i=$((i+1))
  [ "$V" = "-" ] && V=""
  python - "$V" "$i" <<'PY' || exit 1
import sys; sys.path.insert(0, "hashnerf-pytorch_amd")
import build
build.build_variant(sys.argv[1].split(), f"/tmp/hn_vtest{sys.argv[2]}.so")
PY
  HN_LIB_PATH=/tmp/hn_vtest$i.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "$K" --timeout 120 \
      --timeout-method thread > $OUT/vtest$i.log 2>&1
  RC=$?
  echo "variant [$V] rc=$RC: $(tail -1 $OUT/vtest$i.log)"
  [ $RC -le 1 ] || exit $RC
done
