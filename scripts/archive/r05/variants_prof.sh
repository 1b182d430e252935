#!/bin/bash
# Diagnostic: per-kernel average durations over the TIMED steps (the last 10
# dispatches of each kernel, rocprofv3 --kernel-trace) of a bench run for each
# -D build variant of the library.
#   usage: scripts/variants_prof.sh "-DFOO=1" "-DFOO=2" ...     ("-" = the default build)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for V in "$@"; do
  i=$((i+1))
  [ "$V" = "-" ] && V=""
  python - "$V" "$i" <<'PY' || exit 1
import sys; sys.path.insert(0, "hashnerf-pytorch_amd")
import build
defs = sys.argv[1].split()
build.build_variant(defs, f"/tmp/hn_vprof{sys.argv[2]}.so")
PY
  HN_LIB_PATH=/tmp/hn_vprof$i.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d $OUT/vprof$i -o p -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
      > $OUT/vprof$i.log 2>&1 || { echo "variant $i failed"; tail -3 $OUT/vprof$i.log; exit 1; }
  T=$(ls $OUT/vprof$i/*kernel_trace.csv $OUT/vprof$i/*/*kernel_trace.csv 2>/dev/null | head -1)
  echo "variant [$V]: $(grep -o '"value": [0-9.]*' $OUT/vprof$i.log | head -1)"
  python3 scripts/trace_tail_stats.py $T 10 | python3 -c "
import csv, sys
for r in csv.DictReader(sys.stdin):
    if 'hn::' in r['Name']:
        print(f'   {float(r[\"AverageNs\"])/1e3:9.2f} us  {r[\"Name\"][:60]}')"
  rm -f $T
done
