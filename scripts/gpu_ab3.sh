#!/bin/bash
# Interleaved A/B of (library, bench flags) variants on one box: short bench
# lines, then one rocprofv3 kernel trace per variant.
#   usage: scripts/gpu_ab3.sh TAG "name:lib.so:flags" ...   (lib "-" = the in-tree library)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
run() {   # name lib flags -> env for the library
  if [ "$2" = "-" ]; then echo ""; else echo "HN_LIB_PATH=hashnerf-pytorch_amd/build/$2"; fi
}
for r in $(seq 1 ${REPS:-2}); do
  for V in "$@"; do
    IFS=: read -r N LIBF FL <<< "$V"
    env $(run $N $LIBF) timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline $FL > $O/${N}_$r.json 2> $O/${N}_$r.err || { tail -5 $O/${N}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${N}_$r.json'));print('$N', $r, d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
  done
done
if [ -n "$PROF" ]; then
  for V in "$@"; do
    IFS=: read -r N LIBF FL <<< "$V"
    env $(run $N $LIBF) timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$N -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $FL > $O/prof_$N.log 2>&1 || { tail -5 $O/prof_$N.log; exit 1; }
    F=$(find $O/prof_$N -name "*kernel_trace.csv" | head -1)
    python3 scripts/trace_tail_stats.py $F 10 > $O/kernel_stats_$N.csv && rm -rf $O/prof_$N
    python3 - $O/kernel_stats_$N.csv $N <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("render_fwd_kernel", "render_bwd_kernel", "scatter_bins", "bin_reduce", "comp_bwd")):
        print(sys.argv[2], n.split("(")[0].replace("void ", "").replace("hn::", ""), round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
  done
fi
