#!/bin/bash
# Kernel-level profile of a short bench run; prints the top kernels.
#   usage: scripts/gpu_prof.sh TAG [bench args...]
set -o pipefail
TAG=${1:-p}
shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
python hashnerf-pytorch_amd/build.py > $OUT/build_$TAG.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $OUT/prof_$TAG.log 2>&1 || { echo "prof failed"; tail $OUT/prof_$TAG.log; exit 1; }
python3 - "$OUT/prof_$TAG" <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.3f} ms {r["Calls"]:>5} avg {float(r["AverageNs"])/1e3:9.2f} us {float(r["Percentage"]):5.1f}%  {r["Name"][:70]}')
print("total GPU ms", round(tot / 1e6, 3))
EOF
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv   # per-dispatch rows: large
