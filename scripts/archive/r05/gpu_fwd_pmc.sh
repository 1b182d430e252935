#!/bin/bash
# Forward-kernel bottleneck counters (config 2): one rocprofv3 --pmc pass per
# group (MI355X_MICROARCH.md: separate passes, --kernel-trace only), each
# under its own time limit; a pass whose counters this pool does not know is
# skipped.  Per-dispatch averages of render_fwd_kernel over the last 4 dispatches.
#   usage: scripts/gpu_fwd_pmc.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for P in "TA_BUSY_avr TA_BUSY_max" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
         "TD_BUSY_avr" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$i -o pmc -- \
      python3 bench.py --steps 4 --warmup 2 --pretrain 200 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1
  echo "pass $i [$P] rc=$?"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
raw = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if "render_fwd_kernel" not in name:
            continue
        raw[r["Counter_Name"]][int(r.get("Dispatch_Id", 0) or 0)] += float(r["Counter_Value"])
with open(f"{out}/fwd_counters.txt", "w") as fo:
    for c, d in sorted(raw.items()):
        ids = sorted(d)[-4:]
        line = f"{c:40s} {sum(d[i] for i in ids) / len(ids):.6g}"
        print(line); fo.write(line + "\n")
PY
rm -rf $OUT/p*/
