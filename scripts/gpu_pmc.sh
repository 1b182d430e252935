#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 run, --kernel-trace only,
# as MI355X_MICROARCH.md prescribes) over a short bench; per-kernel averages
# per dispatch go to gpurun_out/pmc_<tag>.txt.
#   usage: scripts/gpu_pmc.sh TAG [bench args...]
set -o pipefail
TAG=${1:-m}
shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
# the in-tree library is built on the CPU side before the call (no build here)
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
# counter groups, one rocprofv3 pass each; PMC_PASSES="A B;C D" overrides
if [ -n "$PMC_PASSES" ]; then
  IFS=';' read -r -a PASSES <<< "$PMC_PASSES"
else
  PASSES=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum"
          "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32"
          "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS")
fi
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/pmc_${TAG}_$i -o pmc -- \
      python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline "$@" > $OUT/pmc_${TAG}_$i.log 2>&1 \
      || { echo "pass $i ($P) failed: $(tail -2 $OUT/pmc_${TAG}_$i.log)"; exit 1; }
done
python3 - "$OUT" "$TAG" "$*" <<'EOF' | tee $OUT/pmc_$TAG.txt
import csv, glob, json, os, sys, collections
out, tag, bench_args = sys.argv[1], sys.argv[2], sys.argv[3]
# only the last PMC_LAST dispatches of each kernel (the timed steps; the
# bench's untimed pretraining steps come first in dispatch order)
last = int(os.environ.get("PMC_LAST", "4"))
raw = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{out}/pmc_{tag}_*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", r.get("Kernel-Name", ""))
        if "hn::" not in name:
            continue
        key = name.split("(")[0].split("<")[0].replace("void ", "")   # render_bwd_kernel<CAP> -> one key
        did = int(r.get("Dispatch_Id", r.get("Dispatch-Id", 0)) or 0)
        raw[key][r["Counter_Name"]].append((did, float(r["Counter_Value"])))
agg = collections.defaultdict(dict)
for k, cs in raw.items():
    for c, v in cs.items():
        # several rows per dispatch (per-XCD/SE instances) are summed
        per = collections.defaultdict(float)
        for did, x in v:
            per[did] += x
        ids = sorted(per)[-last:]
        agg[k][c] = [per[i] for i in ids]
for k, cs in sorted(agg.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} avg/dispatch {sum(v)/len(v):.6g}  (n={len(v)})")
# per-dispatch HBM-side bytes for bench.py's roofline.traffic (KB -> B);
# FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 reports half of a
# 128-B request); the correction is uncalibrated for 8-B gathers.
traffic = {"bench_args": bench_args, "source": f"pmc_{tag}", "kernels": {}}
for k, cs in agg.items():
    f, w = cs.get("FETCH_SIZE"), cs.get("WRITE_SIZE")
    ent = {}
    if f and w:
        ent = {"fetch_bytes": 2 * 1024 * sum(f) / len(f), "write_bytes": 1024 * sum(w) / len(w)}
        a = cs.get("TCC_EA0_ATOMIC_sum")
        if a:
            ent["atomic_requests"] = sum(a) / len(a)
    # MFMA-pipe busy cycles (all SIMDs) and GRBM_GUI_ACTIVE (sum over the 8
    # XCDs): bench.py's mfma busy fraction = busy / (1024 * grbm / 8)
    for c, key in (("SQ_VALU_MFMA_BUSY_CYCLES", "mfma_busy_cycles"), ("GRBM_GUI_ACTIVE", "grbm_gui_active")):
        v = cs.get(c)
        if v:
            ent[key] = sum(v) / len(v)
    if ent:
        traffic["kernels"][k.replace("hn::", "")] = ent
json.dump(traffic, open(f"{out}/traffic_{tag}.json", "w"), indent=1)
EOF
# the raw per-dispatch CSVs (every pretraining dispatch too) are tens of MB:
# keep only the summaries (gpurun copies back at most 64 MiB)
rm -rf $OUT/pmc_${TAG}_*/
