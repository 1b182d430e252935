#!/bin/bash
# r03y: PSNR@5k on the final round-3 library.  Seed 0 paired in full, its
# reference curve compared with r03k's seed-0 run (the cache's premise); then
# seeds 1-4 HIP-only against their r03k/r03l reference curves, then seeds 5-6
# paired in full.
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_psnr_seq.sh r03y 0 || exit 1
python - <<'PY' || exit 1
import json
a = json.load(open("gpurun_out/psnr_r03y/psnr_5k_r03y_seed0.json"))
b = json.load(open("profiles/r03/psnr_r03k/psnr_5k_r03k_seed0.json"))
rb = {c["iter"]: c["psnr_ref"] for c in b["curve"]}
d = [abs(c["psnr_ref"] - rb[c["iter"]]) for c in a["curve"] if c["iter"] in rb]
print("reference curve vs r03k seed 0:", len(d), "common evaluations, max |diff|", max(d))
json.dump({"common_evals": len(d), "max_abs_diff_db": max(d)}, open("gpurun_out/psnr_r03y/ref_cache_check.json", "w"))
assert max(d) <= 1e-4, "the reference path is not repeatable across runs: do not use the cache"
PY
bash scripts/gpu_psnr_seq.sh r03y c1 c2 c3 c4 5 6
