"""Per-kernel duration statistics over the LAST n dispatches of each kernel in
a rocprofv3 --kernel-trace CSV: the timed steps of a bench run whose untimed
pretraining steps come first.  Complements rocprofv3's --stats summary, which
averages over every dispatch of the run.

Only dispatches inside the timed window count: the window opens at the first
of the last N dispatches of the anchor kernel (the fused forward, which runs
once per step), so kernels of the data set-up or the pretraining (torch ops of
the procedural scene, say) are left out and Calls is the count per N steps.

  usage: python scripts/trace_tail_stats.py prof_kernel_trace.csv N [anchor] > tail.csv
"""
import collections
import csv
import sys

path, n = sys.argv[1], int(sys.argv[2])
anchor = sys.argv[3] if len(sys.argv) > 3 else "hn::render_fwd_kernel"
rows = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    rows[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
anchors = sorted(i for name, v in rows.items() if name.startswith(anchor) for i, _ in v)
start = anchors[-n] if len(anchors) >= n else 0
out = []
for name, v in rows.items():
    v = [d for i, d in sorted(v) if i >= start]
    if v:
        out.append((sum(v), name, len(v), sum(v) / len(v), min(v), max(v)))
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
tot = sum(o[0] for o in out)
for s, name, c, avg, mn, mx in sorted(out, reverse=True):
    w.writerow([name, c, s, round(avg, 1), mn, mx, round(100.0 * s / tot, 2)])
