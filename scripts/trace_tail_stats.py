"""Per-kernel duration statistics over the LAST n dispatches of each kernel in
a rocprofv3 --kernel-trace CSV: the timed steps of a bench run whose untimed
pretraining steps come first.  Complements rocprofv3's --stats summary, which
averages over every dispatch of the run.

  usage: python scripts/trace_tail_stats.py prof_kernel_trace.csv N > tail.csv
"""
import collections
import csv
import sys

path, n = sys.argv[1], int(sys.argv[2])
rows = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    rows[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
out = []
for name, v in rows.items():
    v = [d for _, d in sorted(v)][-n:]
    out.append((sum(v), name, len(v), sum(v) / len(v), min(v), max(v)))
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
tot = sum(o[0] for o in out)
for s, name, c, avg, mn, mx in sorted(out, reverse=True):
    w.writerow([name, c, s, round(avg, 1), mn, mx, round(100.0 * s / tot, 2)])
