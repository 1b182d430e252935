"""Diagnostic: the dispatch timeline of the last timed step of a bench run
from a rocprofv3 --kernel-trace CSV: per dispatch its start offset within the
step, its duration and the idle gap before it (ns), and the step's totals.
A step is delimited by the sampler's first kernel (morton_count_kernel).
   usage: python scripts/trace_timeline.py kernel_trace.csv [steps=1]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    starts = [i for i, r in enumerate(rows) if "morton_count_kernel" in r["Kernel_Name"]]
    if len(starts) < steps + 1:
        print("not enough steps in the trace")
        return
    for s in range(steps):
        a, b = starts[-steps - 1 + s], starts[-steps + s]
        seg = rows[a:b]
        t0 = int(seg[0]["Start_Timestamp"])
        busy = gaps = 0
        prev_end = t0
        print(f"step {s}: {len(seg)} dispatches")
        for r in seg:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = max(0, st - prev_end)
            gaps += gap
            busy += en - st
            name = r["Kernel_Name"].replace("void ", "")
            name = name.split("(")[0][:48] if "hn::" in name else name[:48]
            print(f"  +{(st - t0) / 1e3:8.1f} us  {(en - st) / 1e3:8.1f} us  gap {gap / 1e3:6.1f} us  {name}")
            prev_end = max(prev_end, en)
        total = int(rows[b]["Start_Timestamp"]) - t0
        print(f"  step {total / 1e3:.1f} us: kernels {busy / 1e3:.1f} us, gaps {gaps / 1e3:.1f} us "
              f"(+ {(int(rows[b]['Start_Timestamp']) - prev_end) / 1e3:.1f} us to the next step)")


if __name__ == "__main__":
    main()
