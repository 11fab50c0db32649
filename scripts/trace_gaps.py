"""Per-kernel mean duration and the mean idle gap before each launch (start minus the previous
kernel's end on the same queue) from a rocprofv3 kernel trace: where a latency-bound chain of
short launches (the PPO update's minibatches) spends its time.
  python scripts/trace_gaps.py run_kernel_trace.csv [min_calls]"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
min_calls = int(sys.argv[2]) if len(sys.argv) > 2 else 50
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = (r["Kernel_Name"].split("(")[0][:60], int(r["Grid_Size_X"]))
    dur[k].append((e - s) / 1e3)
    if prev_end is not None and 0 <= s - prev_end < 50_000:
        gap[k].append((s - prev_end) / 1e3)
    prev_end = e
print(f"{'kernel':62s} {'grid':>8s} {'calls':>6s} {'mean us':>8s} {'median':>8s} {'gap before':>10s}")
for k, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    if len(d) < min_calls:
        continue
    gp = statistics.mean(gap[k]) if gap[k] else float("nan")
    print(f"{k[0]:62s} {k[1]:8d} {len(d):6d} {statistics.mean(d):8.2f} {statistics.median(d):8.2f} {gp:10.2f}")
