"""Kernel-trace durations grouped by (kernel, grid size): bench.py runs the headline workload
(65,536 walkers) and the smaller BASELINE shapes in one command, so rocprofv3's per-name
--stats averages mix launch sizes; this separates them.
  python scripts/trace_by_grid.py gpurun_out/prof_r02/trace/run_kernel_trace.csv > profiles/r02_kernel_stats_by_grid.csv"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
g = collections.defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]),
           int(r["Workgroup_Size_X"]))
    g[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
w = csv.writer(sys.stdout)
w.writerow(["kernel", "grid_threads", "workgroup", "calls", "total_us", "mean_us", "median_us", "min_us", "max_us"])
for (k, grid, wg), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([k, grid, wg, len(d), round(sum(d), 1), round(statistics.mean(d), 3),
                round(statistics.median(d), 3), round(min(d), 3), round(max(d), 3)])
