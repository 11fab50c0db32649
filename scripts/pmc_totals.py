"""Per-launch totals of every counter in gpurun_out/pmc/p*/run_counter_collection.csv
(summed over the device's SEs/CUs by rocprofv3, averaged over the matched dispatches)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
tot, disp = collections.defaultdict(float), collections.defaultdict(set)
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / len(disp[k]):16.1f} per launch ({len(disp[k])} launches)")
