"""Per-dispatch average of each counter over every run_counter_collection.csv under a directory
(rocprofv3 sums over the device's units): python scripts/pmc_agg.py DIR [kernel-substring]."""
import collections, csv, glob, sys
root = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else ""
tot, disp = collections.defaultdict(float), collections.defaultdict(set)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if key and key not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / len(disp[k]):18.1f} per dispatch ({len(disp[k])} dispatches)")
