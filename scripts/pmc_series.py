"""Per-dispatch series of one rocprofv3 --pmc counter for the rollout kernel (MiB), in dispatch
order.  usage: pmc_series.py counter_collection.csv COUNTER [kernel-substring]"""
import csv
import sys

path, name = sys.argv[1], sys.argv[2]
sub = sys.argv[3] if len(sys.argv) > 3 else "k_env_side<true, true, false"
per = {}
for r in csv.DictReader(open(path)):
    if r["Counter_Name"] == name and sub in r["Kernel_Name"]:
        d = int(r["Dispatch_Id"])
        per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
print(name, " ".join(f"{per[d] / 1024:.1f}" for d in sorted(per)))
