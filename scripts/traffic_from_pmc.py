"""Per-launch HBM bytes of the rollout kernel from separate rocprofv3 --pmc passes.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes
of a wide coalesced read -> x2; WRITE_SIZE is exact for dword stores.  Both are KiB.
usage: traffic_from_pmc.py FETCH.csv WRITE.csv walkers horizon out.json
"""
import csv
import json
import sys

fetch_csv, write_csv, walkers, horizon, out = sys.argv[1:6]


def read(path, name):
    """mean over the rollout dispatches (the counting replay's k_env_step is not one) of the
    counter summed over its per-unit rows"""
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name and "k_env_side<true, true, false" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sum(per.values()) / len(per), len(per)


f_kib, nf = read(fetch_csv, "FETCH_SIZE")
w_kib, nw = read(write_csv, "WRITE_SIZE")
res = {"kernel": "k_env_side<true,true,false> (rollout: physics + policy)", "walkers": int(walkers), "horizon": int(horizon),
       "fetch_size_kib": f_kib, "write_size_kib": w_kib,
       "hbm_bytes_per_launch": (2.0 * f_kib + w_kib) * 1024.0,
       "launches": [nf, nw],
       "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported; KiB -> bytes"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
