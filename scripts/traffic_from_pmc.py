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
    """per rollout dispatch (the counting replay's k_env_step is not one), in dispatch order,
    the counter summed over its per-unit rows"""
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name and "k_env_side<true, true, false" in r["Kernel_Name"]:
            d = int(r["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    return [per[d] for d in sorted(per)]


fs = read(fetch_csv, "FETCH_SIZE")
ws = read(write_csv, "WRITE_SIZE")
f_mean, w_mean = sum(fs) / len(fs), sum(ws) / len(ws)
# the timed launch: bench.py --steps 1 --warmup 0 --no-extras runs its regime iterations first and
# the timed iteration last, so the last rollout dispatch is the launch the bench line's roofline
# times; the earlier ones start from fresh walkers (more resets, another lane order)
res = {"kernel": "k_env_side<true,true,false> (rollout: physics + policy)", "walkers": int(walkers), "horizon": int(horizon),
       "fetch_size_kib": fs[-1], "write_size_kib": ws[-1],
       "hbm_bytes_per_launch": (2.0 * fs[-1] + ws[-1]) * 1024.0,
       "hbm_bytes_per_launch_mean": (2.0 * f_mean + w_mean) * 1024.0,
       "fetch_size_kib_series": [round(v, 1) for v in fs], "write_size_kib_series": [round(v, 1) for v in ws],
       "launches": [len(fs), len(ws)],
       "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported; KiB -> bytes; the timed (last) launch, the mean over all alongside"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
