"""Summarise gpurun_out/pmc/p*/run_counter_collection.csv: counters per wave per substep.
  python scripts/pmc_summary.py [substeps_per_launch]"""
import csv
import glob
import sys

sub = int(sys.argv[1]) if len(sys.argv) > 1 else 400
agg, meta = {}, None
for f in sorted(glob.glob("gpurun_out/pmc/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta = r
waves = int(meta["Grid_Size"]) // 64
dur = (int(meta["End_Timestamp"]) - int(meta["Start_Timestamp"])) / 1e6
print(f"grid {meta['Grid_Size']} waves {waves} vgpr {meta['VGPR_Count']} sgpr {meta['SGPR_Count']} "
      f"scratch {meta['Scratch_Size']} dur {dur:.2f} ms")
quad = {"SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"}
for k in sorted(agg):
    v = agg[k] * (4 if k in quad else 1)
    print(f"  {k:28s} {agg[k]:16.0f}  per wave-substep {v / max(1, waves) / sub:10.1f}")
