"""Summarise tools/pmc_syrk.sh output: per-dispatch counters of one kernel."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "syrks_q_kernel"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{out}/*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
last = {}
for (f, _), v in agg.items():
    last[f] = v  # last dispatch of each pass
c = {}
for v in last.values():
    c.update(v)
for k in sorted(c):
    print(f"{k:28s} {c[k]:.4e}")
if "TCC_HIT_sum" in c:
    print(f"L2 hit rate {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
    print(f"MFMA busy per SIMD / GUI_ACTIVE per XCD: "
          f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (c['GRBM_GUI_ACTIVE'] / 8):.3f}")
if "SQ_WAVE_CYCLES" in c:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in c:
            print(f"{k} / WAVE_CYCLES {c[k] / c['SQ_WAVE_CYCLES']:.3f}")
