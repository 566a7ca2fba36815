"""Summarise rocprofv3 PMC CSVs for one kernel: per-dispatch averages + derived metrics.
usage: python scripts/pmc_summary.py gpurun_out/prof_TAG [kernel-substring]"""
import csv
import glob
import importlib
import json
import os
import sys
from collections import Counter, defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

root = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
# The bench run renders other variants too after its timed region (the reference-leaks leg, r06):
# only the most dispatched kernel whose name contains kname -- the workload's own -- is summarised.
names = Counter()
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            names[r["Kernel_Name"]] += 1
full = names.most_common(1)[0][0] if names else kname
vals = defaultdict(list)
durs = []
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"] == full or (not names and kname in r["Kernel_Name"]):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"] == full:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
avg = {k: sum(v) / len(v) for k, v in vals.items()}
# The kernel build these counters belong to (bench.py checks it before using them): the hash the
# library was built with (embedded by make, spt_build_sources_sha16; SPT_LIB selects an A/B build),
# which must equal the tree's -- a summary of counters from other sources is refused.
spt = importlib.import_module("small-pathtracer_amd")
built, tree = spt.build_sources_sha16(), spt.kernel_sources_sha16()
if built != tree:
    sys.exit(f"pmc_summary: {spt.LIB_PATH} was built from kernel sources {built}, the tree has {tree}; "
             f"rebuild it (or summarise on the tree it was built from)")
out = {"kernel": full, "dispatches": {k: len(v) for k, v in vals.items()}, "counters": avg,
       "kernel_sources_sha16": built}
if durs:
    out["avg_duration_ms"] = 1e3 * sum(durs) / len(durs)
d = out.get("avg_duration_ms")
g = lambda k: avg.get(k)  # noqa: E731
der = {}
if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
    der["valu_insts_per_wave"] = g("SQ_INSTS_VALU") / g("SQ_WAVES")
if g("SQ_INSTS_VALU") and d:
    # wave-instructions/s x 64 lanes vs peak 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6e12
    der["valu_lane_slots_per_s"] = g("SQ_INSTS_VALU") * 64 / (d * 1e-3)
    der["valu_issue_frac_of_peak"] = der["valu_lane_slots_per_s"] / 78.6432e12
if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
    der["valu_lane_utilization"] = g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU"))
if g("GRBM_GUI_ACTIVE") and d:
    der["effective_clock_ghz"] = g("GRBM_GUI_ACTIVE") / 8 / (d * 1e-3) / 1e9
for k in ("SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
    if g(k) and g("SQ_INSTS_VALU"):
        der[k.lower() + "_per_valu"] = g(k) / g("SQ_INSTS_VALU")
if g("SQ_WAIT_INST_ANY") and g("SQ_WAVE_CYCLES"):
    der["wait_inst_any_frac"] = g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES")
if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
    der["wait_any_frac"] = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
if g("SQ_ACTIVE_INST_ANY") and g("SQ_WAVE_CYCLES"):
    der["active_inst_any_frac"] = g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES")
if g("FETCH_SIZE") is not None:
    der["fetch_bytes_corrected"] = 2 * g("FETCH_SIZE") * 1024  # gfx950: FETCH_SIZE reads 1/2, KB
if g("WRITE_SIZE") is not None:
    der["write_bytes"] = g("WRITE_SIZE") * 1024
out["derived"] = der
print(json.dumps(out, indent=1))
