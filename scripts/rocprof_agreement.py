#!/usr/bin/env python3
"""profiles/<ROUND>_rocprof_agreement.json from one profiling session (scripts/profile.sh TAG): the
render dispatches of the kernel-trace pass in order, the average of the bench's timed ones, and the
bench line's own kernel_ms from the same run (its JSON line in trace.log).
usage: python scripts/rocprof_agreement.py TAG ROUND   (e.g. r05 r05)"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, rnd = sys.argv[1], sys.argv[2]
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
rows = list(csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_trace.csv"))))
rows = [r for r in rows if "render_kernel" in r["Kernel_Name"]]
main_name = max({r["Kernel_Name"] for r in rows}, key=lambda n: sum(r["Kernel_Name"] == n for r in rows))
all_names = sorted({r["Kernel_Name"][:160] for r in rows})
rows = [r for r in rows if r["Kernel_Name"] == main_name]  # the workload's own variant
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
line = next(json.loads(l) for l in open(os.path.join(src, "trace.log")) if l.startswith("{"))
warm, steps = line["warmup"], line["steps"]
timed = ms[warm:warm + steps]
sys.path.insert(0, ROOT)
summ = json.load(open(os.path.join(ROOT, "profiles", f"{rnd}_pmc_summary.json")))
out = {
    "command": f"scripts/profile.sh {tag}: rocprofv3 --kernel-trace --stats -- python3 bench.py --steps {steps} "
               f"--warmup {warm} --no-cpu-baseline --frames-in-flight 1 (C3)",
    "render_dispatches_ms": [round(x, 4) for x in ms],
    "order": f"{warm} warm-up launches, the {steps} timed launches, then the renders after the timed region "
             "(the reference-leaks leg of paths.leak_end -- another kernel variant, kernel_names -- and "
             "the quality renders)",
    "kernel_names": all_names,
    "main_kernel": main_name[:160],
    "timed_dispatches_avg_ms": round(sum(timed) / len(timed), 3),
    "bench_kernel_ms_same_run": line["roofline"]["kernel_ms"],
    "all_dispatches_avg_ms": round(sum(ms) / len(ms), 4),
    "all_dispatches_median_ms": round(statistics.median(ms), 4),
    "note": "the summary CSV's average (all dispatches) includes the warm-up and the launches after idle "
            "gaps, which run while the GPU's clocks ramp",
    "kernel_sources_sha16": summ["kernel_sources_sha16"],
}
json.dump(out, open(os.path.join(ROOT, "profiles", f"{rnd}_rocprof_agreement.json"), "w"), indent=1)
print(json.dumps({k: out[k] for k in ("timed_dispatches_avg_ms", "bench_kernel_ms_same_run",
                                      "all_dispatches_avg_ms", "all_dispatches_median_ms")}))
