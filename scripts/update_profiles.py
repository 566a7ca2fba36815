#!/usr/bin/env python3
"""Copy one profiling session (scripts/profile.sh TAG -> gpurun_out/prof_TAG) into the tracked
profiles/ files that bench.py attaches and DESIGN.md cites:
  profiles/<ROUND>_rocprof_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary
  profiles/<ROUND>_pmc_summary.json          per-dispatch PMC averages + derived VALU metrics
  profiles/traffic_c3.json                   HBM bytes per render launch (FETCH_SIZE x2 gfx950 correction)
usage: python scripts/update_profiles.py TAG ROUND   (e.g. r02 r02)"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
prof = os.path.join(ROOT, "profiles")
shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"),
            os.path.join(prof, f"{rnd}_rocprof_kernel_stats.csv"))
summ = json.loads(subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), src],
                                 check=True, capture_output=True, text=True).stdout)
summ["session"] = f"scripts/profile.sh {tag} (bench.py c3, --steps 6 --warmup 2 --frames-in-flight 1)"
json.dump(summ, open(os.path.join(prof, f"{rnd}_pmc_summary.json"), "w"), indent=1)
c = summ["counters"]
fetch = 2 * c["FETCH_SIZE"] * 1024
write = c["WRITE_SIZE"] * 1024
json.dump({
    "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, render kernel of "
              f"bench.py c3 (profiles/{rnd}_pmc_summary.json, scripts/profile.sh {tag})",
    "fetch_size_kb": c["FETCH_SIZE"], "write_size_kb": c["WRITE_SIZE"],
    "correction": "gfx950 (MI355X_MICROARCH.md HBM section): FETCH_SIZE counts 1/2 of the bytes of "
                  "wide reads -> x2; KB -> bytes x1024; WRITE_SIZE as reported",
    "hbm_bytes_per_launch": fetch + write,
    "kernel_sources_sha16": summ["kernel_sources_sha16"],
    "note": "writes are the unit slots (one 24-byte owner store of three 64-bit fixed-point sums per "
            "work unit; C3 since round 4: 96-sample units, 6 passes x 786,432 pixels = 4.72 M units "
            "= 113 MB) plus the 64-bit atomics of the ranges stolen in the tail (three per range, "
            "each a whole-sector write)",
}, open(os.path.join(prof, "traffic_c3.json"), "w"), indent=1)
print("kernel avg ms", summ["avg_duration_ms"], "hbm bytes/launch", fetch + write)
