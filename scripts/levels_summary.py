#!/usr/bin/env python3
"""Collect scripts/levels.sh's bench lines (gpurun_out/TAG_level_*.json) into
profiles/TAG_kernel_levels_c3.json: per level the workload, value, isolated kernel time, its ratio to
the literal HEAD kernel's (c3 / c2), and the same ratio per traced ray (edits change the work per
sample: a larger light ends more paths early).  usage: python scripts/levels_summary.py TAG"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
tag = sys.argv[1] if len(sys.argv) > 1 else "r06"
lines = {}
for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"{tag}_level_*.json"))):
    name = os.path.basename(f)[len(tag) + 7:-5]
    txt = [l for l in open(f).read().splitlines() if l.startswith("{")]
    if txt:
        lines[name] = json.loads(txt[-1])
out = {}
for name, d in lines.items():
    base = lines.get("c2" if name.startswith("c2") else "c3")
    p, r = d["paths"], d["roofline"]
    e = {"workload": d["config"]["workload"], "value_Msamples_s": d["value"],
         "ms_per_step": d["ms_per_step"], "kernel_ms_isolated": r["kernel_ms"], "frac": r["frac"],
         "frac_executed": r["frac_executed"], "vertices_per_sample": p["vertices_per_sample"],
         "rays_traced_per_sample": p["rays_traced_per_sample"],
         "shadow_proven_per_sample": p["shadow_proven_per_sample"]}
    if base is not None:
        bk, bp = base["roofline"]["kernel_ms"], base["paths"]
        e["kernel_ratio"] = round(r["kernel_ms"] / bk, 4)
        e["kernel_ratio_per_traced_ray"] = round(
            (r["kernel_ms"] / p["rays_traced_per_sample"]) / (bk / bp["rays_traced_per_sample"]), 4)
    lk = p.get("leak_end") or {}
    if "kernel_ms_reference_leaks" in lk:
        e["kernel_ms_reference_leaks"] = lk["kernel_ms_reference_leaks"]
        e["value_reference_leaks"] = lk["value_reference_leaks"]
    out[name] = e
spt = __import__("importlib").import_module("small-pathtracer_amd")
out["_session"] = (f"scripts/levels.sh (TAG={tag}): bench.py --steps 5 --warmup 2 --no-cpu-baseline "
                   f"per level, one box; kernel_ms_isolated = 3 launches one at a time after the timed "
                   f"region")
out["_kernel_sources_sha16"] = spt.kernel_sources_sha16()
out["_libspt_build_sources_sha16"] = spt.build_sources_sha16()
json.dump(out, open(os.path.join(ROOT, "profiles", f"{tag}_kernel_levels_c3.json"), "w"), indent=1)
for k, v in out.items():
    if not k.startswith("_"):
        print(f"{k:22s} {v['kernel_ms_isolated']:8.3f} ms  x{v.get('kernel_ratio', 0):.3f}  "
              f"per-ray x{v.get('kernel_ratio_per_traced_ray', 0):.3f}  proven {v['shadow_proven_per_sample']}")
