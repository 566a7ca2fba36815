#!/usr/bin/env python3
"""The shadow-ray slot model's inputs: which light-accepted NEE
shadow rays the HEAD NEE kernel still traces (early_nee_proven fails), by outcome and by the
predicate's failing clause, from the oracle (the same contract and Philox streams as the kernel).
Writes profiles/r06_shadow_census.json.  usage: python tools/shadow_census.py [W H SPP]"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402  (test infrastructure: the checker, not the product)

w, h, spp = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 192, 32)
p = oracle.default_params(width=w, height=h, spp=spp, seed=3)
oracle.proof_check(True)
try:
    _, st = oracle.counter_render(oracle.scene_cornell(), oracle.camera(w / h), p)
    claims, bad = oracle.proof_counts()
finally:
    oracle.proof_check(False)
c = oracle.shadow_census()
n = w * h * spp
per = lambda v: round(v / n, 4)  # noqa: E731
traced = c[0] + c[1]
out = {
    "workload": f"HEAD scene, NEE (C3's estimator), {w}x{h} @ {spp} spp, seed 3, oracle counter mode",
    "per_sample": {
        "path_rays": per(st["path_rays"]), "vertices": per(st["vertices"]),
        "nee_light_hits": per(st["nee_light_hits"]),
        "shadow_light_accepted": per(st["shadow_traced"]),
        "shadow_proven_in_iteration": per(claims),
        "shadow_traced_iterations": per(traced),
        "lane_iterations": per(st["path_rays"] + traced),
        "traced_reached": per(c[0]), "traced_blocked": per(c[1]),
        "traced_blocked_vertex_outside_room": per(c[3]),
        "traced_blocked_self_hit_inside": per(c[4]), "traced_blocked_self_hit_outside": per(c[5]),
        "traced_reached_short_box_clause_failed": per(c[6]),
        "traced_reached_tall_box_clause_failed": per(c[7]),
        "traced_reached_both_clauses_failed": per(c[8]),
    },
    "proof_contradictions": bad,
    "how": "spt_oracle_shadow_census (proof mode 1): every light-accepted shadow ray the early "
           "resolve does not prove is classified by the contract's own intersect",
}
out["traced_share_of_lane_iterations"] = round(traced / (st["path_rays"] + traced), 4)
json.dump(out, open(os.path.join(ROOT, "profiles", "r06_shadow_census.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
