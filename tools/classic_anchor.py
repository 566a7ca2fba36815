#!/usr/bin/env python3
"""Diagnostic (not a gate): the classic smallpt sphere box (spt_scene_smallpt_classic) rendered on
the GPU against the reference's shipped renders of that scene (tests/golden/
shipped_sphere_box_k32.npz: 32x32-block means of /root/reference/image*.ppm, 512x512, made by
tests/golden/make_golden.py --shipped).

The shipped images come from older revisions of the reference whose
source is not in the tree: their estimators (sphere-light NEE, "total random" scattering) and
any constants beyond those mined from src/a.exe are unknown. So this only reports how far a
converged render of the rebuilt scene is from each of them: per-channel image-mean difference and
block RMSE, beside each image's own noise (its within-block pixel variance / 1024, an upper bound
since it includes the block's signal gradient).

  python tools/classic_anchor.py [--spp 1024] > profiles/r02_classic_anchor.json
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def blocks(img, k):
    h, w, _ = img.shape
    v = np.floor(np.power(np.clip(img.astype(np.float64), 0, 1), 1 / 2.2) * 255 + 0.5)
    return ((v / 255.0) ** 2.2).reshape(h // k, k, w // k, k, 3).mean(axis=(1, 3))


# shipped render -> (our estimator, its spp): the old revision's cosine ("importance") and
# "total random" (the uniform hemisphere of :352-359) estimators are pure path tracing, so the
# rebuilt scene must reproduce them; its explicit-light estimator sampled the sphere light with
# code that is not in the reference tree.
SAME_SPP = [("image2_32pps_importancesampl", "cosine", 32), ("image1_16ssp_importsampl", "cosine", 16),
            ("image_32pps_totalrandom", "uniform", 32)]


def same_spp_z(spt, f, name, est, spp, w, h, k, cam, seeds=16):
    """z of the shipped image's global mean per channel and mean z^2 over blocks, against `seeds`
    renders of ours at the shipped spp (their sample mean and spread)."""
    flags = spt.FLAG_UNIFORM_SCATTER if est == "uniform" else 0
    own = []
    for seed in range(1, seeds + 1):
        p = spt.default_params(width=w, height=h, spp=spp, nee_prob=0.0, flags=flags, seed=seed)
        own.append(blocks(spt.render(spt.smallpt_classic_scene(), cam, p), k))
    own = np.array(own)
    ref = f[f"{name}_mean"]
    mu, sd = own.mean(0), own.std(0, ddof=1)
    g_mu, g_sd = own.mean(axis=(1, 2)).mean(0), own.mean(axis=(1, 2)).std(0, ddof=1)
    ok = sd > 0
    zb = (ref - mu)[ok] / (sd[ok] * np.sqrt(1 + 1.0 / seeds))
    return {"estimator": est, "spp": spp, "seeds": seeds,
            "global_z": [round(float(x), 2) for x in (ref.mean(axis=(0, 1)) - g_mu) / (g_sd * np.sqrt(1 + 1.0 / seeds))],
            "rel_mean_diff": [round(float(x), 4) for x in (ref.mean(axis=(0, 1)) - g_mu) / g_mu],
            "block_mean_z2": round(float((zb ** 2).mean()), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--png", default="", help="also save the renders (8-bit, gamma as :319-321)")
    ap.add_argument("--seeds", type=int, default=16)
    args = ap.parse_args()
    spt = importlib.import_module("small-pathtracer_amd")
    f = np.load(os.path.join(ROOT, "tests", "golden", "shipped_sphere_box_k32.npz"))
    w, h, k = (int(v) for v in f["shape"])
    cam = spt.Camera(aspect=1.0)
    renders = {}
    for name, flags in (("cosine", 0), ("uniform", spt.FLAG_UNIFORM_SCATTER)):
        p = spt.default_params(width=w, height=h, spp=args.spp, nee_prob=0.0, flags=flags)
        img, st = spt.render(spt.smallpt_classic_scene(), cam, p, return_stats=True)
        renders[name] = (blocks(img, k), st)
        if args.png:
            from PIL import Image
            v = np.floor(np.power(np.clip(img, 0, 1), 1 / 2.2) * 255 + 0.5).astype(np.uint8)
            Image.fromarray(v).save(args.png.replace(".png", f"_{name}.png"))
    out = {"scene": "spt_scene_smallpt_classic (matte .999 balls)", "size": [w, h], "spp": args.spp,
           "estimators": {n: {"kernel_ms": round(st["kernel_ms"], 2),
                              "vertices_per_sample": round(st["vertices"] / st["samples"], 3)}
                          for n, (_, st) in renders.items()},
           "images": {}}
    for name in [str(n) for n in f["names"]]:
        ref, var = f[f"{name}_mean"], f[f"{name}_var"]
        noise = np.sqrt((var / (k * k)).mean(axis=(0, 1)))
        row = {"shipped_mean": [round(float(x), 4) for x in ref.mean(axis=(0, 1))],
               "block_noise_bound": [round(float(x), 4) for x in noise]}
        for est, (own, _) in renders.items():
            # a global exposure factor (least squares own ~ g * ref) and the block RMSE left after it
            g = float((own * ref).sum() / max((ref * ref).sum(), 1e-30))
            row[est] = {"scale_own_over_shipped": round(g, 4),
                        "block_rmse_after_scale": [round(float(x), 4) for x in
                                                   np.sqrt(((own / g - ref) ** 2).mean(axis=(0, 1)))],
                        "mean_diff": [round(float(x), 4) for x in (own - ref).mean(axis=(0, 1))],
                        "rel_mean_diff": [round(float(x), 4) for x in
                                          ((own - ref).mean(axis=(0, 1)) / ref.mean(axis=(0, 1)))],
                        "block_rmse": [round(float(x), 4) for x in
                                       np.sqrt(((own - ref) ** 2).mean(axis=(0, 1)))]}
        out["images"][name] = row
    # Same-spp statistics for the shipped pure-path-tracing renders: the reference clamps each
    # pixel estimate (:538), so a shipped 16/32-spp image and a converged render differ in
    # expectation; compare the shipped image with the distribution of OUR images at its spp.
    out["same_spp"] = {}
    for name, est, spp in SAME_SPP:
        z = same_spp_z(spt, f, name, est, spp, w, h, k, cam, seeds=args.seeds)
        out["same_spp"][name] = z
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
