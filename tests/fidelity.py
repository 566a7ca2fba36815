"""P2 estimator-fidelity statistics against the reference's own runs (tests/golden/
ref_fidelity_256x192_s256.npz, made by tests/golden/make_golden.py from oracle/_ref/smallpt_*_xs).

Both sides are reduced the same way: the image is quantised as the reference writes it (toInt
:319-321), linearised ((v/255)^2.2), and averaged over 16x16 blocks, once per independent seed.
Two pooled-variance t statistics compare the seed populations (the same estimator has the same
variance: per-pixel noise 0.1419 vs the reference's 0.1421, measured):
  * global: per channel, t of the image-mean difference. Bar |t| < 4.
  * blocks: mean of t^2 over every block and channel. Unbiased runs give the variance of a t with
    nR + nO - 2 degrees of freedom, dof/(dof-2) = 1.07-1.13 here; a 0.5 % darkening of one region
    or of the whole image gives 3+. Bar < 1.6.
Calibration, 4 / 8 own seeds: the fp32 contract before the plane_k rule scores
global t -13 / -18 (cosine) and -8.5 / -10.8 (NEE), blocks 2.8-3.1 / 4.1-4.2; with the rule
|t| < 0.9 and blocks 1.08-1.31.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "ref_fidelity_256x192_s256.npz")
GLOBAL_Z_MAX = 4.0
BLOCK_Z2_MAX = 1.6


# Estimators pinned in the fixture: {name: (scene, spt_params keyword arguments, reference build)}.
# Every reference build is oracle/_ref/smallpt_{name}_xs (oracle/build_ref.sh); the scene names
# the product's builder (cornell_scene / spheres32_scene; the reference's own rect[] / the same
# 32 spheres in the reference's own Sphere class).
ESTIMATORS = {
    "nee": ("cornell", dict(nee_prob=1.0)),                 # HEAD :464 q < 1
    "cos": ("cornell", dict(nee_prob=0.0)),                 # :464 q < 0
    "uni": ("cornell", dict(nee_prob=1.0, flags=1)),        # uniform hemisphere :352-359
    "q05": ("cornell", dict(nee_prob=0.5)),                 # :464 q < 0.5 (NEE-mix Q)
    "sph": ("spheres32", dict(nee_prob=1.0)),               # C5's scene, no depth cap
    "sph16": ("spheres32", dict(nee_prob=1.0, max_depth=16)),  # C5: depth cap 16 (:447 + return)
}


def load_fixture():
    f = np.load(FIXTURE)  # plain arrays, allow_pickle=False
    w, h, spp, k = (int(v) for v in f["shape"])
    out = {"w": w, "h": h, "spp": spp, "k": k}
    for est in ESTIMATORS:
        if f"{est}_blocks" in f:
            out[est] = f[f"{est}_blocks"]
    return out


def params_of(est):
    """spt_params keyword arguments of an estimator name (ESTIMATORS)."""
    return dict(ESTIMATORS[est][1])


def scene_of(spt, est):
    """The scene (prim list) of an estimator, from the product's builders."""
    return spt.spheres32_scene() if ESTIMATORS[est][0] == "spheres32" else spt.cornell_scene()


def blocks(img, k):
    """(h, w, 3) linear framebuffer -> (h/k, w/k, 3) block means of the reference's 8-bit output."""
    h, w, _ = img.shape
    v = np.floor(np.power(np.clip(np.asarray(img, np.float64), 0, 1), 1 / 2.2) * 255 + 0.5)
    lin = (v / 255.0) ** 2.2
    return lin.reshape(h // k, k, w // k, k, 3).mean(axis=(1, 3))


def compare(ref_blocks, own_blocks):
    """-> (global z per channel (3,), block mean z^2). Inputs: (seeds, by, bx, 3)."""
    R, O = np.asarray(ref_blocks), np.asarray(own_blocks)
    nR, nO = len(R), len(O)

    def t(a, b):  # pooled two-sample t over axis 0
        s2 = ((nR - 1) * a.var(0, ddof=1) + (nO - 1) * b.var(0, ddof=1)) / (nR + nO - 2)
        se = np.sqrt(s2 * (1.0 / nR + 1.0 / nO))
        ok = se > 0  # blocks black in every run carry no information
        return (b.mean(0) - a.mean(0))[ok] / se[ok]

    zg = t(R.mean(axis=(1, 2)), O.mean(axis=(1, 2)))
    zb = t(R, O)
    return zg, float((zb ** 2).mean())
