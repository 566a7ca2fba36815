"""Regenerate tests/golden/ from the reference itself (run in the dev container only).

Builds oracle/_ref/smallpt_{nee,cos} from /root/reference/src/smallpt.cpp via oracle/build_ref.sh
(the SURVEY.md Appendix A patch streamed through sed into g++ -O3; no reference source is copied),
runs it, and stores (`--counter-only`: only the counter-mode pins, after a contract change):
  ref_64x48_s4_{nee,cos}.ppm   the reference's own output PPMs (data fixtures)
  golden.json                  md5s of the reference PPMs for 64x48@4 and 256x192@4 (NEE, cosine),
                               the build recipe, known-answer values, and counter-mode md5s
  counter_64x48_s16_{nee,cos}.npy  counter-mode contract images from oracle/ (regression pins for
                               the GPU kernel; produced by the oracle, not by the reference)
  ref_fidelity_256x192_s256.npz  the reference's estimator statistics (P2 fixture): 16 runs each of
                               oracle/_ref/smallpt_{nee,cos}_xs (row streams seeded too, so the runs
                               are independent) at 256x192@256, seeds 101..116, as 16x16-block means
                               of the linearised PPM ((v/255)^2.2): per-seed block means
                               {est}_blocks (16, 12, 16, 3); uni_blocks (the uniform-hemisphere
                               build smallpt_uni_xs), q05_blocks (Q = 0.5), sph_blocks and
                               sph16_blocks (config 5's 32-sphere scene in the reference's own
                               Sphere class, uncapped / depth cap 16) added by `--fidelity-add <est>`
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def md5(path):
    return hashlib.md5(open(path, "rb").read()).hexdigest()


def read_ppm(path):
    tok = open(path, "rb").read().split()
    w, h = int(tok[1]), int(tok[2])
    return np.array(tok[4:4 + w * h * 3], dtype=np.float64).reshape(h, w, 3)


def fidelity_fixture(ref, tmp, w=256, h=192, spp=256, seeds=range(101, 117), k=16):
    """16x16-block means of the reference's linearised PPMs, one set per independent seed."""
    from concurrent.futures import ThreadPoolExecutor
    jobs = [(est, s) for est in ("nee", "cos") for s in seeds]

    def run(job):
        est, s = job
        path = os.path.join(tmp, f"fid_{est}_{s}.ppm")
        subprocess.run([os.path.join(ref, f"smallpt_{est}_xs"), str(w), str(h), str(spp), str(s), path],
                       check=True, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        lin = (read_ppm(path) / 255.0) ** 2.2
        return lin.reshape(h // k, k, w // k, k, 3).mean(axis=(1, 3))

    with ThreadPoolExecutor(max(1, (os.cpu_count() or 2) - 1)) as ex:
        blocks = list(ex.map(run, jobs))
    n = len(seeds)
    np.savez(os.path.join(HERE, f"ref_fidelity_{w}x{h}_s{spp}.npz"),
             nee_blocks=np.array(blocks[:n]), cos_blocks=np.array(blocks[n:]),
             seeds=np.array(list(seeds)), shape=np.array([w, h, spp, k]))


def fidelity_add(ref, tmp, est, w=256, h=192, spp=256, seeds=range(101, 117), k=16):
    """Add {est}_blocks (16 independent runs of oracle/_ref/smallpt_{est}_xs) to the existing P2
    fixture, leaving its other arrays as they are (`--fidelity-add uni`)."""
    from concurrent.futures import ThreadPoolExecutor
    path = os.path.join(HERE, f"ref_fidelity_{w}x{h}_s{spp}.npz")
    old = dict(np.load(path))  # plain arrays, allow_pickle=False
    assert [int(v) for v in old["shape"]] == [w, h, spp, k]
    assert list(old["seeds"]) == list(seeds)

    def run(s):
        p = os.path.join(tmp, f"fid_{est}_{s}.ppm")
        subprocess.run([os.path.join(ref, f"smallpt_{est}_xs"), str(w), str(h), str(spp), str(s), p],
                       check=True, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        lin = (read_ppm(p) / 255.0) ** 2.2
        return lin.reshape(h // k, k, w // k, k, 3).mean(axis=(1, 3))

    with ThreadPoolExecutor(max(1, (os.cpu_count() or 2) - 1)) as ex:
        old[f"{est}_blocks"] = np.array(list(ex.map(run, seeds)))
    np.savez(path, **old)


def counter_pins(out):
    """Counter-mode contract pins (oracle output) for the GPU regression tests."""
    from oracle import oracle as o
    o.build()
    prims = o.scene_cornell()
    out["counter_md5"] = {}
    out["counter_stats"] = {}
    for est, q, fl in (("nee", 1.0, 0), ("cos", 0.0, 0), ("uni", 1.0, 1)):
        p = o.default_params(width=64, height=48, spp=16, seed=1, nee_prob=q, flags=fl)
        img, st = o.counter_render(prims, o.camera(64 / 48), p)
        if est != "uni":
            np.save(os.path.join(HERE, f"counter_64x48_s16_{est}.npy"), img)
        out["counter_md5"][est] = hashlib.md5(img.tobytes()).hexdigest()
        out["counter_stats"][est] = st


def variant_pins():
    """md5s of the reference variants that need a scene or threshold argument in the restatement
    (`--variant-pins`): smallpt_q05 (:464 q < 0.5), smallpt_sph (C5's 32 spheres in the reference's
    own Sphere class), smallpt_sph16 (the same with the depth-16 cap), at 64x48@4 and 256x192@4,
    seed 1, added to golden.json["reference_md5"] as {w}x{h}_s4_seed1_{variant}."""
    subprocess.run([os.path.join(ROOT, "oracle", "build_ref.sh")], check=True)
    ref = os.path.join(ROOT, "oracle", "_ref")
    tmp = "/tmp/spt_golden"
    os.makedirs(tmp, exist_ok=True)
    path = os.path.join(HERE, "golden.json")
    out = json.load(open(path))
    for w, h in ((64, 48), (256, 192)):
        for est in ("q05", "sph", "sph16"):
            ppm = os.path.join(tmp, f"ref_{w}x{h}_s4_{est}.ppm")
            subprocess.run([os.path.join(ref, f"smallpt_{est}"), str(w), str(h), "4", "1", ppm],
                           check=True, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            out["reference_md5"][f"{w}x{h}_s4_seed1_{est}"] = md5(ppm)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


def quality_c3(ref, tmp, w=1024, h=768, spp=512, seeds=range(201, 217), k=32, est="nee", cfg="c3"):
    """bench.py's `quality` fixture (`--quality-c3`): the reference's own C3 image (HEAD NEE,
    1024x768 @ 512 spp, the bench's config) as 32x32-block means of its linearised PPM, one set
    per independent run of oracle/_ref/smallpt_nee_xs (16 runs): ref_c3_blocks_k32.npz. The runs
    use the bench's spp because the reference clamps each PIXEL estimate to [0, 1] (:538): the
    clamp removes more of a noisier estimate, so images at different spp differ in expectation
    (measured: 64-spp runs are 0.4 % darker than a 512-spp image).
    `--quality-c2` (est "cos", cfg "c2"): the same for C2, 16 runs of smallpt_cos_xs (the cosine
    estimator :474-477) at 1024x768 @ 64 spp: ref_c2_blocks_k32.npz."""
    from concurrent.futures import ThreadPoolExecutor

    def run(s):
        path = os.path.join(tmp, f"q_{cfg}_{s}.ppm")
        subprocess.run([os.path.join(ref, f"smallpt_{est}_xs"), str(w), str(h), str(spp), str(s), path],
                       check=True, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        lin = (read_ppm(path) / 255.0) ** 2.2
        os.remove(path)
        return lin.reshape(h // k, k, w // k, k, 3).mean(axis=(1, 3))

    with ThreadPoolExecutor(max(1, (os.cpu_count() or 2) - 2)) as ex:
        blocks = np.array(list(ex.map(run, seeds)))
    np.savez(os.path.join(HERE, f"ref_{cfg}_blocks_k{k}.npz"), blocks=blocks, seeds=np.array(list(seeds)),
             shape=np.array([w, h, spp, k]))


SHIPPED = ["image_512pps_explicitlight", "image_512pps_explicitlight_test", "image_512pps_random_test",
           "image2_32pps_importancesampl", "image2_32pps_explicitsampling", "image_32pps_totalrandom",
           "image_32pps_halflighthalfimportance", "image1_16ssp_importsampl",
           "image2_16ssp_explicitsampling"]


def shipped_blocks(k=32):
    """`--shipped`: the reference's shipped renders of the classic sphere box (/root/reference/*.ppm,
    512x512 P3; renders of an older revision) as data: per image the
    32x32-block means and within-block pixel variances of the linearised PPM ((v/255)^2.2):
    shipped_sphere_box_k32.npz {name}_mean, {name}_var (16, 16, 3)."""
    out = {}
    for name in SHIPPED:
        lin = (read_ppm(os.path.join("/root/reference", name + ".ppm")) / 255.0) ** 2.2
        h, w, _ = lin.shape
        b = lin.reshape(h // k, k, w // k, k, 3)
        out[f"{name}_mean"] = b.mean(axis=(1, 3))
        out[f"{name}_var"] = b.var(axis=(1, 3), ddof=1)
    out["names"] = np.array(SHIPPED)
    out["shape"] = np.array([512, 512, k])
    np.savez(os.path.join(HERE, f"shipped_sphere_box_k{k}.npz"), **out)


def main():
    if "--shipped" in sys.argv:
        shipped_blocks()
        return
    if "--quality-c3" in sys.argv:
        subprocess.run([os.path.join(ROOT, "oracle", "build_ref.sh")], check=True)
        tmp = "/tmp/spt_golden"
        os.makedirs(tmp, exist_ok=True)
        quality_c3(os.path.join(ROOT, "oracle", "_ref"), tmp)
        return
    if "--quality-c2" in sys.argv:
        subprocess.run([os.path.join(ROOT, "oracle", "build_ref.sh")], check=True)
        tmp = "/tmp/spt_golden"
        os.makedirs(tmp, exist_ok=True)
        quality_c3(os.path.join(ROOT, "oracle", "_ref"), tmp, spp=64, seeds=range(301, 317), est="cos",
                   cfg="c2")
        return
    if "--variant-pins" in sys.argv:
        variant_pins()
        return
    if "--fidelity-add" in sys.argv:  # one more estimator in the P2 fixture (e.g. uni)
        est = sys.argv[sys.argv.index("--fidelity-add") + 1]
        subprocess.run([os.path.join(ROOT, "oracle", "build_ref.sh")], check=True)
        tmp = "/tmp/spt_golden"
        os.makedirs(tmp, exist_ok=True)
        fidelity_add(os.path.join(ROOT, "oracle", "_ref"), tmp, est)
        return
    if "--counter-only" in sys.argv:  # contract change: re-pin the oracle's images, keep the rest
        path = os.path.join(HERE, "golden.json")
        out = json.load(open(path))
        counter_pins(out)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out["counter_md5"], indent=1))
        return
    if not os.path.exists("/root/reference/src/smallpt.cpp"):
        sys.exit("reference not present: golden fixtures can only be regenerated in the dev container")
    subprocess.run([os.path.join(ROOT, "oracle", "build_ref.sh")], check=True)
    ref = os.path.join(ROOT, "oracle", "_ref")
    out = {"recipe": "oracle/build_ref.sh: sed patch of smallpt.cpp (:424-442 deleted, srand(seed), "
                     "argv w h spp seed out, :517 skipped; cosine: :464 q<1 -> q<0; uni: :340-347 out, "
                     ":351/:360 comment markers out) | g++ -O3 (x86-64 baseline, g++ 11.4)", "reference_md5": {}}
    tmp = "/tmp/spt_golden"
    os.makedirs(tmp, exist_ok=True)
    for w, h, spp in ((64, 48, 4), (256, 192, 4)):
        for est in ("nee", "cos", "uni"):
            path = os.path.join(tmp, f"ref_{w}x{h}_s{spp}_{est}.ppm")
            subprocess.run([os.path.join(ref, f"smallpt_{est}"), str(w), str(h), str(spp), "1", path],
                           check=True, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            out["reference_md5"][f"{w}x{h}_s{spp}_seed1_{est}"] = md5(path)
            if w == 64:
                with open(path, "rb") as f, open(os.path.join(HERE, os.path.basename(path)), "wb") as g:
                    g.write(f.read())
    # Row-seeded variants (statistics builds): their PPMs pin oracle.compat_render(row_seed=True).
    for est in ("nee", "cos"):
        path = os.path.join(tmp, f"ref_xs_64x48_s4_seed5_{est}.ppm")
        subprocess.run([os.path.join(ref, f"smallpt_{est}_xs"), "64", "48", "4", "5", path],
                       check=True, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        out["reference_md5"][f"xs_64x48_s4_seed5_{est}"] = md5(path)
    fidelity_fixture(ref, tmp)
    # Known answers (measured by calling the reference's own functions).
    out["kat"] = {
        "camera_aspect1": {"llc": [49.362929701805115, 39.362929701805115, 167],
                           "horizontal": [1.2741405963897705, -0.0, 0], "vertical": [0, 1.2741405963897705, 0]},
        "camera_aspect4_3": {"llc": [49.150572896003723, 39.362929701805115, 167],
                             "horizontal": [1.6988542079925537, -0.0, 0], "vertical": [0, 1.2741405963897705, 0]},
        "erand48_row_seeds": {"0": [3.907985046680551e-14, 0.00098539467465030839, 0.041631001594613082],
                              "1": [0.90010070800785158, 0.041650067526212808, 0.81001784241492558],
                              "3385": [0.84089660644535158, 0.65090299721371281, 0.031087178352425582],
                              "2303": [0.93193054199222658, 0.65172697182308781, 0.63652541077430058]},
        "glibc_srand1_first3": [1804289383, 846930886, 1681692777],
        # Random123 kat_vectors, philox4x32 R=10
        "philox4x32_10": [
            {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]},
            {"ctr": [0xffffffff] * 4, "key": [0xffffffff] * 2, "out": [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]},
            {"ctr": [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], "key": [0xa4093822, 0x299f31d0],
             "out": [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]},
        ],
    }
    counter_pins(out)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["reference_md5"], indent=1))


if __name__ == "__main__":
    main()
