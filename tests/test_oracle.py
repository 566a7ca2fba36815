"""Pin the CPU oracle before trusting it (CPU only).

P0: the fp64 compat restatement reproduces the reference's own PPMs byte for byte
(golden md5s made by running the reference itself, tests/golden/make_golden.py), plus
known-answer tests for each primitive on the path (SURVEY.md §4 test plan items 1-2).
"""
import ctypes
import hashlib
import json
import math
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))
REF_DIR = os.path.join(os.path.dirname(HERE), "oracle", "_ref")


def _md5_of_ppm(oracle, img, tmp_path, name):
    path = str(tmp_path / name)
    oracle.write_ppm(path, img)
    return hashlib.md5(open(path, "rb").read()).hexdigest()


@pytest.mark.parametrize("w,h,est", [(64, 48, "nee"), (64, 48, "cos"), (64, 48, "uni"),
                                     (256, 192, "nee"), (256, 192, "cos"), (256, 192, "uni")])
def test_compat_restatement_matches_reference_md5(oracle, tmp_path, w, h, est):
    """est: nee = HEAD; cos = :464 q<0; uni = HEAD with the uniform hemisphere of :352-359."""
    img = oracle.compat_render(w, h, 4, seed=1, nee=(est != "cos"), uniform=(est == "uni"))
    assert _md5_of_ppm(oracle, img, tmp_path, "c.ppm") == GOLD["reference_md5"][f"{w}x{h}_s4_seed1_{est}"]


@pytest.mark.parametrize("est", ["nee", "cos", "uni"])
def test_reference_ppm_fixture_matches(oracle, tmp_path, est):
    """The committed reference PPM (data) equals the restatement's bytes."""
    img = oracle.compat_render(64, 48, 4, seed=1, nee=(est != "cos"), uniform=(est == "uni"))
    path = str(tmp_path / "c.ppm")
    oracle.write_ppm(path, img)
    assert open(path, "rb").read() == open(os.path.join(HERE, "golden", f"ref_64x48_s4_{est}.ppm"), "rb").read()


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_DIR, "smallpt_nee")),
                    reason="oracle/_ref not built (reference absent)")
@pytest.mark.parametrize("seed,w,h,spp", [(7, 40, 30, 3), (123, 33, 17, 5)])
def test_compat_restatement_matches_reference_binary_other_seeds(oracle, tmp_path, seed, w, h, spp):
    """Beyond the committed md5s: odd sizes and other seeds against the live reference binary."""
    for est in ("nee", "cos", "uni"):
        ref_path = str(tmp_path / f"ref_{est}.ppm")
        subprocess.run([os.path.join(REF_DIR, f"smallpt_{est}"), str(w), str(h), str(spp), str(seed),
                        ref_path], check=True, cwd=str(tmp_path), stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL)
        img = oracle.compat_render(w, h, spp, seed=seed, nee=(est != "cos"), uniform=(est == "uni"))
        assert _md5_of_ppm(oracle, img, tmp_path, "c.ppm") == hashlib.md5(open(ref_path, "rb").read()).hexdigest()


@pytest.mark.parametrize("w,h", [(64, 48), (256, 192)])
@pytest.mark.parametrize("est", ["q05", "sph", "sph16"])
def test_compat_restatement_matches_reference_variants_md5(oracle, spt, tmp_path, w, h, est):
    """P0 for the reference variants built by oracle/build_ref.sh beyond HEAD: NEE-mix Q = 0.5
    (:464 `q < 0.5`), config 5's 32 spheres in the reference's own Sphere class (:223-254, fp64,
    eps 1e-4), and the same with the depth-16 cap."""
    prims = spt.spheres32_scene() if est.startswith("sph") else None
    img = oracle.compat_render(w, h, 4, seed=1, prims=prims, qthr=0.5 if est == "q05" else 1.0,
                               max_depth=16 if est == "sph16" else 0)
    assert _md5_of_ppm(oracle, img, tmp_path, "c.ppm") == GOLD["reference_md5"][f"{w}x{h}_s4_seed1_{est}"]


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_DIR, "smallpt_sph")),
                    reason="oracle/_ref not built (reference absent)")
@pytest.mark.parametrize("est", ["q05", "sph", "sph16"])
def test_compat_variants_match_reference_binary_other_seeds(oracle, spt, tmp_path, est):
    """The same variants against the live reference binaries at an odd size and other seeds, plus
    their row-seeded (_xs) builds (the P2 fixture's runs)."""
    prims = spt.spheres32_scene() if est.startswith("sph") else None
    kw = dict(prims=prims, qthr=0.5 if est == "q05" else 1.0, max_depth=16 if est == "sph16" else 0)
    for seed, xs in ((7, False), (9, True)):
        ref_path = str(tmp_path / "ref.ppm")
        subprocess.run([os.path.join(REF_DIR, f"smallpt_{est}" + ("_xs" if xs else "")), "33", "17",
                        "5", str(seed), ref_path], check=True, cwd=str(tmp_path),
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        img = oracle.compat_render(33, 17, 5, seed=seed, row_seed=xs, **kw)
        assert _md5_of_ppm(oracle, img, tmp_path, "c.ppm") == hashlib.md5(open(ref_path, "rb").read()).hexdigest()


def test_erand48_kat(oracle):
    for xi2, expect in GOLD["kat"]["erand48_row_seeds"].items():
        got = oracle.erand48_seq(int(xi2), 3)
        assert got == expect


def test_row_seed_is_y_cubed_truncated():
    # :530 Xi = {0, 0, y*y*y} truncated to unsigned short; y=41 -> 3385, y=767 -> 2303
    assert (41 ** 3) & 0xFFFF == 3385 and (767 ** 3) & 0xFFFF == 2303


def test_glibc_rand_restatement_matches_libc(oracle):
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 2, 12345, 0):
        libc.srand(seed)
        want = [libc.rand() for _ in range(2000)]
        assert oracle.glibc_rand(seed, 2000) == want
    assert oracle.glibc_rand(1, 3) == GOLD["kat"]["glibc_srand1_first3"]


def test_philox_random123_kat(oracle):
    for kat in GOLD["kat"]["philox4x32_10"]:
        assert oracle.philox(kat["ctr"], kat["key"]) == kat["out"]


def _philox_py(ctr, key, rounds):
    """Philox4x32-R as published (Salmon et al., SC'11, Random123's constants), in Python big-integer
    arithmetic: an implementation independent of the oracle's C (spt_oracle_philox_r)."""
    m0, m1, w0, w1, mask = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85, 0xFFFFFFFF
    x, (k0, k1) = list(ctr), key
    for _ in range(rounds):
        p0, p1 = m0 * x[0], m1 * x[2]
        x = [((p1 >> 32) ^ x[1] ^ k0) & mask, p1 & mask, ((p0 >> 32) ^ x[3] ^ k1) & mask, p0 & mask]
        k0, k1 = (k0 + w0) & mask, (k1 + w1) & mask
    return x


def test_philox7_known_answers(oracle):
    """The contract's generator at its own round count (SPT_PHILOX_ROUNDS = 7, include/spt.h): the
    Python restatement reproduces Random123's 10-round vectors, and the committed 7-round vectors it
    made (golden.json philox4x32_7) equal both it and the oracle's C function."""
    hdr = open(os.path.join(os.path.dirname(HERE), "include", "spt.h")).read()
    assert "#define SPT_PHILOX_ROUNDS 7" in hdr
    for kat in GOLD["kat"]["philox4x32_10"]:
        assert _philox_py(kat["ctr"], kat["key"], 10) == kat["out"]
    for kat in GOLD["kat"]["philox4x32_7"]:
        assert _philox_py(kat["ctr"], kat["key"], 7) == kat["out"]
        assert oracle.philox_r(kat["ctr"], kat["key"], 7) == kat["out"]
    rng = np.random.default_rng(7)
    for _ in range(200):
        ctr = [int(v) for v in rng.integers(0, 1 << 32, 4)]
        key = [int(v) for v in rng.integers(0, 1 << 32, 2)]
        assert oracle.philox_r(ctr, key, 7) == _philox_py(ctr, key, 7)


@pytest.mark.parametrize("aspect,key", [(1.0, "camera_aspect1"), (4 / 3, "camera_aspect4_3")])
def test_camera_kat(oracle, aspect, key):
    c = oracle.camera(aspect)
    k = GOLD["kat"][key]
    assert list(c.lower_left_corner) == k["llc"]
    assert list(c.horizontal) == k["horizontal"]
    assert list(c.vertical) == k["vertical"]


def test_sincos_polynomial_accuracy(oracle):
    xs = np.concatenate([np.arange(0, 1 << 24, 4099) / float(1 << 24), [0.125, 0.25, 0.5, 0.75, 1 - 2 ** -24]])
    err = 0.0
    for xi in xs:
        s, c = oracle.sincos2pi(float(np.float32(xi)))
        err = max(err, abs(s - math.sin(2 * math.pi * xi)), abs(c - math.cos(2 * math.pi * xi)))
    assert err < 3e-7


def test_disk_dir_octant_mapping(oracle):
    """The contract's azimuth (spt_oracle_disk_dir): (cos, sin) of the angle the word's bits name —
    octant by bits 31..29, theta = u * (pi/2) * 2^-22 from bits 28..8 — within 3e-7, unit length,
    and every octant equally often."""
    rng = np.random.default_rng(5)
    words = np.concatenate([rng.integers(0, 1 << 32, 20000, dtype=np.uint64),
                            [0, 0xFFFFFFFF, 0x1FFFFF00, 0x20000000, 0xE0000000]]).astype(np.uint64)
    err = 0.0
    for w in words:
        w = int(w)
        th = ((w >> 8) & 0x1FFFFF) * (math.pi / 2) * 2.0 ** -22
        c, s = math.cos(th), math.sin(th)
        if w & 0x20000000:
            c, s = s, c
        c = -c if w & 0x80000000 else c
        s = -s if w & 0x40000000 else s
        gc, gs = oracle.disk_dir(w)
        err = max(err, abs(gc - c), abs(gs - s), abs(gc * gc + gs * gs - 1.0))
    assert err < 3e-7
    phi = np.array([math.atan2(*oracle.disk_dir(int(w))[::-1]) for w in words[:20000]])
    counts = np.histogram(np.mod(phi, 2 * math.pi), bins=8, range=(0, 2 * math.pi))[0]
    assert counts.min() > 2300 and counts.max() < 2700, counts


def test_rect_intersect_kats(oracle, spt):
    """Ray-rect cases of :102-112 incl. the no-epsilon self-hit and the float in-plane rounding."""
    light = oracle.scene_cornell()[6]  # Rectangle_xz(32,68,63,96,81.5)
    arr = (spt.spt_prim * 1)(light)
    f = lambda o, d: oracle.lib().spt_oracle_prim_intersect(arr, (ctypes.c_double * 3)(*o), (ctypes.c_double * 3)(*d))  # noqa
    assert f((50, 40, 80), (0, 1, 0)) == pytest.approx(41.5)
    assert f((50, 40, 80), (0, -1, 0)) == 0          # behind -> t < 0 -> 0
    assert f((10, 40, 80), (0, 1, 0)) == 0           # outside x range
    assert f((50, 81.5, 80), (0, 1, 0)) == 0         # origin on the plane: t = 0 -> miss
    assert f((32, 40, 63), (0, 1, 0)) == pytest.approx(41.5)  # closed bounds (edge hits)


def test_light_sampling_wraps_like_glibc(oracle):
    """light_sampling :365-366 computes rand()*36 in int: with glibc RAND_MAX=2^31-1 it wraps, so
    x lies in [31,33] (not [32,68]). The compat restatement reproduces it (md5 tests above);
    here the arithmetic itself: (int32)(r*36) / RAND_MAX for r in the glibc stream."""
    r = np.array(oracle.glibc_rand(1, 100000), dtype=np.int64)
    wrapped = ((r * 36) & 0xFFFFFFFF).astype(np.uint32).astype(np.int32)
    x = 32 + wrapped / 2147483647.0
    assert 31.0 <= x.min() < 31.01 and 32.99 < x.max() <= 33.0


def test_counter_mode_pins(oracle):
    """The counter-mode contract (what the GPU must match) is stable: committed images/md5s."""
    prims = oracle.scene_cornell()
    for est, q, fl in (("nee", 1.0, 0), ("cos", 0.0, 0), ("uni", 1.0, 1)):
        p = oracle.default_params(width=64, height=48, spp=16, seed=1, nee_prob=q, flags=fl)
        img, st = oracle.counter_render(prims, oracle.camera(64 / 48), p)
        assert hashlib.md5(img.tobytes()).hexdigest() == GOLD["counter_md5"][est]
        assert st == GOLD["counter_stats"][est]


@pytest.mark.parametrize("est,q", [("nee", 1.0), ("cos", 0.0)])
def test_parallel_pairs_equal_per_rect_tests(oracle, est, q):
    """The contract's parallel-pair rect tests (one plane of a box's opposite faces per ray), its
    room test (the nearest of the three wall pairs, one box check widened by 2^-8: contract v5) and
    its box slabs (contract v6) against testing every rectangle on its own (intersect :323-335 as
    written). The skipped plane of a pair is never the nearest hit outside ulp-level edge grazes;
    the room rule differs only for rays from outside the room (leaked paths) that pass within 2^-8
    of a wall's edge; a box slab differs from its five faces only for rays grazing an edge within
    rounding (0 of 382k random rays and 168k rays from box-face vertices, self-hits included).
    Pinned at 128x96, seed 7 (the measured values, not loose tolerances): NEE 6 of
    12288 pixels differ, 3.9e-7 of the image sum, path rays 6787723 vs 6787725, every other counter
    within 4, misses 346989 vs 346968; cosine-only 1 pixel, 7.4e-7 of the sum, counters within 1,
    misses 362143 vs 362122 (the room rule: rays from outside the room near a wall's edge)."""
    prims = oracle.scene_cornell()
    p = oracle.default_params(width=128, height=96, spp=128 if est == "nee" else 64, seed=7,
                              nee_prob=q)
    oracle.set_leak_end(False)  # (needs the room: compare like with like)
    try:
        a, sa = oracle.counter_render(prims, oracle.camera(128 / 96), p)
        oracle.set_pairs(False)
        b, sb = oracle.counter_render(prims, oracle.camera(128 / 96), p)
    finally:
        oracle.set_pairs(True)
        oracle.set_leak_end(True)
    d = np.abs(a.astype(np.float64) - b)
    max_pixels, max_frac, max_count = (6, 4e-7, 4) if est == "nee" else (1, 8e-7, 1)
    assert (d.max(axis=2) > 0).sum() <= max_pixels
    assert d.sum() <= max_frac * a.sum()
    assert sa["samples"] == sb["samples"]
    for k in ("path_rays", "vertices", "nee_light_hits", "cosine_samples", "shadow_traced",
              "nee_events", "shadow_rays"):
        assert abs(sa[k] - sb[k]) <= max_count, (k, sa[k], sb[k])
    assert abs(sa["misses"] - sb["misses"]) <= 25, (sa["misses"], sb["misses"])


@pytest.mark.parametrize("pairs", [True, False])
def test_early_nee_resolve_proof_holds(oracle, pairs):
    """The HEAD NEE kernel's early shadow-ray resolve (spt_kernel.hip early_nee_proven) claims the
    light is the nearest hit at the light's own t. Every claim is checked against the contract's
    intersect (and with pairs=False against the per-rect tests of :323-335 as written): none is
    contradicted, and the claims cover well over half of the shadow rays that reach the light."""
    prims = oracle.scene_cornell()
    w, h, spp = (256, 192, 48) if pairs else (192, 144, 32)
    p = oracle.default_params(width=w, height=h, spp=spp, seed=11)
    oracle.set_pairs(pairs)
    oracle.proof_check(True)
    try:
        _, st = oracle.counter_render(prims, oracle.camera(w / h), p)
        claims, bad = oracle.proof_counts()
    finally:
        oracle.proof_check(False)
        oracle.set_pairs(True)
    assert bad == 0, (claims, bad)
    assert claims > 0.55 * st["nee_light_hits"], (claims, st["nee_light_hits"])


def test_early_nee_resolve_proof_holds_with_reference_leaks(oracle, spt):
    """SPT_FLAG_REFERENCE_LEAKS: leaked paths wander on from the miss vertex (the origin) and across
    the walls' outer faces as the reference's (:371-377), and those vertices take NEE samples too.
    The HEAD NEE kernel's early resolve must still never claim a shadow ray its intersect would not
    give the light; and the flag is the test hook's set_leak_end(False), bit for bit."""
    prims = oracle.scene_cornell()
    w, h, spp = 192, 144, 32
    p = oracle.default_params(width=w, height=h, spp=spp, seed=13, flags=spt.FLAG_REFERENCE_LEAKS)
    oracle.proof_check(True)
    try:
        img, st = oracle.counter_render(prims, oracle.camera(w / h), p)
        claims, bad = oracle.proof_counts()
    finally:
        oracle.proof_check(False)
    assert bad == 0, (claims, bad)
    assert claims > 0.55 * st["nee_light_hits"], (claims, st["nee_light_hits"])
    p0 = oracle.default_params(width=w, height=h, spp=spp, seed=13)
    oracle.set_leak_end(False)
    try:
        img0, st0 = oracle.counter_render(prims, oracle.camera(w / h), p0)
    finally:
        oracle.set_leak_end(True)
    assert np.array_equal(img, img0) and st == st0
    img1, st1 = oracle.counter_render(prims, oracle.camera(w / h), p0)
    assert st["misses"] > 2 * st1["misses"] and not np.array_equal(img, img1)


def test_early_nee_resolve_proof_holds_spheres(oracle, spt):
    """The sphere NEE kernel's early resolve (early_room_proven: the HEAD room, vertices above
    every sphere's top + 1 = 13 in the C5 scene) against the contract's intersect, depth cap 16."""
    prims = spt.spheres32_scene()
    p = oracle.default_params(width=160, height=120, spp=32, seed=5, max_depth=16)
    oracle.proof_check(True, sphere_y0=13.0)
    try:
        _, st = oracle.counter_render(prims, oracle.camera(160 / 120), p)
        claims, bad = oracle.proof_counts()
    finally:
        oracle.proof_check(False)
    assert bad == 0, (claims, bad)
    assert claims > 0.3 * st["nee_light_hits"], (claims, st["nee_light_hits"])


def test_counter_mode_thread_invariance(oracle):
    prims = oracle.scene_cornell()
    p = oracle.default_params(width=40, height=24, spp=8, seed=3)
    a, sa = oracle.counter_render(prims, oracle.camera(40 / 24), p, threads=1)
    b, sb = oracle.counter_render(prims, oracle.camera(40 / 24), p, threads=4)
    assert np.array_equal(a, b) and sa == sb


def test_fast_plane_distance_equals_the_fma(oracle):
    """The oracle computes the contract's plane distance fma(n, inv, -2^-149) without the fma's
    denormal addend (an x86 assist that made it 10x slower): same bits on exact rounding ties
    (where the fma picks the lower neighbour), zeros, signs, infinities, NaN, tiny and huge
    products, and random operands."""
    f32 = np.float32
    rng = np.random.default_rng(11)
    # exact ties: (1 + 2^-12 m)(1 + 2^-12 m') has its 2^-24 bit as the only bit below the ulp
    m = np.arange(1, 200, dtype=np.float64)
    a = (1 + m * 2.0 ** -12).astype(f32)
    ties_n = np.concatenate([a, -a, a * f32(2 ** 20), a * f32(2 ** -20), -a * f32(3)])
    ties_i = np.concatenate([a, a, a, a, a])
    special = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-30, 1e-38, 3e38, 1e-45],
                       dtype=f32)
    sn, si = np.meshgrid(special, special)
    rn = (rng.standard_normal(200000) * rng.choice([1e-3, 1, 1e3], 200000)).astype(f32)
    ri = (1 / rng.standard_normal(200000)).astype(f32)
    num = np.concatenate([ties_n, sn.ravel(), rn])
    inv = np.concatenate([ties_i, si.ravel(), ri])
    assert oracle.plane_t_mismatches(num, inv) == 0


def test_plane_k_rule(oracle):
    """Contract plane coordinates (spt_oracle_plane_k; kernel spt_cornell.h plane_k): fp32-exact
    values stay; otherwise the neighbouring float with the double's last significand bit."""
    f32 = np.float32
    assert f32(oracle.plane_k(81.6)) == f32(81.600006103515625)  # (float)81.6 = 81.59999847 is odd
    for k in (0.0, 1.0, 99.0, 170.0, 81.5, 12.0, 1e30, -3.25):
        assert f32(oracle.plane_k(k)) == f32(k)
    for k in (81.6, -81.6, 0.1, 1 / 3, 2.2, 1e-3, 33.3, 170.17):
        f = f32(oracle.plane_k(k))
        lo, hi = np.nextafter(f32(k), f32(-np.inf)), np.nextafter(f32(k), f32(np.inf))
        assert f in (f32(k), lo, hi) and abs(float(f) - k) < 2 * abs(float(hi) - float(lo))
        m, _ = math.frexp(k)
        bit64 = int(math.ldexp(abs(m), 53)) & 1
        bit32 = int(math.ldexp(abs(math.frexp(float(f))[0]), 24)) & 1
        assert bit32 == bit64, (k, f)


@pytest.mark.parametrize("est", ["nee", "cos"])
def test_compat_row_seeded_matches_reference_binary(oracle, tmp_path, est):
    """compat_render(row_seed=True) == oracle/_ref/smallpt_{est}_xs (rows seeded {0, seed, y^3})."""
    img = oracle.compat_render(64, 48, 4, seed=5, nee=(est == "nee"), row_seed=True)
    assert _md5_of_ppm(oracle, img, tmp_path, "c.ppm") == GOLD["reference_md5"][f"xs_64x48_s4_seed5_{est}"]


@pytest.mark.parametrize("nee", [True, False])
def test_contract_path_statistics_match_reference(oracle, nee):
    """The fp32 contract leaks out of the room as often as the fp64 reference: paths that left
    through a self-hit (:103-106 has no epsilon) per sample, and vertices per sample up to a
    path's first miss, at 128x96@16, 2 seeds. The contract ends a leaked path at its first miss
    (c_find_leak_end); the reference goes on from the miss vertex, and with the rule off the
    contract's misses and vertices match those of the reference too. Before the plane_k rule the
    contract had +17 % misses (the ceiling at y=81.6 leaked 26x)."""
    w, h, spp = 128, 96, 16
    ref = {"vertices": 0, "misses": 0, "first_misses": 0, "vertices_pre": 0}
    own = {"vertices": 0, "misses": 0}
    full = {"vertices": 0, "misses": 0}
    for seed in (1, 2):
        _, st = oracle.compat_render(w, h, spp, seed=seed, nee=nee, row_seed=True, stats=True)
        ref = {k: ref[k] + st[k] for k in ref}
        p = oracle.default_params(width=w, height=h, spp=spp, seed=seed, nee_prob=1.0 if nee else 0.0)
        # compat's radiance() re-traces the light ray after a NEE hit; the contract carries it
        _, cs = oracle.counter_render(oracle.scene_cornell(), oracle.camera(w / h), p)
        own = {k: own[k] + cs[k] for k in own}
        oracle.set_leak_end(False)
        try:
            _, cs = oracle.counter_render(oracle.scene_cornell(), oracle.camera(w / h), p)
        finally:
            oracle.set_leak_end(True)
        full = {k: full[k] + cs[k] for k in full}
    n = 2 * w * h * spp
    assert abs(own["misses"] / ref["first_misses"] - 1) < 0.03, (own, ref)
    assert abs(own["vertices"] / ref["vertices_pre"] - 1) < 0.01, (own, ref)
    assert abs(full["misses"] / ref["misses"] - 1) < 0.03, (full, ref)
    assert abs(full["vertices"] / ref["vertices"] - 1) < 0.01, (full, ref)
    assert 0.02 < ref["first_misses"] / n < 0.2 and 0.1 < ref["misses"] / n < 1.0


# "sph" (the 32 spheres without a depth cap) is the one estimator left to the GPU P2 test
# (tests/test_gpu_fidelity.py, 16 seeds through the sphere kernels): its uncapped paths make 4 CPU
# seeds cost ~10 CPU-minutes, and sph16 pins the same fp32 sphere test here.
@pytest.mark.parametrize("est", ["nee", "cos", "uni", "q05", "sph16"])
def test_contract_fidelity_vs_reference_runs(oracle, spt, est):
    """P2 for the contract itself (the CPU statement the GPU is bit-exact with): 4 seeds (sph16: 2)
    at 256x192@256 against 16 independent runs of the reference binary (tests/fidelity.py).
    sph16: the 32-sphere scene of config 5 (depth cap 16), whose fp32 sphere test (eps 2e-3) is
    pinned here against the reference's own fp64 Sphere::intersect (eps 1e-4, :229-239)."""
    import fidelity
    fx = fidelity.load_fixture()
    w, h, spp, k = fx["w"], fx["h"], fx["spp"], fx["k"]
    prims = fidelity.scene_of(spt, est)
    own = []
    # sph16 with 2 seeds: its depth-16 sphere paths cost the CPU suite ~2 minutes at 4; the GPU P2
    # test (tests/test_gpu_fidelity.py) runs the same contract with 16 seeds, bit-exact with this one
    for seed in ((1, 2) if est == "sph16" else (1, 2, 3, 4)):
        p = oracle.default_params(width=w, height=h, spp=spp, seed=seed, **fidelity.params_of(est))
        img, _ = oracle.counter_render(prims, oracle.camera(w / h), p)
        own.append(fidelity.blocks(img, k))
    zg, z2 = fidelity.compare(fx[est], own)
    assert np.all(np.abs(zg) < fidelity.GLOBAL_Z_MAX), zg
    assert z2 < fidelity.BLOCK_Z2_MAX, z2


def test_box_rule_finds_standing_boxes_only(oracle, spt):
    """Contract v6 (oracle c_find_boxes): the HEAD scene's two boxes; in a scene with three boxes
    on the floor and one floating, the three; none without pairs. Boxes on vs face by face: the
    same image but for rays grazing an edge (here: none at 48x36 @ 8)."""
    import test_gpu_parity as tg
    p = oracle.default_params(width=48, height=36, spp=8, seed=3)
    assert oracle.scene_boxes(oracle.scene_cornell(), p) == 2
    prims = tg._box_scene(spt, tg.BOXES3)
    assert oracle.scene_boxes(prims, p) == 3
    oracle.set_pairs(False)
    try:
        assert oracle.scene_boxes(prims, p) == 0
    finally:
        oracle.set_pairs(True)
    a, sa = oracle.counter_render(prims, oracle.camera(48 / 36), p)
    oracle.set_boxes(False)
    try:
        b, sb = oracle.counter_render(prims, oracle.camera(48 / 36), p)
    finally:
        oracle.set_boxes(True)
    assert np.array_equal(a, b) and sa == sb


@pytest.mark.parametrize("nee", [1.0, 0.0])
def test_leaked_paths_end_at_their_first_miss(oracle, nee):
    """Contract v6 ends a path at its first miss (c_find_leak_end: the miss vertex lies outside the
    closed room, nothing outside emits). With the rule off the path goes on from the miss vertex as
    the reference's (:373-374): the image then differs only by the light that a leaked path
    collects after rounding back into the room through a wall's outer face -- a few pixels by one
    sample each, under 1e-4 of the image mean (measured 8e-6 at 256x192 @ 64); cosine-only: none
    -- while the leaked paths' vertices (4 %) are not executed."""
    prims = oracle.scene_cornell()
    p = oracle.default_params(width=160, height=120, spp=32, seed=9, nee_prob=nee)
    a, sa = oracle.counter_render(prims, oracle.camera(160 / 120), p)
    oracle.set_leak_end(False)
    try:
        b, sb = oracle.counter_render(prims, oracle.camera(160 / 120), p)
    finally:
        oracle.set_leak_end(True)
    d = a.astype(np.float64) - b
    assert (np.abs(d).max(axis=2) > 0).sum() <= 0.01 * a.shape[0] * a.shape[1]
    assert abs(d.mean()) < 1e-4 * b.mean() and d.max() <= 1e-12  # dropped light only, never added
    if nee == 0.0:
        assert np.array_equal(a, b)
    assert sa["misses"] < sb["misses"] and sa["vertices"] < 0.98 * sb["vertices"]
    assert sa["samples"] == sb["samples"]


def _move_boxes(spt, short=(0.0, 0.0), tall=(0.0, 0.0)):
    """rect[] with the short box (prims 12-16) and the tall box (7-11) moved by (dx, dz)."""
    prims = [spt.spt_prim.from_buffer_copy(p) for p in spt.cornell_scene()]
    for base, (dx, dz) in ((12, short), (7, tall)):
        for i in (base, base + 1):       # XY faces: x bounds geom[0:2], plane z = geom[4]
            prims[i].geom[0] += dx; prims[i].geom[1] += dx; prims[i].geom[4] += dz
        for i in (base + 2, base + 3):   # YZ faces: z bounds geom[2:4], plane x = geom[4]
            prims[i].geom[2] += dz; prims[i].geom[3] += dz; prims[i].geom[4] += dx
        t = prims[base + 4]              # XZ top: x bounds geom[0:2], z bounds geom[2:4]
        t.geom[0] += dx; t.geom[1] += dx; t.geom[2] += dz; t.geom[3] += dz
    return prims


EDITS = [dict(short=(1.0, 0.0)), dict(short=(-20.0, 0.0)), dict(short=(-35.0, 0.0)),
         dict(short=(0.0, 30.0), tall=(40.0, -10.0)), dict(tall=(-5.0, 60.0))]


@pytest.mark.parametrize("edit", range(len(EDITS)))
def test_early_nee_resolve_proof_holds_edited_geometry(oracle, spt, edit):
    """The uploaded-geometry HEAD-topology NEE kernel's early resolve (early_geo_proven, clauses by
    c_find_early_clauses from each box's position relative to the reference's wrapped light
    samples) against the contract's intersect on edited rect[]s -- boxes moved so that every
    clause (x <= x0, x >= x1, z <= z0, z >= z1, top only) occurs: no claim contradicted."""
    prims = _move_boxes(spt, **EDITS[edit])
    p = oracle.default_params(width=128, height=96, spp=32, seed=7)
    assert oracle.scene_boxes(prims, p) == 2
    oracle.proof_check(True, edited=True)
    try:
        _, st = oracle.counter_render(prims, oracle.camera(128 / 96), p)
        claims, bad = oracle.proof_counts()
    finally:
        oracle.proof_check(False)
    assert bad == 0, (claims, bad)
    assert claims > 0.3 * st["nee_light_hits"], (claims, st["nee_light_hits"])


def _tall_box_height(spt, prims, hgt):
    """rect[] with the tall box (prims 7-11) raised to height hgt."""
    out = [spt.spt_prim.from_buffer_copy(p) for p in prims]
    for i in (7, 8):   # XY faces: y bounds geom[2:4]
        out[i].geom[3] = hgt
    for i in (9, 10):  # YZ faces: y bounds geom[0:2]
        out[i].geom[1] = hgt
    out[11].geom[4] = hgt
    return out


# Round 6: edits of the light and the room (early_geo_setup / c_find_early_clauses). on = whether
# the scene meets the clause conditions (a light plane 0.02 under the ceiling, a box top 0.3 under
# the light plane, a light 0.5 from a wall: no clause, nothing resolved early, still exact).
EDITS_LR = [
    (dict(light=dict(x=(30, 66), z=(65, 99))), True),
    (dict(light=dict(x=(28, 72), z=(60, 100), y=80.0, e=15)), True),
    (dict(room=dict(depth=150.0, width=(2.0, 98.0))), True),
    (dict(room=dict(height=90.0), light=dict(y=81.0)), True),
    (dict(room=dict(depth=160.0), light=dict(x=(30, 70), y=81.0), short=(-20.0, 0.0)), True),
    (dict(light=dict(y=81.58)), False),
    (dict(tall=81.2), False),
    (dict(tall=80.9), True),
    (dict(light=dict(x=(1.5, 40))), False),
]


def edited_scene(spt, light=None, room=None, short=(0.0, 0.0), tall=None):
    prims = _move_boxes(spt, short=short)
    if tall is not None:
        prims = _tall_box_height(spt, prims, tall)
    if room is not None:
        prims = spt.edit_room(prims, **room)
    if light is not None:
        prims = spt.edit_light(prims, **light)
    return prims


@pytest.mark.parametrize("edit", range(len(EDITS_LR)))
def test_early_nee_resolve_proof_holds_edited_light_and_room(oracle, spt, edit):
    """The early resolve of an edited rect[] whose light or room moved as well (round 6): the room
    clause from the room's own box and the light plane, the box clauses as before. No claim is
    contradicted by the contract's intersect, and a scene outside the margins gets no claim."""
    kw, on = EDITS_LR[edit]
    prims = edited_scene(spt, **kw)
    p = oracle.default_params(width=128, height=96, spp=24, seed=17 + edit)
    assert oracle.scene_boxes(prims, p) == 2
    oracle.proof_check(True, edited=True)
    try:
        _, st = oracle.counter_render(prims, oracle.camera(128 / 96), p)
        claims, bad = oracle.proof_counts()
    finally:
        oracle.proof_check(False)
    assert bad == 0, (claims, bad)
    if on:
        assert claims > 0.3 * st["nee_light_hits"], (claims, st["nee_light_hits"])
    else:
        assert claims == 0 and st["nee_light_hits"] > 0, (claims, st["nee_light_hits"])


def test_shadow_census_accounts_for_every_traced_shadow_ray(oracle):
    """The slot model's census (tools/shadow_census.py): every light-accepted shadow
    ray the HEAD early resolve does not prove is counted once, as reached or blocked, and the
    sub-classes never exceed their class."""
    w, h, spp = 64, 48, 16
    p = oracle.default_params(width=w, height=h, spp=spp, seed=23)
    oracle.shadow_census()  # reset
    oracle.proof_check(True)
    try:
        _, st = oracle.counter_render(oracle.scene_cornell(), oracle.camera(w / h), p)
        claims, bad = oracle.proof_counts()
    finally:
        oracle.proof_check(False)
    c = oracle.shadow_census()
    assert bad == 0
    assert c[0] + c[1] == st["shadow_traced"] - claims, (c[:2], st["shadow_traced"], claims)
    assert c[0] == st["nee_light_hits"] - claims  # every traced ray that reached the light
    assert c[3] + c[4] <= c[1] and c[5] <= c[3]  # blocked: vertex outside the room; self-hits
    # reached: by failing box clause; a vertex outside the room never reaches the light (its own
    # wall's slab candidate is the entry at a tiny t)
    assert c[6] + c[7] + c[8] <= c[0] and c[2] == 0
