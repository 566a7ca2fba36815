"""The C ABI library loads, exports every symbol include/spt.h declares, and its host helpers match
the reference's host API (restated independently by the oracle). No GPU compute here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "spt.h")).read()
    return sorted(set(re.findall(r"\b(spt_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol(spt):
    declared = _declared_symbols()
    assert sorted(spt.EXPORTS) == declared
    out = subprocess.run(["nm", "-D", "--defined-only", spt.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (spt_\w+)", out))
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    lib = spt.load_library()
    for s in declared:
        assert getattr(lib, s) is not None


def test_abi_version_and_status_strings(spt):
    lib = spt.load_library()
    assert lib.spt_abi_version() == 5
    assert len(lib.spt_build_sources_sha16()) == 16
    for code, text in spt.STATUS.items():
        assert lib.spt_status_string(code).decode() == text


def test_library_is_gfx950_code_object(spt):
    """The HIP fat binary of libspt.so holds gfx950 code objects and no other target (offload
    bundle entry ids `hipv4-amdgcn-amd-amdhsa--<arch>`; no tool needed, runs on the CPU)."""
    import re
    data = open(spt.LIB_PATH, "rb").read()
    archs = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert archs == {b"gfx950"}, archs


def test_scene_builder_matches_reference_scene(spt, oracle):
    mine = spt.cornell_scene()
    ref = oracle.scene_cornell()
    assert len(mine) == len(ref) == 17
    for a, b in zip(mine, ref):
        assert bytes(a) == bytes(b)


def test_python_ctor_mirror_matches(spt, oracle):
    ref = oracle.scene_cornell()
    assert bytes(spt.Rectangle_xy(1, 99, 0, 81.6, 0, spt.Vec(), spt.Vec(.75, .75, .75), spt.DIFF)) == bytes(ref[0])
    assert bytes(spt.Rectangle_xz(32, 68, 63, 96, 81.5, spt.Vec(12, 12, 12), spt.Vec(), spt.DIFF)) == bytes(ref[6])
    assert bytes(spt.Rectangle_yz(0, 25, 63, 88, 88, spt.Vec(), spt.Vec(1, 1, 1), spt.DIFF)) == bytes(ref[15])


@pytest.mark.parametrize("w,h", [(512, 512), (256, 192), (1024, 768), (4096, 4096), (37, 11)])
def test_camera_init_matches_reference_ctor(spt, oracle, w, h):
    mine = spt.Camera(aspect=float(np.float32(w) / np.float32(h)))
    ref = oracle.camera(float(np.float32(w) / np.float32(h)))
    assert bytes(mine._c) == bytes(ref)


def test_default_params_match_oracle(spt, oracle):
    assert bytes(spt.default_params()) == bytes(oracle.default_params())


@pytest.mark.parametrize("h,T,n", [(768, 8, 8), (768, 8, 1), (100, 8, 3), (7, 8, 2), (4096, 16, 8), (1, 8, 4)])
def test_shard_rows_partition_the_image(spt, h, T, n):
    seen = []
    for k in range(n):
        rows = spt.shard_rows(spt.default_params(height=h, tile_rows=T, shard_index=k, shard_count=n))
        assert np.all(np.diff(rows) > 0)
        assert all(((r // T) % n) == k for r in rows)
        seen.extend(rows.tolist())
    assert sorted(seen) == list(range(h))


def test_invalid_arguments_fail_loudly(spt):
    cam = spt.Camera(aspect=1.0)
    with pytest.raises(spt.SptError) as e:
        spt.render(spt.cornell_scene(), cam, spt.default_params(width=0))
    assert e.value.status == 1
    bad = spt.cornell_scene()
    bad[3].refl = 7  # not a Refl_t (:72-74)
    with pytest.raises(spt.SptError) as e:
        spt.render(bad, cam, spt.default_params(width=8, height=8, spp=1))
    assert e.value.status == 1
    with pytest.raises(spt.SptError) as e:
        spt.render(spt.cornell_scene(), cam, spt.default_params(width=8, height=8, spp=1, flags=8))
    assert e.value.status == 1


@pytest.mark.parametrize("rad", [0.0, -6.0, float("inf"), float("nan")])
def test_sphere_radius_must_be_positive(spt, rad):
    """Sphere::normal (:248) is (x - p).norm(); the contract's (x - p) * (1/r) equals it only for
    r > 0 (a negative radius would flip the geometric normal of the REFR test :485)."""
    cam = spt.Camera(aspect=1.0)
    scene = spt.spheres32_scene()
    scene[9].geom[0] = rad
    with pytest.raises(spt.SptError) as e:
        spt.render(scene, cam, spt.default_params(width=8, height=8, spp=1))
    assert e.value.status == 1 and "radius" in spt.load_library().spt_last_error().decode()


def test_nee_needs_an_emitting_light(spt):
    """NEE (nee_prob > 0) weights shadow rays reaching prims[light_id] as light hits: a light id
    that is absent or does not emit is rejected (the classic box's HEAD id 6 is a ball there)."""
    cam = spt.Camera(aspect=1.0)
    classic = spt.smallpt_classic_scene()
    for kw in (dict(), dict(light_id=40), dict(light_id=-1)):
        with pytest.raises(spt.SptError) as e:
            spt.render(classic, cam, spt.default_params(width=8, height=8, spp=1, **kw))
        assert e.value.status == 1 and "light" in spt.load_library().spt_last_error().decode()


def test_kernel_level_flag_is_validated(spt):
    cam = spt.Camera(aspect=1.0)
    with pytest.raises(spt.SptError) as e:  # bits 8-9 hold the level, bit 10 is not a flag
        spt.render(spt.cornell_scene(), cam, spt.default_params(width=8, height=8, spp=1,
                                                                flags=1 << 10))
    assert e.value.status == 1
    assert spt.kernel_flag("generic") == 1 << 8 and spt.kernel_flag("head") == 0


def test_classic_scenes_differ_only_in_ball_materials(spt):
    a, b = spt.smallpt_classic_scene(), spt.smallpt_mirror_glass_scene()
    assert len(a) == len(b) == 9
    assert [p.refl for p in a] == [0] * 9 and [p.refl for p in b] == [0] * 6 + [1, 2, 0]
    for p, q in zip(a, b):
        p.refl = q.refl = 0
        assert bytes(p) == bytes(q)
    assert a[8].e[0] == 12 and a[6].c[0] == .999


def test_no_device_is_an_error_not_a_fallback(spt):
    """Without a GPU (this container) rendering must fail with NO_DEVICE, never compute on CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(spt.SptError) as e:
        spt.render(spt.cornell_scene(), spt.Camera(aspect=1.0), spt.default_params(width=8, height=8, spp=1))
    assert e.value.status in (2, 3)


def test_oracle_p3_writer_byte_identical_to_reference_file(oracle):
    """The writer checker (oracle encode_image, P3) reproduces the reference's own PPM bytes."""
    img = oracle.compat_render(64, 48, 4, seed=1, nee=True)
    ref = open(os.path.join(ROOT, "tests", "golden", "ref_64x48_s4_nee.ppm"), "rb").read()
    assert oracle.encode_image(img, 0) == ref


def test_oracle_p6_pfm_layout(oracle):
    import struct
    rgb = np.random.default_rng(3).random((5, 7, 3), dtype=np.float32)
    p3 = oracle.encode_image(rgb, 0)
    p6 = oracle.encode_image(rgb, 1)
    vals = [int(v) for v in p3.split(b"\n", 3)[3].split()]
    hd6 = p6[: p6.index(b"255\n") + 4]  # "P6\n7 5<spaces>\n255\n", padded to 16 bytes
    assert hd6.split() == [b"P6", b"7", b"5", b"255"] and len(hd6) % 16 == 0
    assert list(p6[len(hd6):]) == vals
    pfm = oracle.encode_image(rgb, 2)
    hd = pfm[: pfm.index(b"\n", pfm.index(b"\n", 3) + 1) + 1]
    assert hd.startswith(b"PF\n7 5\n-1.0") and len(hd) % 16 == 0 and float(hd.split()[3]) == -1.0
    data = np.frombuffer(pfm[len(hd):], dtype="<f4").reshape(5, 7, 3)
    assert np.array_equal(data[::-1], rgb) and struct.calcsize("<f") == 4


def test_writers_need_the_gpu(spt, tmp_path):
    """No CPU fallback for the writers either: without a device they fail loudly."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(spt.SptError):
        spt.write_ppm(str(tmp_path / "x.ppm"), np.zeros((2, 2, 3), np.float32))
