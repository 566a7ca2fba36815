"""The C++ drop-in host program (small-pathtracer_amd/csrc/smallpt_main.cpp over smallpt.hpp):
the reference's main() (/root/reference/src/smallpt.cpp:502-556) with the pixel loop :528-542
replaced by one spt_render() call and the P3 writer :548-551 kept.

CPU: the `main` INTEGRATION.md gives a maintainer compiles and links against smallpt.hpp/libspt.so.
GPU: `smallpt_amd W H SPP SEED OUT` run as a fresh process writes the bytes the oracle's
restatement of the writer produces for the counter-mode render (bit-exact), for the HEAD NEE
estimator, --cos, --p6, --pfm (the linear framebuffer itself) and --devices 1 (spt_render_multi).
"""
import hashlib
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "small-pathtracer_amd", "csrc")
PROG = os.path.join(ROOT, "small-pathtracer_amd", "smallpt_amd")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
HIPCC = "/opt/rocm/bin/hipcc"


def _integration_main():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = text.index("The reference's `main` becomes:")
    m = re.search(r"```cpp\n(.*?)```", text[i:], re.S)
    return m.group(1)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="needs hipcc")
def test_integration_main_compiles_and_links(tmp_path):
    """The INTEGRATION.md patch for the reference's main() builds against the shipped header."""
    src = tmp_path / "main.cpp"
    src.write_text(_integration_main())
    lib_dir = os.path.join(ROOT, "small-pathtracer_amd")
    if not os.path.exists(os.path.join(lib_dir, "libspt.so")):
        import __graft_entry__
        __graft_entry__.build()
    r = subprocess.run([HIPCC, "-O1", "-std=c++17", "-I", CSRC, str(src), "-o", str(tmp_path / "main"),
                        "-L", lib_dir, "-lspt", f"-Wl,-rpath,{lib_dir}"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert os.path.exists(tmp_path / "main")


def _run(tmp_path, *args, name="out.ppm"):
    out = tmp_path / name
    r = subprocess.run([PROG, *[str(a) for a in args[:4]], str(out), *args[4:]],
                       capture_output=True, text=True, timeout=120, cwd=tmp_path)
    assert r.returncode == 0, (r.stdout + r.stderr)[-2000:]
    assert "DURATION" in r.stdout  # the reference's timing print (:554-556)
    return out.read_bytes()


def _pfm_image(data):
    """A PFM file (spt_image.hip: 'PF', w h, -scale, padded header; rows bottom to top) as (h,w,3)."""
    parts = data.split(b"\n", 3)
    assert parts[0] == b"PF"
    w, h = (int(v) for v in parts[1].split())
    assert float(parts[2]) < 0  # little-endian
    raster = np.frombuffer(data[len(data) - w * h * 12:], dtype="<f4").reshape(h, w, 3)
    return np.ascontiguousarray(raster[::-1])


@pytest.fixture(scope="module")
def counter_images():
    from oracle import oracle as o
    o.lib()
    prims = o.scene_cornell()
    out = {}
    for est, q in (("nee", 1.0), ("cos", 0.0)):
        p = o.default_params(width=64, height=48, spp=16, seed=1, nee_prob=q)
        img, _ = o.counter_render(prims, o.camera(64 / 48), p)
        out[est] = img
    return o, out


@pytest.mark.gpu
@pytest.mark.parametrize("est,flags", [("nee", []), ("cos", ["--cos"])])
def test_smallpt_amd_p3_bit_exact(tmp_path, counter_images, est, flags):
    o, imgs = counter_images
    assert hashlib.md5(imgs[est].tobytes()).hexdigest() == GOLD["counter_md5"][est]
    got = _run(tmp_path, 64, 48, 16, 1, *flags)
    assert got == o.encode_image(imgs[est], 0)


@pytest.mark.gpu
def test_smallpt_amd_p6_and_devices(tmp_path, counter_images):
    o, imgs = counter_images
    assert _run(tmp_path, 64, 48, 16, 1, "--p6", name="out.p6") == o.encode_image(imgs["nee"], 1)
    # one process driving a device list (spt_render_multi: ncclCommInitAll + the gather)
    assert _run(tmp_path, 64, 48, 16, 1, "--devices", "1", name="multi.ppm") == o.encode_image(imgs["nee"], 0)


@pytest.mark.gpu
@pytest.mark.parametrize("est,flags", [("nee", []), ("cos", ["--cos"])])
def test_smallpt_amd_pfm_is_the_pinned_framebuffer(tmp_path, counter_images, est, flags):
    o, imgs = counter_images
    data = _run(tmp_path, 64, 48, 16, 1, "--pfm", *flags, name="out.pfm")
    assert data == o.encode_image(imgs[est], 2)
    img = _pfm_image(data)
    assert hashlib.md5(np.ascontiguousarray(img, dtype=np.float32).tobytes()).hexdigest() == \
        GOLD["counter_md5"][est]
