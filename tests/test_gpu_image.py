"""GPU image encoder (spt_image.hip) against the oracle's C restatement of the reference writer
(/root/reference/src/smallpt.cpp:313-321 toInt/clamp, :548-551 the P3 fprintf loop).

Bar: byte-identical files. P3 is also checked against the reference's own PPM (tests/golden).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FMTS = [("p3", 0), ("p6", 1), ("pfm", 2)]


def _gpu_bytes(spt, rgb, fmt):
    import torch
    h, w, _ = rgb.shape
    src = torch.from_numpy(np.ascontiguousarray(rgb, dtype=np.float32)).cuda()
    cap = spt.Encoder.bound(w, h, fmt)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    enc = spt.Encoder(0)
    try:
        n = enc.encode(src.data_ptr(), w, h, fmt, out.data_ptr(), cap)
        torch.cuda.synchronize()
    finally:
        enc.close()
    return bytes(out[:n].cpu().numpy())


def _edge_values():
    f = np.float32
    thr = []
    # every toInt step of the reference formula, +-3 ulps around it (toInt is monotone)
    x = np.arange(0, 2 ** 30, 2 ** 14, dtype=np.uint32).view(np.float32)  # dense sweep of [0, 2)
    v = np.floor(np.power(np.clip(x.astype(np.float64), 0, 1), 1 / 2.2) * 255 + 0.5)
    steps = x[1:][np.diff(v) != 0]
    for s in steps:
        b = np.array([s], dtype=np.float32).view(np.uint32)[0]
        lo = max(0, int(b) - 2 ** 14)
        thr.append(np.arange(lo, int(b) + 4, dtype=np.uint32).view(np.float32))
    special = np.array([0.0, -0.0, -1.0, 1.0, 1.0000001, 2.0, 1e-45, 1e-38, np.inf, -np.inf,
                        np.nan, 0.5, 0.999999], dtype=f)
    return np.concatenate(thr + [special])


@pytest.mark.parametrize("name,fmt", FMTS)
def test_encoder_matches_oracle_on_edge_values(spt, oracle, name, fmt):
    vals = _edge_values()
    n = (len(vals) + 2) // 3 * 3
    vals = np.concatenate([vals, np.zeros(n - len(vals), np.float32)])
    w = 777  # odd width, many encoder blocks with unaligned byte ranges
    h = (n // 3 + w - 1) // w
    rgb = np.zeros((h * w * 3,), np.float32)
    rgb[: len(vals)] = vals
    rgb = rgb.reshape(h, w, 3)
    assert _gpu_bytes(spt, rgb, name) == oracle.encode_image(rgb, fmt)


@pytest.mark.parametrize("w,h", [(1, 1), (3, 1), (1, 5), (1023, 3), (1024, 768)])
@pytest.mark.parametrize("name,fmt", FMTS)
def test_encoder_matches_oracle_sizes(spt, oracle, name, fmt, w, h):
    rgb = np.random.default_rng(w * 31 + h).random((h, w, 3), dtype=np.float32) * 1.2 - 0.1
    assert _gpu_bytes(spt, rgb, name) == oracle.encode_image(rgb, fmt)


def test_write_ppm_reproduces_reference_file(spt, oracle, tmp_path):
    """spt.write_ppm on the reference's own image == the reference's PPM (64x48@4, NEE)."""
    img = oracle.compat_render(64, 48, 4, seed=1, nee=True).astype(np.float32)
    ref = open(os.path.join(HERE, "golden", "ref_64x48_s4_nee.ppm"), "rb").read()
    assert oracle.encode_image(img, 0) == ref  # float32 framebuffer prints the same bytes here
    path = str(tmp_path / "out.ppm")
    spt.write_ppm(path, img)
    assert open(path, "rb").read() == ref


def test_rendered_image_all_formats(spt, oracle, tmp_path):
    p = spt.default_params(width=64, height=48, spp=16, seed=1)
    img = spt.render(spt.cornell_scene(), spt.Camera(aspect=64 / 48), p)
    for name, fmt in FMTS:
        path = str(tmp_path / f"r.{name}")
        spt.write_image(path, img, name)
        assert open(path, "rb").read() == oracle.encode_image(img, fmt)


def test_encode_into_too_small_buffer_fails(spt):
    import torch
    rgb = torch.zeros((4, 4, 3), dtype=torch.float32, device="cuda")
    out = torch.empty(8, dtype=torch.uint8, device="cuda")
    enc = spt.Encoder(0)
    try:
        with pytest.raises(spt.SptError):
            enc.encode(rgb.data_ptr(), 4, 4, "p3", out.data_ptr(), 8)
    finally:
        enc.close()


def test_encoder_reuse_across_nan_and_clean_images(spt, oracle):
    """P3 in passes: a NaN anywhere sends the whole encode down the exact slow path (the encode's
    epoch in the NaN word); the next encode with the same Encoder, without a NaN, takes the fast
    path again. Every output byte-identical to the oracle's writer."""
    import torch
    h, w = 200, 311  # 186,600 values: 23 text blocks, the last one partial
    rng = np.random.default_rng(7)
    clean = rng.random((h, w, 3), dtype=np.float32) * 1.2 - 0.1
    mid_nan = clean.copy()
    mid_nan[97, 150, 1] = np.nan
    last_nan = clean.copy()
    last_nan[-1, -1, -1] = np.nan
    enc = spt.Encoder(0)
    try:
        for img in (clean, mid_nan, clean, last_nan, clean):
            src = torch.from_numpy(np.ascontiguousarray(img)).cuda()
            cap = spt.Encoder.bound(w, h, "p3")
            out = torch.empty(cap, dtype=torch.uint8, device="cuda")
            n = enc.encode(src.data_ptr(), w, h, "p3", out.data_ptr(), cap)
            torch.cuda.synchronize()
            assert bytes(out[:n].cpu().numpy()) == oracle.encode_image(img, 0)
    finally:
        enc.close()


@pytest.mark.parametrize("name,fmt", FMTS)
def test_unaligned_framebuffer_rejected_before_any_work(spt, oracle, name, fmt):
    """A framebuffer that is not 16-byte aligned is refused (SPT_ERR_INVALID_ARG) before anything is
    queued: the output buffer keeps its bytes, and the same Encoder then encodes correctly."""
    import torch
    h, w = 4, 5
    rgb = np.random.default_rng(3).random((h, w, 3), dtype=np.float32)
    buf = torch.zeros(h * w * 3 + 4, dtype=torch.float32, device="cuda")
    buf[1:1 + h * w * 3].copy_(torch.from_numpy(rgb.reshape(-1)))
    cap = spt.Encoder.bound(w, h, name)
    out = torch.full((cap,), 0xAB, dtype=torch.uint8, device="cuda")
    enc = spt.Encoder(0)
    try:
        with pytest.raises(spt.SptError, match="aligned"):
            enc.encode(buf.data_ptr() + 4, w, h, name, out.data_ptr(), cap)
        torch.cuda.synchronize()
        assert bool((out == 0xAB).all())
        src = torch.from_numpy(np.ascontiguousarray(rgb)).cuda()
        n = enc.encode(src.data_ptr(), w, h, name, out.data_ptr(), cap)
        torch.cuda.synchronize()
        assert bytes(out[:n].cpu().numpy()) == oracle.encode_image(rgb, fmt)
    finally:
        enc.close()
