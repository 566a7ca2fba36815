"""The multi-GPU path on the MI355X, as far as one GPU can drive it:

* spt_render_multi (one process, n devices, RCCL gather) with the box's one device equals the
  1-GPU render bit for bit;
* the de-interleave rank 0 runs after the RCCL transfers, fed with 8 shards rendered on the
  device, rebuilds the 1-GPU image bit for bit (the row mapping of every rank count);
* spt_comm (one process per GPU, the bench's path) with nranks = 1;
* two ranks (processes) on the one GPU, each rendering its shard through the product (C ABI),
  gathered over gloo to rank 0: the same image as one GPU.
"""
import importlib
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _full(spt, w, h, spp, **kw):
    cam = spt.Camera(aspect=float(np.float32(w) / np.float32(h)))
    p = spt.default_params(width=w, height=h, spp=spp, **kw)
    return cam, p, spt.render(spt.cornell_scene(), cam, p)


def test_render_multi_one_device_equals_render(spt):
    cam, p, full = _full(spt, 96, 64, 8)
    img, st = spt.render_multi(spt.cornell_scene(), cam, p, [0], return_stats=True)
    assert np.array_equal(img, full)
    assert st["samples"] == 96 * 64 * 8 and st["kernel_ms"] > 0


def test_render_multi_rejects_duplicate_devices(spt):
    cam, p, _ = _full(spt, 8, 8, 1)
    with pytest.raises(spt.SptError):
        spt.render_multi(spt.cornell_scene(), cam, p, [0, 0])


@pytest.mark.parametrize("n,tile,h", [(8, 8, 768), (3, 4, 50), (5, 8, 20)])
def test_deinterleave_rebuilds_image_from_shards(spt, n, tile, h):
    """rank 0's de-interleave: shard k (its compact rows) -> image rows, for n ranks (incl. ranks
    that own no rows: 5 ranks, 20 rows, tiles of 8)."""
    import torch
    w = 64
    cam, p1, full = _full(spt, w, h, 2, tile_rows=tile)
    shards = []
    for k in range(n):
        p = spt.default_params(width=w, height=h, spp=2, tile_rows=tile, shard_index=k, shard_count=n)
        rows = spt.shard_rows(p)
        t = torch.zeros((max(1, len(rows)), w, 3), dtype=torch.float32, device="cuda")
        if len(rows):
            t[: len(rows)] = torch.from_numpy(spt.render(spt.cornell_scene(), cam, p)).cuda()
        shards.append(t)
    img = torch.full((h, w, 3), -1.0, dtype=torch.float32, device="cuda")
    p = spt.default_params(width=w, height=h, spp=2, tile_rows=tile, shard_count=n)
    spt.deinterleave_rows(p, [s.data_ptr() for s in shards], img.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(img.cpu().numpy(), full)


def test_comm_single_rank_gather(spt):
    """spt_comm_create / spt_gather_framebuffer with nranks = 1: the RCCL communicator of the
    bench's one-process-per-GPU path, the shard de-interleaved into the image."""
    import torch
    w, h = 64, 40
    cam, p, full = _full(spt, w, h, 4)
    comm = spt.Comm(spt.comm_unique_id(), 1, 0, 0)
    try:
        comm.reserve(p)
        ren = spt.Renderer(0)
        shard = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
        img = torch.zeros_like(shard)
        s = torch.cuda.current_stream().cuda_stream
        ren.render_async(spt.cornell_scene(), cam, p, shard.data_ptr(), s)
        comm.gather(p, shard.data_ptr(), img.data_ptr(), s)
        ren.stats()
        torch.cuda.synchronize()
        assert np.array_equal(img.cpu().numpy(), full)
        ren.close()
    finally:
        comm.close()


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_two_ranks_render_product_shards_and_gather(spt, tmp_path):
    """Two processes share the one GPU; each renders its row tiles through the C ABI and rank 0
    gathers them (gloo; on an 8-GPU node the bench uses spt_comm's RCCL gather instead)."""
    w, h, spp = 80, 48, 8
    out = str(tmp_path / "full.npy")
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    worker = os.path.join(ROOT, "tests", "multi_rank_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, str(w), str(h), str(spp), out],
                              env=dict(env, RANK=str(r)), cwd=ROOT) for r in range(2)]
    codes = [pr.wait(timeout=100) for pr in procs]
    assert codes == [0, 0], codes
    _, _, full = _full(spt, w, h, spp)
    assert np.array_equal(np.load(out), full)
