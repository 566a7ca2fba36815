"""Multi-rank path on CPU (gloo, world_size 2 and 3): row-tile sharding + the single gather to
rank 0 reassemble the exact single-process image. The shards are rendered by the CPU oracle's
counter-mode contract (which the GPU matches bit for bit), so this checks the distributed
plumbing bench.py uses with RCCL, without a GPU."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, w, h, spp, tile, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spt = importlib.import_module("small-pathtracer_amd")
        sd = importlib.import_module("small-pathtracer_amd.distributed")
        from oracle import oracle
        rows_of = sd.shard_row_lists(h, tile, world)
        p = oracle.default_params(width=w, height=h, spp=spp, seed=5, tile_rows=tile,
                                  shard_index=rank, shard_count=world)
        # the library's row rule and the python one agree
        assert np.array_equal(spt.shard_rows(p), rows_of[rank])
        img, _ = oracle.counter_render(oracle.scene_cornell(), oracle.camera(w / h), p,
                                       rows=rows_of[rank].astype(np.int32), threads=1)
        shard = torch.zeros((sd.max_rows(rows_of), w, 3), dtype=torch.float32)
        shard[: len(rows_of[rank])] = torch.from_numpy(img)
        full = torch.zeros((h, w, 3), dtype=torch.float32) if rank == 0 else None
        res = sd.gather_rows(shard, rows_of, full)
        if rank == 0:
            np.save(out_path, res.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,h,tile", [(2, 20, 4), (3, 17, 2)])
def test_row_tile_gather_reassembles_image(tmp_path, oracle, world, h, tile):
    w, spp = 24, 4
    out = str(tmp_path / "full.npy")
    mp.start_processes(_worker, args=(world, _free_port(), w, h, spp, tile, out), nprocs=world,
                       join=True, start_method="spawn")
    full = np.load(out)
    p = oracle.default_params(width=w, height=h, spp=spp, seed=5)
    ref, _ = oracle.counter_render(oracle.scene_cornell(), oracle.camera(w / h), p, threads=1)
    assert np.array_equal(full, ref)


def test_shard_row_lists_partition():
    sd = importlib.import_module("small-pathtracer_amd.distributed")
    for h, t, n in [(768, 8, 8), (100, 8, 3), (5, 8, 4)]:
        rows = sd.shard_row_lists(h, t, n)
        assert sorted(np.concatenate(rows).tolist()) == list(range(h))


def test_shard_zero_is_the_largest_shard(spt):
    """spt_multi.hip sizes rank 0's receive slots (and bench.py its padded shard buffers) by shard 0:
    with cyclic tiles (tile t -> rank t mod n) shard 0 never owns fewer rows than any other shard,
    ragged last tiles and ranks without rows included (checked through the C ABI spt_shard_rows)."""
    sd = importlib.import_module("small-pathtracer_amd.distributed")
    cases = 0
    for h in list(range(1, 70)) + [767, 768, 769, 1000, 4095, 4096, 4097]:
        for t in (1, 2, 3, 7, 8, 16):
            for n in (1, 2, 3, 5, 7, 8, 16):
                counts = []
                for k in range(n):
                    p = spt.default_params(width=3, height=h, spp=1, tile_rows=t, shard_index=k,
                                           shard_count=n)
                    counts.append(len(spt.shard_rows(p)))
                assert counts[0] == max(counts), (h, t, n, counts)
                assert sum(counts) == h
                assert sd.max_rows(sd.shard_row_lists(h, t, n)) == counts[0]
                cases += 1
    assert cases > 3000


def test_gather_plan_reassembles_image(spt):
    """The transfers spt_gather_framebuffer posts (spt_gather_plan: what spt_multi.hip executes
    inside its ncclGroupStart/End) and the de-interleave's row map (spt_deinterleave_source: the
    kernel's own row_source), simulated on the host for every (h, tile, n <= 8): every send has a
    matching receive of the same size, the receives land in disjoint slots inside rank 0's staging
    buffer, and de-interleaving from shard 0 and the staging buffer rebuilds every image row."""
    w = 3
    cases = 0
    for h in list(range(1, 41)) + [95, 96, 97, 767, 768, 769]:
        for t in (1, 2, 3, 7, 8, 16):
            for n in range(1, 9):
                ps = [spt.default_params(width=w, height=h, spp=1, tile_rows=t, shard_index=k,
                                         shard_count=n) for k in range(n)]
                rows = [spt.shard_rows(p) for p in ps]
                # shard k's compact buffer: row r's 3*w floats all hold r
                shards = [np.repeat(r.astype(np.float64), 3 * w) for r in rows]
                staging = np.full(spt.gather_staging_floats(ps[0], n), -1.0)
                sends = {}
                for k in range(1, n):
                    plan = spt.gather_plan(ps[k], n, k)
                    assert all(op[0] == spt.GATHER_SEND and op[1] == 0 and op[3] == 0 for op in plan)
                    assert [op[2] for op in plan] == ([len(rows[k]) * 3 * w] if len(rows[k]) else [])
                    if plan:
                        sends[k] = plan[0][2]
                recvs = spt.gather_plan(ps[0], n, 0)
                assert {op[1]: op[2] for op in recvs} == sends
                src = {0: (shards[0], 0)}
                used = np.zeros(len(staging), dtype=bool)
                for kind, peer, count, off in recvs:
                    assert kind == spt.GATHER_RECV and off + count <= len(staging)
                    assert not used[off:off + count].any()
                    used[off:off + count] = True
                    staging[off:off + count] = shards[peer]  # the transfer
                    src[peer] = (staging, off)
                for r in range(h):
                    k, j = spt.deinterleave_source(ps[0], n, r)
                    buf, off = src[k]
                    seg = buf[off + j * 3 * w: off + (j + 1) * 3 * w]
                    assert len(seg) == 3 * w and (seg == r).all(), (h, t, n, r, k, j)
                cases += 1
    assert cases > 2000
