"""One rank of tests/test_gpu_multi.py::test_two_ranks_render_product_shards_and_gather:
renders its row tiles on cuda:0 through the product (C ABI), gathers to rank 0 over gloo.
Usage (env RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT): multi_rank_worker.py W H SPP OUT.npy"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    w, h, spp, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    try:
        spt = importlib.import_module("small-pathtracer_amd")
        sd = importlib.import_module("small-pathtracer_amd.distributed")
        rows_of = sd.shard_row_lists(h, 8, world)
        p = spt.default_params(width=w, height=h, spp=spp, tile_rows=8, shard_index=rank,
                               shard_count=world)
        assert np.array_equal(spt.shard_rows(p), rows_of[rank])
        cam = spt.Camera(aspect=float(np.float32(w) / np.float32(h)))
        img = spt.render(spt.cornell_scene(), cam, p)
        shard = torch.zeros((sd.max_rows(rows_of), w, 3), dtype=torch.float32)
        shard[: len(rows_of[rank])] = torch.from_numpy(img)
        full = torch.zeros((h, w, 3), dtype=torch.float32) if rank == 0 else None
        res = sd.gather_rows(shard, rows_of, full)
        if rank == 0:
            np.save(out, res.numpy())
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
