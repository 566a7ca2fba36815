#!/usr/bin/env python3
"""Render the finalize pass's two extreme shapes a few times each, for rocprofv3 --kernel-trace
--stats (the finalize kernels' durations): C3 on one GPU (786 K pixels, 11 chunks per pixel) and
one rank's shard of the 8-GPU weak-scaled C3 (shard 0 of 8: 98 K pixels at 8 x 512 spp, ~84
chunks per pixel). SPT_LIB selects the library build.

  rocprofv3 --kernel-trace --stats -d gpurun_out/fin -o fin -- python3 tools/finalize_probe.py
"""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    spt = importlib.import_module("small-pathtracer_amd")
    prims = spt.cornell_scene()
    cam = spt.Camera(aspect=float(np.float32(1024) / np.float32(768)))
    for name, kw in (("c3", dict(spp=512)), ("c3_shard0of8_weak", dict(spp=4096, shard_index=0, shard_count=8))):
        p = spt.default_params(width=1024, height=768, tile_rows=8, **kw)
        for _ in range(3):
            img = spt.render(prims, cam, p)
        print(name, img.shape, float(img.mean()), flush=True)


if __name__ == "__main__":
    main()
