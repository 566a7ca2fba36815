#!/usr/bin/env python3
"""Does the next frame's render fill the previous frame's tail? K renders of one config, either on
one stream (each launch starts after the previous one ends) or alternating over two streams and two
render contexts (the next launch's blocks take the CU slots the previous launch's waves free), with
per-frame output buffers. Prints Msamples/s for both. Images are checked equal to a single render.

  python tools/overlap_probe.py [c3|c2] [K]
"""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    spt = importlib.import_module("small-pathtracer_amd")
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    k_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    w, h = 1024, 768
    spp, nee = (512, 1.0) if cfg == "c3" else (64, 0.0)
    prims = spt.cornell_scene()
    cam = spt.Camera(aspect=float(np.float32(w) / np.float32(h)))
    p = spt.default_params(width=w, height=h, spp=spp, nee_prob=nee, tile_rows=8)
    ref = spt.render(prims, cam, p)
    rens = [spt.Renderer(0), spt.Renderer(0)]
    for r in rens:
        r.reserve(len(prims), p)
    outs = [torch.zeros((h, w, 3), dtype=torch.float32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for mode in ("one_stream", "two_streams", "one_stream", "two_streams"):
        for i in range(2):  # warm both contexts
            rens[i].render_async(prims, cam, p, outs[i].data_ptr(), streams[0].cuda_stream)
            rens[i].stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(k_steps):
            s = streams[0] if mode == "one_stream" else streams[k % 2]
            rens[k % 2].render_async(prims, cam, p, outs[k % 2].data_ptr(), s.cuda_stream)
            if k > 0:
                rens[(k - 1) % 2].stats()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rens[(k_steps - 1) % 2].stats()
        ok = all(np.array_equal(o.cpu().numpy(), ref) for o in outs)
        print(f"{cfg} {mode}: {w * h * spp * k_steps / dt / 1e6:.1f} Msamples/s, "
              f"{dt / k_steps * 1e3:.3f} ms/frame, images equal: {ok}", flush=True)
    for r in rens:
        r.close()


if __name__ == "__main__":
    main()
