#!/usr/bin/env python3
"""Per-wave dump of one render with a -DSPT_DIAG=2 library (spt_diag.h: SPT_WAVE_TIMES): renders the
config twice through one Renderer (the second launch's dump is kept: SPT_WAVE_DUMP is rewritten by
every spt_context_stats) and prints the residency summary of tools/wave_tail.py plus the waves' work
by age: a wave's age rank is its start order among the waves of its CU (0 = the first block the CU
received), compared with blockIdx / n_cu.

  SPT_LIB=build/ab/diag2.so python tools/wave_dump.py c3 gpurun_out/waves_c3.bin
"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    cfg, path = sys.argv[1], sys.argv[2]
    os.environ["SPT_WAVE_DUMP"] = path
    import torch

    spt = importlib.import_module("small-pathtracer_amd")
    bench = importlib.import_module("bench")
    c = bench.CONFIGS[cfg]
    w, h = c["width"], c["height"]
    p = spt.default_params(width=w, height=h, spp=c["spp"], nee_prob=c["nee_prob"],
                           max_depth=c["max_depth"])
    cam = spt.Camera(aspect=float(np.float32(w) / np.float32(h)))
    prims = spt.cornell_scene() if c["scene"] == "cornell" else spt.spheres32_scene()
    r = spt.Renderer(0)
    out = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
    for _ in range(2):
        r.render_async(prims, cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        st = r.stats()
    r.close()
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 3)
    wid = np.nonzero(a[:, 1] > 0)[0]
    a = a[wid]
    t0, t1 = a[:, 0].astype(np.int64), a[:, 1].astype(np.int64)
    cu = (a[:, 2] >> 32).astype(np.int64)
    iters = (a[:, 2] & 0xFFFFFFFF).astype(np.int64)
    start, span = t0.min(), t1.max() - t0.min()
    block = wid // 4
    n_cu = int(cu.max()) + 1
    # age rank: start order of the wave's block among the blocks on its CU
    rank = np.zeros(len(a), dtype=np.int64)
    for k in np.unique(cu):
        m = np.nonzero(cu == k)[0]
        blocks = np.unique(block[m])
        bstart = {b: t0[m][block[m] == b].min() for b in blocks}
        order = {b: i for i, b in enumerate(sorted(blocks, key=lambda b: bstart[b]))}
        rank[m] = [order[b] for b in block[m]]
    res = {"config": cfg, "kernel_ms": st["kernel_ms"], "waves": int(len(a)), "span_us": span / 100.0,
           "mean_resident_frac": float((t1 - t0).sum() / (len(a) * span)),
           "iters_total": int(iters.sum()),
           # a resident wave's time per loop iteration, and the span if every wave slot stayed
           # resident to the end at that rate (the residency-limited bound of a perfectly balanced tail)
           "wave_ns_per_iter": float((t1 - t0).sum() * 10.0 / iters.sum()),
           "balanced_span_us": float((t1 - t0).sum() / len(a) / 100.0),
           "end_quantiles_frac_of_span": {str(q): float(np.quantile((t1 - start) / span, q))
                                          for q in (0.01, 0.1, 0.5, 0.9, 0.99)},
           "by_age_rank": {}}
    for k in range(int(rank.max()) + 1):
        m = rank == k
        res["by_age_rank"][k] = {"waves": int(m.sum()), "iters_mean": float(iters[m].mean()),
                                 "iters_share": float(iters[m].sum() / iters.sum()),
                                 "end_frac_mean": float(((t1[m] - start) / span).mean()),
                                 "end_frac_p99": float(np.quantile((t1[m] - start) / span, 0.99)),
                                 "rank_eq_block_div_ncu": float(np.mean(block[m] // max(1, len(np.unique(cu))) == k))}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
