#!/usr/bin/env python3
"""Per-wave residency of a -DSPT_DIAG=2 build (spt_diag.h: SPT_WAVE_TIMES) (SPT_WAVE_DUMP file): how much of the kernel's
span the waves are resident, and how the last waves straggle (queue tail).

  python tools/wave_tail.py gpurun_out/waves_c2.bin
"""
import json
import sys

import numpy as np


def main():
    a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 3)
    a = a[a[:, 1] > 0]
    t0, t1 = a[:, 0].astype(np.int64), a[:, 1].astype(np.int64)
    iters = (a[:, 2] & 0xFFFFFFFF).astype(np.int64)
    start, end = t0.min(), t1.max()
    span = end - start  # 100 MHz ticks
    dur = t1 - t0
    ends = np.sort(t1 - start) / span
    out = {
        "waves": int(len(a)),
        "span_us": span / 100.0,
        "mean_resident_frac": float(dur.sum() / (len(a) * span)),
        "start_spread_us": float((t0.max() - start) / 100.0),
        "end_quantiles_frac_of_span": {q: float(np.quantile(ends, q)) for q in (0.01, 0.1, 0.5, 0.9, 0.99)},
        "iters_mean": float(iters.mean()), "iters_max": int(iters.max()), "iters_min": int(iters.min()),
        "iter_ns": float(dur.sum() * 10.0 / iters.sum()),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
