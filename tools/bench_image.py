#!/usr/bin/env python3
"""Image-encoder microbench (spt_image.hip): P3 / P6 / PFM of a synthetic 4096x4096 fp32
framebuffer (the C4/C5 image size), device to device. Prints one JSON line per format."""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    spt = importlib.import_module("small-pathtracer_amd")
    w = h = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rgb = torch.rand((h, w, 3), dtype=torch.float32, device="cuda")
    enc = spt.Encoder(0)
    stream = torch.cuda.current_stream().cuda_stream
    for fmt in ("p3", "p6", "pfm"):
        cap = spt.Encoder.bound(w, h, fmt)
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        n = enc.encode(rgb.data_ptr(), w, h, fmt, out.data_ptr(), cap, stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            n = enc.encode(rgb.data_ptr(), w, h, fmt, out.data_ptr(), cap, stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps({"format": fmt, "w": w, "h": h, "bytes": n, "ms_per_encode": round(dt * 1e3, 4)}))
    enc.close()


if __name__ == "__main__":
    main()
