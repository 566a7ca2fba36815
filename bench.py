#!/usr/bin/env python3
"""bench.py — throughput of the MI355X smallpt sampling loop (BASELINE.json metric: Msamples/s).

A "step" = one render of the workload through the C ABI (spt_render_async: scene upload, queue
reset, render kernel, fixed-point -> float finalize) into a device framebuffer, plus (N > 1) the
single RCCL gather of the fp32 row tiles to rank 0. Inputs (scene, camera) are built once; the
framebuffers stay resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--no-cpu-baseline]
  torchrun --nproc-per-node N bench.py --gpus N ...        (one rank per GPU, RCCL)

Workloads (BASELINE.json configs):
  c2  1024x768 @ 64 spp, cosine-weighted (:474-477)
  c3  1024x768 @ 512 spp, explicit light sampling (:464-473)   <- default, the north-star config
  c4  4096x4096 @ 1024 spp, NEE                                 (8-GPU config; strong by default)
  c5  4096x4096 @ 4096 spp, 32-sphere scene, max depth 16       (8-GPU config; strong by default)
Weak scaling (default for c2/c3): each of N GPUs renders 1/N of the rows at N x spp, so per-GPU
work is the single-GPU workload and the N-GPU job is the same image at N x the samples.
"""
from __future__ import annotations

import argparse
import importlib
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec (w×h×spp/s) on Cornell box; per-channel RMSE vs ref PPM"
PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (v_fma_f32 on all lanes)
CONFIGS = {
    "c2": dict(width=1024, height=768, spp=64, nee_prob=0.0, scene="cornell", max_depth=0,
               scaling="weak", desc="C2: 1024x768 @ 64 spp, cosine-weighted importance sampling"),
    "c3": dict(width=1024, height=768, spp=512, nee_prob=1.0, scene="cornell", max_depth=0,
               scaling="weak", desc="C3: 1024x768 @ 512 spp, Cornell box + explicit light sampling"),
    "c4": dict(width=4096, height=4096, spp=1024, nee_prob=1.0, scene="cornell", max_depth=0,
               scaling="strong", desc="C4: 4096x4096 @ 1024 spp, NEE, row-tile shards"),
    "c5": dict(width=4096, height=4096, spp=4096, nee_prob=1.0, scene="spheres32", max_depth=16,
               scaling="strong", desc="C5: 4096x4096 @ 4096 spp, 32-sphere scene, max depth 16"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads() -> int:
    """CPU-baseline threads: the cores this process may run on, capped at 16 = one GPU's share of a
    GPU-box host (the gpurun pool gives each GPU 16 cores; nproc reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


QUALITY_FIXTURE = os.path.join(ROOT, "tests", "golden", "ref_c3_blocks_k32.npz")
# per config: the fixture and the reference binary its runs came from (tests/golden/make_golden.py
# --quality-c3 / --quality-c2)
QUALITY_FIXTURES = {"c3": (QUALITY_FIXTURE, "smallpt_nee_xs"),
                    "c2": (os.path.join(ROOT, "tests", "golden", "ref_c2_blocks_k32.npz"), "smallpt_cos_xs")}


def quality(img: np.ndarray, spp: int, extra_images=(), config: str = "c3"):
    """The metric's quality half (BASELINE.json: per-channel RMSE vs the reference PPM) at C3:
    the GPU image, quantised and linearised as the reference's P3 (toInt :319-321, (v/255)^2.2),
    as 32x32-block means against the pooled block means of 16 independent runs of the reference
    itself (oracle/_ref/smallpt_nee_xs, 1024x768 @ 512 spp each; tests/golden/ref_c3_blocks_k32.npz,
    made by tests/golden/make_golden.py --quality-c3). Both images are Monte-Carlo estimates, so
    the RMSE has a noise floor: the expected RMSE of two unbiased estimates at these sample counts,
    from the spread of the 16 runs (per block: var_run * (spp_ref/spp + 1/16)); and the same RMSE
    between the two halves of the reference runs (reference vs reference).
    extra_images: further GPU renders of the same config with other seeds (the bench image is
    seed 1). Pooled with it, they give the comparison at a matched budget -- as many 512-spp runs
    on each side -- whose noise floor is below the north star's 1e-3 tolerance. (Runs are pooled
    rather than rendered at 16x the spp: the per-pixel clamp of :538 makes an image depend on its
    own spp.)
    config "c2": the same against 16 runs of oracle/_ref/smallpt_cos_xs at C2's 1024x768 @ 64 spp
    (tests/golden/ref_c2_blocks_k32.npz)."""
    fixture, ref_bin = QUALITY_FIXTURES[config]
    if not os.path.exists(fixture):
        return None
    f = np.load(fixture)  # plain arrays (allow_pickle=False)
    blocks, (w, h, spp_ref, k) = f["blocks"], [int(v) for v in f["shape"]]
    if img.shape != (h, w, 3):
        return None
    def block_means(im):
        q = np.floor(np.power(np.clip(im.astype(np.float64), 0, 1), 1 / 2.2) * 255 + 0.5)
        return ((q / 255.0) ** 2.2).reshape(h // k, k, w // k, k, 3).mean(axis=(1, 3))

    own = block_means(img)
    n = len(blocks)
    ref = blocks.mean(0)
    var_run = blocks.var(0, ddof=1)
    rmse = np.sqrt(((own - ref) ** 2).mean(axis=(0, 1)))
    floor = np.sqrt((var_run * (spp_ref / spp + 1.0 / n)).mean(axis=(0, 1)))
    half = np.sqrt(((blocks[: n // 2].mean(0) - blocks[n // 2:].mean(0)) ** 2).mean(axis=(0, 1)))
    half_floor = np.sqrt((var_run * (4.0 / n)).mean(axis=(0, 1)))
    matched = None
    if extra_images and spp == spp_ref:
        gpu = np.stack([own] + [block_means(im) for im in extra_images])
        m = len(gpu)
        rm = np.sqrt(((gpu.mean(0) - ref) ** 2).mean(axis=(0, 1)))
        # expected RMSE of two unbiased pooled estimates: the reference runs' and the GPU runs' own
        # block variances (the GPU's from its m seeds)
        fl = np.sqrt((var_run / n + gpu.var(0, ddof=1) / m).mean(axis=(0, 1)))
        matched = {"gpu_runs": m, "reference_runs": n, "spp_each": spp,
                   "rmse_vs_reference": [round(float(x), 6) for x in rm],
                   "noise_floor": [round(float(x), 6) for x in fl],
                   "ratio_to_floor": [round(float(a / b), 3) for a, b in zip(rm, fl)],
                   "mean_diff": [round(float(x), 6) for x in (gpu.mean(0) - ref).mean(axis=(0, 1))],
                   "seeds": f"1..{m} (Philox stream seed; the reference runs use their own seeds)"}
    return {"rmse_vs_reference": [round(float(x), 6) for x in rmse],
            "noise_floor": [round(float(x), 6) for x in floor],
            "ratio_to_floor": [round(float(a / b), 3) for a, b in zip(rmse, floor)],
            "reference_halves_rmse": [round(float(x), 6) for x in half],
            "reference_halves_floor": [round(float(x), 6) for x in half_floor],
            "mean_diff": [round(float(x), 6) for x in (own - ref).mean(axis=(0, 1))],
            "rmse_vs_contract": None,
            "matched_budget": matched,
            "space": f"linear, quantised as the reference's P3, {k}x{k}-block means, per channel (R,G,B)",
            "reference": f"{n} runs of oracle/_ref/{ref_bin} at {w}x{h} @ {spp_ref} spp "
                         f"({n * spp_ref} spp pooled), tests/golden/{os.path.basename(fixture)}"}


def cpu_baseline(spt, prims, cam, params, gpu_img, budget_s: float):
    """Counter-mode oracle (the same algorithm and random stream as the kernel) on the host cores,
    OpenMP over an evenly spread pixel subset, sized to ~budget_s; also checks those pixels
    bit-exactly against the GPU image. (Pixels, not rows: one C5 row is 4096 x 4096 samples.)"""
    from oracle import oracle

    threads = host_threads()
    h, w, spp = params.height, params.width, params.spp
    npix = h * w
    # Grow the subset until one timed run takes >= budget_s / 2 (the first, small run also absorbs
    # library load and OpenMP start-up).
    n = 4 * threads
    while True:
        pixels = np.unique(np.linspace(0, npix - 1, min(n, npix)).round().astype(np.uint32))
        t0 = time.perf_counter()
        img, st = oracle.counter_render_pixels(prims, cam._c, params, pixels, threads=threads)
        dt = time.perf_counter() - t0
        if dt >= budget_s / 2 or len(pixels) >= npix:
            break
        n = int(min(npix, max(2 * n, round(n * budget_s / max(dt, 1e-3)))))
    samples = len(pixels) * spp
    exact = gpu_img is not None and np.array_equal(gpu_img.reshape(-1, 3)[pixels], img)
    return {"value": round(samples / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
            "host_cpus": os.cpu_count(), "kind": "port",
            "sample": f"{len(pixels)} of {npix} pixels evenly spread, {spp} spp each = "
                      f"{samples} samples in {dt:.1f} s; oracle/spt_oracle.c counter mode, "
                      f"OpenMP dynamic pixels",
            "gpu_pixels_bit_exact": bool(exact)}


def reference_baseline(cfg, budget_s: float, threads: int = 1):
    """The reference itself (oracle/_ref/smallpt_*: /root/reference/src/smallpt.cpp compiled by
    oracle/build_ref.sh with the SURVEY Appendix A patch) with spp scaled to a bounded sample of
    ~budget_s; None when the binary is absent (it is built only where the reference is).
    threads == 1: the build as shipped (its OpenMP pragma :526 is commented out). threads > 1: the
    reference's own OpenMP loop (smallpt_*_omp: pragma :526 enabled, row loop :528 made canonical)
    on that many host cores (HEAD scene only).
    C1-C4 (the HEAD scene): smallpt_nee / smallpt_cos. C5 (32 spheres, depth cap 16): smallpt_sph16,
    the reference's own Sphere class (:223-254) in C5's scene with the cap. The 4096^2 configs run
    the reference at 1024^2 (the same square camera, so the same distribution of pixel-sample work):
    one 4096^2 pass of the reference is ~25 s (C4) or minutes (C5) plus a 200 MB P3 write."""
    import subprocess
    import tempfile

    if cfg["scene"] == "cornell" and cfg["max_depth"] == 0:
        est = "nee" if cfg["nee_prob"] >= 1 else "cos"
    elif cfg["scene"] == "spheres32" and cfg["max_depth"] == 16 and cfg["nee_prob"] >= 1:
        if threads > 1:
            return None
        est = "sph16"
    else:
        return None
    binary = os.path.join(ROOT, "oracle", "_ref", f"smallpt_{est}" + ("_omp" if threads > 1 else ""))
    if not os.path.exists(binary):
        return None
    w, h = cfg["width"], cfg["height"]
    if w * h > 1024 * 1024:
        w, h = w * 1024 // max(w, h), h * 1024 // max(w, h)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    with tempfile.TemporaryDirectory() as tmp:
        def run(spp):
            t0 = time.perf_counter()
            subprocess.run([binary, str(w), str(h), str(spp), "1", os.path.join(tmp, "o.ppm")],
                           check=True, cwd=tmp, env=env, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
            return time.perf_counter() - t0
        spp = 1
        dt = run(spp)
        if dt < budget_s / 2:
            spp = max(2, int(budget_s / 2 / dt + 0.5))
            dt = run(spp)
    how = ("single thread as shipped" if threads == 1 else
           f"the reference's OpenMP loop (:526 enabled) on {threads} threads; its libc rand() is one "
           f"locked global generator, so it scales negatively")
    return {"value": round(w * h * spp / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
            "host_cpus": os.cpu_count(), "kind": "reference",
            "sample": f"{w}x{h} @ {spp} spp = {w * h * spp} samples in {dt:.1f} s (whole image incl. "
                      f"its P3 write{'' if (w, h) == (cfg['width'], cfg['height']) else ', at 1024^2: same camera aspect'}); "
                      f"{os.path.relpath(binary, ROOT)} = the reference compiled from its own sources, "
                      f"g++ -O3, {how}"}


def image_writer(spt, full, w, h, with_cpu: bool):
    """§8(f) output formats: the GPU encoder (spt_image.hip) on the resident framebuffer, P3 as the
    reference writes it (:548-551) and P6/PFM; HBM bytes = 12 B/pixel read + encoded bytes written
    (P3 also re-reads the framebuffer in its write pass). CPU leg: the oracle's fprintf-format
    restatement of the same writer on the same image (single thread)."""
    import torch
    from oracle import oracle

    enc = spt.Encoder(torch.cuda.current_device())
    out = {}
    p3_dev = b""  # the GPU encoder's P3 bytes of the bench image (compared with the CPU writer's)
    try:
        for name in ("p3", "p6", "pfm"):
            cap = spt.Encoder.bound(w, h, name)
            buf = torch.empty(cap, dtype=torch.uint8, device="cuda")
            stream = torch.cuda.current_stream().cuda_stream
            n = enc.encode(full.data_ptr(), w, h, name, buf.data_ptr(), cap, stream)  # warm-up
            torch.cuda.synchronize()
            reps = 10
            t0 = time.perf_counter()
            for _ in range(reps):
                n = enc.encode(full.data_ptr(), w, h, name, buf.data_ptr(), cap, stream)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            if name == "p3" and with_cpu:
                p3_dev = buf[:n].cpu().numpy().tobytes()
            moved = w * h * 12 * (2 if name == "p3" else 1) + n
            out[name] = {"bytes": n, "ms": round(dt * 1e3, 4), "GBps": round(moved / dt / 1e9, 1)}
        # the C4/C5 image size (4096^2, 201 MB of fp32) with synthetic data, P3
        big = torch.rand((4096, 4096, 3), dtype=torch.float32, device="cuda")
        cap = spt.Encoder.bound(4096, 4096, "p3")
        buf = torch.empty(cap, dtype=torch.uint8, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        enc.encode(big.data_ptr(), 4096, 4096, "p3", buf.data_ptr(), cap, stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            n = enc.encode(big.data_ptr(), 4096, 4096, "p3", buf.data_ptr(), cap, stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        out["p3_4096x4096_synthetic"] = {"bytes": n, "ms": round(dt * 1e3, 3),
                                          "GBps": round((4096 * 4096 * 24 + n) / dt / 1e9, 1)}
        del big, buf
        if with_cpu:
            img = full.cpu().numpy()
            t0 = time.perf_counter()
            b = oracle.encode_image(img, 0)
            out["p3"]["cpu_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
            out["p3"]["cpu_kind"] = "oracle snprintf restatement of :548-551, 1 thread"
            # byte for byte: the device buffer the GPU encoder wrote against the CPU writer's bytes
            out["p3"]["bytes_equal_cpu"] = bool(b == p3_dev)
    finally:
        enc.close()
    return out


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, timeout_s: float, env=None) -> int:
    """`bench.py --gpus N` without a launcher: start N copies of this script as child processes,
    one rank per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N, MASTER_ADDR = 127.0.0.1, a free
    MASTER_PORT), and wait for them. The parent never touches the GPU (no torch import, no HIP
    call): it only starts processes, so nothing is exec'd from a process that initialised the GPU.
    The parent reads every child's stdout: rank 0's JSON lines are its own stdout, everything else
    (gloo's connection messages, which it prints on stdout) goes to stderr, so the parent's stdout
    holds exactly the one JSON line. Returns 0 when every rank exits 0. Otherwise it returns the first failing rank's status
    (124 when the ranks outlive `timeout_s`), after ending the remaining children: each runs in its
    own process group, and the parent kills exactly those groups. No retry.
    The reference's own parallel construct is an OpenMP pragma over rows (smallpt.cpp:526-528)."""
    import signal
    import subprocess
    import threading

    base = dict(os.environ if env is None else env)
    base.update(WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(free_port()), SPT_BENCH_SPAWNED="1")
    procs, readers = [], []

    def forward(rank, pipe):
        for line in iter(pipe.readline, b""):
            if rank == 0 and line.lstrip().startswith(b"{"):
                sys.stdout.buffer.write(line)
                sys.stdout.flush()
            else:
                sys.stderr.buffer.write(line)
                sys.stderr.flush()
        pipe.close()

    for i in range(n):
        e = dict(base, RANK=str(i), LOCAL_RANK=str(i))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=e, start_new_session=True, stdout=subprocess.PIPE))
        readers.append(threading.Thread(target=forward, args=(i, procs[-1].stdout), daemon=True))
        readers[-1].start()
    deadline = time.monotonic() + timeout_s
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc  # -N (signal N) -> 128 + N
                log(f"bench.py: rank {procs.index(p)} exited with status {rc}; ending the other ranks")
        if status != 0 or time.monotonic() > deadline:
            if status == 0:
                status = 124
                log(f"bench.py: ranks still running after {timeout_s:.0f} s; ending them (status 124)")
            for p in live:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
            for p in live:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    p.wait()
            break
        time.sleep(0.05)
    for t in readers:
        t.join(timeout=10)
    return status


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None)
    ap.add_argument("--spp", type=int, default=0, help="override spp (per-GPU for weak scaling)")
    ap.add_argument("--chunk", type=int, default=int(os.environ.get("SPT_CHUNK", "0")),
                    help="samples per work unit (0 = auto; A/B scripts set SPT_CHUNK)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_c3.json"),
                    help="PMC traffic summary (HBM bytes per render launch) to attach, if present")
    ap.add_argument("--save-ppm", default="")
    ap.add_argument("--kernel-level", default="auto", help="A/B only: cap the kernel specialisation "
                    "(auto | generic | cornell | const; spt_params.flags, never changes results)")
    ap.add_argument("--move-box", type=float, default=0.0,
                    help="edit rect[] (:287-311): move the short box by this many units in x (the "
                         "HEAD topology with uploaded geometry; 0 = the reference's table)")
    ap.add_argument("--light-y", type=float, default=None,
                    help="edit rect[] (:294): the light's plane y (81.5 in the reference; the light "
                         "uploaded, the room literal: KV_UPBOX_*)")
    ap.add_argument("--light-grow", type=float, default=0.0,
                    help="edit rect[] (:294): grow the light rectangle by this much on every side")
    ap.add_argument("--room-depth", type=float, default=None,
                    help="edit rect[] (:288-293): the back wall's z (170 in the reference; the room "
                         "uploaded too: KV_CORNELL_*)")
    ap.add_argument("--camera", choices=["reference", "tilted"], default="reference",
                    help="tilted: Camera(lookfrom (50,40,168), lookat (56,36,5), vup (0,1,0)), not "
                         "axis-aligned (the literal kernels' any-camera forms, Cfg CAMAX 2)")
    ap.add_argument("--drop-short-box", action="store_true",
                    help="edit rect[] (:287-311): remove the short box (:305-309), another topology "
                         "(the uploaded-geometry rect-only kernels)")
    ap.add_argument("--reference-leaks", action="store_true",
                    help="leaked paths go on from the miss vertex as the reference's (:371-377; "
                         "SPT_FLAG_REFERENCE_LEAKS) instead of ending at their first miss (contract v6)")
    ap.add_argument("--verify-gather", dest="verify_gather", action="store_true", default=None,
                    help="rank 0 re-renders the whole image alone and checks the gathered one bit for "
                         "bit (default on for N > 1: the RCCL gather has not run on hardware before)")
    ap.add_argument("--no-verify-gather", dest="verify_gather", action="store_false")
    ap.add_argument("--gather", choices=["spt", "torch"], default="spt",
                    help="N > 1 over nccl: the library's gather (spt_comm: grouped ncclSend/ncclRecv "
                         "+ de-interleave kernel) or torch.distributed.gather of the shards (RCCL) "
                         "with the de-interleave as torch indexing on rank 0")
    ap.add_argument("--frames-in-flight", type=int, choices=[1, 2, 3, 4], default=2,
                    help="N > 1: consecutive frames render on N streams, so a frame's launch fills the "
                         "CU slots the previous frames' tails free (1: one stream, frame after frame)")
    ap.add_argument("--init-timeout", type=float, default=300.0,
                    help="seconds allowed for the RCCL / process-group set-up; past it the rank "
                         "prints an error and exits with status 3 (no retry)")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="--gpus N > 1 without a launcher: seconds the spawned ranks may run in all "
                         "before they are ended (exit status 124)")
    ap.add_argument("--no-extras", action="store_true",
                    help="profiling sessions only: skip everything after the timed region that launches "
                         "the render kernel again (the reference-leaks leg, the quality renders), so a "
                         "rocprofv3 summary of the run averages the warm-up and timed dispatches only")
    ap.add_argument("--probe-env", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun: start the N ranks here, before anything loads HIP (launch_ranks)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))
    if args.probe_env:
        # CPU test hook (tests/test_bench_launch.py): report the rank environment, no GPU work
        rk = os.environ.get("RANK", "0")
        print(json.dumps({k: os.environ.get(k) for k in
                          ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                           "SPT_BENCH_SPAWNED")}), flush=True)
        if os.environ.get("SPT_PROBE_HANG_RANK") == rk:
            time.sleep(3600)
        sys.exit(int(os.environ.get("SPT_PROBE_EXIT", "0")) if
                 os.environ.get("SPT_PROBE_FAIL_RANK") == rk else 0)

    import datetime
    import threading

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.verify_gather is None:
        args.verify_gather = world > 1

    # Bounded set-up: a rank that cannot join the process group or the RCCL communicator (a peer
    # missing, a wrong address) exits with a clear error instead of hanging the job.
    def init_expired():
        log(f"bench.py: rank {os.environ.get('RANK', '0')}: process-group / RCCL set-up did not "
            f"finish within {args.init_timeout:.0f} s; exiting with status 3")
        os._exit(3)
    watchdog = threading.Timer(args.init_timeout, init_expired)
    watchdog.daemon = True
    if world > 1:
        watchdog.start()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # SPT_DIST_BACKEND=gloo: rehearsal mode for >1 rank on a 1-GPU box (ranks share the device,
    # the gather goes through host memory); the real path is nccl = RCCL over xGMI.
    backend = os.environ.get("SPT_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        tmo = datetime.timedelta(seconds=args.init_timeout)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)

    spt = importlib.import_module("small-pathtracer_amd")
    sd = importlib.import_module("small-pathtracer_amd.distributed")
    cfg = dict(CONFIGS[args.config])
    scaling = args.scaling or cfg["scaling"]
    spp = args.spp or cfg["spp"]
    if scaling == "weak":
        spp *= world
    prims = spt.cornell_scene() if cfg["scene"] == "cornell" else spt.spheres32_scene()
    if args.move_box:
        assert cfg["scene"] == "cornell", "--move-box edits the Cornell scene"
        prims = spt.move_short_box(prims, args.move_box)
    if args.drop_short_box:
        assert cfg["scene"] == "cornell", "--drop-short-box edits the Cornell scene"
        prims = spt.drop_short_box(prims)
    if args.room_depth is not None:
        assert cfg["scene"] == "cornell", "--room-depth edits the Cornell scene"
        prims = spt.edit_room(prims, depth=args.room_depth)
    if args.light_y is not None or args.light_grow:
        assert cfg["scene"] == "cornell", "--light-y / --light-grow edit the Cornell scene"
        gl = args.light_grow
        prims = spt.edit_light(prims, x=(32 - gl, 68 + gl), z=(63 - gl, 96 + gl),
                               y=81.5 if args.light_y is None else args.light_y)
    edited = bool(args.move_box or args.drop_short_box or args.room_depth is not None
                  or args.light_y is not None or args.light_grow)
    w, h = cfg["width"], cfg["height"]
    cam_kw = dict(lookat=(56, 36, 5)) if args.camera == "tilted" else {}
    cam = spt.Camera(aspect=float(np.float32(w) / np.float32(h)), **cam_kw)
    edited = edited or args.camera != "reference"
    leak_flag = spt.FLAG_REFERENCE_LEAKS if args.reference_leaks else 0
    params = spt.default_params(width=w, height=h, spp=spp, nee_prob=cfg["nee_prob"],
                                max_depth=cfg["max_depth"], tile_rows=8, shard_index=rank,
                                shard_count=world, device=local, chunk=args.chunk,
                                flags=spt.kernel_flag(args.kernel_level) | leak_flag)
    rows_of = sd.shard_row_lists(h, 8, world)
    my_rows = rows_of[rank]
    assert np.array_equal(spt.shard_rows(params), my_rows)
    max_rows = sd.max_rows(rows_of)

    # Frames in flight: frame k renders into buffer k % nfly on stream k % nfly; the gathers (N > 1)
    # run in frame order on one stream behind an event of their render, and a frame buffer is not
    # rendered into again before its previous gather has read it.
    nfly = args.frames_in_flight
    # Render contexts used in turn, one per frame in flight (two at least): a step's statistics
    # (kernel time, event counts) are read `lag` steps later, after the steps in flight behind it
    # are queued, so reading them never stalls the streams between steps. Context k % n_ctx always
    # runs on the same stream (n_ctx == nfly) or on the one stream (nfly == 1).
    n_ctx = max(2, nfly)
    lag = max(1, nfly - 1)
    rens = [spt.Renderer(local) for _ in range(n_ctx)]
    for r_ in rens:
        r_.reserve(len(prims), params)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nfly - 1)]
    stream = streams[0]
    comm_stream = torch.cuda.Stream() if (world > 1 and nfly > 1) else stream
    shards = [torch.zeros((max_rows, w, 3), dtype=torch.float32, device="cuda") for _ in range(nfly)]
    fulls = ([torch.zeros((h, w, 3), dtype=torch.float32, device="cuda") for _ in range(nfly)]
             if rank == 0 else [None] * nfly)
    shard, full = shards[0], fulls[0]
    gather_done = [None] * nfly
    comm = None
    use_torch_gather = world > 1 and backend == "nccl" and args.gather == "torch"
    # torch.distributed.gather into rank 0's pre-allocated slots, de-interleaved on the device
    # (distributed.gather_rows, the path the gloo tests cover)
    slots = [torch.zeros_like(shard) for _ in range(world)] if use_torch_gather and rank == 0 else None
    comm_error = ""
    if world > 1 and backend == "nccl" and not use_torch_gather:
        # the framebuffer gather of SURVEY §8e in the library (spt_comm: C++ over RCCL, grouped
        # ncclSend/ncclRecv to rank 0 + the de-interleave kernel); torch.distributed only carries
        # the RCCL unique id from rank 0 to the others
        uid = [spt.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        try:  # (a rank whose communicator fails to come up takes the torch fallback below)
            comm = spt.Comm(uid[0], world, rank, local)
            comm.reserve(params)
        except Exception as e:  # noqa: BLE001
            comm, comm_error = None, f"{type(e).__name__}: {e}"
            log(f"bench.py: rank {rank}: spt_comm set-up failed ({comm_error})")
        up = torch.tensor([1 if comm is not None else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(up, op=dist.ReduceOp.MIN)
        if int(up.item()) == 0:
            if comm is not None:
                comm.close()
            comm = None
            use_torch_gather = True
            slots = [torch.zeros_like(shard) for _ in range(world)] if rank == 0 else None
    gather_mode = "spt (RCCL send/recv)" if comm is not None else (
        "torch (dist.gather)" if use_torch_gather else ("host (gloo)" if world > 1 else "none"))
    if world > 1 and backend == "nccl" and args.gather == "spt" and comm is None:
        gather_mode = ("torch (dist.gather; spt_comm set-up failed on a rank"
                       + (f": {comm_error})" if comm_error else ")"))
    if comm is not None:
        # The library gather has not run on >1 GPU before the driver's scaling run: check it on a
        # known pattern (every rank's rows, exact in fp32) before anything is timed, and fall back
        # to torch's gather for the whole run if it raises or mismatches (recorded in the line).
        ok, why = True, ""
        try:
            rr = torch.as_tensor(my_rows, device="cuda", dtype=torch.int64).view(-1, 1, 1)
            xx = torch.arange(w, device="cuda", dtype=torch.int64).view(1, -1, 1)
            cc = torch.arange(3, device="cuda", dtype=torch.int64).view(1, 1, -1)
            shard.zero_()
            shard[: len(my_rows)] = ((rr * 7 + xx * 3 + cc) % 65521).to(torch.float32)
            if rank == 0:
                full.fill_(-1.0)
            comm.gather(params, shard.data_ptr(), full.data_ptr() if rank == 0 else 0,
                        stream.cuda_stream)
            torch.cuda.synchronize()
            if rank == 0:
                ra = torch.arange(h, device="cuda", dtype=torch.int64).view(-1, 1, 1)
                want = ((ra * 7 + xx * 3 + cc) % 65521).to(torch.float32)
                if not torch.equal(full, want):
                    ok, why = False, "pattern mismatch"
        except Exception as e:  # noqa: BLE001
            ok, why = False, f"{type(e).__name__}: {e}"
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            log(f"bench.py: rank {rank}: library gather check failed ({why or 'on another rank'}); "
                f"using torch.distributed.gather")
            comm = None
            use_torch_gather = True
            slots = [torch.zeros_like(shard) for _ in range(world)] if rank == 0 else None
            gather_mode = f"torch (dist.gather; library gather check failed: {why or 'another rank'})"
        else:
            gather_mode = "spt (RCCL send/recv; pattern check passed)"
    kstats = []
    n_step = [0]

    def step(p_=None):
        k = n_step[0]
        n_step[0] += 1
        i = k % nfly
        s_ = streams[i]
        if gather_done[i] is not None:  # buffer i's previous gather must have read it
            s_.wait_event(gather_done[i])
        rens[k % n_ctx].render_async(prims, cam, params if p_ is None else p_, shards[i].data_ptr(),
                                     s_.cuda_stream)
        if k >= lag:  # the statistics of the step `lag` back (its context's last launch)
            kstats.append(rens[(k - lag) % n_ctx].stats())
        if comm is not None or use_torch_gather:
            ev = torch.cuda.Event()
            ev.record(s_)
            comm_stream.wait_event(ev)
            if comm is not None:  # one RCCL gather to rank 0
                comm.gather(params, shards[i].data_ptr(), fulls[i].data_ptr() if rank == 0 else 0,
                            comm_stream.cuda_stream)
            else:  # torch.distributed.gather over RCCL, de-interleave on rank 0
                with torch.cuda.stream(comm_stream):
                    sd.gather_rows(shards[i], rows_of, fulls[i], gather_list=slots)
            gd = torch.cuda.Event()
            gd.record(comm_stream)
            gather_done[i] = gd
        elif world > 1:
            with torch.cuda.stream(s_):
                host = sd.gather_rows(shards[i].cpu(), rows_of, fulls[i].cpu() if rank == 0 else None)
                if rank == 0:
                    fulls[i].copy_(host)
        else:
            with torch.cuda.stream(s_):
                fulls[i].copy_(shards[i][: len(my_rows)])

    watchdog.cancel()  # set-up done (the first gather below has its own collective timeout)
    def drain():  # the statistics of the last `lag` queued steps
        for j in range(max(0, n_step[0] - lag), n_step[0]):
            kstats.append(rens[j % n_ctx].stats())
        n_step[0] = 0

    # every context's first launch allocates its unit slots: warm both up, whatever --warmup says
    n_warm = max(args.warmup, len(rens))
    for _ in range(n_warm):
        step()
    drain()
    kstats.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    drain()
    assert len(kstats) == args.steps, (len(kstats), args.steps)
    last = (args.steps - 1) % nfly
    shard, full = shards[last], fulls[last]
    # The roofline's kernel time: with two frames in flight a launch's HIP-event span also covers
    # the neighbouring frame's overlap, so the per-launch time is measured on 3 launches run one at
    # a time after the timed region (the same kernel and work; rocprofv3 sees them as well).
    kms_flight = float(np.mean([s["kernel_ms"] for s in kstats]))
    iso = []
    for _ in range(3 if nfly > 1 else 0):
        rens[0].render_async(prims, cam, params, shards[0].data_ptr(), streams[0].cuda_stream)
        iso.append(rens[0].stats())
    torch.cuda.synchronize()
    kst = iso if iso else kstats
    kms = np.array([s["kernel_ms"] for s in kst])
    per_rank = None
    if world > 1:
        # Per-rank evidence for the N > 1 line: each rank's isolated kernel time, its timed-region
        # wall time and the gather alone (3 gathers after a barrier each, the fastest; the image
        # they gather is the frame just rendered into buffer 0, so nothing checked changes).
        gms = []
        for _ in range(3):
            dist.barrier()
            torch.cuda.synchronize()
            t_ = time.perf_counter()
            if comm is not None:
                comm.gather(params, shards[0].data_ptr(), fulls[0].data_ptr() if rank == 0 else 0,
                            streams[0].cuda_stream)
            elif use_torch_gather:
                sd.gather_rows(shards[0], rows_of, fulls[0], gather_list=slots)
            else:
                host = sd.gather_rows(shards[0].cpu(), rows_of, fulls[0].cpu() if rank == 0 else None)
                if rank == 0:
                    fulls[0].copy_(host)
            torch.cuda.synchronize()
            gms.append((time.perf_counter() - t_) * 1e3)
        dev = "cuda" if backend == "nccl" else "cpu"
        mine = torch.tensor([float(kms.mean()), kms_flight, elapsed * 1e3, min(gms)],
                            dtype=torch.float64, device=dev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        every = np.stack([e.cpu().numpy() for e in every])
        per_rank = {"kernel_ms": [round(float(x), 3) for x in every[:, 0]],
                    "kernel_ms_min": round(float(every[:, 0].min()), 3),
                    "kernel_ms_max": round(float(every[:, 0].max()), 3),
                    "kernel_ms_in_flight": [round(float(x), 3) for x in every[:, 1]],
                    "timed_region_ms": [round(float(x), 2) for x in every[:, 2]],
                    "gather_ms": [round(float(x), 3) for x in every[:, 3]],
                    "gather_ms_source": "3 gathers alone after the timed region, each after a "
                                        "barrier, fastest (wall clock incl. the barrier release)",
                    "launcher": ("bench.py (spawned ranks)" if os.environ.get("SPT_BENCH_SPAWNED")
                                 else "external (torch.distributed.run or equivalent)")}
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_per_step = w * h * spp  # all ranks together (each rank renders its rows at spp)
    value = samples_per_step * args.steps / elapsed / 1e6
    flop = np.array([s["flop"] for s in kst])
    flop_x = np.array([s["flop_executed"] for s in kst])
    achieved = float((flop / (kms * 1e-3)).mean() / 1e12)
    achieved_x = float((flop_x / (kms * 1e-3)).mean() / 1e12)
    s0 = kstats[-1]
    my_samples = len(my_rows) * w * spp
    assert s0["samples"] == my_samples, (s0["samples"], my_samples)

    traffic, traffic_file = None, None
    if os.path.exists(args.traffic) and args.config == "c3" and world == 1:
        try:
            traffic_file = json.load(open(args.traffic))
            traffic = traffic_file.get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None
    # Hardware-counter figures come from a committed rocprofv3 session (scripts/session.sh, copied
    # into profiles/ by scripts/update_profiles.py), not from this run: each file records the hash
    # of the kernel sources it profiled, and a file taken on other sources is not used.
    this_sha = spt.kernel_sources_sha16()
    hw_notes = []

    def current_profile(pattern):
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
        if not files:
            return None, None
        d_ = json.load(open(files[-1]))
        name = f"profiles/{os.path.basename(files[-1])}"
        if d_.get("kernel_sources_sha16") != this_sha:
            hw_notes.append(f"{name} profiled kernel sources {d_.get('kernel_sources_sha16')}, this "
                            f"build is {this_sha}: not used")
            return None, name
        return d_, name

    pmc = {}
    if args.config == "c3" and world == 1:
        try:
            d_, name = current_profile("r[0-9][0-9]_pmc_summary.json")
            if d_ is not None:
                der = d_["derived"]
                pmc = {"valu_issue_frac": round(der["valu_issue_frac_of_peak"], 3),
                       "valu_lane_utilization": round(der["valu_lane_utilization"], 3),
                       "source": f"{name} (SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU; a committed profile "
                                 f"session of this kernel build, not this run)"}
        except Exception:  # noqa: BLE001
            pmc = {}

    # the hardware's own count: SQ_INSTS_VALU_FLOPS_FP32 of the newest round's
    # C3 instruction-class passes (scripts/session.sh classes) counts FP32 operations per
    # wave-instruction; x 64 lanes x the measured lane utilisation = FLOP executed per launch
    hw = {}
    if args.config == "c3" and world == 1:
        try:
            d_, name = current_profile("r[0-9][0-9]_pmc_c3_classes.json")
            if d_ is not None:
                c_ = d_["counters"]
                lu = c_["SQ_THREAD_CYCLES_VALU"] / (64.0 * c_["SQ_ACTIVE_INST_VALU"])
                hw_flop = c_["SQ_INSTS_VALU_FLOPS_FP32"] * 64.0 * lu
                hw = {"frac_hw": round(hw_flop / (float(kms.mean()) * 1e-3) / 1e12 / PEAK_FP32_TFLOPS, 4),
                      "hw_flop_per_launch": round(hw_flop, -6),
                      "hw_source": f"{name}: SQ_INSTS_VALU_FLOPS_FP32 x 64 x lane utilisation {lu:.3f} "
                                   f"over this run's kernel time",
                      "hw_counters_from": "a committed profile session of this kernel build "
                                          f"(kernel sources {this_sha}), not this run"}
        except Exception:  # noqa: BLE001
            hw = {}
    if traffic_file is not None and traffic_file.get("kernel_sources_sha16") != this_sha:
        hw_notes.append(f"{os.path.relpath(args.traffic, ROOT)} profiled kernel sources "
                        f"{traffic_file.get('kernel_sources_sha16')}, this build is {this_sha}: not used")
        traffic = None
    if hw_notes:
        hw["hw_stale"] = "; ".join(hw_notes)

    gather_exact = None
    if rank == 0:
        img = full.cpu().numpy()
        if args.verify_gather:  # the whole image on this GPU alone (1 shard) must equal the gather
            p1 = spt.default_params(width=w, height=h, spp=spp, nee_prob=cfg["nee_prob"],
                                    max_depth=cfg["max_depth"], tile_rows=8, device=local,
                                    flags=leak_flag)
            one = spt.render(prims, cam, p1)
            gather_exact = bool(np.array_equal(one, img))
            assert gather_exact, "gathered image differs from the 1-GPU render"
        cpu = None
        port = None
        if not args.no_cpu_baseline and world == 1:
            # (the reference binaries hold the unedited table: no reference leg for an edited scene)
            cpu = None if edited else reference_baseline(cfg, args.cpu_budget)
            omp = None if edited else reference_baseline(cfg, args.cpu_budget, threads=host_threads())
            port = cpu_baseline(spt, prims, cam, params, img, args.cpu_budget)
            if cpu is not None and omp is not None:
                cpu["openmp"] = omp
            if cpu is None:
                cpu = port
            else:
                cpu["port"] = port
        if args.save_ppm:
            spt.write_ppm(args.save_ppm, img)
        writer = image_writer(spt, full, w, h, with_cpu=not args.no_cpu_baseline)
        qual = None
        if (args.config in QUALITY_FIXTURES and world == 1 and not edited and not args.no_extras
                and os.path.exists(QUALITY_FIXTURES[args.config][0])):
            # 15 more seeds of the same render (after the timed region): the matched-budget RMSE
            extra = [spt.render(prims, cam, spt.default_params(
                width=w, height=h, spp=spp, nee_prob=cfg["nee_prob"], max_depth=cfg["max_depth"],
                tile_rows=8, device=local, seed=sd_, flags=leak_flag)) for sd_ in range(2, 17)]
            qual = quality(img, spp, extra, config=args.config)
        if qual is not None and port is not None:
            # the bench's own rows re-rendered by the CPU contract (cpu_baseline.port): exact
            qual["rmse_vs_contract"] = 0.0 if port.get("gpu_pixels_bit_exact") else None
        # Contract v6's leak-end rule, quantified on this workload: the same workload
        # with leaked paths going on as the reference's (SPT_FLAG_REFERENCE_LEAKS; the same Philox
        # streams, so only the leaked paths differ), timed after everything above has read the
        # bench image: K steps through the same pipeline (value_reference_leaks) and 3 isolated
        # launches (kernel_ms_reference_leaks), VERDICT r05 item 4
        leak = None
        if world == 1 and cfg["scene"] == "cornell" and not args.no_extras:
            if args.reference_leaks:
                leak = {"rule": "off: leaked paths go on from the miss vertex as the reference's "
                                "(:371-377, SPT_FLAG_REFERENCE_LEAKS)"}
            else:
                pr = spt.default_params(width=w, height=h, spp=spp, nee_prob=cfg["nee_prob"],
                                        max_depth=cfg["max_depth"], tile_rows=8, device=local,
                                        chunk=args.chunk,
                                        flags=spt.kernel_flag(args.kernel_level) | spt.FLAG_REFERENCE_LEAKS)
                saved = list(kstats)
                kstats.clear()
                for _ in range(n_warm):
                    step(pr)
                drain()
                kstats.clear()
                torch.cuda.synchronize()
                t_r = time.perf_counter()
                for _ in range(args.steps):
                    step(pr)
                torch.cuda.synchronize()
                el_r = time.perf_counter() - t_r
                drain()
                st_r = kstats[-1]
                img_r = fulls[(args.steps - 1) % nfly].cpu().numpy()
                iso_r = []
                for _ in range(3):
                    rens[0].render_async(prims, cam, pr, shards[0].data_ptr(), streams[0].cuda_stream)
                    iso_r.append(rens[0].stats()["kernel_ms"])
                torch.cuda.synchronize()
                kstats[:] = saved
                leak = {"rule": "contract v6: a leaked path ends at its first miss (DESIGN.md §3); "
                                "the reference wanders on from the miss vertex (:371-377)",
                        "value_reference_leaks": round(samples_per_step * args.steps / el_r / 1e6, 3),
                        "ms_per_step_reference_leaks": round(el_r / args.steps * 1e3, 3),
                        "kernel_ms_reference_leaks": round(float(np.mean(iso_r)), 3),
                        "kernel_ratio_reference_leaks": round(float(np.mean(iso_r)) / float(kms.mean()), 4),
                        "reference_vertices_per_sample": round(st_r["vertices"] / my_samples, 4),
                        "reference_vertices_skipped_frac": round(1 - s0["vertices"] / st_r["vertices"], 4),
                        "reference_path_rays_skipped_frac": round(1 - s0["path_rays"] / st_r["path_rays"], 4),
                        "image_mean_rel_diff": float(f"{(img.mean() - img_r.mean()) / img_r.mean():.3g}"),
                        "how": f"the same workload with SPT_FLAG_REFERENCE_LEAKS (same seed, same random "
                               f"streams) after the timed region: {args.steps} steps through the same "
                               f"pipeline ({nfly} frames in flight) after {n_warm} warm-up steps, and 3 "
                               f"launches one at a time for the kernel time"}
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": n_warm,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic: the reference's Cornell-box scene (smallpt.cpp:287-311)"
                     if cfg["scene"] == "cornell" else
                     "synthetic: C5's 32-sphere scene (the room and light of smallpt.cpp:288-294 plus "
                     "32 DIFF spheres of the reference's Sphere class :223-254)")
                    + " and camera (:521), Philox4x32-7 stream seed 1",
            "config": {"workload": cfg["desc"] + (f", weak-scaled to {spp} spp over {world} GPUs"
                                                   if scaling == "weak" and world > 1 else "")
                       + (f", short box moved {args.move_box:g} in x (edited rect[])" if args.move_box else "")
                       + (", short box removed (edited rect[])" if args.drop_short_box else "")
                       + (f", back wall at z = {args.room_depth:g} (edited rect[])"
                          if args.room_depth is not None else "")
                       + (f", light at y = {81.5 if args.light_y is None else args.light_y:g} grown by "
                          f"{args.light_grow:g} (edited rect[])"
                          if args.light_y is not None or args.light_grow else "")
                       + (", tilted camera (lookat (56,36,5))" if args.camera == "tilted" else "")
                       + (", leaked paths as the reference's" if args.reference_leaks else ""),
                       "width": w, "height": h, "spp": spp,
                       "estimator": "nee" if cfg["nee_prob"] >= 1 else "cosine",
                       "frames_in_flight": nfly,
                       "parallelism": (f"row-tile x{world} (tile 8 rows, cyclic) + one gather to rank 0 "
                                       f"({('RCCL, ' + ('torch.distributed.gather' if use_torch_gather else 'spt_comm grouped send/recv')) if backend == 'nccl' else backend})")
                                      if world > 1 else "1 GPU"},
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                         # the same model with only the shadow rays the kernel traces charged a
                         # scene test (the rest are rejected exactly by the light pre-test)
                         "achieved_executed": round(achieved_x, 3),
                         "frac_executed": round(achieved_x / PEAK_FP32_TFLOPS, 4),
                         **hw,
                         "traffic": traffic,
                         "hbm_gbs": (round(traffic / (kms.mean() * 1e-3) / 1e9, 2)
                                     if traffic else None),
                         "hbm_frac": (round(traffic / (kms.mean() * 1e-3) / 8e12, 5)
                                      if traffic else None),
                         # SURVEY §8(d) asks for both denominators; profiles/r01_valu_rates.txt
                         # measures v_fma_f32 at full rate and v_pk_fma_f32 at half rate on gfx950,
                         # so 157.3 (non-packed fma on all lanes) is the binding peak, not 78.6.
                         "frac_vs_78p6": round(achieved / (PEAK_FP32_TFLOPS / 2), 4),
                         "valu_pmc": pmc or None,
                         "kernel": "spt::render_kernel",
                         "kernel_ms": round(float(kms.mean()), 3),
                         "kernel_ms_source": ("3 launches one at a time after the timed region"
                                              if iso else "the timed launches"),
                         # frames in flight: the same FLOP over the GPU time per frame of the
                         # timed run (elapsed / steps, the neighbouring frame filling each tail)
                         "frac_pipelined": round(float(flop.mean()) / (elapsed / args.steps)
                                                 / 1e12 / PEAK_FP32_TFLOPS, 4),
                         "kernel_ms_in_flight": round(kms_flight, 3),
                         "flop_per_launch": float(flop.mean()),
                         "flop_per_sample": round(float(flop.mean()) / my_samples, 1)},
            "paths": {"vertices_per_sample": round(s0["vertices"] / my_samples, 4),
                      "rays_per_sample": round((s0["path_rays"] + s0["shadow_rays"]) / my_samples, 4),
                      "rays_traced_per_sample": round((s0["path_rays"] + s0["shadow_traced"]
                                                       - s0["shadow_proven"]) / my_samples, 4),
                      "shadow_proven_per_sample": round(s0["shadow_proven"] / my_samples, 4),
                      # contract v6: a leaked path ends at its first miss, so every miss is a
                      # path leaving the room (the reference re-misses from its miss vertex,
                      # :373-374: 0.22 misses but ~0.047 leaked paths per sample at C3)
                      "misses_per_sample": round(s0["misses"] / my_samples, 4),
                      "misses": ("every miss (leaked paths go on as the reference's)" if args.reference_leaks
                                 else "first misses: leaked paths end there (contract v6, DESIGN.md §3)"),
                      "leak_end": leak},
            "quality": qual,
            "gather_equals_1gpu_render": gather_exact,
            "gather": gather_mode,
            "ranks": per_rank,
            "cpu_baseline": cpu,
            "image_writer": writer,
            # the kernel build this line measured (the GPU test record profiles/rNN_gpu_tests.json
            # carries the same hash)
            "build": {"kernel_sources_sha16": spt.kernel_sources_sha16(),
                      "libspt_build_sources_sha16": spt.build_sources_sha16()},
        }
        print(json.dumps(out), flush=True)
    for r_ in rens:
        r_.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
