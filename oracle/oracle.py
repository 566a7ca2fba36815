"""ctypes front end of the CPU oracle (oracle/libspt_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker. The product package never imports this module.
"""
from __future__ import annotations

import ctypes
import importlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libspt_oracle.so")
_spt = importlib.import_module("small-pathtracer_amd")
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        L.spt_oracle_compat_render.argtypes = [P(_spt.spt_prim), ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_uint,
                                               ctypes.c_int, P(ctypes.c_double)]
        L.spt_oracle_counter_render.argtypes = [P(_spt.spt_prim), ctypes.c_int,
                                                P(_spt.spt_camera), P(_spt.spt_params),
                                                P(ctypes.c_int32), ctypes.c_int,
                                                P(ctypes.c_float), P(ctypes.c_uint64), ctypes.c_int]
        L.spt_oracle_write_ppm_d.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                             P(ctypes.c_double)]
        L.spt_oracle_write_ppm_f.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                             P(ctypes.c_float)]
        L.spt_oracle_erand48.argtypes = [P(ctypes.c_ushort)]
        L.spt_oracle_erand48.restype = ctypes.c_double
        L.spt_oracle_glibc_rand.argtypes = [ctypes.c_uint, ctypes.c_int, P(ctypes.c_int32)]
        L.spt_oracle_philox.argtypes = [P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32)]
        L.spt_oracle_philox_r.argtypes = [P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32),
                                          ctypes.c_int]
        L.spt_oracle_set_pairs.argtypes = [ctypes.c_int]
        L.spt_oracle_disk_dir.argtypes = [ctypes.c_uint32, P(ctypes.c_float), P(ctypes.c_float)]
        L.spt_oracle_sincos2pi.argtypes = [ctypes.c_float, P(ctypes.c_float), P(ctypes.c_float)]
        L.spt_oracle_camera.argtypes = [P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_double),
                                        P(ctypes.c_double), ctypes.c_float, ctypes.c_float]
        L.spt_oracle_scene_cornell.argtypes = [P(_spt.spt_prim)]
        L.spt_oracle_default_params.argtypes = [P(_spt.spt_params)]
        L.spt_oracle_camera_spt.argtypes = [P(_spt.spt_camera), ctypes.c_float]
        L.spt_oracle_prim_intersect.argtypes = [P(_spt.spt_prim), P(ctypes.c_double),
                                                P(ctypes.c_double)]
        L.spt_oracle_prim_intersect.restype = ctypes.c_double
        L.spt_oracle_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def scene_cornell():
    arr = (_spt.spt_prim * 17)()
    n = lib().spt_oracle_scene_cornell(arr)
    return [arr[i] for i in range(n)]


def default_params(**kw):
    p = _spt.spt_params()
    lib().spt_oracle_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def camera(aspect: float):
    c = _spt.spt_camera()
    lib().spt_oracle_camera_spt(ctypes.byref(c), ctypes.c_float(aspect))
    return c


def compat_render(w: int, h: int, spp: int, seed: int = 1, nee: bool = True, prims=None,
                  uniform: bool = False, row_seed: bool = False, stats: bool = False,
                  qthr: float = None, max_depth: int = 0):
    """fp64 restatement of the reference (bit-exact with the patched oracle). (h, w, 3) float64.

    row_seed: seed erand48's row streams with the seed too (oracle/_ref/smallpt_cos_xs); without it
    the reference's scattering/RR draws are the same for every seed. stats: also return
    {"vertices", "misses", "first_misses", "vertices_pre"} over all radiance() calls (first_misses:
    samples whose path missed; vertices_pre: vertices up to and with a path's first miss). qthr: the NEE-mix threshold of :464
    (default 1 if nee else 0; oracle/_ref/smallpt_q05 is 0.5). max_depth: the depth cap of
    oracle/_ref/smallpt_sph16 (0 = none, the reference)."""
    prims = prims or scene_cornell()
    arr = (_spt.spt_prim * len(prims))(*prims)
    out = np.zeros((h, w, 3), dtype=np.float64)
    st = (ctypes.c_uint64 * 4)()
    flags = (2 if uniform else 0) | (4 if row_seed else 0)
    if qthr is None:
        qthr = 1.0 if nee else 0.0
    L = lib()
    L.spt_oracle_compat_render_ex.argtypes = [
        ctypes.POINTER(_spt.spt_prim), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_uint, ctypes.c_int, ctypes.c_double, ctypes.c_int,
        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    L.spt_oracle_compat_render_ex(arr, len(prims), w, h, spp, seed, flags, qthr, max_depth,
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), st)
    if stats:
        return out, {"vertices": int(st[0]), "misses": int(st[1]), "first_misses": int(st[2]),
                     "vertices_pre": int(st[3])}
    return out


def plane_k(k: float) -> float:
    """The contract's fp32 plane coordinate of a rectangle at k (spt_oracle_plane_k)."""
    L = lib()
    L.spt_oracle_plane_k.restype = ctypes.c_float
    L.spt_oracle_plane_k.argtypes = [ctypes.c_double]
    return float(np.float32(L.spt_oracle_plane_k(k)))


def scene_boxes(prims, params) -> int:
    """Boxes of contract v6 that the oracle finds in the scene (spt_oracle_scene_boxes)."""
    arr = (_spt.spt_prim * len(prims))(*prims)
    L = lib()
    L.spt_oracle_scene_boxes.restype = ctypes.c_int
    return int(L.spt_oracle_scene_boxes(arr, len(prims), ctypes.byref(params)))


def set_boxes(on: bool) -> None:
    """Test hook: False = boxes tested face by face (pairs and a top), True = the contract."""
    lib().spt_oracle_set_boxes(int(bool(on)))


def set_leak_end(on: bool) -> None:
    """Test hook: False = leaked paths go on from the miss vertex as the reference's (:373-374),
    True = the contract (c_find_leak_end: they end at their first miss)."""
    lib().spt_oracle_set_leak_end(int(bool(on)))


def plane_t_mismatches(num, inv) -> int:
    """Operands (float32 arrays) on which the oracle's fast plane distance differs in its bits from
    the contract's fma(n, inv, -2^-149) (spt_oracle_plane_t_mismatches)."""
    num = np.ascontiguousarray(num, dtype=np.float32)
    inv = np.ascontiguousarray(inv, dtype=np.float32)
    L = lib()
    L.spt_oracle_plane_t_mismatches.restype = ctypes.c_int
    L.spt_oracle_plane_t_mismatches.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return int(L.spt_oracle_plane_t_mismatches(num.ctypes.data, inv.ctypes.data, len(num)))


def counter_render(prims, cam, params, rows=None, threads: int = 0):
    """Counter-mode contract on the CPU. Returns ((nrows, w, 3) float32, stats dict)."""
    if rows is None:
        rows = np.arange(params.height, dtype=np.int32)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    arr = (_spt.spt_prim * len(prims))(*prims)
    out = np.zeros((len(rows), params.width, 3), dtype=np.float32)
    st = (ctypes.c_uint64 * 10)()
    lib().spt_oracle_counter_render(arr, len(prims), ctypes.byref(cam), ctypes.byref(params),
                                    rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(rows),
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), st, threads)
    return out, dict(zip(_spt.STAT_KEYS, [int(v) for v in st]))


def counter_render_pixels(prims, cam, params, pixels, threads: int = 0):
    """Counter-mode contract at the listed pixels (y * w + x). Returns ((npix, 3) float32, stats)."""
    pixels = np.ascontiguousarray(pixels, dtype=np.uint32)
    arr = (_spt.spt_prim * len(prims))(*prims)
    out = np.zeros((len(pixels), 3), dtype=np.float32)
    st = (ctypes.c_uint64 * 10)()
    L = lib()
    L.spt_oracle_counter_render_pixels.argtypes = [
        ctypes.POINTER(_spt.spt_prim), ctypes.c_int, ctypes.POINTER(_spt.spt_camera),
        ctypes.POINTER(_spt.spt_params), ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
        ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    rc = L.spt_oracle_counter_render_pixels(
        arr, len(prims), ctypes.byref(cam), ctypes.byref(params),
        pixels.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(pixels),
        out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), st, threads)
    assert rc == 0
    return out, dict(zip(_spt.STAT_KEYS, [int(v) for v in st]))


def proof_check(on: bool, sphere_y0=None, edited=False) -> None:
    """Test hook: check the early shadow-ray resolve of the HEAD NEE kernel (spt_kernel.hip
    early_nee_proven) or, with sphere_y0, of the sphere NEE kernel (early_room_proven with that
    threshold), or with edited=True of the uploaded-geometry HEAD-topology NEE kernel
    (early_geo_proven, clauses by c_find_early_clauses), restated as c_early_nee_proven, against
    c_intersect during counter renders; resets the counts."""
    L = lib()
    L.spt_oracle_proof_check.argtypes = [ctypes.c_int, ctypes.c_float]
    mode = 0 if not on else (3 if edited else (2 if sphere_y0 is not None else 1))
    L.spt_oracle_proof_check(mode, float(sphere_y0 or 0.0))


def proof_counts() -> tuple:
    """(claims, contradicted claims) since proof_check(True)."""
    out = (ctypes.c_uint64 * 2)()
    lib().spt_oracle_proof_counts(out)
    return int(out[0]), int(out[1])


def shadow_census() -> list:
    """Test hook (tools/shadow_census.py): the light-accepted shadow rays the HEAD early resolve
    left to a trace since the last call, by outcome and failing clause (spt_oracle_shadow_census,
    proof mode 1); resets the counts."""
    out = (ctypes.c_uint64 * 16)()
    L = lib()
    L.spt_oracle_shadow_census.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    L.spt_oracle_shadow_census(out)
    return [int(v) for v in out]


def set_pairs(on: bool) -> None:
    """Test hook: parallel-pair rect tests on (the contract) or off (every rect on its own)."""
    lib().spt_oracle_set_pairs(1 if on else 0)


def write_ppm(path: str, rgb: np.ndarray) -> None:
    h, w, _ = rgb.shape
    if rgb.dtype == np.float64:
        lib().spt_oracle_write_ppm_d(path.encode(), w, h,
                                     np.ascontiguousarray(rgb).ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    else:
        a = np.ascontiguousarray(rgb, dtype=np.float32)
        lib().spt_oracle_write_ppm_f(path.encode(), w, h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))


def encode_image(rgb: np.ndarray, fmt: int) -> bytes:
    """P3 (0) / P6 (1) / PFM (2) file bytes from the C restatement of :548-551 (the checker)."""
    h, w, _ = rgb.shape
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    L = lib()
    L.spt_oracle_encode_image.restype = ctypes.c_size_t
    L.spt_oracle_encode_image.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    ptr = a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    need = L.spt_oracle_encode_image(ptr, w, h, fmt, None, 0)
    buf = ctypes.create_string_buffer(need)
    n = L.spt_oracle_encode_image(ptr, w, h, fmt, buf, need)
    return buf.raw[:n]


def erand48_seq(xi2: int, n: int):
    xs = (ctypes.c_ushort * 3)(0, 0, xi2 & 0xFFFF)
    return [lib().spt_oracle_erand48(xs) for _ in range(n)]


def glibc_rand(seed: int, n: int):
    out = (ctypes.c_int32 * n)()
    lib().spt_oracle_glibc_rand(seed, n, out)
    return list(out)


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().spt_oracle_philox(c, k, o)
    return list(o)


def philox_r(ctr, key, rounds: int):
    """Philox4x32 with `rounds` rounds (the contract uses SPT_PHILOX_ROUNDS = 7)."""
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().spt_oracle_philox_r(c, k, o, rounds)
    return list(o)


def disk_dir(ra: int):
    """(cos phi, sin phi) of the contract's azimuth from one Philox word (octant symmetry)."""
    c, s = ctypes.c_float(), ctypes.c_float()
    lib().spt_oracle_disk_dir(ctypes.c_uint32(ra), ctypes.byref(c), ctypes.byref(s))
    return c.value, s.value


def sincos2pi(xi: float):
    s, c = ctypes.c_float(), ctypes.c_float()
    lib().spt_oracle_sincos2pi(ctypes.c_float(xi), ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def threads() -> int:
    return lib().spt_oracle_threads()


def set_unit_dirs(mode) -> None:
    """Test hook: None = the contract (unit directions iff the scene has a sphere or a REFR prim),
    True/False = force normalised / free-scale directions (diagnostics only)."""
    lib().spt_oracle_set_unit_dirs(-1 if mode is None else (1 if mode else 0))
