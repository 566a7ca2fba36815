"""small-pathtracer_amd — MI355X-native drop-in for the smallpt per-pixel sampling loop.

Python mirror of the reference's host API over the C ABI in ``include/spt.h`` (libspt.so):

=====================================  ==================================================
reference (/root/reference/src/...)    here
=====================================  ==================================================
``Rectangle_xz/xy/yz`` smallpt.cpp:92-221  ``Rectangle_xz/xy/yz`` (same ctor argument order)
``Sphere`` :223-254                     ``Sphere``
``Refl_t {DIFF, SPEC, REFR}`` :72-74    ``DIFF, SPEC, REFR``
``Camera`` :256-285                     ``Camera`` (constructor semantics via spt_camera_init)
``Hitable *rect[]`` :287-311            ``cornell_scene()``
pixel loop :528-542 (+ radiance :419)   ``render()`` / ``Renderer`` (HIP kernel, gfx950)
``toInt`` :319-321 + PPM writer :548-551  ``write_ppm()`` / ``write_image()`` / ``Encoder``
                                        (GPU encoder: byte-identical P3, plus P6 and PFM)
=====================================  ==================================================

The product path is the HIP kernel only: ``render()`` and the writers raise if libspt.so or a
gfx950 device is missing — there is no CPU fallback in this package.
"""
from __future__ import annotations

import atexit
import ctypes
import os
from typing import Iterable, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SPT_LIB overrides the library (A/B builds in tools/ab.sh); the default is the in-tree build.
LIB_PATH = os.environ.get("SPT_LIB") or os.path.join(_HERE, "libspt.so")

DIFF, SPEC, REFR = 0, 1, 2
RECT_XY, RECT_XZ, RECT_YZ, SPHERE = 0, 1, 2, 3
LIGHT_GLIBC_WRAP, LIGHT_UNIFORM = 0, 1
PHILOX_KEY1 = 0x53505431

STATUS = {0: "ok", 1: "invalid argument", 2: "HIP runtime error", 3: "no usable gfx950 device",
          4: "device out of memory", 5: "unsupported feature", 6: "RCCL error"}


class SptError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        super().__init__(f"spt error {status} ({STATUS.get(status, '?')}): {msg}")
        self.status = status


# ---------------------------------------------------------------------------------------------
# ctypes mirror of include/spt.h
# ---------------------------------------------------------------------------------------------
class spt_prim(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("refl", ctypes.c_int32),
                ("geom", ctypes.c_double * 5), ("e", ctypes.c_double * 3),
                ("c", ctypes.c_double * 3)]


class spt_camera(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_double * 3), ("lower_left_corner", ctypes.c_double * 3),
                ("horizontal", ctypes.c_double * 3), ("vertical", ctypes.c_double * 3)]


class spt_params(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("seed", ctypes.c_uint32), ("nee_prob", ctypes.c_float),
                ("rr_depth", ctypes.c_int32), ("max_depth", ctypes.c_int32),
                ("light_id", ctypes.c_int32),
                ("light_x0", ctypes.c_float), ("light_dx", ctypes.c_float),
                ("light_z0", ctypes.c_float), ("light_dz", ctypes.c_float),
                ("light_y", ctypes.c_float), ("light_area", ctypes.c_float),
                ("light_mode", ctypes.c_int32),
                ("tile_rows", ctypes.c_int32), ("shard_index", ctypes.c_int32),
                ("shard_count", ctypes.c_int32), ("chunk", ctypes.c_int32),
                ("device", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class spt_stats(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_uint64), ("path_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("vertices", ctypes.c_uint64),
                ("nee_events", ctypes.c_uint64), ("nee_light_hits", ctypes.c_uint64),
                ("cosine_samples", ctypes.c_uint64), ("misses", ctypes.c_uint64),
                ("shadow_traced", ctypes.c_uint64), ("sphere_vertices", ctypes.c_uint64),
                ("shadow_proven", ctypes.c_uint64), ("flop", ctypes.c_double), ("flop_executed", ctypes.c_double),
                ("kernel_ms", ctypes.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class spt_gather_op(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("peer", ctypes.c_int32), ("count", ctypes.c_uint64),
                ("offset", ctypes.c_uint64)]


GATHER_SEND, GATHER_RECV = 0, 1

STAT_KEYS = ["samples", "path_rays", "shadow_rays", "vertices", "nee_events", "nee_light_hits",
             "cosine_samples", "misses", "shadow_traced", "sphere_vertices"]

# Every entry point declared in include/spt.h (checked by tests/test_capi.py).
EXPORTS = ["spt_default_params", "spt_camera_init", "spt_scene_cornell", "spt_scene_spheres32",
           "spt_scene_cornell_specular", "spt_scene_smallpt_classic", "spt_scene_smallpt_mirror_glass",
           "spt_shard_rows", "spt_render", "spt_context_create", "spt_context_destroy",
           "spt_context_reserve", "spt_render_async", "spt_context_stats", "spt_abi_version",
           "spt_status_string", "spt_last_error", "spt_device_count", "spt_image_bound",
           "spt_encoder_create", "spt_encoder_destroy", "spt_encode_image", "spt_write_image",
           "spt_comm_unique_id", "spt_comm_create", "spt_comm_destroy", "spt_comm_reserve",
           "spt_gather_framebuffer", "spt_deinterleave_rows", "spt_render_multi", "spt_shutdown",
           "spt_gather_plan", "spt_gather_staging_floats", "spt_deinterleave_source",
           "spt_build_sources_sha16"]
IMAGE_FORMATS = {"p3": 0, "p6": 1, "pfm": 2}
FLAG_UNIFORM_SCATTER = 1  # spt_params.flags: random_scattering from the uniform code of :352-359
# spt_params.flags: leaked paths go on from the miss vertex as the reference's (:371-377) instead of
# ending at their first miss (contract v6's leak-end rule, the default where it applies)
FLAG_REFERENCE_LEAKS = 4
# spt_params.flags bits 8-9: cap on the kernel specialisation (A/B and tests; never changes results).
# "head"/"auto": the most specialised kernel the host can prove applicable.
KERNEL_LEVELS = {"auto": 0, "head": 0, "generic": 1, "cornell": 2, "const": 3}


def kernel_flag(name: str) -> int:
    """spt_params.flags bits selecting the kernel specialisation cap `name` (KERNEL_LEVELS)."""
    return KERNEL_LEVELS[name] << 8

_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libspt.so (built by __graft_entry__.build()). Fails loudly if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SptError(2, f"{path} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1
    # (same SONAMEs as /opt/rocm's). Loading torch first makes libspt bind to torch's copy, so
    # device pointers and streams from torch are valid here; loading libspt first would pin the
    # system runtime and torch's later HIP init fails ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    P, I32, U32 = ctypes.POINTER, ctypes.c_int32, ctypes.c_uint32
    lib.spt_default_params.argtypes = [P(spt_params)]
    lib.spt_camera_init.argtypes = [P(spt_camera), P(ctypes.c_double), P(ctypes.c_double),
                                    P(ctypes.c_double), ctypes.c_float, ctypes.c_float]
    lib.spt_scene_cornell.argtypes = [P(spt_prim), I32, P(I32)]
    lib.spt_scene_spheres32.argtypes = [P(spt_prim), I32, P(I32)]
    lib.spt_scene_cornell_specular.argtypes = [P(spt_prim), I32, P(I32)]
    lib.spt_scene_smallpt_classic.argtypes = [P(spt_prim), I32, P(I32)]
    lib.spt_scene_smallpt_mirror_glass.argtypes = [P(spt_prim), I32, P(I32)]
    lib.spt_shard_rows.argtypes = [P(spt_params), P(I32), I32]
    lib.spt_shard_rows.restype = I32
    lib.spt_render.argtypes = [P(spt_prim), I32, P(spt_camera), P(spt_params),
                               P(ctypes.c_float), P(spt_stats)]
    lib.spt_context_create.argtypes = [I32, P(ctypes.c_void_p)]
    lib.spt_context_destroy.argtypes = [ctypes.c_void_p]
    lib.spt_context_reserve.argtypes = [ctypes.c_void_p, I32, P(spt_params)]
    lib.spt_render_async.argtypes = [ctypes.c_void_p, P(spt_prim), I32, P(spt_camera),
                                     P(spt_params), ctypes.c_void_p, ctypes.c_void_p]
    lib.spt_context_stats.argtypes = [ctypes.c_void_p, P(spt_stats)]
    lib.spt_abi_version.restype = I32
    lib.spt_build_sources_sha16.restype = ctypes.c_char_p
    lib.spt_status_string.argtypes = [I32]
    lib.spt_status_string.restype = ctypes.c_char_p
    lib.spt_last_error.restype = ctypes.c_char_p
    lib.spt_device_count.restype = I32
    U64 = ctypes.c_uint64
    lib.spt_image_bound.argtypes = [I32, I32, I32]
    lib.spt_image_bound.restype = U64
    lib.spt_encoder_create.argtypes = [I32, P(ctypes.c_void_p)]
    lib.spt_encoder_destroy.argtypes = [ctypes.c_void_p]
    lib.spt_encode_image.argtypes = [ctypes.c_void_p, ctypes.c_void_p, I32, I32, I32,
                                     ctypes.c_void_p, U64, P(U64), ctypes.c_void_p]
    lib.spt_write_image.argtypes = [I32, ctypes.c_void_p, I32, I32, I32, ctypes.c_char_p]
    for name in ("spt_encoder_create", "spt_encoder_destroy", "spt_encode_image",
                 "spt_write_image"):
        getattr(lib, name).restype = I32
    VP = ctypes.c_void_p
    lib.spt_comm_unique_id.argtypes = [P(ctypes.c_uint8)]
    lib.spt_comm_create.argtypes = [P(ctypes.c_uint8), I32, I32, I32, P(VP)]
    lib.spt_comm_destroy.argtypes = [VP]
    lib.spt_comm_reserve.argtypes = [VP, P(spt_params)]
    lib.spt_gather_framebuffer.argtypes = [VP, P(spt_params), VP, VP, VP]
    lib.spt_deinterleave_rows.argtypes = [P(spt_params), I32, P(VP), VP, VP]
    lib.spt_render_multi.argtypes = [P(spt_prim), I32, P(spt_camera), P(spt_params), P(I32), I32,
                                     P(ctypes.c_float), P(spt_stats)]
    lib.spt_gather_plan.argtypes = [P(spt_params), I32, I32, P(spt_gather_op), I32]
    lib.spt_gather_plan.restype = I32
    lib.spt_gather_staging_floats.argtypes = [P(spt_params), I32]
    lib.spt_gather_staging_floats.restype = U64
    lib.spt_deinterleave_source.argtypes = [P(spt_params), I32, I32, P(I32), P(I32)]
    lib.spt_shutdown.argtypes = []
    for name in ("spt_comm_unique_id", "spt_comm_create", "spt_comm_destroy", "spt_comm_reserve",
                 "spt_gather_framebuffer", "spt_deinterleave_rows", "spt_render_multi",
                 "spt_deinterleave_source", "spt_shutdown"):
        getattr(lib, name).restype = I32
    for name in ("spt_default_params", "spt_camera_init", "spt_scene_cornell",
                 "spt_scene_spheres32", "spt_scene_cornell_specular", "spt_scene_smallpt_classic",
                 "spt_scene_smallpt_mirror_glass",
                 "spt_render", "spt_context_create",
                 "spt_context_destroy", "spt_context_reserve", "spt_render_async",
                 "spt_context_stats"):
        getattr(lib, name).restype = I32
    del U32
    _lib = lib
    # spt_render's cached per-device contexts (unit slots: ~200-400 MB) are returned when the
    # interpreter exits, not held until the process dies (a no-op when spt_render never ran)
    atexit.register(_release_dropin_contexts)
    return lib


# The sources the render kernel is compiled from: their hash identifies a kernel build, so a PMC
# profile committed under profiles/ can say which kernel it measured (bench.py omits hardware-counter
# figures whose profile was taken on other sources).
KERNEL_SOURCES = ("csrc/spt_kernel.hip", "csrc/spt_device.h", "csrc/spt_cornell.h", "csrc/spt_diag.h",
                  "csrc/Makefile", "../include/spt.h", "../include/spt_flops.h")


def kernel_sources_sha16() -> str:
    import hashlib

    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(_HERE, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_sources_sha16() -> str:
    """kernel_sources_sha16() of the sources the loaded libspt.so was built from (embedded by make)."""
    return load_library().spt_build_sources_sha16().decode()


def _release_dropin_contexts() -> None:
    if _lib is not None:
        try:
            _lib.spt_shutdown()
        except Exception:  # noqa: BLE001 -- interpreter shutdown: nothing left to report to
            pass


def _check(status: int) -> None:
    if status != 0:
        msg = (load_library().spt_last_error() or b"").decode(errors="replace")
        raise SptError(status, msg)


# ---------------------------------------------------------------------------------------------
# Reference-shaped host API
# ---------------------------------------------------------------------------------------------
def _v3(v) -> tuple:
    if isinstance(v, (int, float)):
        return (float(v), 0.0, 0.0)
    t = tuple(float(x) for x in v)
    return t + (0.0,) * (3 - len(t))


class Vec(tuple):
    """Vec :24-62 (only what scene construction needs: Vec(x=0, y=0, z=0), * scalar)."""

    def __new__(cls, x=0.0, y=0.0, z=0.0):
        return super().__new__(cls, (float(x), float(y), float(z)))

    def __mul__(self, b):
        return Vec(self[0] * b, self[1] * b, self[2] * b)

    __rmul__ = __mul__


def _prim(kind, geom, e, c, refl) -> spt_prim:
    p = spt_prim()
    p.kind, p.refl = kind, int(refl)
    for i, g in enumerate(geom):
        p.geom[i] = float(g)
    for i, x in enumerate(_v3(e)):
        p.e[i] = x
    for i, x in enumerate(_v3(c)):
        p.c[i] = x
    return p


def Rectangle_xz(x1, x2, z1, z2, y, e, c, refl=DIFF) -> spt_prim:  # :97-98
    return _prim(RECT_XZ, (x1, x2, z1, z2, y), e, c, refl)


def Rectangle_xy(x1, x2, y1, y2, z, e, c, refl=DIFF) -> spt_prim:  # :142
    return _prim(RECT_XY, (x1, x2, y1, y2, z), e, c, refl)


def Rectangle_yz(y1, y2, z1, z2, x, e, c, refl=DIFF) -> spt_prim:  # :185
    return _prim(RECT_YZ, (y1, y2, z1, z2, x), e, c, refl)


def Sphere(rad, p, e, c, refl=DIFF) -> spt_prim:  # :228
    pp = _v3(p)
    return _prim(SPHERE, (rad, pp[0], pp[1], pp[2], 0.0), e, c, refl)


LOOKFROM = Vec(50, 40, 168)  # :65


class Camera:
    """Camera :256-285: Camera(lookfrom, lookat, vup, vfov, aspect); get_ray(s, t)."""

    def __init__(self, lookfrom=LOOKFROM, lookat=(50, 40, 5), vup=(0, 1, 0), vfov=65.0,
                 aspect=1.0):
        lib = load_library()
        self._c = spt_camera()
        arr = lambda v: (ctypes.c_double * 3)(*_v3(v))  # noqa: E731
        _check(lib.spt_camera_init(ctypes.byref(self._c), arr(lookfrom), arr(lookat), arr(vup),
                                   float(vfov), float(aspect)))

    @property
    def origin(self):
        return tuple(self._c.origin)

    @property
    def lower_left_corner(self):
        return tuple(self._c.lower_left_corner)

    @property
    def horizontal(self):
        return tuple(self._c.horizontal)

    @property
    def vertical(self):
        return tuple(self._c.vertical)

    def get_ray(self, s: float, t: float):  # :276-279
        o, l, h, v = self.origin, self.lower_left_corner, self.horizontal, self.vertical
        return o, tuple(l[i] + h[i] * s + v[i] * t - o[i] for i in range(3))


def cornell_scene() -> list:
    """rect[] of :287-311 via the library's builder (17 primitives)."""
    lib = load_library()
    arr = (spt_prim * 64)()
    n = ctypes.c_int32()
    _check(lib.spt_scene_cornell(arr, 64, ctypes.byref(n)))
    return [arr[i] for i in range(n.value)]


def smallpt_classic_scene() -> list:
    """spt_scene_smallpt_classic(): the classic smallpt sphere box of the reference's older revision
    and its shipped image*.ppm (walls of radius 1e5, fp64-tested; two matte white balls; the
    radius-600 light sphere, prim 8). Render with nee_prob = 0 (no light rectangle)."""
    lib = load_library()
    arr = (spt_prim * 16)()
    n = ctypes.c_int32()
    _check(lib.spt_scene_smallpt_classic(arr, 16, ctypes.byref(n)))
    return [arr[i] for i in range(n.value)]


def smallpt_mirror_glass_scene() -> list:
    """spt_scene_smallpt_mirror_glass(): the same box with smallpt's mirror (SPEC) and glass (REFR)
    balls."""
    lib = load_library()
    arr = (spt_prim * 16)()
    n = ctypes.c_int32()
    _check(lib.spt_scene_smallpt_mirror_glass(arr, 16, ctypes.byref(n)))
    return [arr[i] for i in range(n.value)]


def spheres32_scene() -> list:
    lib = load_library()
    arr = (spt_prim * 64)()
    n = ctypes.c_int32()
    _check(lib.spt_scene_spheres32(arr, 64, ctypes.byref(n)))
    return [arr[i] for i in range(n.value)]


def move_short_box(prims: list, dx: float) -> list:
    """rect[] of :287-311 with the short box (:305-309, prims 12-16) moved by dx along x: the HEAD
    topology with edited geometry (the uploaded-geometry kernels; the compile-time one matches only
    the unedited table)."""
    out = [spt_prim.from_buffer_copy(p) for p in prims]
    for i in (12, 13, 16):  # XY faces and the XZ top: x bounds geom[0:2]
        out[i].geom[0] += dx
        out[i].geom[1] += dx
    for i in (14, 15):  # YZ faces: plane x = geom[4]
        out[i].geom[4] += dx
    return out


def edit_light(prims: list, x=(32.0, 68.0), z=(63.0, 96.0), y=81.5, e=None) -> list:
    """rect[] of :287-311 with the light (:294, prim 6) moved or resized: Rectangle_xz(x0, x1, z0,
    z1, y) and optionally its emission e. The room and the boxes stay (the boxes-only-uploaded
    kernels take the light from LDS; the early shadow-ray resolve needs the light's plane at most
    81.5 and its rectangle >= 1 inside the walls)."""
    out = [spt_prim.from_buffer_copy(p) for p in prims]
    g = out[6].geom
    g[0], g[1], g[2], g[3], g[4] = float(x[0]), float(x[1]), float(z[0]), float(z[1]), float(y)
    if e is not None:
        for i, v in enumerate(_v3(e)):
            out[6].e[i] = v
    return out


def edit_room(prims: list, depth: float = 170.0, width=(1.0, 99.0), height: float = 81.6) -> list:
    """rect[] of :287-311 with the room (:288-293, prims 0-5) resized: back wall at z = depth, side
    walls at x = width, ceiling at y = height, every wall's extents to match (a closed room, the
    HEAD topology)."""
    out = [spt_prim.from_buffer_copy(p) for p in prims]
    x0, x1 = float(width[0]), float(width[1])
    for i in (0, 1):  # Front / Back: Rectangle_xy(x0, x1, 0, height, z)
        g = out[i].geom
        g[0], g[1], g[3] = x0, x1, float(height)
    out[1].geom[4] = float(depth)
    for i, xw in ((2, x0), (3, x1)):  # Left / Right: Rectangle_yz(0, height, 0, depth, x)
        g = out[i].geom
        g[1], g[3], g[4] = float(height), float(depth), xw
    for i in (4, 5):  # Bottom / Top: Rectangle_xz(x0, x1, 0, depth, y)
        g = out[i].geom
        g[0], g[1], g[3] = x0, x1, float(depth)
    out[5].geom[4] = float(height)
    return out


def drop_short_box(prims: list) -> list:
    """rect[] of :287-311 without the short box (:305-309, prims 12-16): another topology (the
    uploaded-geometry rect-only kernels)."""
    return [spt_prim.from_buffer_copy(p) for p in prims[:12]]


def cornell_specular_scene() -> list:
    """Room + light of :288-294 with smallpt's mirror (SPEC) and glass (REFR) balls (:296-297)."""
    lib = load_library()
    arr = (spt_prim * 16)()
    n = ctypes.c_int32()
    _check(lib.spt_scene_cornell_specular(arr, 16, ctypes.byref(n)))
    return [arr[i] for i in range(n.value)]


def default_params(**kw) -> spt_params:
    p = spt_params()
    _check(load_library().spt_default_params(ctypes.byref(p)))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown spt_params field {k!r}")
        setattr(p, k, v)
    return p


def shard_rows(params: spt_params) -> np.ndarray:
    lib = load_library()
    n = lib.spt_shard_rows(ctypes.byref(params), None, 0)
    rows = (ctypes.c_int32 * max(n, 1))()
    lib.spt_shard_rows(ctypes.byref(params), rows, n)
    return np.frombuffer(rows, dtype=np.int32, count=n).copy()


def _scene_array(prims: Sequence[spt_prim]):
    arr = (spt_prim * len(prims))()
    for i, p in enumerate(prims):
        arr[i] = p
    return arr


def render(prims: Sequence[spt_prim], cam: Camera, params: spt_params, return_stats=False):
    """Drop-in for :528-542: returns (rows, w, 3) float32 linear clamped RGB (rows = this shard's
    rows, the whole image when shard_count == 1), y=0 top row. Runs on the GPU only."""
    lib = load_library()
    rows = int(lib.spt_shard_rows(ctypes.byref(params), None, 0))
    out = np.empty((rows, params.width, 3), dtype=np.float32)
    st = spt_stats()
    _check(lib.spt_render(_scene_array(prims), len(prims), ctypes.byref(cam._c),
                          ctypes.byref(params),
                          out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(st)))
    return (out, st.as_dict()) if return_stats else out


class Renderer:
    """Persistent device context for repeated renders into device buffers (torch tensors or raw
    pointers) on a given HIP stream — what bench.py and the multi-GPU path use."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        self._ctx = ctypes.c_void_p()
        _check(self.lib.spt_context_create(int(device), ctypes.byref(self._ctx)))
        self.device = device

    def close(self):
        if self._ctx:
            self.lib.spt_context_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # at interpreter exit module globals (ctypes) may already be gone
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def reserve(self, n_prims: int, params: spt_params):
        _check(self.lib.spt_context_reserve(self._ctx, int(n_prims), ctypes.byref(params)))

    def render_async(self, prims, cam: Camera, params: spt_params, rgb_dev_ptr: int,
                     stream_ptr: int = 0):
        self._prims = _scene_array(prims)
        _check(self.lib.spt_render_async(self._ctx, self._prims, len(prims), ctypes.byref(cam._c),
                                         ctypes.byref(params), ctypes.c_void_p(rgb_dev_ptr),
                                         ctypes.c_void_p(stream_ptr)))

    def stats(self) -> dict:
        st = spt_stats()
        _check(self.lib.spt_context_stats(self._ctx, ctypes.byref(st)))
        return st.as_dict()


def render_multi(prims: Sequence[spt_prim], cam: Camera, params: spt_params, devices,
                 return_stats=False):
    """One process, len(devices) GPUs (spt_render_multi): shard k on devices[k], one RCCL gather to
    devices[0]. Returns the full (h, w, 3) image, bit-identical to render() on one GPU."""
    lib = load_library()
    devs = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
    out = np.empty((params.height, params.width, 3), dtype=np.float32)
    st = spt_stats()
    _check(lib.spt_render_multi(_scene_array(prims), len(prims), ctypes.byref(cam._c),
                                ctypes.byref(params), devs, len(devices),
                                out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                ctypes.byref(st)))
    return (out, st.as_dict()) if return_stats else out


COMM_ID_BYTES = 128


def comm_unique_id() -> bytes:
    """spt_comm_unique_id(): the RCCL unique id rank 0 hands to every rank."""
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    _check(load_library().spt_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """One rank of the framebuffer gather (spt_comm_*): RCCL over xGMI, rank 0 receives."""

    def __init__(self, unique_id: bytes, nranks: int, rank: int, device: int):
        self.lib = load_library()
        self._c = ctypes.c_void_p()
        idb = (ctypes.c_uint8 * COMM_ID_BYTES)(*unique_id)
        _check(self.lib.spt_comm_create(idb, int(nranks), int(rank), int(device),
                                        ctypes.byref(self._c)))
        self.nranks, self.rank, self.device = nranks, rank, device

    def close(self):
        if self._c:
            self.lib.spt_comm_destroy(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def reserve(self, params: spt_params):
        _check(self.lib.spt_comm_reserve(self._c, ctypes.byref(params)))

    def gather(self, params: spt_params, shard_dev_ptr: int, image_dev_ptr: int, stream_ptr: int = 0):
        """Enqueue the gather of this rank's shard (rank 0: into image_dev_ptr) on the stream."""
        _check(self.lib.spt_gather_framebuffer(self._c, ctypes.byref(params),
                                               ctypes.c_void_p(shard_dev_ptr),
                                               ctypes.c_void_p(image_dev_ptr or None),
                                               ctypes.c_void_p(stream_ptr or None)))


def gather_plan(params: spt_params, nranks: int, rank: int) -> list:
    """spt_gather_plan(): the (kind, peer, count, offset) transfers `rank` posts in one framebuffer
    gather (pure host function, no device)."""
    ops = (spt_gather_op * 64)()
    n = load_library().spt_gather_plan(ctypes.byref(params), int(nranks), int(rank), ops, 64)
    if n < 0:
        raise SptError(1, "spt_gather_plan: bad arguments")
    return [(ops[i].kind, ops[i].peer, int(ops[i].count), int(ops[i].offset)) for i in range(n)]


def gather_staging_floats(params: spt_params, nranks: int) -> int:
    return int(load_library().spt_gather_staging_floats(ctypes.byref(params), int(nranks)))


def deinterleave_source(params: spt_params, nranks: int, row: int) -> tuple:
    """(rank, compact row) the de-interleave kernel reads image row `row` from."""
    k, j = ctypes.c_int32(), ctypes.c_int32()
    _check(load_library().spt_deinterleave_source(ctypes.byref(params), int(nranks), int(row),
                                                  ctypes.byref(k), ctypes.byref(j)))
    return k.value, j.value


def shutdown() -> None:
    """spt_shutdown(): release spt_render's cached per-device contexts."""
    _check(load_library().spt_shutdown())


def deinterleave_rows(params: spt_params, shard_dev_ptrs, image_dev_ptr: int, stream_ptr: int = 0):
    """spt_deinterleave_rows(): shard k's compact rows (device pointers) -> the image."""
    arr = (ctypes.c_void_p * len(shard_dev_ptrs))(*[ctypes.c_void_p(int(x)) for x in shard_dev_ptrs])
    _check(load_library().spt_deinterleave_rows(ctypes.byref(params), len(shard_dev_ptrs), arr,
                                                ctypes.c_void_p(image_dev_ptr),
                                                ctypes.c_void_p(stream_ptr or None)))


# ---------------------------------------------------------------------------------------------
# Output (:313-321 toInt/clamp, :548-551 the P3 writer): encoded on the GPU (spt_image.hip)
# ---------------------------------------------------------------------------------------------
def _format(fmt) -> int:
    return IMAGE_FORMATS[fmt] if isinstance(fmt, str) else int(fmt)


def write_image(path: str, rgb: np.ndarray, fmt="p3", device: int = 0) -> None:
    """Write an (h, w, 3) float32 framebuffer as P3 (byte-identical to :548-551), P6 or PFM."""
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w, _ = a.shape
    _check(load_library().spt_write_image(device, a.ctypes.data, w, h, _format(fmt),
                                          path.encode()))


def write_ppm(path: str, rgb: np.ndarray, device: int = 0) -> None:
    """The reference's writer (:548-551): ASCII P3, '%d %d %d ' per pixel."""
    write_image(path, rgb, "p3", device)


class Encoder:
    """spt_encoder: device framebuffer -> file bytes in a device buffer (spt_encode_image)."""

    def __init__(self, device: int = 0):
        self._e = ctypes.c_void_p()
        _check(load_library().spt_encoder_create(device, ctypes.byref(self._e)))

    def close(self):
        if self._e:
            load_library().spt_encoder_destroy(self._e)
            self._e = None

    @staticmethod
    def bound(w: int, h: int, fmt="p3") -> int:
        return int(load_library().spt_image_bound(w, h, _format(fmt)))

    def encode(self, rgb_dev_ptr: int, w: int, h: int, fmt, out_dev_ptr: int, cap: int,
               stream: int = 0) -> int:
        n = ctypes.c_uint64()
        _check(load_library().spt_encode_image(self._e, rgb_dev_ptr, w, h, _format(fmt),
                                               out_dev_ptr, cap, ctypes.byref(n), stream or None))
        return int(n.value)


def flop_model(stats: dict, prims: Iterable[spt_prim], executed: bool = False) -> float:
    """include/spt_flops.h model (same as the C side): `flop`, or with executed=True
    `flop_executed` (only the traced shadow rays charged a scene test)."""
    scene = sum(19 if p.kind == SPHERE else 6 for p in prims)
    shadow = (stats["shadow_traced"] - stats.get("shadow_proven", 0)) if executed else stats["shadow_rays"]
    return (stats["samples"] * 40 + (stats["path_rays"] + shadow) * scene
            + stats["vertices"] * 11 + stats["sphere_vertices"] * 13
            + (stats["vertices"] - stats["samples"]) * 12
            + stats["cosine_samples"] * 65 + stats["nee_events"] * 19
            + stats["nee_light_hits"] * 14)


__all__ = [n for n in dir() if not n.startswith("_")]
