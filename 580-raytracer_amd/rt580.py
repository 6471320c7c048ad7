"""ctypes binding of lib580rt.so (include/rt580.h) — the Python-side FFI a
maintainer would add next to the reference's class surface.

The product path is native: every render goes through rt_gpu_* into the HIP
kernels. If the library or a GPU is missing, calls raise RuntimeError; there is
no CPU fallback here.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib580rt.so")

RT_SUCCESS, RT_FAILURE, RT_INVALID_ARG = 0, 1, 2
RT_RNG_MINSTD_RAND0, RT_RNG_MT19937 = 0, 1
RT580_ABI_VERSION = 1


class RenderParams(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("depth", ctypes.c_int32), ("ao_samples", ctypes.c_int32),
        ("ao_enabled", ctypes.c_int32), ("rng_engine", ctypes.c_int32),
        ("rng_seed", ctypes.c_uint32), ("view_inverse_ok", ctypes.c_int32),
        ("view_inv", ctypes.c_float * 9), ("cam_from", ctypes.c_float * 3),
        ("ndc_kx", ctypes.c_double), ("ndc_ky", ctypes.c_double),
        ("ao_angle_max", ctypes.c_float),
        ("row_begin", ctypes.c_int32), ("row_end", ctypes.c_int32), ("row_step", ctypes.c_int32),
    ]


class RenderStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls")] + \
        [(n, ctypes.c_double) for n in ("ms_count", "ms_scan", "ms_render", "ms_total")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class Prim(ctypes.Structure):
    _fields_ = [("p0", ctypes.c_float * 3), ("d", ctypes.c_float), ("p1", ctypes.c_float * 3),
                ("area", ctypes.c_float), ("p2", ctypes.c_float * 3), ("kind", ctypes.c_int32),
                ("nrm", ctypes.c_float * 3), ("shape", ctypes.c_int32)]


class SceneSoa(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("n_prims", ctypes.c_int32),
                ("prims", ctypes.POINTER(Prim)), ("shade", ctypes.c_void_p),
                ("n_materials", ctypes.c_int32), ("materials", ctypes.c_void_p),
                ("n_lights", ctypes.c_int32), ("lights", ctypes.c_void_p)]


# (name, restype, argtypes) of every symbol in include/rt580.h
SIGNATURES = [
    ("rt_gpu_init", ctypes.c_int, [ctypes.c_int]),
    ("rt_gpu_upload_scene", ctypes.c_int, [ctypes.POINTER(SceneSoa)]),
    ("rt_gpu_scene_id", ctypes.c_uint64, []),
    ("rt_gpu_set_stream", ctypes.c_int, [ctypes.c_void_p]),
    ("rt_gpu_own_stream", ctypes.c_void_p, []),
    ("rt_gpu_render", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p]),
    ("rt_gpu_render_device", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.POINTER(ctypes.c_void_p)]),
    ("rt_gpu_render_async", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p]),
    ("rt_gpu_render_async_ppm", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p]),
    ("rt_gpu_count_rows", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p]),
    ("rt_gpu_shade_rows", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_void_p]),
    ("rt_gpu_last_stats", ctypes.c_int, [ctypes.POINTER(RenderStats)]),
    ("rt_gpu_profile", ctypes.c_int, [ctypes.c_int]),
    ("rt_gpu_profile_read", ctypes.c_int, [ctypes.POINTER(ctypes.c_double)] * 4 + [ctypes.POINTER(ctypes.c_int)]),
    ("rt_gpu_profile_ao_kernel", ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                                 ctypes.POINTER(ctypes.c_uint64)]),
    ("rt_gpu_set_accel", ctypes.c_int, [ctypes.c_int]),
    ("rt_gpu_render_multi", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p]),
    ("rt_gpu_render_multi_async", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_int,
                                                  ctypes.c_void_p]),
    ("rt_gpu_deinterleave_ppm", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_void_p, ctypes.c_void_p]),
    ("rt_gpu_shade_rows_ppm", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p]),
    ("rt_gpu_rank_unique_id", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    ("rt_gpu_rank_init", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]),
    ("rt_gpu_render_rank_async", ctypes.c_int, [ctypes.POINTER(RenderParams), ctypes.c_void_p]),
    ("rt_gpu_rank_share_body", ctypes.c_int, [ctypes.c_int]),
    ("rt_gpu_rank_finish", ctypes.c_int, []),
    ("rt_gpu_rank_shutdown", ctypes.c_int, []),
    ("rt580_rank_rehearse", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("rt_gpu_device_count", ctypes.c_int, []),
    ("rt_gpu_gamma_u8", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    ("rt_gpu_row_bases", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p]),
    ("rt_gpu_accel_active", ctypes.c_int, []),
    ("rt580_set_chunk_log2", ctypes.c_int, [ctypes.c_int]),
    ("rt580_set_ao_order", ctypes.c_int, [ctypes.c_int]),
    ("rt_gpu_host_register", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    ("rt_gpu_host_unregister", ctypes.c_int, [ctypes.c_void_p]),
    ("rt580_selftest_math", ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    ("rt580_eval_powf", ctypes.c_int, [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_uint64]),
    ("rt_gpu_last_error", ctypes.c_char_p, []),
    ("rt_gpu_synchronize", ctypes.c_int, []),
    ("rt_gpu_copy_to_host", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    ("rt_gpu_shutdown", None, []),
    ("rt580_create", ctypes.c_void_p, [ctypes.c_int, ctypes.c_int]),
    ("rt580_destroy", None, [ctypes.c_void_p]),
    ("rt580_set_assets_root", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    ("rt580_load_scene_json", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    ("rt580_initialize_renderer", ctypes.c_int, [ctypes.c_void_p]),
    ("rt580_render", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    ("rt580_flush_ppm", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    ("rt580_set_depth", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("rt580_set_ao", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    ("rt580_set_rng", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("rt580_set_rows", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    ("rt580_set_gpus", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("rt580_framebuffer", ctypes.POINTER(ctypes.c_int16), [ctypes.c_void_p]),
    ("rt580_get_render_params", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(RenderParams)]),
    ("rt580_get_scene", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(SceneSoa)]),
    ("rt580_last_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(RenderStats)]),
]

_lib = None


def copy_to_host(device_ptr, nbytes, dtype):
    """Copy nbytes from a device pointer the library handed out (e.g.
    rt_gpu_render_device's framebuffer) into a new numpy array of dtype, after
    the work queued on the shim's stream (rt_gpu_copy_to_host: staged through
    the library's pinned buffer)."""
    import numpy as np
    out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype=dtype)
    check(load().rt_gpu_copy_to_host(out.ctypes.data, device_ptr, nbytes), "rt_gpu_copy_to_host")
    return out


def _preload_torch_hip_runtime():
    """PyTorch-ROCm wheels bundle their own libamdhip64.so and librccl.so. A
    process must hold ONE HIP runtime (device pointers, streams and events are
    runtime objects) and one RCCL: lib580rt.so loaded first would bind
    /opt/rocm's copies, and a later `import torch` would add its own (two
    RCCLs tear each other's state down at exit: "double free or corruption";
    preloading torch's two libraries by path before torch does not avoid it
    either). So when torch is installed it is imported first: lib580rt.so's
    libamdhip64.so.7 and its dlopen("librccl.so.1") then bind to torch's
    copies (same SONAMEs). Without torch, /opt/rocm's are used."""
    import importlib.util
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def load(path=None):
    """Load lib580rt.so (built by `make -C 580-raytracer_amd`); raise if absent.
    $RT580_LIB selects another build (the diagnostic timing library, A/B only)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("RT580_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError("lib580rt.so not built (%s); run __graft_entry__.build()" % path)
    _preload_torch_hip_runtime()
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(status, what=""):
    if status != RT_SUCCESS:
        msg = load().rt_gpu_last_error()
        raise RuntimeError("%s failed with status %d: %s" % (what, status, msg.decode() if msg else ""))


class Raytracer:
    """The reference's class surface (Raytracer.h:572-588) over the C ABI."""

    def __init__(self, width, height, assets_root="."):
        self.lib = load()
        self.width, self.height = width, height
        self.h = self.lib.rt580_create(width, height)
        if not self.h:
            raise RuntimeError("rt580_create failed")
        self.lib.rt580_set_assets_root(self.h, os.fsencode(assets_root))

    def close(self):
        if self.h:
            self.lib.rt580_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def LoadSceneJSON(self, path):
        return self.lib.rt580_load_scene_json(self.h, os.fsencode(path))

    def InitializeRenderer(self):
        return self.lib.rt580_initialize_renderer(self.h)

    def Render(self, output_name=""):
        return self.lib.rt580_render(self.h, os.fsencode(output_name))

    def FlushFrameBufferToPPM(self, output_name):
        return self.lib.rt580_flush_ppm(self.h, os.fsencode(output_name))

    def set_depth(self, d):
        check(self.lib.rt580_set_depth(self.h, d), "set_depth")

    def set_ao(self, samples, enabled=True):
        check(self.lib.rt580_set_ao(self.h, samples, int(bool(enabled))), "set_ao")

    def set_rng(self, engine):
        check(self.lib.rt580_set_rng(self.h, engine), "set_rng")

    def set_rows(self, row_begin, row_end):
        check(self.lib.rt580_set_rows(self.h, row_begin, row_end), "set_rows")

    def set_gpus(self, n):
        check(self.lib.rt580_set_gpus(self.h, n), "set_gpus")

    def framebuffer(self):
        """Pixel[w*h] as a (h, w, 3) int16 numpy array (copy)."""
        import numpy as np
        ptr = self.lib.rt580_framebuffer(self.h)
        n = self.width * self.height * 3
        return np.ctypeslib.as_array(ptr, shape=(n,)).copy().reshape(self.height, self.width, 3)

    def render_params(self):
        p = RenderParams()
        check(self.lib.rt580_get_render_params(self.h, ctypes.byref(p)), "get_render_params")
        return p

    def scene(self):
        s = SceneSoa()
        check(self.lib.rt580_get_scene(self.h, ctypes.byref(s)), "get_scene")
        return s

    def stats(self):
        s = RenderStats()
        check(self.lib.rt580_last_stats(self.h, ctypes.byref(s)), "last_stats")
        return s.as_dict()


_GAMMA_LUT = None


def gamma_lut():
    """(unsigned char)(powf(c/255.0f, 1.0f/2.2f)*255.0f) for c in 0..255 with
    this machine's glibc powf (FlushFrameBufferToPPM, Raytracer.cpp:816-818)."""
    global _GAMMA_LUT
    if _GAMMA_LUT is None:
        import numpy as np
        libm = ctypes.CDLL("libm.so.6")
        libm.powf.restype = ctypes.c_float
        libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
        e = np.float32(1.0) / np.float32(2.2)
        lut = []
        for c in range(256):
            v = np.float32(libm.powf(float(np.float32(c) / np.float32(255.0)), float(e))) * np.float32(255.0)
            lut.append(int(np.float32(v)))
        _GAMMA_LUT = np.array(lut, dtype=np.uint8)
    return _GAMMA_LUT


def ppm_bytes(fb):
    """P6 bytes of an int16 (h, w, 3) framebuffer exactly as the reference's
    FlushFrameBufferToPPM writes them (pixels are clamped to [0, 255])."""
    import numpy as np
    h, w, _ = fb.shape
    fb = np.asarray(fb)
    if fb.min() < 0 or fb.max() > 255:
        raise ValueError("framebuffer outside [0,255]")
    body = gamma_lut()[fb.astype(np.int64)].astype(np.uint8).tobytes()
    return b"P6\n%d %d\n255\n" % (w, h) + body
