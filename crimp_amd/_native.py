"""ctypes binding of libcrimp_hip.so (include/crimp_hip.h).

The shipped path has no CPU fallback: if the library is missing, cannot be
loaded, or no HIP device is visible, every hot-path call raises
``CrimpNativeError``. Buffers may be NumPy arrays (host; the library stages them)
or torch CUDA tensors (device; passed by pointer on torch's current stream).
"""
import contextlib
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CRIMP_LIB=<path> loads another build of the library (A/B measurements of kernel builds)
LIB_PATH = os.environ.get("CRIMP_LIB") or os.path.join(_HERE, "lib", "libcrimp_hip.so")

FLAG_DEVICE_PTRS = 1
FLAG_SYNC = 2
FLAG_FORCE_MFMA = 8
FLAG_TIME_KERNELS = 128
FLAG_F64 = 256
FLAG_NO_FIXUP = 1024
FLAG_ASYNC = 2048
FLAG_NUFFT = 4096
FLAG_EXACT = 8192
FLAG_TIME_DAYS = 16384
FLAG_FOLD_RADIANS = 32768

STAT_Z2 = 0
STAT_H = 1

MODEL_IDS = {"fourier": 0, "cauchy": 1, "vonmises": 2}
MAX_GLITCH = 32
MAX_WAVE = 64
MAX_COMP = 16


class CrimpNativeError(RuntimeError):
    """Raised when the HIP library is unavailable or a native call fails."""


class TimingModel(ctypes.Structure):
    _fields_ = [("pepoch", ctypes.c_double), ("f", ctypes.c_double * 13), ("n_glitch", ctypes.c_int32),
                ("glitch", (ctypes.c_double * 7) * MAX_GLITCH), ("n_wave", ctypes.c_int32),
                ("wave_epoch", ctypes.c_double), ("wave_om", ctypes.c_double),
                ("wave_ab", (ctypes.c_double * 2) * MAX_WAVE)]


SHAPE_SUMS = 4 + 3 * MAX_COMP  # CRIMP_SHAPE_SUMS


class Template(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int32), ("ncomp", ctypes.c_int32), ("amp", ctypes.c_double * MAX_COMP),
                ("loc", ctypes.c_double * MAX_COMP), ("wid", ctypes.c_double * MAX_COMP),
                ("i0", ctypes.c_double * MAX_COMP), ("amp_shift", ctypes.c_double)]


EXPORTS = ("crimp_version", "crimp_last_error", "crimp_last_kernel_ms", "crimp_last_kernel_times", "crimp_last_fixups",
           "crimp_last_search_path", "crimp_last_nufft_plan", "crimp_last_nufft_work", "crimp_last_toa_grid_norms", "crimp_last_toa_grid_fast", "crimp_release_scratch",
           "crimp_device_count", "crimp_calcphase", "crimp_search", "crimp_search_best", "crimp_best", "crimp_search_sets", "crimp_toa_points",
           "crimp_toa_grid", "crimp_toa_fit", "crimp_toa_redchi2", "crimp_toa_fit_redchi2", "crimp_toa_shape_points", "crimp_binphases",
           "crimp_is_sorted", "crimp_select_intervals", "crimp_gather_ranges")

_lib = None
_lock = threading.Lock()
_dev_ok = None


def load(require_device=True):
    """Load the library (and, by default, insist on a visible HIP device)."""
    global _lib, _dev_ok
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise CrimpNativeError("libcrimp_hip.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
            try:
                L = ctypes.CDLL(LIB_PATH)
            except OSError as e:  # pragma: no cover - environment specific
                raise CrimpNativeError("cannot load %s: %s" % (LIB_PATH, e))
            P = ctypes.c_void_p
            i64, i32, u32 = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32
            L.crimp_version.restype = ctypes.c_int
            L.crimp_last_error.restype = ctypes.c_char_p
            L.crimp_last_kernel_ms.restype = ctypes.c_double
            L.crimp_last_fixups.restype = ctypes.c_int64
            L.crimp_last_toa_grid_norms.restype = ctypes.c_int64
            L.crimp_last_toa_grid_fast.restype = ctypes.c_int64
            L.crimp_last_kernel_times.argtypes = [ctypes.POINTER(ctypes.c_double), i32]
            L.crimp_last_nufft_plan.argtypes = [ctypes.POINTER(i64), ctypes.POINTER(i32), ctypes.POINTER(i32)]
            L.crimp_last_nufft_work.argtypes = [ctypes.POINTER(ctypes.c_double), i32]
            L.crimp_device_count.argtypes = [ctypes.POINTER(i32)]
            L.crimp_calcphase.argtypes = [P, i64, ctypes.POINTER(TimingModel), i32, P, P, u32, P]
            L.crimp_search.argtypes = [P, i64, ctypes.c_double, P, i64, P, i64, i32, i32, i64, i64, P, u32, P]
            L.crimp_search_sets.argtypes = [P, P, i64, P, i32, i32, P, u32, P]
            L.crimp_best.argtypes = [P, i64, P, u32, P]
            L.crimp_search_best.argtypes = [P, i64, ctypes.c_double, P, i64, P, i64, i32, i32, i64, i64, P, P, u32, P]
            L.crimp_toa_points.argtypes = [P, P, i64, ctypes.POINTER(Template), P, P, P, i64, P, u32, P]
            L.crimp_toa_grid.argtypes = [P, P, i64, ctypes.POINTER(Template), P, i64, P, i64, P, P, u32, P]
            L.crimp_toa_fit.argtypes = [P, P, i64, ctypes.POINTER(Template), P, ctypes.c_double, i32, i32, P, u32, P]
            L.crimp_toa_shape_points.argtypes = [P, P, i64, ctypes.POINTER(Template), P, P, P, P, i64, P, u32, P]
            L.crimp_binphases.argtypes = [P, P, i64, P, i32, P, u32, P]
            L.crimp_is_sorted.argtypes = [P, i64, ctypes.POINTER(i32), u32, P]
            L.crimp_select_intervals.argtypes = [P, i64, P, P, i64, P, P, P, u32, P]
            L.crimp_gather_ranges.argtypes = [P, i64, P, P, i64, P, u32, P]
            L.crimp_toa_redchi2.argtypes = [P, P, i64, ctypes.POINTER(Template), P, P, P, P, i32, i32, P, u32, P]
            L.crimp_toa_fit_redchi2.argtypes = [P, P, i64, ctypes.POINTER(Template), P, ctypes.c_double, i32, i32, P, P,
                                                i32, i32, P, P, u32, P]
            for name in EXPORTS:
                if name not in ("crimp_last_error", "crimp_last_kernel_ms", "crimp_last_fixups",
                                "crimp_last_toa_grid_norms", "crimp_last_toa_grid_fast"):
                    getattr(L, name).restype = ctypes.c_int
            _lib = L
        if require_device and not _dev_ok:
            n = ctypes.c_int32(0)
            _lib.crimp_device_count(ctypes.byref(n))
            if n.value < 1:
                raise CrimpNativeError("no HIP device visible: the CRIMP hot path runs only on the GPU "
                                       "(there is no CPU fallback)")
            _dev_ok = True
    return _lib


def last_nufft_plan():
    """(FFT length, moments, spread form: 'gather' | 'mfma') of the last NUFFT search (crimp_last_nufft_plan)."""
    L = load(require_device=False)
    n, p, g = ctypes.c_int64(0), ctypes.c_int32(0), ctypes.c_int32(0)
    L.crimp_last_nufft_plan(ctypes.byref(n), ctypes.byref(p), ctypes.byref(g))
    return int(n.value), int(p.value), "gather" if g.value else "mfma"


def last_nufft_work():
    """The last NUFFT search's algorithmic work (crimp_last_nufft_work): the spread's fp64 flops and the HBM bytes of
    each kernel class."""
    L = load(require_device=False)
    w = (ctypes.c_double * 7)()
    L.crimp_last_nufft_work(w, 7)
    return {"spread_flops": w[0], "spread_bytes": w[1], "merge_bytes": w[2], "pass1_bytes": w[3], "pass2_bytes": w[4],
            "combine_bytes": w[5], "finalize_bytes": w[6]}


NUFFT_CLASSES = ("cellstart", "spread", "merge", "pass1", "pass2", "combine", "finalize")


def last_kernel_times():
    """Every timed span (ms) of the last native call made with FLAG_TIME_KERNELS (crimp_last_kernel_times)."""
    L = load(require_device=False)
    buf = (ctypes.c_double * 64)()
    n = L.crimp_last_kernel_times(buf, 64)
    return [buf[i] for i in range(min(n, 64))]


def check(rc):
    if rc != 0:
        msg = _lib.crimp_last_error().decode(errors="replace") if _lib is not None else "library not loaded"
        raise CrimpNativeError("libcrimp_hip: %s (status %d)" % (msg, rc))


# ------------------------------------------------------------------ buffer helpers
def _is_torch(a):
    return type(a).__module__.startswith("torch") and hasattr(a, "data_ptr")


class Buffers:
    """Collects the pointers for one call; all-host or all-device (torch CUDA) arrays. Device tensors must all
    live on one GPU: the call runs with that GPU current (``device_guard``) on its current torch stream."""

    def __init__(self):
        self.keep = []
        self.device = None
        self.tdev = None

    def arg(self, a, dtype, writable=False, allow_none=False):
        if a is None:
            if allow_none:
                return None
            raise ValueError("missing array argument")
        if _is_torch(a):
            import torch
            if not a.is_cuda:
                a = a.cpu().numpy()
            else:
                tdt = {np.float64: torch.float64, np.int64: torch.int64}[np.dtype(dtype).type]
                if a.dtype != tdt or not a.is_contiguous():
                    if writable:
                        raise ValueError("output tensors must be contiguous %s" % tdt)
                    a = a.to(tdt).contiguous()
                self._mode(True)
                if self.tdev is None:
                    self.tdev = a.device
                elif a.device != self.tdev:
                    raise ValueError("device tensors of one call must be on one GPU (%s and %s)" % (self.tdev, a.device))
                self.keep.append(a)
                return ctypes.c_void_p(a.data_ptr())
        arr = np.asarray(a)
        if writable:
            if arr.dtype != dtype or not arr.flags.c_contiguous or not arr.flags.writeable:
                raise ValueError("output arrays must be writable C-contiguous %s" % np.dtype(dtype))
        else:
            arr = np.ascontiguousarray(arr, dtype=dtype)
        self._mode(False)
        self.keep.append(arr)
        return ctypes.c_void_p(arr.ctypes.data)

    def _mode(self, dev):
        if self.device is None:
            self.device = dev
        elif self.device != dev:
            raise ValueError("mix of host arrays and device tensors in one call")

    def flags(self, extra=0):
        return (FLAG_DEVICE_PTRS if self.device else 0) | extra

    def stream(self):
        if self.device:
            import torch
            raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
            if raw is not None and self.tdev.index is not None:  # the handle itself, no Stream object (~2 us less)
                return ctypes.c_void_p(raw(self.tdev.index))
            return ctypes.c_void_p(torch.cuda.current_stream(self.tdev).cuda_stream)
        return None

    def device_guard(self):
        """Context making the tensors' GPU the current HIP device for the native call (the library allocates its
        scratch and launches on the current device); nothing to switch when it already is."""
        if self.device and self.tdev is not None:
            import torch
            if self.tdev.index is not None and torch.cuda.current_device() == self.tdev.index:
                return contextlib.nullcontext()
            return torch.cuda.device(self.tdev)
        return contextlib.nullcontext()
