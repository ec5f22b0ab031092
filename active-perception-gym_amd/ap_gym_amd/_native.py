"""Bindings of the gfx950 C ABI (include/apgym_capi.h) in _lib/libapgym_hip.so.

* `lib()` — ctypes over every entry point (setup, tests, render, utility calls);
* `torch_ops()` — the TORCH_LIBRARY(apgym) custom ops of _lib/libapgym_torch.so
  (csrc/apg_torch_ops.cpp), which the envs' reset/step hot path calls: one C++ op call per step,
  launched on PyTorch's current HIP stream (CUDA-graph capturable);
* `fast()` — METH_FASTCALL wrappers of the per-step C-ABI calls (_lib/_apgfast*.so, csrc/apg_pyfast.cpp) that the
  envs' eager steps use: ~0.1 us per call instead of ctypes' ~2.5 us of argument marshalling.

The library is the ONLY compute path of this package: there is no CPU fallback.  Both loaders raise
NativeLibraryError when their shared object is missing or cannot be loaded.
"""

from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "_lib")
LIB_PATH = os.environ.get("APG_LIBRARY") or os.path.join(LIB_DIR, "libapgym_hip.so")  # override: tuning builds
TORCH_LIB_PATH = os.path.join(LIB_DIR, "libapgym_torch.so")

APG_OK = 0
APG_E_INVALID = -1  # apgym_capi.h: invalid argument / configuration (raised as ValueError)
APG_ERR_NAN_ACTION = 1
APG_ERR_NAN_PREDICTION = 2
APG_ERR_MAPGEN = 4
APG_ERR_OOB_Y = 8
APG_ERR_OOB_X = 16
APG_ERR_PREFETCH = 32
APG_ERR_NO_FREE_CELL = 64
APG_MAP_ROOMS = 0
APG_MAP_MAZE = 1
APG_MAP_POOL = 2
APG_DRAW_UNIFORM = 0
APG_DRAW_INTEGERS = 1
APG_IMAGE_CLASSIFY = 0
APG_IMAGE_LOCALIZE = 1
APG_POOL_U8 = 0
APG_POOL_F32 = 1
APG_POOL_U8_TILED = 2  # RGBX in 8 x 4-pixel 128-byte tiles (apgym_capi.h)
APG_U8_POOL_PAD = 16  # readable bytes after a u8 image pool (apgym_capi.h)
APG_DS_CIRCLE_SQUARE = 0
APG_DS_DOUBLE_CIRCLE_SQUARE = 1


class NativeLibraryError(RuntimeError):
    pass


class ApgError(RuntimeError):
    pass


_vp = ctypes.c_void_p


class Pcg64(ctypes.Structure):
    _fields_ = [("state_hi", ctypes.c_uint64), ("state_lo", ctypes.c_uint64), ("inc_hi", ctypes.c_uint64),
                ("inc_lo", ctypes.c_uint64), ("has_uint32", ctypes.c_uint32), ("uinteger", ctypes.c_uint32)]


class LidarConfig(ctypes.Structure):
    _fields_ = [("num_envs", ctypes.c_int32), ("height", ctypes.c_int32), ("width", ctypes.c_int32),
                ("map_kind", ctypes.c_int32), ("is_static", ctypes.c_int32), ("static_map_index", ctypes.c_int32),
                ("beams", ctypes.c_int32), ("step_limit", ctypes.c_int32), ("max_rooms", ctypes.c_int32),
                ("door_width", ctypes.c_int32), ("lidar_range", ctypes.c_float), ("loss_scale", ctypes.c_float),
                ("loss_offset", ctypes.c_float), ("branching_prob", ctypes.c_double), ("log_stats", ctypes.c_int32),
                ("sparse", ctypes.c_int32), ("out_row_bytes", ctypes.c_int32), ("pool_len", ctypes.c_int32),
                ("stream_len", ctypes.c_int64)]


class LidarState(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("pos", "init_pos", "elapsed", "flags", "rng", "it_rng", "occ", "scratch", "stack",
                                   "map_idx", "beam_dirs", "stats_hist", "prefetch", "prefetcher", "pool_occ",
                                   "pool_free")]


class LidarOutputs(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("lidar", "odometry", "time_step", "map_obs", "reward", "terminated", "truncated",
                                   "base_reward", "target", "loss", "info_mask", "map_idx", "reset_mask", "err",
                                   "stats", "stats_len", "weight")]


class LidarRenderState(ctypes.Structure):
    _fields_ = [("num_tracked", ctypes.c_int32), ("scan_points", ctypes.c_int32)] + [
        (n, _vp) for n in ("env", "scan_xy", "scan_norm", "obs_map", "traj", "traj_len", "pose", "has_last",
                           "lidar_dist")]


class LidarSizes(ctypes.Structure):
    _fields_ = [("occ_bytes", ctypes.c_size_t), ("scratch_bytes", ctypes.c_size_t),
                ("stack_bytes", ctypes.c_size_t), ("wpr", ctypes.c_int32), ("maze_frames", ctypes.c_int32),
                ("prefetch_bytes", ctypes.c_size_t)]


class ImageConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("num_envs", "kind", "height", "width", "pool_channels", "channels",
                                              "pool_dtype", "sensor_h", "sensor_w", "step_limit", "num_classes",
                                              "invert_labels", "top_k", "unique_points", "num_envs_total",
                                              "env_offset")] + [
        ("pool_len", ctypes.c_int64), ("sensor_scale", ctypes.c_double), ("max_step", ctypes.c_double * 2),
        ("cell", ctypes.c_double * 2), ("ce_scale", ctypes.c_double), ("ce_offset", ctypes.c_double),
        ("mse_scale", ctypes.c_float), ("mse_offset", ctypes.c_float), ("log_stats", ctypes.c_int32),
        ("sparse", ctypes.c_int32), ("out_row_bytes", ctypes.c_int32)]


class ImageState(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("pool", "pool_labels", "unique_grid", "index", "label", "inverted", "pos",
                                   "target", "rng", "scratch_i64", "scratch_f64", "top_k", "rng_work",
                                   "stats_hist", "ahead_i64", "ahead_f64", "rng_saved")]


class ImageOutputs(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("glimpse", "glimpse_pos", "time_step", "target_glimpse", "reward", "base_reward",
                                   "target", "label_target", "loss_f64", "loss_f32", "err", "stats",
                                   "stats_idx")]


class CircleSquareConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("kind", "height", "width", "show_gradient_a", "show_gradient_b",
                                              "pad_")] + [
        ("num_positions", ctypes.c_int64), ("half_extent", ctypes.c_double), ("max_dist", ctypes.c_double)]


class HideAndSeekArgs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("num_envs", "height", "width", "resetting", "terminated",
                                              "mask_prediction", "sparse", "pad_")] + [
        ("lim", ctypes.c_double * 2)] + [(n, _vp) for n in ("index", "glimpse_pos", "base_reward_in", "reward_in",
                                                              "loss", "base_reward_out", "reward_out", "additional")]


class LightDarkConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("num_envs", "step_limit", "log_stats", "sparse")] + [
        ("loss_scale", ctypes.c_float), ("loss_offset", ctypes.c_float)]


class LightDarkState(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("pos", "elapsed", "flags", "rng", "stats_hist")]


class LightDarkOutputs(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("noisy_position", "time_step", "reward", "terminated", "truncated", "base_reward",
                                   "target", "loss", "info_mask", "reset_mask", "err", "stats", "stats_len",
                                   "weight")]


# (name, restype, argtypes) for every symbol declared in include/apgym_capi.h
SYMBOLS = [
    ("apg_version", ctypes.c_char_p, []),
    ("apg_last_error", ctypes.c_char_p, []),
    ("apg_lidar_query_sizes", ctypes.c_int, [ctypes.POINTER(LidarConfig), ctypes.POINTER(LidarSizes)]),
    ("apg_lidar_init", ctypes.c_int, [ctypes.POINTER(LidarConfig), ctypes.POINTER(LidarState), _vp]),
    ("apg_lidar_reset", ctypes.c_int, [ctypes.POINTER(LidarConfig), ctypes.POINTER(LidarState), ctypes.c_uint64,
                                       ctypes.c_int, ctypes.POINTER(LidarOutputs), _vp]),
    ("apg_lidar_step", ctypes.c_int, [ctypes.POINTER(LidarConfig), ctypes.POINTER(LidarState), _vp, _vp,
                                      ctypes.POINTER(LidarOutputs), _vp]),
    ("apg_lidar_step_profiled", ctypes.c_int, [ctypes.POINTER(LidarConfig), ctypes.POINTER(LidarState), _vp, _vp,
                                               ctypes.POINTER(LidarOutputs), _vp, _vp, _vp]),
    ("apg_lidar_prefetcher_create", ctypes.c_int, [ctypes.POINTER(LidarConfig), ctypes.POINTER(_vp)]),
    ("apg_lidar_prefetcher_destroy", ctypes.c_int, [_vp]),
    ("apg_lidar_prefetcher_stats", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64)]),
    ("apg_lidar_peek_map_index", ctypes.c_int, [ctypes.POINTER(LidarConfig), ctypes.POINTER(LidarState),
                                                ctypes.c_uint64, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    ("apg_maze_frames", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("apg_map_generate", ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_double, _vp, _vp, _vp, _vp, _vp]),
    ("apg_lidar_scan_batch", ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int, _vp, _vp,
                                            _vp]),
    ("apg_lidar_render_track", ctypes.c_int, [ctypes.POINTER(LidarConfig), ctypes.POINTER(LidarState), _vp,
                                              ctypes.POINTER(LidarOutputs), ctypes.POINTER(LidarRenderState), _vp]),
    ("apg_rng_draws", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                     _vp, _vp]),
    ("apg_rng_fill_work_elems", ctypes.c_int64, [ctypes.c_int64, ctypes.c_uint64]),
    ("apg_rng_fill", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int, _vp, _vp, ctypes.c_int64,
                                    ctypes.c_uint64, _vp, _vp, _vp]),
    ("apg_image_seed", ctypes.c_int, [ctypes.POINTER(ImageConfig), ctypes.POINTER(ImageState), ctypes.c_uint64,
                                      _vp]),
    ("apg_image_reset", ctypes.c_int, [ctypes.POINTER(ImageConfig), ctypes.POINTER(ImageState),
                                       ctypes.POINTER(ImageOutputs), _vp]),
    ("apg_image_step", ctypes.c_int, [ctypes.POINTER(ImageConfig), ctypes.POINTER(ImageState), _vp, _vp,
                                      ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ImageOutputs), _vp]),
    ("apg_image_draw_ahead", ctypes.c_int, [ctypes.POINTER(ImageConfig), ctypes.POINTER(ImageState), _vp]),
    ("apg_image_discard_ahead", ctypes.c_int, [ctypes.POINTER(ImageConfig), ctypes.POINTER(ImageState), _vp]),
    ("apg_image_glimpse", ctypes.c_int, [ctypes.POINTER(ImageConfig), _vp, _vp, _vp, ctypes.c_int, ctypes.c_int32,
                                         _vp, _vp, _vp]),
    ("apg_image_unique_top_k", ctypes.c_int, [ctypes.POINTER(ImageConfig), _vp, _vp, _vp, ctypes.c_int32,
                                              ctypes.c_int32, _vp, _vp, _vp]),
    ("apg_loss_ce", ctypes.c_int, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double, _vp,
                                   _vp]),
    ("apg_loss_mse", ctypes.c_int, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_float, _vp,
                                    _vp]),
    ("apg_circle_square_pool", ctypes.c_int, [ctypes.POINTER(CircleSquareConfig), _vp, ctypes.c_int64,
                                              ctypes.c_int64, _vp, _vp, _vp]),
    ("apg_hide_and_seek_reward", ctypes.c_int, [ctypes.POINTER(HideAndSeekArgs), _vp]),
    ("apg_light_dark_reset", ctypes.c_int, [ctypes.POINTER(LightDarkConfig), ctypes.POINTER(LightDarkState),
                                            ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(LightDarkOutputs), _vp]),
    ("apg_light_dark_step", ctypes.c_int, [ctypes.POINTER(LightDarkConfig), ctypes.POINTER(LightDarkState), _vp, _vp,
                                           ctypes.POINTER(LightDarkOutputs), _vp]),
    ("apg_standard_normal_draws", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _vp]),
]

_lib = None


def lib():
    """Load the native library (raises NativeLibraryError if it is absent: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). ap_gym_amd has no CPU fallback.")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the ROCm runtime
            raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, res, args in SYMBOLS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


_fast = None


def fast():
    """The CPython fast-call entry points of the per-step C-ABI calls (_lib/_apgfast*.so, csrc/apg_pyfast.cpp:
    ~0.1 us per call against ~2.5 us through ctypes), loaded after the C-ABI library it links.  Raises when it is
    missing, like lib()."""
    global _fast
    if _fast is None:
        import importlib.machinery
        import importlib.util
        import sysconfig

        lib()  # (an APG_LIBRARY variant, loaded first, also serves this module's libapgym_hip.so dependency)
        path = os.path.join(LIB_DIR, "_apgfast" + sysconfig.get_config_var("EXT_SUFFIX"))
        if not os.path.exists(path):
            raise NativeLibraryError(f"{path} not found: build it with "
                                     "`python -c 'import __graft_entry__ as g; g.build()'`")
        loader = importlib.machinery.ExtensionFileLoader("_apgfast", path)
        spec = importlib.util.spec_from_file_location("_apgfast", path, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _fast = mod
    return _fast


def addr(obj) -> int:
    """Address of a ctypes structure (the fast-call entry points take plain ints)."""
    return ctypes.addressof(obj)


_torch_ops = None


def torch_ops():
    """torch.ops.apgym (loads _lib/libapgym_torch.so once, after the C-ABI library it links)."""
    global _torch_ops
    if _torch_ops is None:
        import torch

        lib()  # the ops library resolves libapgym_hip.so through its rpath; load (and check) it first
        if not os.path.exists(TORCH_LIB_PATH):
            raise NativeLibraryError(f"{TORCH_LIB_PATH} not found: build it with "
                                     "`python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            torch.ops.load_library(TORCH_LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the ROCm runtime
            raise NativeLibraryError(f"cannot load {TORCH_LIB_PATH}: {e}") from e
        _torch_ops = torch.ops.apgym
    return _torch_ops


def exact_device(device):
    """`device` with its index filled in (tensors report cuda:0, never a bare cuda)."""
    import torch

    if device.type == "cuda" and device.index is None:
        return torch.device("cuda", torch.cuda.current_device())
    return device


def as_device_f32(x, dev, numel: int, shape=None, name: str = "input"):
    """`x` as a contiguous float32 tensor on `dev` (an exact_device): `x` itself when it already is one
    with `numel` elements (the step hot path: no tensor constructions), else converted.  The size is
    checked here because the C ABI takes raw pointers (the torch ops check it in check_io)."""
    import torch

    if (type(x) is torch.Tensor and x.dtype is torch.float32 and x.device == dev and x.is_contiguous()
            and x.numel() == numel):
        return x
    t = torch.as_tensor(x, dtype=torch.float32, device=dev)
    t = (t if shape is None or t.numel() != numel else t.reshape(shape)).contiguous()
    if t.numel() != numel:
        raise RuntimeError(f"{name} must have {numel} elements, got {t.numel()}")
    return t


def wrong_current_device(dev) -> bool:
    """True when HIP's current device is not `dev` (an exact_device): direct C-ABI launches run on the
    current device."""
    import torch

    return torch._C._cuda_getDevice() != dev.index


def current_stream_ptr(dev) -> int:
    """Raw HIP stream of torch's current stream on `dev` (an exact_device), the stream the torch ops use."""
    import torch

    return torch._C._cuda_getCurrentRawStream(dev.index)


def op_buffers(tensors, device):
    """Buffer list for an env handle: None -> a 0-element tensor (NULL in the C struct)."""
    import torch

    empty = torch.empty(0, dtype=torch.uint8, device=device)
    return [empty if t is None else t for t in tensors]


def check(rc: int, what: str = "apg call") -> None:
    if rc != APG_OK:
        msg = lib().apg_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        raise ApgError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_handle(device) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


_hip = None


def hip():
    """The HIP runtime torch already loaded (ctypes: the event calls below)."""
    global _hip
    if _hip is None:
        h = ctypes.CDLL("libamdhip64.so")
        h.hipEventRecord.argtypes = [_vp, _vp]
        h.hipEventRecord.restype = ctypes.c_int
        h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(_vp), ctypes.c_uint]
        h.hipEventCreateWithFlags.restype = ctypes.c_int
        h.hipStreamWaitEvent.argtypes = [_vp, _vp, ctypes.c_uint]
        h.hipStreamWaitEvent.restype = ctypes.c_int
        h.hipEventDestroy.argtypes = [_vp]
        h.hipEventDestroy.restype = ctypes.c_int
        _hip = h
    return _hip


def event_record(event, stream) -> None:
    """hipEventRecord(event, stream) through the HIP runtime torch already loaded (bench timing of
    the step op on its own stream; torch.cuda.Event would only see torch's current stream object)."""
    if hip().hipEventRecord(event, stream) != 0:
        raise ApgError("hipEventRecord failed")


class DeviceEvent:
    """A hipEvent for ordering two streams of one device (no timing, no host inspection): recorded with a
    device-scope release (hipEventReleaseToDevice), so the marker skips the system-scope cache writeback a
    default event (torch.cuda.Event) pays on every record -- measured as a ~6-8 us idle gap on the recording
    stream after the image env's batch-autoreset step.  record(stream) / wait(stream) take raw HIP streams."""

    FLAGS = 0x2 | 0x40000000  # hipEventDisableTiming | hipEventReleaseToDevice

    def __init__(self):
        ev = _vp()
        if hip().hipEventCreateWithFlags(ctypes.byref(ev), self.FLAGS) != 0:
            raise ApgError("hipEventCreateWithFlags failed")
        self.handle = ev.value

    def record(self, stream: int) -> None:
        if _hip.hipEventRecord(self.handle, stream) != 0:
            raise ApgError("hipEventRecord failed")

    def wait(self, stream: int) -> None:
        """The stream's later work waits for the last record (none yet: no wait)."""
        if _hip.hipStreamWaitEvent(stream, self.handle, 0) != 0:
            raise ApgError("hipStreamWaitEvent failed")

    def destroy(self) -> None:
        if self.handle is not None:
            _hip.hipEventDestroy(self.handle)
            self.handle = None
