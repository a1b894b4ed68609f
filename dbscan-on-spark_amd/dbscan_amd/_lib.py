"""ctypes binding of libdbscan_hip.so (the C-ABI declared in include/dbscan_hip.h).

There is deliberately no CPU fallback: if the HIP library is missing or no GPU is visible the
calls raise, so a test that passes has run the gfx950 kernels.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
# DBSCAN_LIB_PATH: an alternative build of the same library (A/B measurements of build options)
LIB_PATH = os.environ.get("DBSCAN_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libdbscan_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "dbscan_hip.h")

DBSCAN_OK, DBSCAN_EARG, DBSCAN_EHIP, DBSCAN_EOOM = 0, -1, -2, -3
MODE_NAIVE, MODE_ARCHERY = 0, 1
# LocalDBSCANArchery with its float32 R-tree search box (LocalDBSCANArchery.scala:38-41,118-124):
# local fits only
MODE_ARCHERY_F32BOX = 2

# (name, restype, argtypes) for every symbol include/dbscan_hip.h declares.
_vp, _i32, _i64, _d, _u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, \
    ctypes.c_uint64
SIGNATURES = [
    ("dbscan_last_error", ctypes.c_char_p, []),
    ("dbscan_version", _i32, []),
    ("dbscan_device_count", _i32, []),
    ("dbscan_create", _vp, [_i32]),
    ("dbscan_destroy", None, [_vp]),
    ("dbscan_fit", _i32, [_vp, _vp, _i64, _d, _i32, _i32, _vp, _vp, _vp]),
    ("dbscan_fit_h", _i32, [_vp, _vp, _vp, _i64, _d, _i32, _i32, _vp, _vp, _vp]),
    ("dbscan_fit_device", _i32, [_vp, _vp, _vp, _i64, _d, _i32, _i32, _vp, _vp, _vp]),
    ("dbscan_fit_device_async", _i32, [_vp, _vp, _vp, _i64, _d, _i32, _i32, _vp, _vp, _vp]),
    ("dbscan_sync", _i32, [_vp]),
    ("dbscan_stream", _vp, [_vp]),
    ("dbscan_set_stream", _i32, [_vp, _vp, _i32]),
    ("dbscan_last_stats", _i32, [_vp, _vp, _i32]),
    ("dbscan_profile_enable", _i32, [_vp, _i32]),
    ("dbscan_profile_only", _i32, [_vp, ctypes.c_char_p]),
    ("dbscan_profile_reset", _i32, [_vp]),
    ("dbscan_profile_read", _i32, [_vp, _vp, _i32, _vp, _vp, _i32]),
    ("dbscan_partition", _i64, [_vp, _vp, _vp, _i64, _d, _i64, _vp, _vp, _i64]),
    ("dbscan_partition_device", _i64, [_vp, _vp, _vp, _i64, _d, _i64, _vp, _vp, _i64]),
    ("dbscan_partition_cells", _i64, [_vp, _vp, _vp, _i64, _i64, _d, _vp, _vp, _i64]),
    ("dbscan_csv_read", _i64, [ctypes.c_char_p, _vp, _vp, _i64]),
    ("dbscan_csv_write", _i32, [ctypes.c_char_p, _vp, _vp, _vp, _i64]),
    ("dbscan_format_double", _i32, [_d, ctypes.c_char_p]),
    ("dbscan_scala_range_count", _i64, [_d, _d, _d, _i32]),
    ("dbscan_train_node", _i32, [_vp, _vp, _i64, _d, _i32, _i32, _i32, _vp, _vp, _vp]),
    ("dbscan_selftest_worker_errors", _i32, [_vp, _i32]),
    ("dbscan_train_node_shards", _i32, [_vp, _vp, _vp, _i32]),
    ("dbscan_selftest_node_plan", _i32, [_i32, _i32, _i32, _vp, _vp]),
    ("dbscan_slab_fit_device", _i32, [_vp, _vp, _vp, _vp, _i64, _d, _i32, _vp, _vp]),
    ("dbscan_slab_label_device", _i32, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp]),
    ("dbscan_slab_fit_device_async", _i32, [_vp, _vp, _vp, _vp, _i64, _d, _i32, _vp, _vp]),
    ("dbscan_slab_fit_shared_device_async", _i32,
     [_vp, _vp, _vp, _vp, _i64, _d, _i32, _vp, _i64, _vp, _vp]),
    ("dbscan_slab_label_device_async", _i32, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp]),
    ("dbscan_merge_union_device", _i32, [_vp, _vp, _i64, _vp, _vp]),
    ("dbscan_merge_reset_device", _i32, [_vp, _vp, _i64, _vp, _vp]),
    ("dbscan_slab_merge_roots_device", _i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("dbscan_slab_roots_prepare_device", _i32,
     [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    ("dbscan_slab_label_finish_device_async", _i32, [_vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    ("dbscan_generate_blobs_device", _i32, [_vp, _vp, _vp, _i64, _d, _d, _u64]),
    ("dbscan_set_small_max", _i64, [_vp, _i64]),
    ("dbscan_set_spread_min", _i64, [_vp, _i64]),
    ("dbscan_set_band_max", _i64, [_vp, _i64]),
    ("dbscan_set_band_min", _i64, [_vp, _i64]),
    ("dbscan_set_spread_spin_limit", _i64, [_vp, _i64]),
    ("dbscan_spread_fallbacks", _i64, [_vp]),
    ("dbscan_fit_batch", _i32, [_vp, _vp, _vp, _vp, _i32, _d, _i32, _i32, _vp, _vp, _vp]),
    ("dbscan_fit_batch_device_async", _i32,
     [_vp, _vp, _vp, _vp, _i32, _d, _i32, _i32, _vp, _vp, _vp]),
    ("dbscan_duplicate", _i64, [_vp, _vp, _i64, _vp, _i64, _d, _vp, _vp, _i64]),
    ("dbscan_route_slabs_device", _i64, [_vp, _vp, _vp, _i64, _i64, _vp, _i32, _d, _vp, _i64,
                                         _vp]),
    ("dbscan_slab_select_device", _i64, [_vp, _vp, _vp, _i64, _vp, _i32, _i32, _d, _vp, _vp,
                                         _vp, _vp, _vp, _i64, _vp]),
    ("dbscan_owned_rows_device", _i64, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64]),
    ("dbscan_rows_unpack_device", _i64, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    ("dbscan_label_scatter_device", _i32, [_vp, _vp, _i64, _i64, _i64, _vp, _vp]),
]
SMALL_MAX_POINTS = 8192  # DBSCAN_SMALL_MAX_POINTS

_lib = None
_lock = threading.Lock()


class DBSCANError(RuntimeError):
    pass


def _adopt_torch_runtime() -> None:
    """torch (ROCm wheel) bundles its own libamdhip64.so / libhsa-runtime64.so with the same
    SONAMEs as /opt/rocm's.  Two HIP runtimes in one process cannot share the GPU, so when torch
    is importable we load it first: the dynamic linker then binds our DT_NEEDED
    libamdhip64.so.7 / libhsa-runtime64.so.1 to torch's already-loaded copies."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load() -> ctypes.CDLL:
    """Load libdbscan_hip.so (raises if it has not been built)."""
    global _lib
    with _lock:
        if _lib is None:
            _adopt_torch_runtime()
            if not os.path.exists(LIB_PATH):
                raise DBSCANError(
                    f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                    "g.build()'` (hipcc --offload-arch=gfx950)")
            L = ctypes.CDLL(LIB_PATH)
            ab = bool(os.environ.get("DBSCAN_LIB_PATH"))
            for name, res, args in SIGNATURES:
                # (an A/B build of an older revision, loaded through DBSCAN_LIB_PATH, may lack
                # entry points added since: bind what it has; the in-tree library has them all)
                if ab and not hasattr(L, name):
                    continue
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != DBSCAN_OK:
        msg = load().dbscan_last_error()
        raise DBSCANError(f"libdbscan_hip error {rc}: {msg.decode() if msg else ''}")


class Handle:
    """Owns a dbscan_handle (one HIP stream + grow-only device buffers on one GPU)."""

    def __init__(self, device: int = 0):
        L = load()
        h = L.dbscan_create(int(device))
        if not h:
            raise DBSCANError(f"dbscan_create({device}) failed: {L.dbscan_last_error().decode()}")
        self._h = ctypes.c_void_p(h)
        self.device = int(device)

    @property
    def ptr(self):
        return self._h

    def close(self):
        if self._h:
            load().dbscan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self) -> None:
        """Wait for the handle's stream; settles an asynchronous fit (stats, errors)."""
        check(load().dbscan_sync(self._h))

    @property
    def stream(self) -> int:
        return int(load().dbscan_stream(self._h) or 0)

    def set_small_max(self, max_points: int) -> int:
        """Fits of <= max_points points run the one-workgroup kernel (small.hip); 0 sends every
        fit through the tiled pipeline.  Returns the previous value."""
        r = load().dbscan_set_small_max(self._h, int(max_points))
        if r < 0:
            check(int(r))
        return int(r)

    def set_spread_min(self, min_points: int) -> int:
        """LDS fits of >= min_points points run spread over several workgroups (small.hip,
        spread_fit_kernel); above DBSCAN_SMALL_MAX_POINTS every LDS fit keeps one workgroup.
        Returns the previous value."""
        r = load().dbscan_set_spread_min(self._h, int(min_points))
        if r < 0:
            check(int(r))
        return int(r)

    def set_band_max(self, max_points: int) -> int:
        """Full fits above the LDS capacity and up to max_points points run the band form
        (one launch; 0: never).  Returns the previous value."""
        r = load().dbscan_set_band_max(self._h, int(max_points))
        if r < 0:
            check(int(r))
        return int(r)

    def set_band_min(self, min_points: int) -> int:
        """Fits inside the LDS capacity of >= min_points points also take the band form (0:
        every eligible fit; 1 << 30: none).  Returns the previous value."""
        r = load().dbscan_set_band_min(self._h, int(min_points))
        if r < 0:
            check(int(r))
        return int(r)

    def set_spread_spin_limit(self, polls: int) -> int:
        """Test hook: the spread fit's barrier poll bound (0: every barrier gives up at once and
        the fit is re-run by the one-workgroup kernel).  Returns the previous bound."""
        r = load().dbscan_set_spread_spin_limit(self._h, int(polls))
        if r < 0:
            check(int(r))
        return int(r)

    def spread_fallbacks(self) -> int:
        """Spread fits of this handle re-run by the one-workgroup kernel so far."""
        r = load().dbscan_spread_fallbacks(self._h)
        if r < 0:
            check(int(r))
        return int(r)

    def stats(self) -> dict:
        buf = (ctypes.c_int64 * 14)()
        k = load().dbscan_last_stats(self._h, buf, 14)
        keys = ["n", "finite", "cells", "core", "clusters", "nx", "ny", "key_bits", "grid_mode",
                "tiles", "clique", "pts_small", "pts_medium", "pts_big"]
        return {keys[i]: int(buf[i]) for i in range(k)}

    def profile(self, on: bool = True, kernels: bool = False) -> None:
        """Event timing on the handle's stream: per pipeline stage (event records between
        stages, ~10 us of GPU idle each) or, with kernels=True, per kernel launch (events on
        the dispatch packets: no added gaps)."""
        check(load().dbscan_profile_enable(self._h, (2 if kernels else 1) if on else 0))

    def profile_only(self, kernel=None) -> None:
        """Kernel mode: time only `kernel`'s launches (None: every kernel)."""
        check(load().dbscan_profile_only(self._h, kernel.encode() if kernel else None))

    def profile_reset(self) -> None:
        check(load().dbscan_profile_reset(self._h))

    def profile_read(self) -> dict:
        names = ctypes.create_string_buffer(4096)
        ms = (ctypes.c_double * 64)()
        ln = (ctypes.c_int64 * 64)()
        k = load().dbscan_profile_read(self._h, names, 4096, ms, ln, 64)
        out, parts = {}, names.raw.split(b"\0")
        for i in range(k):
            out[parts[i].decode()] = dict(ms=float(ms[i]), launches=int(ln[i]))
        return out
