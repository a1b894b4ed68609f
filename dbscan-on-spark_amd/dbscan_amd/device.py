"""Device-resident entry points (torch tensors in HBM -> labels in HBM).

torch is plumbing here (allocation, streams); all compute is libdbscan_hip.so."""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _p(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def fit_tensors(x: torch.Tensor, y: torch.Tensor, eps: float, min_points: int, mode: int,
                handle: _lib.Handle, cluster: torch.Tensor = None, flag: torch.Tensor = None):
    """Fit device float64 tensors; returns (cluster int32, flag uint8, n_clusters).

    The caller's pending torch work on x/y must be complete: we synchronize torch's current
    stream before handing the pointers to the library's own stream."""
    assert x.is_cuda and y.is_cuda and x.dtype == torch.float64 and y.dtype == torch.float64
    assert x.shape == y.shape and x.dim() == 1 and x.is_contiguous() and y.is_contiguous()
    n = x.numel()
    if cluster is None:
        cluster = torch.empty(n, dtype=torch.int32, device=x.device)
    if flag is None:
        flag = torch.empty(n, dtype=torch.uint8, device=x.device)
    torch.cuda.current_stream(x.device).synchronize()
    k = ctypes.c_int32(0)
    _lib.check(_lib.load().dbscan_fit_device(handle.ptr, _p(x), _p(y), n, float(eps),
                                             int(min_points), int(mode), _p(cluster), _p(flag),
                                             ctypes.byref(k)))
    return cluster, flag, int(k.value)


def fit_tensors_async(x: torch.Tensor, y: torch.Tensor, eps: float, min_points: int, mode: int,
                      handle: _lib.Handle, cluster: torch.Tensor, flag: torch.Tensor,
                      n_clusters: torch.Tensor = None) -> None:
    """Enqueue a fit on the handle's stream and return at once (dbscan_fit_device_async).
    n_clusters (int32 device tensor of one element) receives the cluster count; call
    handle.sync() (or synchronize the device) before reading any output.  x/y must not be
    written by other streams until then."""
    assert x.is_cuda and y.is_cuda and x.dtype == torch.float64 and y.dtype == torch.float64
    assert x.shape == y.shape and x.dim() == 1 and x.is_contiguous() and y.is_contiguous()
    n = x.numel()
    assert cluster.numel() == n and flag.numel() == n and cluster.dtype == torch.int32 \
        and flag.dtype == torch.uint8
    nk = _p(n_clusters) if n_clusters is not None else None
    _lib.check(_lib.load().dbscan_fit_device_async(handle.ptr, _p(x), _p(y), n, float(eps),
                                                   int(min_points), int(mode), _p(cluster),
                                                   _p(flag), nk))


def fit_batch_tensors_async(x: torch.Tensor, y: torch.Tensor, offsets, eps: float,
                            min_points: int, mode: int, handle: _lib.Handle,
                            cluster: torch.Tensor, flag: torch.Tensor,
                            n_clusters: torch.Tensor) -> None:
    """Enqueue a batch of partition fits (dbscan_fit_batch_device_async): partition p is
    x[offsets[p]:offsets[p+1]] (offsets: host int64 array); n_clusters: int32 device tensor of
    n_parts entries.  handle.sync() before reading the outputs."""
    import numpy as np

    offs = np.ascontiguousarray(offsets, dtype=np.int64)
    if offs.ndim != 1 or offs.size < 1 or offs[0] < 0 or np.any(np.diff(offs) < 0):
        raise ValueError("offsets: n_parts + 1 non-decreasing values from >= 0")
    total = int(offs[-1])
    for name, t, dt, need in (("x", x, torch.float64, total), ("y", y, torch.float64, total),
                              ("cluster", cluster, torch.int32, total),
                              ("flag", flag, torch.uint8, total),
                              ("n_clusters", n_clusters, torch.int32, offs.size - 1)):
        if not (t.is_cuda and t.is_contiguous() and t.dtype == dt and t.device == x.device
                and t.numel() >= need):
            raise ValueError(f"{name}: contiguous {dt} tensor of >= {need} values on {x.device}")
    if x.numel() != y.numel():
        raise ValueError("x and y differ in length")
    _lib.check(_lib.load().dbscan_fit_batch_device_async(
        handle.ptr, _p(x), _p(y), offs.ctypes.data_as(ctypes.c_void_p), offs.size - 1,
        float(eps), int(min_points), int(mode), _p(cluster), _p(flag), _p(n_clusters)))


def generate_blobs(n: int, noise: float, dense: float, seed: int, handle: _lib.Handle,
                   device=None):
    """SURVEY §8d generator on the device (no PCIe): returns (x, y) float64 tensors."""
    dev = device if device is not None else torch.device("cuda", handle.device)
    x = torch.empty(n, dtype=torch.float64, device=dev)
    y = torch.empty(n, dtype=torch.float64, device=dev)
    torch.cuda.current_stream(dev).synchronize()
    _lib.check(_lib.load().dbscan_generate_blobs_device(handle.ptr, _p(x), _p(y), n,
                                                        float(noise), float(dense), int(seed)))
    return x, y


def slab_fit(x: torch.Tensor, y: torch.Tensor, zone: torch.Tensor, eps: float, min_points: int,
             handle: _lib.Handle):
    """Slab fit phase 1 (node path): returns (core uint8, root int32) device tensors."""
    n = x.numel()
    core = torch.empty(n, dtype=torch.uint8, device=x.device)
    root = torch.empty(n, dtype=torch.int32, device=x.device)
    torch.cuda.current_stream(x.device).synchronize()
    _lib.check(_lib.load().dbscan_slab_fit_device(handle.ptr, _p(x), _p(y), _p(zone), n,
                                                  float(eps), int(min_points), _p(core),
                                                  _p(root)))
    return core, root


def slab_merge_roots(zone: torch.Tensor, gid: torch.Tensor, root: torch.Tensor,
                     parent: torch.Tensor, gs_of_root: torch.Tensor, own_roots: torch.Tensor,
                     handle: _lib.Handle) -> int:
    """After a slab fit and the merge union: gs_of_root[p] for every local root p; the global
    roots owned here into own_roots (increasing gid); returns their count."""
    k = ctypes.c_int64(0)
    torch.cuda.current_stream(zone.device).synchronize()
    _lib.check(_lib.load().dbscan_slab_merge_roots_device(handle.ptr, zone.numel(), _p(zone),
                                                          _p(gid), _p(root), _p(parent),
                                                          _p(gs_of_root), _p(own_roots),
                                                          ctypes.byref(k)))
    return int(k.value)


def slab_label(zone: torch.Tensor, gid: torch.Tensor, gs_of_root: torch.Tensor,
               all_roots: torch.Tensor, mode: int, handle: _lib.Handle, cluster=None,
               flag=None):
    """Slab fit phase 2 (after the global merge): (cluster int32, flag uint8) in slab order;
    only zone-0 entries are written.  all_roots: every global component's s(K), sorted."""
    n = zone.numel()
    if cluster is None:
        cluster = torch.zeros(n, dtype=torch.int32, device=zone.device)
    if flag is None:
        flag = torch.full((n,), 3, dtype=torch.uint8, device=zone.device)
    all_roots = all_roots.to(torch.int64).contiguous()
    torch.cuda.current_stream(zone.device).synchronize()
    _lib.check(_lib.load().dbscan_slab_label_device(handle.ptr, _p(zone), _p(gid),
                                                    _p(gs_of_root), _p(all_roots),
                                                    all_roots.numel(), int(mode), _p(cluster),
                                                    _p(flag)))
    return cluster, flag
