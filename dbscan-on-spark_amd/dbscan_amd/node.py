"""Whole-node DBSCAN over N GPUs: spatial slabs with eps halos, exact merge over RCCL.

This is the MI355X restatement of the reference's distributed path:
  DBSCAN.scala:105-137   partition the plane, grow each partition by eps, duplicate points
  DBSCAN.scala:150-155   LocalDBSCANNaive.fit per partition            -> slab fit on one GPU
  DBSCAN.scala:158-222   band points, findAdjacencies, DBSCANGraph, global ids
                                                  -> all-gather of shared core points + merge
  DBSCAN.scala:232-270   relabel inner/outer points                  -> slab label kernel
One process per GPU; slabs are x-ranges at count quantiles snapped to the 2*eps grid
(DBSCAN.scala:289 minimumRectangleSize), one slab per rank.

Exactness (why the result equals ONE fit of the whole data set, bit for bit, including the
Naive noise rule and the cluster numbering -- unlike the reference's merge):
  * zone 0 = the rank's own slab; zone 1 = points within R = max|x'-x| of any accepted pair
    (R >= eps) of the slab; zone 2 = within 2R.  Counts of zone 0/1 points are exact, so their
    core flags are the global ones.
  * every global core-core edge (p, q) has p owned by some rank g and q in g's zone 0/1, so it
    is an edge of g's local graph: global components are unions of local components that share
    a core point.  Shared points (present in zones 0/1 of two ranks: a set fixed per job) are
    all-gathered each step as (gid, local root gid or -1) records -- fixed sizes, one RCCL
    all-gather, no size exchange; every rank runs the same lock-free union-find over the
    records' gids on its GPU (csrc/merge.hip), which gives each local root its global s(K)
    (= min visit index of the component, the reference's cluster-opening order).
  * owned global roots are all-gathered; cluster id = 1 + rank of s(K) among them.
  * border/noise needs min over core neighbours of s(K): done after the merge on the GPU
    (dbscan_slab_label_device), since s(K) is not monotone in the local root.
"""
from __future__ import annotations

import ctypes
import os
import math
import sys
import warnings
from typing import List, Optional

import torch

from . import _lib


def _p(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


OUT = 255  # point not in this rank's slab


def reach(eps: float) -> float:
    """Upper bound of |x'-x| over pairs the fp64 predicate accepts (grid soundness)."""
    return max(abs(eps) * (1.0 + 2.0 ** -40), 2.0 ** -500)


def margin1(c: float, R: float) -> float:
    return R * (1.0 + 2.0 ** -10) + 16.0 * math.ulp(c)


def margin2(c: float, R: float) -> float:
    return 2.0 * margin1(c, R) + 16.0 * math.ulp(c)


def make_cuts(x: torch.Tensor, world: int, eps: float, sample: int = 1 << 20) -> List[float]:
    """world-1 x cuts at count quantiles of the finite x values, snapped down to the 2*eps grid
    (the reference's partition corners, DBSCAN.scala:289,352-353).  Empty if one slab suffices
    or eps*eps is not finite (all-pairs / no-pairs semantics do not shard)."""
    e2 = eps * eps
    if world <= 1 or not math.isfinite(e2):
        return []
    xf = x[torch.isfinite(x)]
    if xf.numel() == 0:
        return []
    step = max(1, xf.numel() // sample)
    xs, _ = torch.sort(xf[::step])
    xs = xs.double().cpu()
    grid = 2.0 * abs(eps)
    cuts = []
    for k in range(1, world):
        q = float(xs[min(xs.numel() - 1, k * xs.numel() // world)])
        c = math.floor(q / grid) * grid if grid > 0 and math.isfinite(q / grid) else q
        if cuts and c < cuts[-1]:
            c = cuts[-1]
        cuts.append(c)
    return cuts


def zones(x: torch.Tensor, rank: int, cuts: List[float], eps: float):
    """Zone of every point for `rank` (0 owned, 1 inner halo, 2 outer halo, 255 outside) and
    the `shared` mask: points that are in zone 0/1 of at least two ranks."""
    world = len(cuts) + 1
    R = reach(eps)
    lo = cuts[rank - 1] if rank > 0 else None
    hi = cuts[rank] if rank < world - 1 else None
    own = torch.ones_like(x, dtype=torch.bool)
    if lo is not None:
        own &= x >= lo
    if hi is not None:
        own &= x < hi
    if rank == 0 and world > 1:
        own |= torch.isnan(x)  # NaN x: owned by rank 0 (isolated: never anyone's neighbour)
    in1 = torch.zeros_like(own)
    in2 = torch.zeros_like(own)
    shared = torch.zeros_like(own)
    if lo is not None:
        m1, m2 = margin1(lo, R), margin2(lo, R)
        in1 |= (x >= lo - m1) & (x < lo)
        in2 |= (x >= lo - m2) & (x < lo - m1)
        shared |= own & (x <= lo + m1)  # zone 1 of rank-1 (same expression there)
    if hi is not None:
        m1, m2 = margin1(hi, R), margin2(hi, R)
        in1 |= (x >= hi) & (x <= hi + m1)
        in2 |= (x > hi + m1) & (x <= hi + m2)
        shared |= own & (x >= hi - m1)  # zone 1 of rank+1
    z = torch.full(x.shape, OUT, dtype=torch.uint8, device=x.device)
    z[in2] = 2
    z[in1] = 1
    z[own] = 0
    shared |= z == 1
    return z, shared


class Comm:
    """Variable-length all-gather over torch.distributed (RCCL for 'nccl', host for 'gloo')."""

    def __init__(self, dist=None):
        self.dist = dist
        # force: run the collectives at one rank too (tests: RCCL's calls on a one-GPU box)
        self.force = False
        if dist is not None and dist.is_initialized():
            self.world, self.rank = dist.get_world_size(), dist.get_rank()
            self.host = dist.get_backend() == "gloo"
        else:
            self.dist, self.world, self.rank, self.host = None, 1, 0, True

    def _local(self) -> bool:  # one rank and no forced collectives: nothing to exchange
        return self.world == 1 and not (self.force and self.dist is not None)

    def sizes(self, k: int) -> List[int]:
        """Every rank's k, in rank order."""
        if self._local():
            return [k]
        n = torch.tensor([k], dtype=torch.int64,
                         device="cpu" if self.host else torch.device("cuda",
                                                                      torch.cuda.current_device()))
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(ns, n)
        return [int(v) for v in torch.cat(ns).cpu().tolist()]

    def allgather_varlen(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate every rank's t along its last dim, in rank order."""
        if self._local():
            return t
        return self.allgather_fixed(t, self.sizes(t.shape[-1]))

    def alltoall_rows(self, t: torch.Tensor, send_counts: List[int]) -> torch.Tensor:
        """t: rows grouped by destination rank (send_counts[d] rows to rank d).  Returns the
        rows every rank sent here, in source-rank order: one all_to_all_single of the counts,
        one of the rows (RCCL over xGMI for 'nccl')."""
        if self._local():
            return t
        dev = t.device
        cdev = "cpu" if self.host else t.device
        sc = torch.tensor(send_counts, dtype=torch.int64, device=cdev)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc)
        rcounts = [int(v) for v in rc.cpu().tolist()]
        tt = t.cpu() if self.host else t.contiguous()
        out = torch.empty((sum(rcounts),) + tuple(t.shape[1:]), dtype=t.dtype, device=tt.device)
        self.dist.all_to_all_single(out, tt, rcounts, list(send_counts))
        return out.to(dev)

    def allgather_fixed(self, t: torch.Tensor, sizes: List[int]) -> torch.Tensor:
        """allgather_varlen when every rank's length is already known (no size exchange)."""
        if self._local():
            return t
        dev = t.device
        tt = t.cpu() if self.host else t.contiguous()
        mx = max(sizes)
        pad = torch.zeros(tt.shape[:-1] + (mx,), dtype=tt.dtype, device=tt.device)
        pad[..., :tt.shape[-1]] = tt
        outs = [torch.empty_like(pad) for _ in range(self.world)]
        self.dist.all_gather(outs, pad)
        res = torch.cat([o[..., :k] for o, k in zip(outs, sizes)], dim=-1)
        return res.to(dev)


class HipSlabOps:
    """The product slab fit and merge: libdbscan_hip.so through device tensors.  The slab fit
    and label run asynchronously on the handle's stream, ordered against torch's current stream
    by stream waits (no host synchronization); the merge kernels run on torch's stream.  A step
    synchronizes the host only for the owned-root count (while the label's first part runs on
    the GPU) and the all-gather sizes."""

    def __init__(self, handle: _lib.Handle, share_stream: bool = True):
        self.h = handle
        if share_stream:
            # the handle's kernels on torch's current stream: no cross-stream waits per step
            # (two event waits that each left the GPU idle ~25 us per step at N = 1)
            self._hs = torch.cuda.current_stream(torch.device("cuda", handle.device))
            _lib.check(_lib.load().dbscan_set_stream(
                handle.ptr, ctypes.c_void_p(self._hs.cuda_stream or None), 0))
        else:
            self._hs = torch.cuda.ExternalStream(handle.stream,
                                                 device=torch.device("cuda", handle.device))
        self._bound = share_stream
        self._out = None
        self._bufs = None
        self._lab = None  # (cluster, flag, zone) reused across the steps of one slab

    def close(self):
        """Give the handle its own stream back (share_stream=True bound it to torch's stream,
        which the caller may destroy later).  Waits for the handle's work first."""
        if self._bound and self.h.ptr:
            self.h.sync()
            _lib.check(_lib.load().dbscan_set_stream(self.h.ptr, None, 1))
            self._bound = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self, _finalizing=sys.is_finalizing):
        # Callers close() explicitly (NodeJob.close, the bench, the tests).  A finalizer may run
        # at interpreter shutdown, after torch has torn down its streams: HIP calls from here are
        # best-effort only, and never once the interpreter is finalizing or the handle is gone.
        # (sys.is_finalizing is bound at definition: module globals may already be None here.)
        if not getattr(self, "_bound", False) or _finalizing() or not getattr(self.h, "_h", None):
            return
        try:
            self.close()
        except Exception as e:  # pragma: no cover - finalizer
            warnings.warn(f"HipSlabOps finalizer could not unbind the handle's stream: {e}")

    def _to_handle(self):
        cur = torch.cuda.current_stream()
        if cur.cuda_stream != self._hs.cuda_stream:
            self._hs.wait_stream(cur)

    def _from_handle(self):
        cur = torch.cuda.current_stream()
        if cur.cuda_stream != self._hs.cuda_stream:
            cur.wait_stream(self._hs)

    def fit(self, x, y, zone, eps, min_points, shared=None):
        """Slab fit.  shared (int64 slab indices): the lean form -- core/root valid only at
        those indices, root[r] == r marking every local root, -1 elsewhere (all the merge
        reads)."""
        n = x.numel()
        if self._out is None or self._out[0].numel() != n:
            self._out = (torch.empty(n, dtype=torch.uint8, device=x.device),
                         torch.empty(n, dtype=torch.int32, device=x.device))
        core, root = self._out
        self._to_handle()
        if shared is None:
            _lib.check(_lib.load().dbscan_slab_fit_device_async(
                self.h.ptr, _p(x), _p(y), _p(zone), n, float(eps), int(min_points), _p(core),
                _p(root)))
        else:
            _lib.check(_lib.load().dbscan_slab_fit_shared_device_async(
                self.h.ptr, _p(x), _p(y), _p(zone), n, float(eps), int(min_points), _p(shared),
                shared.numel(), _p(core), _p(root)))
        self._from_handle()
        return core, root

    def route(self, x, y, start, cuts, eps):
        """from_chunk's rows (dbscan_route_slabs_device): (rows int64[k, 3], counts per rank)."""
        import numpy as np

        L = _lib.load()
        m = x.numel()
        c = np.ascontiguousarray(cuts, dtype=np.float64)
        counts = np.zeros(len(cuts) + 1, np.int64)
        self._to_handle()
        vp = ctypes.c_void_p
        args = (self.h.ptr, _p(x), _p(y), m, int(start), c.ctypes.data_as(vp), len(cuts),
                float(eps))
        total = L.dbscan_route_slabs_device(*args, None, 0, counts.ctypes.data_as(vp))
        if total < 0:
            _lib.check(int(total))
        rows = torch.empty((max(1, total), 3), dtype=torch.int64, device=x.device)
        got = L.dbscan_route_slabs_device(*args, _p(rows), total, counts.ctypes.data_as(vp))
        if got < 0:
            _lib.check(int(got))
        self._from_handle()
        return rows[:total], [int(v) for v in counts]

    def select(self, x, y, cuts, rank, eps):
        """from_global's slab (dbscan_slab_select_device): (x, y, zone, gid, shared slab
        indices) of slab `rank`, in input order."""
        import numpy as np

        L = _lib.load()
        n = x.numel()
        c = np.ascontiguousarray(cuts, dtype=np.float64)
        ns = ctypes.c_int64(0)
        vp = ctypes.c_void_p
        self._to_handle()
        args = (self.h.ptr, _p(x), _p(y), n, c.ctypes.data_as(vp), len(cuts), int(rank),
                float(eps))
        m = L.dbscan_slab_select_device(*args, None, None, None, None, None, 0, ctypes.byref(ns))
        if m < 0:
            _lib.check(int(m))
        dev = x.device
        sx = torch.empty(max(1, m), dtype=torch.float64, device=dev)
        sy = torch.empty_like(sx)
        sz = torch.empty(max(1, m), dtype=torch.uint8, device=dev)
        sg = torch.empty(max(1, m), dtype=torch.int64, device=dev)
        sh = torch.empty(max(1, ns.value), dtype=torch.int64, device=dev)
        got = L.dbscan_slab_select_device(*args, _p(sx), _p(sy), _p(sz), _p(sg), _p(sh), m,
                                          ctypes.byref(ns))
        if got < 0:
            _lib.check(int(got))
        self._from_handle()
        return sx[:m], sy[:m], sz[:m], sg[:m], sh[:ns.value]

    def unpack(self, rows):
        """from_chunk's received rows -> (x, y, zone, gid, shared slab indices)
        (dbscan_rows_unpack_device)."""
        k = rows.shape[0]
        dev = rows.device
        rows = rows.contiguous()
        sx = torch.empty(max(1, k), dtype=torch.float64, device=dev)
        sy = torch.empty_like(sx)
        sz = torch.empty(max(1, k), dtype=torch.uint8, device=dev)
        sg = torch.empty(max(1, k), dtype=torch.int64, device=dev)
        sh = torch.empty(max(1, k), dtype=torch.int64, device=dev)
        self._to_handle()
        ns = _lib.load().dbscan_rows_unpack_device(self.h.ptr, _p(rows), k, _p(sx), _p(sy),
                                                   _p(sz), _p(sg), _p(sh))
        if ns < 0:
            _lib.check(int(ns))
        self._from_handle()
        return sx[:k], sy[:k], sz[:k], sg[:k], sh[:ns]

    def owned_rows(self, zone, gid, cluster, flag):
        """chunk_labels' rows (dbscan_owned_rows_device): (gid, cluster << 8 | flag) of the
        zone-0 points, slab order (ascending gid)."""
        m = zone.numel()
        rows = torch.empty((max(1, m), 2), dtype=torch.int64, device=zone.device)
        self._to_handle()
        k = _lib.load().dbscan_owned_rows_device(self.h.ptr, _p(zone), _p(gid), _p(cluster),
                                                 _p(flag), m, _p(rows), m)
        if k < 0:
            _lib.check(int(k))
        self._from_handle()
        return rows[:k]

    def label_scatter(self, rows, start, m):
        """The chunk owner's labels from the received rows (dbscan_label_scatter_device)."""
        dev = rows.device
        cl = torch.empty(m, dtype=torch.int32, device=dev)
        fl = torch.empty(m, dtype=torch.uint8, device=dev)
        rows = rows.contiguous()
        self._to_handle()
        _lib.check(_lib.load().dbscan_label_scatter_device(self.h.ptr, _p(rows), rows.shape[0],
                                                           int(start), int(m), _p(cl), _p(fl)))
        self._from_handle()
        return cl, fl

    def fit_whole(self, x, y, eps, min_points, mode):
        """One rank, nothing to merge: the slab is the whole data set, so the node step is the
        direct fit (dbscan_fit_device_async) -- labels in slab order, the cluster count."""
        n = x.numel()
        cl = torch.empty(n, dtype=torch.int32, device=x.device)
        fl = torch.empty(n, dtype=torch.uint8, device=x.device)
        nk = torch.zeros(1, dtype=torch.int32, device=x.device)
        self._to_handle()
        _lib.check(_lib.load().dbscan_fit_device_async(
            self.h.ptr, _p(x), _p(y), n, float(eps), int(min_points), int(mode), _p(cl), _p(fl),
            _p(nk)))
        self._from_handle()
        return cl, fl, int(nk.item())

    @staticmethod
    def _stream():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def merge(self, a, b, parent):
        _lib.check(_lib.load().dbscan_merge_union_device(_p(a), _p(b), a.numel(), _p(parent),
                                                         self._stream()))

    def merge_reset(self, a, b, parent):
        _lib.check(_lib.load().dbscan_merge_reset_device(_p(a), _p(b), a.numel(), _p(parent),
                                                         self._stream()))

    def merge_roots(self, zone, gid, root, parent, gs_of_root, mode=None):
        """The owned global roots.  With mode given, the label's first part (which needs only
        gs_of_root) is enqueued behind the count and runs while the host gathers and numbers
        the roots (dbscan_slab_roots_prepare_device); label() then finishes it."""
        n = zone.numel()
        if self._bufs is None or self._bufs.numel() < max(1, n):
            self._bufs = torch.empty(max(1, n), dtype=torch.int64, device=zone.device)
        k = ctypes.c_int64(0)
        self._to_handle()
        if mode is None:
            _lib.check(_lib.load().dbscan_slab_merge_roots_device(
                self.h.ptr, n, _p(zone), _p(gid), _p(root), _p(parent), _p(gs_of_root),
                _p(self._bufs), ctypes.byref(k)))  # synchronizes the handle stream (the count)
        else:
            _lib.check(_lib.load().dbscan_slab_roots_prepare_device(
                self.h.ptr, n, _p(zone), _p(gid), _p(root), _p(parent), _p(gs_of_root),
                int(mode), _p(self._bufs), ctypes.byref(k)))  # waits for the count only
        self._prepared = mode
        return self._bufs[:int(k.value)]

    def label(self, zone, gid, gs_of_root, all_roots, mode):
        n = zone.numel()
        prepared = getattr(self, "_prepared", None) == mode
        if prepared and self._lab is not None and self._lab[2] is zone:
            # the same slab again (a job's steps): zone 1/2 entries still hold their fill
            cluster, flag = self._lab[0], self._lab[1]
        else:
            cluster = torch.zeros(n, dtype=torch.int32, device=zone.device)
            flag = torch.full((n,), 3, dtype=torch.uint8, device=zone.device)
            self._lab = (cluster, flag, zone) if prepared else None
        all_roots = all_roots.to(torch.int64).contiguous()
        self._to_handle()
        if prepared:
            _lib.check(_lib.load().dbscan_slab_label_finish_device_async(
                self.h.ptr, _p(zone), _p(gs_of_root), _p(all_roots), all_roots.numel(),
                _p(cluster), _p(flag)))
        else:
            _lib.check(_lib.load().dbscan_slab_label_device_async(
                self.h.ptr, _p(zone), _p(gid), _p(gs_of_root), _p(all_roots), all_roots.numel(),
                int(mode), _p(cluster), _p(flag)))
        self._prepared = None
        self._from_handle()
        return cluster, flag


class NodeJob:
    """One rank's share of a whole-node fit.  run() is one step (timed by bench.py)."""

    def __init__(self, x, y, zone, gid, shared, eps, min_points, mode, comm: Comm, ops,
                 n_total: int, sh_idx=None, tick=None):
        tick = tick or (lambda name: None)
        self.x, self.y, self.zone, self.gid, self.shared = x, y, zone, gid, shared
        self.eps, self.min_points, self.mode = float(eps), int(min_points), int(mode)
        self.comm, self.ops = comm, ops
        self.cluster = self.flag = None
        self.n_clusters = 0
        self._cs = None  # the roots' gather stream (N > 1, device tensors)
        # Static per job: the shared points (slab indices), the a-side of every rank's records
        # and the record counts, so each step exchanges only the b-side at known sizes.
        dev = x.device
        self.sh_idx = torch.nonzero(shared).flatten() if sh_idx is None else sh_idx
        a = gid[self.sh_idx]
        tick("job: shared points")
        self.rec_sizes = comm.sizes(a.numel())
        self.all_a = comm.allgather_fixed(a, self.rec_sizes)
        tick("job: a-side records all-gathered")
        self.parent = torch.full((max(1, int(n_total)),), -1, dtype=torch.int32, device=dev)
        self.gs_of_root = torch.zeros(max(1, x.numel()), dtype=torch.int64, device=dev)
        tick("job: merge arrays")

    @classmethod
    def from_global(cls, x_all, y_all, eps, min_points, mode, comm: Comm, ops,
                    cuts: Optional[List[float]] = None, tick=None) -> "NodeJob":
        """Select this rank's slab (zones 0/1/2, global visit order kept) from the global
        arrays.  Setup, not part of a step.  tick(name): called after each phase (traces)."""
        tick = tick or (lambda name: None)
        if cuts is None:
            cuts = make_cuts(x_all, comm.world, eps)
        tick("cuts")
        assert len(cuts) == comm.world - 1 or (not cuts), "one slab per rank"
        if (x_all.is_cuda and hasattr(ops, "select") and math.isfinite(eps * eps)
                and (cuts or comm.world == 1)):
            # the plan kernels (ordered compaction on the GPU): no torch pass per zone
            sx, sy, sz, sg, sh_idx = ops.select(x_all, y_all, cuts, comm.rank, eps)
            tick("zones + slab selection")
            job = cls(sx, sy, sz, sg, None, eps, min_points, mode, comm, ops, x_all.numel(),
                      sh_idx=sh_idx, tick=tick)
            job.cuts = cuts
            return job
        if not cuts and comm.world > 1:  # unshardable eps: everything on rank 0
            own = torch.full(x_all.shape, OUT, dtype=torch.uint8, device=x_all.device)
            if comm.rank == 0:
                own[:] = 0
            z, sh = own, torch.zeros_like(own, dtype=torch.bool)
        else:
            z, sh = zones(x_all, comm.rank, cuts, eps)
        tick("zones")
        idx = torch.nonzero(z != OUT).flatten()  # ascending: global visit order preserved
        sx, sy, sz = x_all[idx].contiguous(), y_all[idx].contiguous(), z[idx].contiguous()
        sg, ss = idx.to(torch.int64).contiguous(), sh[idx].contiguous()
        tick("slab selection")
        job = cls(sx, sy, sz, sg, ss, eps, min_points, mode, comm, ops, x_all.numel(), tick=tick)
        job.cuts = cuts
        return job

    @staticmethod
    def chunk_bounds(n_total: int, world: int) -> List[int]:
        """Rank r's contiguous chunk of the global input is [b[r], b[r+1])."""
        return [r * n_total // world for r in range(world + 1)]

    @classmethod
    def from_chunk(cls, x, y, start: int, n_total: int, eps, min_points, mode, comm: Comm, ops,
                   sample: int = 1 << 20, tick=None) -> "NodeJob":
        """Host-to-slab path: each rank holds only the contiguous chunk [start, start + len(x))
        of the global input (global visit order), e.g. just copied from host memory.  The cuts
        come from an all-gathered sample of every chunk; every point goes to the ranks whose
        zones 0/1/2 hold it in ONE all_to_all of 24-B records (x, y bits, gid/zone/shared),
        so a rank receives its slab in ascending gid (segments in source-rank order, each
        ascending): the same slab from_global selects, without any rank holding all points."""
        tick = tick or (lambda name: None)
        world = comm.world
        m = x.numel()
        dev = x.device
        if comm._local():  # one rank, nothing to route: the chunk is the whole slab, all owned
            job = cls(x.contiguous(), y.contiguous(), torch.zeros(m, dtype=torch.uint8, device=dev),
                      torch.arange(start, start + m, dtype=torch.int64, device=dev),
                      torch.zeros(m, dtype=torch.bool, device=dev), eps, min_points, mode, comm,
                      ops, n_total, sh_idx=torch.zeros(0, dtype=torch.int64, device=dev))
            job.cuts = []
            return job
        if world > 1:
            # every rank's strided sample of its chunk (finite values), all-gathered: the same
            # cuts on every rank
            per = max(1, sample // world)
            smp = x[::max(1, m // per)][:per]
            smp = smp[torch.isfinite(smp)].contiguous()
            allx = comm.allgather_varlen(smp)
            cuts = make_cuts(allx, world, eps, sample=max(1, allx.numel()))
        else:  # (one slab: no cuts whatever the sample)
            cuts = []
        tick("chunk: sample + cuts")
        if x.is_cuda and hasattr(ops, "route") and (cuts or (world == 1 and math.isfinite(eps * eps))):
            # one kernel pass per direction: every destination's rows, grouped and ordered
            rows, counts = ops.route(x, y, start, cuts, eps)
        else:
            rows, counts = cls._route_torch(x, y, start, cuts, eps, world)
        tick("chunk: route rows")
        recv = comm.alltoall_rows(rows, counts)
        tick("chunk: all_to_all rows")
        if recv.is_cuda and hasattr(ops, "unpack"):
            sx, sy, sz, sg, sh_idx = ops.unpack(recv)
            del recv
            tick("chunk: columns")
            job = cls(sx, sy, sz, sg, None, eps, min_points, mode, comm, ops, n_total,
                      sh_idx=sh_idx, tick=tick)
            job.cuts = cuts
            return job
        code = recv[:, 2].contiguous()
        sx = recv[:, 0].contiguous().view(torch.float64)
        sy = recv[:, 1].contiguous().view(torch.float64)
        tick("chunk: columns")
        job = cls(sx, sy, ((code >> 1) & 3).to(torch.uint8), code >> 3, (code & 1) != 0, eps,
                  min_points, mode, comm, ops, n_total, tick=tick)
        job.cuts = cuts
        return job

    @staticmethod
    def _route_torch(x, y, start, cuts, eps, world):
        """from_chunk's rows by torch ops (host tensors: the gloo tests' path; device tensors go
        through ops.route, the HIP kernels of dbscan_route_slabs_device)."""
        m = x.numel()
        dev = x.device
        gid = torch.arange(start, start + m, dtype=torch.int64, device=dev)
        xb, yb = x.contiguous().view(torch.int64), y.contiguous().view(torch.int64)
        recs, counts = [], []
        for d in range(world):
            if cuts:
                z, sh = zones(x, d, cuts, eps)
            else:  # unshardable eps: everything on rank 0
                z = torch.full(x.shape, OUT if d else 0, dtype=torch.uint8, device=dev)
                sh = torch.zeros(x.shape, dtype=torch.bool, device=dev)
            idx = torch.nonzero(z != OUT).flatten()
            code = gid[idx] * 8 + z[idx].long() * 2 + sh[idx].long()
            recs.append(torch.stack([xb[idx], yb[idx], code], 1))
            counts.append(int(idx.numel()))
        return torch.cat(recs), counts

    def chunk_labels(self, start: int, m: int, bounds: List[int], tick=None):
        """The labels of the chunk [start, start + m) this rank holds, in input order: every
        rank sends its owned (gid, cluster, flag) to the chunk owner (one all_to_all), which
        scatters them into place.  Returns (cluster int32[m], flag uint8[m]) on the device."""
        tick = tick or (lambda name: None)
        if self.comm._local():  # one rank: the slab is the chunk, in order, every point owned
            return self.cluster, self.flag
        if self.zone.is_cuda and hasattr(self.ops, "owned_rows"):
            # one ordered compaction (the slab is in ascending gid, so are the rows): the
            # destination of every row is its chunk, the counts a search of the bounds
            rec = self.ops.owned_rows(self.zone, self.gid, self.cluster, self.flag)
            b = torch.tensor(bounds[1:-1], dtype=torch.int64, device=rec.device)
            ends = torch.searchsorted(rec[:, 0].contiguous(), b).cpu().tolist()
            counts = [e - s_ for s_, e in zip([0] + ends, ends + [rec.shape[0]])]
            tick("labels: records")
            recv = self.comm.alltoall_rows(rec, counts)
            tick("labels: all_to_all")
            out = self.ops.label_scatter(recv, start, m)
            tick("labels: scatter")
            return out
        gid, cl, fl = self.owned()
        tick("labels: owned points")
        dev = gid.device
        b = torch.tensor(bounds[1:-1], dtype=torch.int64, device=dev)
        dest = torch.searchsorted(b, gid, right=True)
        counts = torch.bincount(dest, minlength=self.comm.world).cpu().tolist()
        rec = torch.stack([gid, (cl.to(torch.int64) << 8) | fl.to(torch.int64)], 1)
        tick("labels: records")
        recv = self.comm.alltoall_rows(rec, counts)
        tick("labels: all_to_all")
        loc = recv[:, 0] - start
        out_cl = torch.zeros(m, dtype=torch.int32, device=dev)
        out_fl = torch.zeros(m, dtype=torch.uint8, device=dev)
        out_cl[loc] = (recv[:, 1] >> 8).to(torch.int32)
        out_fl[loc] = (recv[:, 1] & 255).to(torch.uint8)
        tick("labels: scatter")
        return out_cl, out_fl

    @classmethod
    def synthetic(cls, n_total, noise, dense, seed, eps, min_points, handle, dist,
                  mode: int = 0, force: bool = False, tick=None) -> "NodeJob":
        """bench.py setup: every rank generates the same G(n_total) on its GPU (device
        generator), then keeps its slab.  force: Comm.force (collectives at one rank too)."""
        from . import device as D

        tick = tick or (lambda name: None)
        x_all, y_all = D.generate_blobs(n_total, noise, dense, seed, handle)
        tick("generate")
        comm = Comm(dist)
        comm.force = force
        ops = HipSlabOps(handle)
        tick("slab ops")
        job = cls.from_global(x_all, y_all, eps, min_points, mode, comm, ops, tick=tick)
        del x_all, y_all
        torch.cuda.empty_cache()
        return job

    def run(self, tick=None) -> int:
        """One step.  tick(name), if given, is called after each phase (tools/node_breakdown.py
        synchronizes and times there)."""
        tick = tick or (lambda name: None)
        if self.comm._local() and not getattr(self, "cuts", None) and hasattr(self.ops, "fit_whole"):
            # one rank and one slab (every point owned): the direct fit IS the node step
            self.cluster, self.flag, self.n_clusters = self.ops.fit_whole(
                self.x, self.y, self.eps, self.min_points, self.mode)
            tick("slab_fit")
            return self.n_clusters
        core, root = self.ops.fit(self.x, self.y, self.zone, self.eps, self.min_points,
                                  shared=self.sh_idx)
        tick("slab_fit")
        # records: (gid of each shared point, gid of its local root, or -1 if not core here)
        rs = root[self.sh_idx].long().clamp(min=0)
        b = torch.where(core[self.sh_idx] != 0, self.gid[rs], torch.full_like(rs, -1))
        all_b = self.comm.allgather_fixed(b, self.rec_sizes)
        tick("records")
        self.ops.merge(self.all_a, all_b, self.parent)
        tick("merge")
        # every local root's global s(K); the zone-0 global roots owned here
        own = self.ops.merge_roots(self.zone, self.gid, root, self.parent, self.gs_of_root,
                                   mode=self.mode)
        tick("roots")
        # cluster id = 1 + rank of s(K) among all ranks' global roots (each rank's list is
        # already in gid order)
        if self.comm.world > 1:
            # DBSCAN_NODE_COMM_STREAM=1: the gather and sort on a stream of their own, so the
            # collectives need not wait for the label's first part still running on the current
            # stream (own is complete: merge_roots waited for it).  Off by default: two gloo
            # ranks sharing one GPU measured 6.0-6.2 ms per step with it, 4.5-4.7 without
            # (tools/node2_ab.sh); the RCCL case is for a multi-GPU A/B.
            if self._cs is None:
                use = own.is_cuda and os.environ.get("DBSCAN_NODE_COMM_STREAM", "0") == "1"
                self._cs = torch.cuda.Stream(device=own.device) if use else False
            main = torch.cuda.current_stream(own.device) if own.is_cuda else None
            if self._cs:
                self._cs.wait_stream(main)  # own was produced on main
                own.record_stream(self._cs)
                with torch.cuda.stream(self._cs):
                    all_roots, _ = torch.sort(self.comm.allgather_varlen(own))
                main.wait_stream(self._cs)
                all_roots.record_stream(main)
            else:
                all_roots, _ = torch.sort(self.comm.allgather_varlen(own))
        else:  # one rank's list is already in gid order
            all_roots = own
        self.ops.merge_reset(self.all_a, all_b, self.parent)
        tick("numbering")
        self.cluster, self.flag = self.ops.label(self.zone, self.gid, self.gs_of_root, all_roots,
                                                 self.mode)
        tick("slab_label")
        self.n_clusters = int(all_roots.numel())
        return self.n_clusters

    def close(self) -> None:
        """Release the slab ops (gives the handle its own stream back)."""
        if self.ops is not None and hasattr(self.ops, "close"):
            self.ops.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def owned(self):
        """(global visit index, cluster, flag) of this rank's owned points."""
        m = self.zone == 0
        return self.gid[m], self.cluster[m], self.flag[m]
