"""Worker processes for the multi-rank node-path tests (spawned by test_node*.py).

Every rank builds its slab of the same global data set, runs one NodeJob step, and writes its
owned (global index, cluster, flag) triples to `out_dir/rank<r>.npz`."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dbscan-on-spark_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


class OracleSlabOps:
    """CPU test double of HipSlabOps: the oracle's restatement of the slab semantics, so the
    merge logic (collectives, global union, numbering) runs under gloo without a GPU."""

    def fit(self, x, y, zone, eps, min_points, shared=None):  # (full outputs either way)
        import oracle as O

        xs, ys, zs = x.numpy(), y.numpy(), zone.numpy()
        core, root = O.slab_fit(xs, ys, zs, eps, min_points, nthreads=2)
        self.state = (xs, ys, zs, eps, core, root)
        return torch.from_numpy(core), torch.from_numpy(root)

    # The merge of csrc/merge.hip restated in numpy: union-find over the records' gids, root =
    # smallest gid of the component; parent is the dense gid-indexed array (-1 = untouched).
    def merge(self, a, b, parent):
        a, b, par = a.numpy(), b.numpy(), parent.numpy()
        ok = b >= 0
        up = {}

        def find(v):
            while up.get(v, v) != v:
                v = up[v]
            return v

        for u, v in zip(a[ok].tolist(), b[ok].tolist()):
            ru, rv = find(u), find(v)
            if ru != rv:
                up[max(ru, rv)] = min(ru, rv)
        for v in set(a[ok].tolist()) | set(b[ok].tolist()):
            par[v] = find(v)

    def merge_reset(self, a, b, parent):
        ok = b >= 0
        parent[a[ok]] = -1
        parent[b[ok]] = -1

    def merge_roots(self, zone, gid, root, parent, gs_of_root, mode=None):
        n = zone.numel()
        lroots = torch.nonzero(root == torch.arange(n, dtype=root.dtype)).flatten()
        g = gid[lroots]
        pg = parent[g].to(torch.int64)
        gs = torch.where(pg >= 0, pg, g)
        gs_of_root[lroots] = gs
        self.lroots = lroots
        return g[(zone[lroots] == 0) & (gs == g)]

    def label(self, zone, gid, gs_of_root, all_roots, mode):
        import oracle as O

        xs, ys, zs, eps, core, root = self.state
        label_of_root = np.zeros(xs.size, np.int32)
        lr = self.lroots.numpy()
        label_of_root[lr] = np.searchsorted(all_roots.numpy(), gs_of_root.numpy()[lr]) + 1
        cl, fl = O.slab_label(xs, ys, zs, eps, core, root, gid.numpy(), gs_of_root.numpy(),
                              label_of_root, mode)
        return torch.from_numpy(cl), torch.from_numpy(fl)


def run(rank, world, port, data_path, out_dir, eps, min_points, mode, use_gpu):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # NODE_WORKER_BACKEND=nccl (one rank per GPU: RCCL refuses two ranks on one GPU) with
    # NODE_WORKER_FORCE_COLLECTIVES=1 runs RCCL's collectives even at world size 1
    backend = os.environ.get("NODE_WORKER_BACKEND", "gloo")
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    from dbscan_amd import node

    d = np.load(data_path)
    x, y = torch.from_numpy(d["x"]), torch.from_numpy(d["y"])
    if use_gpu:
        import dbscan_amd

        torch.cuda.set_device(0)
        h = dbscan_amd.Handle(0)
        # NODE_WORKER_SHARE_STREAM=0: the handle keeps its own stream (event-ordered)
        ops = node.HipSlabOps(h, share_stream=os.environ.get("NODE_WORKER_SHARE_STREAM",
                                                             "1") == "1")
        x, y = x.cuda(), y.cuda()
    else:
        ops = OracleSlabOps()
    comm = node.Comm(dist)
    comm.force = os.environ.get("NODE_WORKER_FORCE_COLLECTIVES") == "1"
    if os.environ.get("NODE_WORKER_CHUNKS") == "1":  # host-to-slab path: this rank's chunk only
        bounds = node.NodeJob.chunk_bounds(x.numel(), world)
        c0, c1 = bounds[rank], bounds[rank + 1]
        job = node.NodeJob.from_chunk(x[c0:c1], y[c0:c1], c0, x.numel(), eps, min_points, mode,
                                      comm, ops)
        k = job.run()
        cl, fl = job.chunk_labels(c0, c1 - c0, bounds)
        cl, fl = cl.clone(), fl.clone()
        k2 = job.run()  # a second step: the same labels again
        cl2, fl2 = job.chunk_labels(c0, c1 - c0, bounds)
        assert torch.equal(cl, cl2) and torch.equal(fl, fl2), "second step's labels differ"
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), gid=np.arange(c0, c1),
                 cluster=cl.cpu().numpy(), flag=fl.cpu().numpy(), k=np.array([k, k2]),
                 n_slab=np.array([job.x.numel()]), cuts=np.array(job.cuts, dtype=np.float64))
        dist.barrier()
        dist.destroy_process_group()
        return
    job = node.NodeJob.from_global(x, y, eps, min_points, mode, comm, ops)
    k = job.run()
    k2 = job.run()  # a second step on the same handle must give the same answer
    g, c, f = (t.cpu().numpy() for t in job.owned())
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), gid=g, cluster=c, flag=f,
             k=np.array([k, k2]), n_slab=np.array([job.x.numel()]),
             cuts=np.array(job.cuts, dtype=np.float64))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    args = sys.argv[1:]
    run(int(args[0]), int(args[1]), int(args[2]), args[3], args[4], float(args[5]),
        int(args[6]), int(args[7]), args[8] == "1")
