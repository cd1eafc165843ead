"""Control plane of a multi-GPU bench job, over
torch.distributed (gloo: CPU tensors and objects only).

The data path is C++: each rank is one node on one GPU (include/wtfnode.h),
an independent shard of the testcase stream (seed + rank), and the nodes
merge their coverage maps with an RCCL MAX all-reduce after every batch
(wtf_amd/host/rccl_exchange.cc; the CPU twin does the same over TCP,
net_exchange.cc). What the Python side does is only:
  * hand rank 0's RCCL communicator id to every rank (share_bytes);
  * reduce the timed region to the job's numbers: max wall time over ranks,
    sum of work over ranks (job_totals).
"""
from __future__ import annotations


def share_bytes(data: bytes | None, dist) -> bytes:
    """Rank 0's bytes on every rank (the RCCL unique id)."""
    if dist is None:
        return data
    box = [data if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def job_totals(dt: float, execs: float, retired: float, dist):
    """(max dt over ranks, sum of execs, sum of retired instructions)."""
    if dist is None:
        return dt, execs, retired
    import torch

    t = torch.tensor([dt, execs, retired], dtype=torch.float64)
    tmax = t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(tmax[0].item()), float(t[1].item()), float(t[2].item())
