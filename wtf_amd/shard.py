"""Multi-GPU sharding of the execution backend.

Testcases are independent (single-testcase determinism, client.cc:88-180), so
each rank (one process per GPU) runs its own stream of testcases on its own
lanes with its own replica of the snapshot page pool: no data-path collective.
The one exchange per batch is the coverage merge: every GPU keeps a uint8
coverage map over the same deterministic executable-page slot table (one byte
per code byte), and the maps are merged with an all-reduce MAX (RCCL over xGMI
on the GPU box, gloo in the CPU tests). Timing follows the bench contract: the
job time is the max over ranks, the work is the sum over ranks.
"""
from __future__ import annotations

MIX = 7919  # per-rank input-stream offset multiplier


def rank_seed(base: int, rank: int) -> int:
    """Seed of rank `rank`'s testcase stream: disjoint streams per shard."""
    return (base + MIX * rank) & 0xFFFFFFFFFFFFFFFF


def merge_coverage_map(cov, dist) -> None:
    """In-place MAX all-reduce of a uint8 coverage map (torch tensor) across ranks.
    After the call every rank's map holds the union of all ranks' coverage."""
    if dist is None:
        return
    dist.all_reduce(cov, op=dist.ReduceOp.MAX)


def job_totals(dt: float, execs: float, retired: float, dist, device="cpu"):
    """(max dt over ranks, sum of execs, sum of retired instructions)."""
    if dist is None:
        return dt, execs, retired
    import torch

    t = torch.tensor([dt, execs, retired], dtype=torch.float64, device=device)
    tmax = t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(tmax[0].item()), float(t[1].item()), float(t[2].item())


def new_rips_from_map(before, after, page_vpns):
    """RIPs whose coverage byte went 0 -> nonzero between two host copies of a
    coverage map (numpy uint8 arrays of len(page_vpns) * 4096): the coverage the
    merge added on this rank, i.e. what the host reports to the master as new."""
    import numpy as np

    idx = np.nonzero((before == 0) & (after != 0))[0]
    vpn = np.asarray(page_vpns, dtype=np.uint64)[idx // 4096]
    return (vpn << np.uint64(12)) | (idx % 4096).astype(np.uint64)
