"""N>1 path on CPU: two ranks over gloo run the sharding helpers bench.py uses
on the GPU box with RCCL (wtf_amd/shard.py): the coverage-map MAX merge, the
new-coverage extraction after a merge, and max-over-ranks / sum-over-ranks
job totals."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from wtf_amd import shard

PAGES = [0x140001, 0x140002, 0x7FF00]


def _rank_cov(rank):
    rng = np.random.default_rng(shard.rank_seed(0x5EED0001, rank))
    m = np.zeros(len(PAGES) * 4096, np.uint8)
    m[rng.choice(m.size, 900, replace=False)] = 1
    return m


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _rank_cov(rank)
        cov = torch.from_numpy(mine.copy())
        shard.merge_coverage_map(cov, dist)
        merged = cov.numpy()
        new = shard.new_rips_from_map(mine, merged, PAGES)
        dt, execs, retired = shard.job_totals(1.0 + rank, 100.0 * (rank + 1), 1e6, dist)
        np.save(os.path.join(out, f"r{rank}_merged.npy"), merged)
        np.save(os.path.join(out, f"r{rank}_new.npy"), new)
        np.save(os.path.join(out, f"r{rank}_tot.npy"), np.array([dt, execs, retired]))
    finally:
        dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_coverage_merge_and_totals(world, tmp_path):
    mp.start_processes(_worker, args=(world, _port(), str(tmp_path)), nprocs=world, start_method="spawn")
    covs = [_rank_cov(r) for r in range(world)]
    union = np.maximum.reduce(covs)
    for r in range(world):
        merged = np.load(tmp_path / f"r{r}_merged.npy")
        assert np.array_equal(merged, union)
        new = set(np.load(tmp_path / f"r{r}_new.npy").tolist())
        # new on rank r = bytes other ranks covered that rank r did not
        idx = np.nonzero((covs[r] == 0) & (union != 0))[0]
        want = {(PAGES[i // 4096] << 12) | (i % 4096) for i in idx}
        assert new == want and new
        dt, execs, retired = np.load(tmp_path / f"r{r}_tot.npy")
        assert dt == float(world)  # max over ranks of 1 + rank
        assert execs == sum(100.0 * (k + 1) for k in range(world))
        assert retired == 1e6 * world


def test_rank_streams_disjoint():
    seeds = {shard.rank_seed(0x5EED0001, r) for r in range(8)}
    assert len(seeds) == 8
