"""The N>1 control plane of bench.py on CPU (world size 2, gloo): rank 0's
RCCL id reaches every rank (wtf_amd/shard.py share_bytes) and the timed
region reduces to max-over-ranks time and sum-over-ranks work (job_totals).
The data-path merge itself (C++ FuzzSession + CoverageExchange_t) is tested
with two twin shards in tests/test_shard_twin.py."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from wtf_amd import shard


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        got = shard.share_bytes(bytes(range(128)) if rank == 0 else None, dist)
        dt, execs, retired = shard.job_totals(1.0 + rank, 100.0 * (rank + 1), 1e6, dist)
        np.save(os.path.join(out, f"r{rank}.npy"), np.array([dt, execs, retired]))
        with open(os.path.join(out, f"r{rank}.id"), "wb") as f:
            f.write(got)
    finally:
        dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_id_broadcast_and_totals(world, tmp_path):
    mp.start_processes(_worker, args=(world, _port(), str(tmp_path)), nprocs=world, start_method="spawn")
    for r in range(world):
        assert (tmp_path / f"r{r}.id").read_bytes() == bytes(range(128))
        dt, execs, retired = np.load(tmp_path / f"r{r}.npy")
        assert dt == float(world)  # max over ranks of 1 + rank
        assert execs == sum(100.0 * (k + 1) for k in range(world))
        assert retired == 1e6 * world
