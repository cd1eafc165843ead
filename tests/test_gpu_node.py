"""The node library (include/wtfnode.h) and the coverage-map merge plumbing
on one MI355X.

  * wtfgpu_coverage_absorb: bytes another shard set in the device map (here
    written straight into it, as an RCCL MAX all-reduce would) come back as
    rips; this context's own commits do not;
  * libwtfnode: tlv_server steps one batch at a time; its counters agree with
    themselves and with the same workload run by `wtfgpu fuzz`.
"""
import ctypes as C
import os

import numpy as np
import pytest

from tests import tlv_harness as H

pytestmark = pytest.mark.gpu


def test_absorb_reports_remote_bytes_only():
    import torch

    from tests.syn_harness import make_engine
    from wtf_amd.tools import syn

    eng, sp, st = make_engine(64)
    try:
        eng.commit_coverage([syn.CODE_VA, syn.CODE_VA + 3])  # own finds
        n = C.c_uint64()
        assert eng.L.wtfgpu_coverage_absorb(eng.ctx, None, 0, C.byref(n)) == 0 and n.value == 0
        p, nb = C.c_void_p(), C.c_uint64()
        assert eng.L.wtfgpu_coverage_device_map(eng.ctx, C.byref(p), C.byref(nb)) == 0
        assert nb.value == 2 * 4096  # code page + exit page slots

        class Buf:
            __cuda_array_interface__ = {"shape": (nb.value,), "typestr": "|u1", "data": (p.value, False),
                                        "version": 2, "strides": None}

        m = torch.as_tensor(Buf(), device="cuda:0")
        # a remote shard's finds: slot 0 is the code page (set_code_pages order)
        m[9] = 1
        m[0x41] = 1
        torch.cuda.synchronize()
        assert eng.L.wtfgpu_coverage_absorb(eng.ctx, None, 0, C.byref(n)) == 0 and n.value == 2
        out = (C.c_uint64 * 2)()
        assert eng.L.wtfgpu_coverage_absorb(eng.ctx, out, 2, C.byref(n)) == 0
        assert list(out) == [syn.CODE_VA + 9, syn.CODE_VA + 0x41]
        assert eng.L.wtfgpu_coverage_absorb(eng.ctx, None, 0, C.byref(n)) == 0 and n.value == 0  # seen now
    finally:
        eng.close()


def test_node_library_steps(tmp_path):
    """libwtfnode steps one slice at a time (continuous batching): counters
    only grow, every testcase it finishes is accounted once. The lanes run in
    two pipelined halves, so a half's results arrive one step after its slice."""
    from wtf_amd.node import Node

    d = H.build_target(str(tmp_path / "tlv"))
    node = Node("tlv_server", d, lanes=4096, limit=100000, seed=1337)
    try:
        node.step()
        node.step()
        s1 = node.stats()
        for _ in range(6):
            node.step()
        s7 = node.stats()
        assert s7["batches"] == 8 and s7["execs"] > s1["execs"] >= 0
        assert s7["retired"] > s1["retired"] >= 0 and s7["kernel_launches"] >= 4  # harvested slices
        assert s7["alg_bytes"] > 0 and s7["group_steps"] > 0 and s7["errors"] == 0
        assert s7["coverage"] > 100 and s7["corpus"] >= 1
        summ = node.summary()
        assert summ["execs"] == s7["execs"] and summ["backend"]["kind"] == "gpu"
    finally:
        node.close()
