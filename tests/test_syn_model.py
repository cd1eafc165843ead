"""The numpy restatement of the SYN loop (wtf_amd/tools/syn.py `model`), which
the headline-config GPU test uses to check all 65,536 lanes of a batch, is
itself checked here against the C oracle, lane by lane: registers, flags,
retired count and scratch page."""
import numpy as np

from tests.syn_harness import oracle_lane
from wtf_amd.abi import EXIT_BREAKPOINT
from wtf_amd.tools import syn

REGS = {"rax": 0, "rcx": 1, "rdx": 2, "rbx": 3, "r8": 8, "r9": 9, "r10": 10}


def test_model_matches_oracle():
    sp, st, _ = syn.build()
    inp = syn.inputs(48, seed=0xABC)
    inp[:40, 1] &= 0x3  # mostly short trips, a few long ones
    table = bytes(sp.pages[sp.translate(syn.TABLE_VA) >> 12])
    regs, scratch = syn.model(inp, table)
    for i in range(len(inp)):
        o, ex = oracle_lane(sp, st, inp[i])
        assert ex.status == EXIT_BREAKPOINT and ex.icount == syn.expected_instructions(inp[i:i + 1])[0]
        r = o.regs()
        for name, k in REGS.items():
            assert int(regs[name][i]) == r.gpr[k], (i, name)
        assert r.rflags == 0x246
        page = np.frombuffer(o.read_virt(syn.SCRATCH_VA, 4096), dtype=np.uint64)
        assert np.array_equal(page, scratch[i]), i
