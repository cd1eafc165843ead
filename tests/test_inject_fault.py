"""Exception delivery through the guest IDT and
PageFaultsMemoryIfNeeded's #PF injection (bochscpu_backend.cc:917-999), on the
HEVD snapshot (IDT + TSS present): the oracle on the CPU; the GPU engine
through wtfgpu_inject_fault against the oracle, register by register and
frame word by frame word."""
import struct

import pytest

from tests.oracle_lib import Oracle
from wtf_amd import abi
from wtf_amd.tools import hevd

ERR = 2 | 4  # ErrorWrite | ErrorUser
ADDR = 0x20000000


@pytest.fixture(scope="module")
def snap(tmp_path_factory):
    sp, st, symbols, _ = hevd.build_space(str(tmp_path_factory.mktemp("hevd")))
    return sp, st, symbols


def _frame(read, rsp):
    return struct.unpack("<6Q", read(rsp, 48))


def test_oracle_delivers_pf_from_user_mode(snap):
    sp, st, symbols = snap
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(abi.regs_from_state(st))
    before = o.regs()
    assert o.inject_fault(14, ERR, ADDR)
    r = o.regs()
    assert r.rip == symbols["nt!KiPageFault"]
    assert r.cr2 == ADDR
    assert r.seg[1].selector == 0x10 and r.seg[2].selector == 0  # ring 0, NULL SS
    rsp0 = (hevd.KSTACK + hevd.KSTACK_PAGES * 0x1000 - 0x40) & ~0xF  # TSS.RSP0 on the privilege change
    assert r.gpr[4] == rsp0 - 48
    err, rip, cs, rflags, rsp, ss = _frame(o.read_virt, r.gpr[4])
    assert (err, rip, cs, rflags, rsp, ss) == (ERR, before.rip, 0x33, before.rflags, before.gpr[4], 0x2B)
    assert not (r.rflags & 0x200)  # interrupt gate: IF cleared
    # a second fault before any instruction retired is a double fault: not delivered
    assert not o.inject_fault(14, ERR, ADDR)


@pytest.mark.gpu
def test_gpu_inject_matches_oracle(snap):
    from wtf_amd.engine import Engine
    sp, st, symbols = snap
    pfns, blob = sp.phys()
    eng = Engine(0)
    try:
        eng.load_pool(pfns, blob)
        eng.alloc_lanes(128, overlay_pages=16, cov_entries=256)
        eng.set_initial_state(abi.regs_from_state(st))
        eng.restore()
        lanes = list(range(0, 128, 3))
        addrs = [ADDR + 0x1000 * i for i in lanes]
        assert all(eng.inject_fault(lanes, 14, ERR, addrs))
        assert not any(eng.inject_fault(lanes[:4], 14, ERR, addrs[:4]))  # double fault
        g = eng.read_gprs()
        for lane, addr in zip(lanes, addrs):
            o = Oracle(pfns=pfns, blob=blob)
            o.restore(abi.regs_from_state(st))
            assert o.inject_fault(14, ERR, addr)
            r = o.regs()
            assert list(g[lane][:16]) == list(r.gpr) and g[lane][16] == r.rip and g[lane][17] == r.rflags
            assert eng.read_regs(lane, 1)[0].cr2 == addr
            assert eng.get_cr(lane, 2) == addr          # GetReg(Cr2): the lane's own
            assert eng.get_cr(lane, 3) == st["cr3"]
            assert eng.read_virt(lane, r.gpr[4], 48) == o.read_virt(r.gpr[4], 48)
        untouched = eng.read_gprs()[1]
        assert untouched[16] == st["rip"]
        assert eng.get_cr(1, 2) == st["cr2"]
        eng.set_cr(1, 2, 0x1234000)                    # SetReg(Cr2)
        assert eng.get_cr(1, 2) == 0x1234000 and eng.read_regs(1, 1)[0].cr2 == 0x1234000
        assert eng.get_cr(2, 2) == st["cr2"]
    finally:
        eng.close()
