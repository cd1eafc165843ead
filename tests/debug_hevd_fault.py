"""Debug aid (not a test): run the HEVD null_deref testcase on one GPU lane and
on the oracle up to nt!KiPageFault and print both delivery frames."""
import struct
import sys
import tempfile

sys.path.insert(0, __file__.rsplit("/tests/", 1)[0])
from tests.oracle_lib import Oracle  # noqa: E402
from wtf_amd import abi  # noqa: E402
from wtf_amd.tools import hevd  # noqa: E402


def main():
    sp, st, symbols, _ = hevd.build_space(tempfile.mkdtemp())
    pfns, blob = sp.phys()
    dbg, kpf = symbols["nt!DbgPrintEx"], symbols["nt!KiPageFault"]
    buf = struct.pack("<I", 0xBAD0B0B0)
    # oracle
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(abi.regs_from_state(st))
    o.set_breakpoints([dbg, kpf])
    r = o.regs()
    r.gpr[2] = 0x222013
    r.gpr[9] = len(buf)
    o.set_regs(r)
    o.write_virt(st["r8"], buf)
    o.write_virt(st["rsp"] + 0x30, struct.pack("<Q", len(buf)))
    skip = False
    while True:
        e = o.run(skip_bp=skip)
        r = o.regs()
        if e.status == abi.EXIT_BREAKPOINT and r.rip == dbg:
            ret = struct.unpack("<Q", o.read_virt(r.gpr[4], 8))[0]
            r.rip, r.gpr[4], r.gpr[0] = ret, r.gpr[4] + 8, 0
            o.set_regs(r)
            skip = False
            continue
        break
    print("oracle", e.status, hex(r.rip), "icount", o.icount(), "rsp", hex(r.gpr[4]), "cs", hex(r.seg[1].selector),
          "frame", [hex(x) for x in struct.unpack("<6Q", o.read_virt(r.gpr[4], 48))])
    # gpu
    from wtf_amd.engine import Engine
    eng = Engine(0)
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(64, overlay_pages=16, cov_entries=256)
    eng.set_initial_state(abi.regs_from_state(st))
    eng.set_breakpoints([dbg, kpf])
    eng.restore()
    g = eng.read_gprs()
    g[0][2] = 0x222013
    g[0][9] = len(buf)
    eng.write_gprs(g)
    eng.write_virt(0, st["r8"], buf)
    eng.write_virt(0, st["rsp"] + 0x30, struct.pack("<Q", len(buf)))
    eng.stop(list(range(1, 64)))
    while True:
        eng.run(0, 64)
        ex = eng.exits(0, 1)[0]
        g = eng.read_gprs(0, 1)
        if ex.status == abi.EXIT_BREAKPOINT and g[0][16] == dbg:
            ret = struct.unpack("<Q", eng.read_virt(0, int(g[0][4]), 8))[0]
            g[0][16], g[0][4], g[0][0] = ret, g[0][4] + 8, 0
            eng.write_gprs(g)
            eng.resume([0], [False])
            continue
        break
    rr = eng.read_regs(0, 1)[0]
    print("gpu   ", ex.status, hex(int(g[0][16])), "icount", ex.icount, "rsp", hex(int(g[0][4])), "cs",
          hex(rr.seg[1].selector), "frame", [hex(x) for x in struct.unpack("<6Q", eng.read_virt(0, int(g[0][4]), 48))])
    eng.close()


if __name__ == "__main__":
    main()
