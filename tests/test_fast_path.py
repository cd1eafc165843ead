"""The fast loop's forms (engine_fast.h: digest + fast_exec) on the CPU.

k_run runs an instruction through its FOp digest first and falls back to the
generic exec() only on a miss. tests/native/sim_lane.cc, in fast mode, runs the
same order on the host-built device code, so every native-execution vector
(integer, SSE, AVX2) is checked through the fast forms too, including the
memory window, and the vector moves the guests' memcpy / memset loops run
(FO_VLD / FO_VST / FO_VMOV / FO_VZU) are checked at every alignment, at page
ends and with the SSE / AVX state switched off, against the generic path and
the oracle.
"""
import ctypes as C
import gzip
import json
import os

import pytest

from tests.golden.gen_native_vectors import splitmix_bytes
from tests.golden.gen_sse_vectors import window_in
from tests.oracle_lib import Oracle
from tests.test_sse import BUF, layout, sim_lib, sim_run
from wtf_amd.abi import EXIT_FAULT

HERE = os.path.dirname(os.path.abspath(__file__))
INT3 = 3


def vectors(name):
    with gzip.open(os.path.join(HERE, "golden", name), "rt") as f:
        return json.load(f)


def run_both(L, sp, regs, win_va, limit=0):
    """(slow result, fast result, instructions the fast forms retired)."""
    cnt = C.c_uint64(0)
    slow = sim_run(L, sp, regs, limit=limit, win_va=win_va)
    fast = sim_run(L, sp, regs, limit=limit, fast=True, counter=cnt, win_va=win_va)
    return slow, fast, cnt.value


def same(a, b):
    return (a.status == b.status and a.vector == b.vector and a.rip == b.rip and a.icount == b.icount and
            list(a.gpr) == list(b.gpr) and a.rflags == b.rflags and list(a.xmm) == list(b.xmm) and
            list(a.ymmh) == list(b.ymmh) and a.nbytes == b.nbytes and bytes(a.win) == bytes(b.win))


def test_integer_vectors_through_fast_forms():
    doc = vectors("native_vectors.json.gz")
    L = sim_lib()
    buf_va = int(doc["buf_va"], 16)
    fails, fast_total = [], 0
    for c in doc["cases"]:
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, splitmix_bytes(int(c["seed"], 16), 256))
        for i in range(16):
            regs.gpr[i] = int(c["in"][i], 16)
        regs.rflags = int(c["fl"], 16) | 0x200
        cnt = C.c_uint64(0)
        out = sim_run(L, sp, regs, fast=True, counter=cnt, win_va=buf_va)
        fast_total += cnt.value
        want = [int(x, 16) for x in c["out"]]
        got = list(out.gpr)
        if c["cls"] == "bsx" and (int(c["flo"], 16) & 0x40):
            got[c["dst"]] = want[c["dst"]]
        win = bytearray(splitmix_bytes(int(c["seed"], 16), 256))
        for i, v in c["diff"]:
            win[i] = v
        if out.status != INT3 or out.icount != 1:
            fails.append((c["name"], "exit", out.status))
        elif got != want or (out.rflags ^ int(c["flo"], 16)) & int(c["fmask"], 16):
            fails.append((c["name"], "regs"))
        elif bytes(out.win[:256]) != bytes(win):
            fails.append((c["name"], "mem"))
    assert not fails, f"{len(fails)} mismatches, first: {fails[:6]}"
    assert fast_total > len(doc["cases"]) // 3, fast_total


@pytest.mark.parametrize("name", ["sse_vectors.json.gz", "avx_vectors.json.gz"])
def test_vector_vectors_fast_equals_slow(name):
    doc = vectors(name)
    L = sim_lib()
    buf_va = int(doc["buf_va"], 16)
    avx = name.startswith("avx")
    fails, fast_total = [], 0
    for c in doc["cases"]:
        win = splitmix_bytes(int(c["seed"], 16), 256) if avx else window_in(int(c["seed"], 16), c["ldmx"])
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, win)
        for i in range(16):
            regs.gpr[i] = int(c["in"][i], 16)
        regs.rflags = int(c["fl"], 16) | 0x200
        if avx:
            ys = [int(v, 16) for v in c["yin"]]
            for i in range(16):
                regs.xmm[i][0], regs.xmm[i][1] = ys[4 * i], ys[4 * i + 1]
                regs.ymmh[i][0], regs.ymmh[i][1] = ys[4 * i + 2], ys[4 * i + 3]
        else:
            xs = [int(v, 16) for v in c["xin"]]
            for i in range(16):
                regs.xmm[i][0], regs.xmm[i][1] = xs[2 * i], xs[2 * i + 1]
            regs.mxcsr = int(c["mx"], 16)
        slow, fast, n = run_both(L, sp, regs, buf_va)
        fast_total += n
        want = bytearray(win)
        for i, v in c["diff"]:
            want[i] = v
        if not same(slow, fast):
            fails.append((c["name"], c["code"], "fast != slow"))
        elif bytes(fast.win[:256]) != bytes(want):
            fails.append((c["name"], c["code"], "mem"))
    assert not fails, f"{len(fails)} mismatches, first: {fails[:6]}"
    assert fast_total > 50, fast_total


# ---- the memcpy / memset forms at every alignment and at page ends
MOVES = {
    "movdqu load": "f30f6f0e",            # movdqu xmm1, [rsi]
    "movdqu store": "f30f7f0f",           # movdqu [rdi], xmm1
    "movups load": "0f100e",
    "movups store": "0f110f",
    "movdqa load": "660f6f0e",            # aligned: #GP when misaligned
    "movdqa store": "660f7f0f",
    "movaps store": "0f290f",
    "vmovdqu ymm load": "c5fe6f0e",
    "vmovdqu ymm store": "c5fe7f0f",
    "vmovdqu xmm load": "c5fa6f0e",       # VEX.128: zeroes bits 255:128
    "vmovdqu xmm store": "c5fa7f0f",
    "vmovdqa ymm load": "c5fd6f0e",
    "vmovdqa ymm store": "c5fd7f0f",
    "vmovups ymm store": "c5fc110f",
    "vmovaps ymm load": "c5fc280e",
    "movdqa reg": "660f6fca",             # movdqa xmm1, xmm2
    "movdqu reg store form": "f30f7fd1",  # movdqu xmm1, xmm2 (0f 7f, r/m = xmm1)
    "vmovdqu ymm reg": "c5fe6fca",
    "vmovdqu xmm reg": "c5fa6fca",
    "pxor zero": "660fefc9",
    "xorps zero": "0f57c9",
    "vpxor zero 128": "c5f1efc9",
    "vpxor zero 256": "c5f5efc9",
    "pxor other": "660fefca",             # not the idiom: generic path
    "vzeroupper": "c5f877",
}


PRIV = "8a078807"  # mov al, [rdi]; mov [rdi], al: the destination page becomes the lane's own first


def move_case(code_hex, off_src, off_dst, cr0=None, cr4=None, xcr0=None):
    code = bytes.fromhex(code_hex)
    page = BUF & ~0xFFF
    sp, regs = layout(code, page, bytes((i * 7 + 3) & 0xFF for i in range(4096)), cr0=cr0, cr4=cr4)
    regs.gpr[6] = page + off_src  # rsi
    regs.gpr[7] = page + off_dst  # rdi
    for k in range(16):
        regs.xmm[k][0], regs.xmm[k][1] = 0x1111111111111111 * (k + 1), 0x0101010101010101 * (k + 3)
        regs.ymmh[k][0], regs.ymmh[k][1] = 0xA0A0A0A0A0A0A0A0 + k, 0xB0B0B0B0B0B0B0B0 + k
    if xcr0 is not None:
        regs.xcr0 = xcr0
    return sp, regs


@pytest.mark.parametrize("name", sorted(MOVES))
def test_moves_fast_equals_slow_and_oracle(name):
    L = sim_lib()
    page = BUF & ~0xFFF
    offsets = [(s, d) for s in (0, 1, 3, 7, 8, 13, 16, 24, 31) for d in (0, 2, 5, 8, 9, 16, 30)]
    offsets += [(4096 - 32, 4096 - 16), (4096 - 16, 4096 - 32), (4096 - 20, 4096 - 9), (4096 - 1, 4096 - 33)]
    fast_runs = 0
    for s, d in offsets:
        sp, regs = move_case(PRIV + MOVES[name], s, d)
        slow, fast, n = run_both(L, sp, regs, page + 0x100 if max(s, d) < 0x100 else page + 4096 - 256)
        fast_runs += n
        assert same(slow, fast), (name, s, d, slow.status, fast.status)
        # the priming moves run fast too (the cold TLB and the copy-on-write are
        # served in place, fast_fill); the vector form runs fast unless it
        # faults, crosses a page or is generic
        size = 32 if name.startswith("v") and "ymm" in name else 16
        off = (d if "store" in name and "reg" not in name else s) if ("load" in name or "store" in name) else 0
        crosses = "reg" not in name and ("load" in name or "store" in name) and off + size > 4096
        assert n == 2 + (0 if slow.status != INT3 or crosses or name == "pxor other" else 1), (name, s, d, n)
        pfns, blob = sp.phys()
        o = Oracle(pfns=pfns, blob=blob)
        o.restore(regs)
        ex = o.run()
        r = o.regs()
        if slow.status == INT3:
            assert ex.status == INT3 and o.icount() == slow.icount, (name, s, d)
            assert [r.xmm[i][h] for i in range(16) for h in range(2)] == list(fast.xmm), (name, s, d)
            assert [r.ymmh[i][h] for i in range(16) for h in range(2)] == list(fast.ymmh), (name, s, d)
            wv = page + 0x100 if max(s, d) < 0x100 else page + 4096 - 256
            assert o.read_virt(wv, 256) == bytes(fast.win[:256]), (name, s, d)
        else:
            assert (ex.status, ex.vector) == (slow.status, slow.vector), (name, s, d)
    # two priming moves per case run fast; "pxor other" itself never does
    assert (fast_runs == 2 * len(offsets)) if name == "pxor other" else fast_runs >= 2 * len(offsets) + 5, (
        name, fast_runs)


def test_vector_moves_defer_to_generic_when_state_is_off():
    """CR0.TS (#NM), CR0.EM / no OSFXSR (#UD), no OSXSAVE or XCR0 (#UD): the
    fast forms leave the lane to exec(), which raises the fault."""
    L = sim_lib()
    cases = [
        ("f30f6f0e", dict(cr0=0x80050031 | 8), 7),
        ("f30f6f0e", dict(cr0=0x80050031 | 4), 6),
        ("f30f6f0e", dict(cr4=0x370678 & ~0x200), 6),
        ("c5fe6f0e", dict(cr4=0x370678 & ~0x40000), 6),
        ("c5fe6f0e", dict(xcr0=3), 6),
        ("c5fe7f0f", dict(cr0=0x80050031 | 8), 7),
        ("c5f877", dict(xcr0=3), 6),
        ("660fefc9", dict(cr0=0x80050031 | 8), 7),
    ]
    for code, kw, vec in cases:
        sp, regs = move_case(code, 0, 64, **kw)
        slow, fast, n = run_both(L, sp, regs, 0)
        assert (fast.status, fast.vector) == (EXIT_FAULT, vec), (code, kw, fast.status, fast.vector)
        assert same(slow, fast) and n == 0, (code, kw)


def test_aligned_forms_fault_when_misaligned_on_fast_path():
    L = sim_lib()
    for code in ("660f6f0e", "660f7f0f", "0f290f", "c5fd6f0e", "c5fd7f0f", "c5fc280e"):
        sp, regs = move_case(code, 8 if code.endswith("0e") else 0, 8)
        slow, fast, _ = run_both(L, sp, regs, 0)
        assert (fast.status, fast.vector) == (EXIT_FAULT, 13), code
        assert same(slow, fast), code


def test_copy_loop_program_fast_equals_slow():
    """The guests' memcpy shape: 32-byte vmovdqu blocks, 16-byte movdqu blocks,
    vzeroupper, at several misalignments, with copy-on-write on first writes."""
    # rcx = count of 32-byte blocks; rsi, rdi
    prog = bytes.fromhex(
        "c5fe6f06"      # vmovdqu ymm0, [rsi]
        "c5fe7f07"      # vmovdqu [rdi], ymm0
        "4883c620"      # add rsi, 32
        "4883c720"      # add rdi, 32
        "48ffc9"        # dec rcx
        "75eb"          # jnz loop
        "c5f877"        # vzeroupper
        "f30f6f06"      # movdqu xmm0, [rsi]
        "f30f7f07"      # movdqu [rdi], xmm0
    )
    L = sim_lib()
    page = BUF & ~0xFFF
    for s, d in ((0, 0), (1, 0), (3, 9), (16, 7), (5, 37)):
        sp, regs = move_case(prog.hex(), s, 0x400 + d)
        regs.gpr[1] = 20
        slow, fast, n = run_both(L, sp, regs, page + 0x400)
        assert same(slow, fast), (s, d)
        assert fast.status == INT3 and n > 60, (s, d, fast.status, n)
        src = bytes((i * 7 + 3) & 0xFF for i in range(4096))
        assert bytes(fast.win[d:d + 656]) == src[s:s + 656][:512 - d], (s, d)


@pytest.mark.parametrize("op", [0x06, 0x07, 0x0E, 0x16, 0x17, 0x1E, 0x1F, 0x27, 0x2F, 0x37, 0x3F, 0x60, 0x61,
                                0x82, 0x9A, 0xD4, 0xD5, 0xD6, 0xEA])
def test_opcodes_invalid_in_64bit_mode_raise_ud(op):
    """SDM opcode map (i64): #UD on the oracle and the engine's code, at the
    instruction, nothing retired (they were engine errors before)."""
    L = sim_lib()
    code = bytes([op, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00])
    sp, regs = layout(code, BUF, bytes(256))
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.step()
    assert (ex.status, ex.vector) == (EXIT_FAULT, 6), hex(op)
    for fast in (False, True):
        out = sim_run(L, sp, regs, fast=fast)
        assert (out.status, out.vector, out.icount, out.rip) == (EXIT_FAULT, 6, 0, regs.rip), (hex(op), fast)


def test_indirect_branches_unary_bit_and_segment_forms_fast_equals_slow():
    """The forms added to the fast path for tlv / HEVD's hot code: fs / gs
    relative moves, not / neg, test with a memory operand, shifts by cl,
    bt / bts with register and immediate bit numbers, call [mem], call reg,
    jmp reg: the fast form gives the generic path's lane, and runs."""
    from tests.test_sse import CODE_VA
    code = bytes.fromhex(
        "65488b042510000000"   # 0  mov rax, gs:[0x10]
        "6548890425 18000000"  # 9  mov gs:[0x18], rax
        "48f7d0"               # 18 not rax
        "48f7d8"               # 21 neg rax
        "48f70705000000"       # 24 test qword [rdi], 5
        "48854708"             # 31 test [rdi+8], rax
        "48d3e0"               # 35 shl rax, cl
        "480fabc8"             # 38 bts rax, rcx
        "480fbae203"           # 42 bt rdx, 3
        "ff5710"               # 47 call qword [rdi+16] -> 60
        .replace(" ", "")) + b"\xcc" * 10
    code += bytes.fromhex(
        "5b"                   # 60 pop rbx
        "488d1d04000000"       # 61 lea rbx, [rip+4] -> 72
        "ffd3"                 # 68 call rbx
        "cccc"                 # 70
        "59"                   # 72 pop rcx
        "488d1503000000"       # 73 lea rdx, [rip+3] -> 83
        "ffe2"                 # 80 jmp rdx
        "cc")                  # 82; 83 is layout's trailing int3
    assert len(code) == 83
    page = BUF & ~0xFFF
    win = bytearray(512)
    win[0:8] = (0x1234).to_bytes(8, "little")
    win[8:16] = (0xF0F0).to_bytes(8, "little")
    win[16:24] = (CODE_VA + 60).to_bytes(8, "little")
    win[0x110:0x118] = (0xDEADBEEF).to_bytes(8, "little")
    L = sim_lib()
    sp, regs = layout(code, page, bytes(win))
    regs.gpr[4], regs.gpr[7], regs.gpr[1], regs.gpr[2] = page + 0x800, page, 5, 0xFF
    regs.seg[5].base = page + 0x100  # gs
    slow, fast, n = run_both(L, sp, regs, page)
    assert same(slow, fast)
    assert fast.status == INT3 and fast.rip == CODE_VA + 83, (fast.status, hex(fast.rip))
    assert n == 16, n  # every instruction but the trailing int3 ran on the fast path
    assert bytes(fast.win[0x118:0x120]) == (0xDEADBEEF).to_bytes(8, "little")


def test_high_byte_register_forms_fast_equals_slow_and_oracle():
    """ah / ch / dh / bh operands (8-bit registers 4..7 without REX) on the fast
    path: read as bits 15:8 of rax..rbx, written merged into those bits, for
    mov / ALU / test / inc / not / neg / shifts / setcc / movzx / movsx and the
    memory forms; the fast forms give the generic path's and the oracle's lane."""
    from tests.test_sse import CODE_VA
    code = bytes.fromhex(
        "f6c510"        # test ch, 0x10
        "88e0"          # mov al, ah
        "88c4"          # mov ah, al
        "8ae1"          # mov ah, cl
        "80c47f"        # add ah, 0x7f
        "28fc"          # sub ah, bh
        "30d6"          # xor dh, dl
        "38ec"          # cmp ah, ch
        "fec4"          # inc ah
        "f6d7"          # not bh
        "f6de"          # neg dh
        "d0e4"          # shl ah, 1
        "c0ef03"        # shr bh, 3
        "0f94c4"        # sete ah
        "0fb6c4"        # movzx eax, ah
        "480fbecd"      # movsx rcx, ch
        "8827"          # mov [rdi], ah
        "8a7701"        # mov dh, [rdi+1]
        "0067 02"       # add [rdi+2], ah
        "8467 03"       # test [rdi+3], ah
        .replace(" ", ""))
    page = BUF & ~0xFFF
    win = bytearray(range(256)) * 2
    L = sim_lib()
    sp, regs = layout(code, page, bytes(win))
    regs.gpr[0], regs.gpr[1], regs.gpr[2], regs.gpr[3] = (0x1122334455667788, 0x99AABBCCDDEEFF10,
                                                          0x0F1E2D3C4B5A6978, 0x8070605040302010)
    regs.gpr[7] = page
    slow, fast, n = run_both(L, sp, regs, page)
    assert same(slow, fast)
    assert n == 20, n  # every form ran fast
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.run()
    r = o.regs()
    assert ex.status == INT3 and o.icount() == fast.icount
    assert [int(x) for x in fast.gpr] == list(r.gpr) and fast.rflags == r.rflags
    assert o.read_virt(page, 256) == bytes(fast.win[:256])


def test_system_call_forms_fast_equals_slow_and_oracle():
    """syscall, swapgs and sysretq (REX.W) between fast-path forms: a user
    syscall into a kernel stub that swaps gs twice and returns; registers, rip,
    rflags match the generic path and the oracle. The system forms stay on the
    generic step (a fast form for them cost more in register pressure than it
    saved); only the mov runs fast. At ring 3,
    swapgs and sysretq raise #GP as exec() does."""
    from tests.test_sse import CODE_VA
    code = bytes.fromhex(
        "0f05"                  # 0  syscall -> lstar = 8
        "cc" "cccccccccc"       # 2  int3 (sysretq returns here)
        "0f01f8"                # 8  swapgs
        "48c7c034120000"        # 11 mov rax, 0x1234
        "0f01f8"                # 18 swapgs
        "480f07")               # 21 sysretq
    page = BUF & ~0xFFF
    L = sim_lib()
    sp, regs = layout(code, page, bytes(256))
    regs.cr4 &= ~(3 << 20)  # no SMEP / SMAP: the stub runs on the test's user code page
    regs.lstar = CODE_VA + 8
    regs.kernel_gs_base = 0xAAAA000
    regs.seg[5].base = 0xBBBB000
    regs.gpr[11] = 0x55
    slow, fast, n = run_both(L, sp, regs, page)
    assert same(slow, fast)
    assert fast.status == INT3 and fast.rip == CODE_VA + 2, (fast.status, hex(fast.rip))
    assert fast.gpr[0] == 0x1234 and fast.gpr[1] == CODE_VA + 2
    assert n == 1, n  # the mov; the system forms run on the generic step
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.run()
    r = o.regs()
    assert ex.status == INT3 and o.icount() == fast.icount
    assert [int(x) for x in fast.gpr] == list(r.gpr) and fast.rflags == r.rflags
    # ring 3: swapgs / sysretq are #GP(0), raised by the slow step
    for op in ("0f01f8", "480f07"):
        sp, regs = layout(bytes.fromhex(op), page, bytes(256))
        slow, fast, n = run_both(L, sp, regs, page)
        assert same(slow, fast) and (fast.status, fast.vector) == (EXIT_FAULT, 13) and n == 0, (op, fast.status)
