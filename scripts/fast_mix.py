"""Which executed instructions the engine's fast path leaves generic
(diagnostic): runs the CPU twin over a corpus with rip traces, reads each rip's
bytes from the snapshot, and classifies it with the engine's own decode +
digest (tests/native libsimlane.so, sim_digest). Counts are weighted by how
often the rip ran.
    python scripts/fast_mix.py <target dir> <inputs dir> <module name> [limit]"""
import collections
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.oracle_lib import Oracle  # noqa: E402
from wtf_amd.abi import regs_from_state  # noqa: E402
from wtf_amd.tools.snapshot import read_kdmp  # noqa: E402

OPS = ("ALU TEST MOV MOVZX MOVSX XCHG XADD CMPXCHG INCDEC NOT NEG SHIFT SHXD MULDIV IMUL BT BSF BSR TZCNT LZCNT "
       "POPCNT CMOV SETCC BSWAP CBW CWD LAHF SAHF FLAGOP NOP JCC JMP CALL RET PUSH POP PUSHF POPF LEAVE STRING INT3 "
       "HLT UD LEA SYS SSE UNIMPL SYS2 LOOP GEXT").split()
LOCS = "NONE GREG RM RAX OPREG IMM ONE CL PUSH POP MOFFS RBPMEM XLAT".split()

target, inputs, name = sys.argv[1], sys.argv[2], sys.argv[3]
limit = sys.argv[4] if len(sys.argv) > 4 else "100000"
tmp = tempfile.mkdtemp()
subprocess.run([os.path.join(ROOT, "oracle", "wtf_twin"), "run", "--name", name, "--target", target, "--input", inputs,
                "--limit", limit, "--trace-path", tmp, "--trace-type", "rip", "--lanes", "64"], check=True,
               stdout=subprocess.DEVNULL)
count = collections.Counter()
for f in os.listdir(tmp):
    if f.endswith(".trace"):
        for line in open(os.path.join(tmp, f)):
            if line.strip():
                count[int(line, 16)] += 1
pfn_off, blob, _ = read_kdmp(os.path.join(target, "state", "mem.dmp"))
pages = {pfn: bytes(blob[off:off + 4096]) for pfn, off in pfn_off.items()}
o = Oracle(pages=pages)
st = json.load(open(os.path.join(target, "state", "regs.json")))
L = C.CDLL(os.path.join(ROOT, "tests", "native", "libsimlane.so"))
L.sim_digest.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32)]
gen = collections.Counter()
total = fast = 0
raw = json.load(open(os.path.join(target, "state", "regs.json")))
conv = {k: int(v, 16) for k, v in raw.items() if isinstance(v, str) and v.startswith("0x")}
r = regs_from_state({"rip": conv["rip"], "rflags": conv["rflags"], **{k: v for k, v in conv.items()}})
r.cr0, r.cr3, r.cr4, r.efer = conv["cr0"], conv["cr3"], conv["cr4"], conv["efer"]
o.restore(r)
for rip, n in count.items():
    try:
        b = o.read_virt(rip, 16)
    except Exception:
        b = o.read_virt(rip, 4096 - (rip & 0xfff))
    out = (C.c_uint32 * 15)()
    L.sim_digest(b, len(b), out)
    total += n
    if out[0] == 0 and out[3] != 0:
        fast += n
        continue
    dr, op, sub, fop, ln, segp, p67, rep, rex, asz, bsz, asrc, bsrc, mem, sup = list(out)
    key = (OPS[op] if op < len(OPS) else op, f"sub{sub:#x}", f"a={LOCS[asrc] if asrc < len(LOCS) else asrc}",
           f"b={LOCS[bsrc] if bsrc < len(LOCS) else bsrc}", "mem" if mem else "reg", f"asz{asz}",
           "seg" if segp else "", "p67" if p67 else "", "rep" if rep else "", b[:ln].hex())
    gen[key] += n
print(f"{total} instructions, fast-path forms {fast} ({100 * fast / max(1, total):.1f}%)")
for k, n in gen.most_common(30):
    print(f"  {n:9d} {100 * n / total:5.2f}%  {' '.join(x for x in k if x)}")
