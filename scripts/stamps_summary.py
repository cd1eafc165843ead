"""Sums the per-launch `wtfgpu stamps` lines of a stamps build into cycles per
wave-step, and the generic ops the slow step ran (O_* numbers of engine_ops.h)."""
import re
import sys

PAT = re.compile(r"wtfgpu stamps \(cycles per wave-step, (\d+) steps\): fast loop (\S+), slow: xlate\+fill (\S+), "
                 r"coverage (\S+), exec (\S+), cross-page ([^;\s]+)(?:; slow steps: miss (\d+), codepage (\d+), "
                 r"ucmiss (\d+), other (\d+))?(?:; fast lookup ([^,\s]+), fast exec ([^,\s]+))?(?:, bp (\S+))?")
OPS = ("ALU TEST MOV MOVZX MOVSX XCHG XADD CMPXCHG INCDEC NOT NEG SHIFT SHXD MULDIV IMUL BT BSF BSR TZCNT LZCNT "
       "POPCNT CMOV SETCC BSWAP CBW CWD LAHF SAHF FLAGOP NOP JCC JMP CALL RET PUSH POP PUSHF POPF LEAVE STRING INT3 "
       "HLT UD LEA SYS SSE UNIMPL SYS2 LOOP GEXT").split()
# 56 + breakpoint action kind (include/wtfgpu.h WTFGPU_BPACT_*): breakpoint hits
OPS = OPS + [str(i) for i in range(len(OPS), 56)] + \
    "BP:host BP:return BP:setgprs BP:feed BP:rdrand BP:stopok BP:stopargs BP:none".split()
for path in sys.argv[1:]:
    steps = 0
    tot = [0.0] * 8
    why = [0] * 4
    ops = {}
    bpc = {}
    for line in open(path):
        if line.startswith("wtfgpu stamps bp_apply cycles by kind:"):
            for kv in line.split(":", 1)[1].split():
                k, v = kv.split(":")
                bpc[int(k)] = bpc.get(int(k), 0) + int(v)
            continue
        if line.startswith("wtfgpu stamps generic ops:"):
            for kv in line.split(":", 1)[1].split():
                k, v = kv.split(":")
                # index: op | why << 6 | covered << 8 (why the fast loop left the
                # group: miss, codepage, ucmiss, other)
                i = int(k)
                name = (OPS[i & 63] if (i & 63) < len(OPS) else str(i & 63)) + ("(cov)" if i & 256 else "") + \
                    "/" + ("miss", "codepage", "ucmiss", "other")[(i >> 6) & 3]
                ops[name] = ops.get(name, 0) + int(v)
            continue
        m = PAT.search(line)
        if not m:
            continue
        n = int(m.group(1))
        steps += n
        for i in range(5):
            tot[i] += float(m.group(2 + i)) * n
        if m.group(11):
            tot[5] += float(m.group(11)) * n
            tot[6] += float(m.group(12)) * n
        if m.group(13):
            tot[7] += float(m.group(13)) * n
        if m.group(7):
            for i in range(4):
                why[i] += int(m.group(7 + i))
    names = ("fast", "xlate+fill", "coverage", "exec", "cross-page", "fast: lookup part", "fast: exec part", "bp")
    print(path, "wave-steps", steps, {k: round(v / max(1, steps)) for k, v in zip(names, tot)},
          "slow steps", dict(zip(("miss", "codepage", "ucmiss", "other"), why)))
    if ops:
        print("  generic ops", dict(sorted(ops.items(), key=lambda kv: -kv[1])))
    if bpc:  # cycles inside bp_apply per wave-step, by action kind
        names = "host return setgprs feed rdrand stopok stopargs none".split()
        print("  bp_apply cycles per wave-step", {names[k]: round(v / max(1, steps)) for k, v in bpc.items() if v})
