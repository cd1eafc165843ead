"""Executed-instruction mix of a CPU twin run (diagnostic for the engine's
fast-path coverage): WTF_OPHIST=<file> oracle/wtf_twin fuzz ... writes
"map opcode modrm.reg memory count" lines at exit; this prints the top forms.
    python scripts/op_mix.py /tmp/oph_tlv.txt [top]"""
import sys

rows = []
for line in open(sys.argv[1]):
    m, op, reg, mem, n = (int(x) for x in line.split())
    rows.append((n, m, op, reg, mem))
total = sum(r[0] for r in rows)
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
print(f"{total} instructions, {len(rows)} forms")
for n, m, op, reg, mem in sorted(rows, reverse=True)[:top]:
    print(f"  {['', '0f ', '0f38 ', '0f3a '][m]}{op:02x} /{reg} {'mem' if mem else 'reg'}  {n}  {100 * n / total:.2f}%")
