"""Sums the per-launch `wtfgpu stamps` lines of a stamps build into cycles per wave-step."""
import re
import sys

PAT = re.compile(r"wtfgpu stamps \(cycles per wave-step, (\d+) steps\): fast loop (\S+), slow: xlate\+fill (\S+), "
                 r"coverage (\S+), exec (\S+), cross-page ([^;\s]+)(?:; slow steps: miss (\d+), codepage (\d+), "
                 r"ucmiss (\d+), other (\d+))?")
for path in sys.argv[1:]:
    steps = 0
    tot = [0.0] * 5
    why = [0] * 4
    for line in open(path):
        m = PAT.search(line)
        if not m:
            continue
        n = int(m.group(1))
        steps += n
        for i in range(5):
            tot[i] += float(m.group(2 + i)) * n
        if m.group(7):
            for i in range(4):
                why[i] += int(m.group(7 + i))
    names = ("fast", "xlate+fill", "coverage", "exec", "cross-page")
    print(path, "wave-steps", steps, {k: round(v / max(1, steps)) for k, v in zip(names, tot)},
          "slow steps", dict(zip(("miss", "codepage", "ucmiss", "other"), why)))
