"""Instruction histogram per kernel of a hipcc --save-temps .s file (diagnostics)."""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2] if len(sys.argv) > 2 else ""
cur, body = None, {}
for line in src:
    m = re.match(r"^(_Z\w+):", line)
    if m:
        cur = m.group(1)
        body[cur] = []
        continue
    if cur and line.startswith(".Lfunc_end"):
        cur = None
        continue
    if cur:
        t = line.strip()
        if t and not t.startswith((".", ";")) and not t.endswith(":"):
            body[cur].append(t)
for name, lines in body.items():
    if pat not in name:
        continue
    c = Counter(l.split()[0] for l in lines)
    print(name, "instructions:", len(lines))
    print("  ", ", ".join(f"{k} {v}" for k, v in c.most_common(40)))
