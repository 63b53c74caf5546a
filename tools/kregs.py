"""VGPR / spill counts per kernel from a hipcc -S listing: python tools/kregs.py x6.s [substring]"""
import re
import sys

name = None
rows = []
for line in open(sys.argv[1]):
    m = re.match(r"\s+\.name:\s+(_Z\S+)", line)
    if m:
        name = m.group(1)
        cur = {}
        continue
    m = re.match(r"\s+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count|agpr_count):\s+(\d+)", line)
    if m and name:
        cur[m.group(1)] = int(m.group(2))
        if m.group(1) == "vgpr_spill_count":
            rows.append((name, cur.get("vgpr_count"), cur.get("vgpr_spill_count")))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for n, v, sp in rows:
    if sub in n:
        print(f"{v:4d} vgpr {sp:4d} spill  {n}")
