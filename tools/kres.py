#!/usr/bin/env python3
"""Per-kernel resources from `llvm-readobj --notes <code object>` on stdin:
one line per kernel (VGPR/AGPR/SGPR counts, spills, static LDS)."""
import re
import sys

KEYS = ("group_segment_fixed_size", "name", "sgpr_count", "sgpr_spill_count", "vgpr_count",
        "vgpr_spill_count", "agpr_count")
rows, cur = [], {}
for line in sys.stdin:
    m = re.match(r"\s+\.(\w+):\s+(\S+)", line)
    if not m or m.group(1) not in KEYS:
        continue
    k, v = m.groups()
    if k == "group_segment_fixed_size" and cur:
        rows.append(cur)
        cur = {}
    cur[k] = v
if cur:
    rows.append(cur)
for r in rows:
    name = re.sub(r"^_ZN10snappy_amd\d+", "", r.get("name", "?"))
    m = re.match(r"[a-z0-9_]+", name)
    name = m.group(0) if m else name
    g = r.get
    print(f"{name:22s} vgpr {g('vgpr_count')} agpr {g('agpr_count')} sgpr {g('sgpr_count')} "
          f"spill v{g('vgpr_spill_count')}/s{g('sgpr_spill_count')} lds {g('group_segment_fixed_size')}")
