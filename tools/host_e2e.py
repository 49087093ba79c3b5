#!/usr/bin/env python3
"""PCIe-inclusive host API rates (bench.host_end_to_end) for a few workloads."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
kinds = sys.argv[2].split(",") if len(sys.argv) > 2 else ["T", "R", "P"]
for kind, seed in (("T", 1234), ("R", 1), ("P", 2)):
    if kind not in kinds:
        continue
    print(kind, json.dumps(bench.host_end_to_end(kind, seed, int(sys.argv[1]) if len(sys.argv) > 1 else 256 << 20)),
          flush=True)
