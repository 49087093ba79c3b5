import sys, os
sys.path.insert(0, "lightweight-snappy_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import json, snappy_amd, oracle
from golden_inputs import make_input
g = json.load(open("tests/golden/golden.json"))
bad = 0
for e in g["entries"]:
    data = make_input(e["spec"])
    out = oracle.compress(data)
    try:
        back = snappy_amd.decompress(out)
        ok = back == data
    except Exception as ex:
        ok = False; back = str(ex)
    if not ok:
        bad += 1
        if bad <= 8:
            print("FAIL", e["name"], len(data), len(out), back if isinstance(back, str) else "mismatch")
print("bad", bad, "of", len(g["entries"]))
