#!/usr/bin/env python3
"""Summarise single rocprofv3 --pmc passes made by tools/gpu_session.sh (steps
`pmc:<tag>:<workload>:<counters>`) into profiles/<round>_pmc_<tag>.json: per
kernel, the mean of every counter over its launches, and the launch count.
Counters are as rocprofv3 reports them (no unit correction here; the HBM-byte
correction of FETCH_SIZE/WRITE_SIZE lives in tools/pmc_summary.py).
Usage: tools/pmc_pass_summary.py <gpurun_out/rNN> <round>"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, rnd = sys.argv[1], sys.argv[2]
for tag in sorted(os.listdir(src)):
    f = os.path.join(src, tag, "run_counter_collection.csv")
    if not tag.startswith("pmc_") or not os.path.exists(f):
        continue
    agg, disp = {}, {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("snappy_amd::", "").replace("void ", "")
        if not k.startswith("k"):
            continue
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        disp.setdefault(k, set()).add(r.get("Dispatch_Id", ""))
    res = {"round": rnd, "pass": tag[4:], "source": "rocprofv3 --pmc, one counter pass, 1-step bench",
           "kernels": {k: {"launches": len(disp[k]),
                           **{c: round(sum(v) / len(disp[k])) for c, v in sorted(cs.items())}}
                       for k, cs in sorted(agg.items())}}
    out = os.path.join(ROOT, "profiles", f"{rnd}_{tag}.json")
    json.dump(res, open(out, "w"), indent=1)
    print(out, json.dumps(res["kernels"])[:600])
