#!/usr/bin/env python3
"""Turn the rocprofv3 passes of tools/profile_round.sh into profiles/:
  <round>_kernel_stats.csv  (copy of --kernel-trace --stats summary)
  <round>_pmc.json          (HBM bytes per launch per kernel, corrected)
  pmc_latest.json           (same, read by bench.py for roofline.traffic)
Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a coalesced streaming
read, so it is doubled; WRITE_SIZE is taken as is."""
import csv, json, os, shutil, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
workload = sys.argv[3] if len(sys.argv) > 3 else "text32k"
out = os.path.join(ROOT, "profiles")
os.makedirs(out, exist_ok=True)
shutil.copyfile(os.path.join(src, "prof_trace", "run_kernel_stats.csv"), os.path.join(out, f"{rnd}_kernel_stats.csv"))


def per_kernel(path, counter):
    agg = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("snappy_amd::", "")
        agg.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


fetch = per_kernel(os.path.join(src, "prof_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
write = per_kernel(os.path.join(src, "prof_write", "run_counter_collection.csv"), "WRITE_SIZE")
res = {"workload": workload, "bytes_per_gpu": 1 << 30, "round": rnd,
       "note": "per launch; FETCH_SIZE KiB x1024 x2 (gfx950 half-count correction), WRITE_SIZE KiB x1024",
       "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    if not k.startswith("k"):
        continue
    f = fetch.get(k, 0.0) * 1024 * 2
    w = write.get(k, 0.0) * 1024
    res["kernels"][k] = {"fetch_bytes": round(f), "write_bytes": round(w), "hbm_bytes": round(f + w)}
for name in (f"{rnd}_pmc.json", "pmc_latest.json"):
    json.dump(res, open(os.path.join(out, name), "w"), indent=1)
print(json.dumps(res, indent=1))
