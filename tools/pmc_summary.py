#!/usr/bin/env python3
"""Turn the rocprofv3 passes of tools/profile_round.sh into profiles/:
  <round>_<W>_bench.json        the bench.py line (roofline.traffic from this round's passes)
  <round>_<W>_kernel_stats.csv  copy of the --kernel-trace --stats summary
  <round>_<W>_pmc.json          per kernel and launch: HBM bytes (FETCH_SIZE,
                                WRITE_SIZE, corrected) and the SQ counters
  pmc_<W>.json                  same, read by bench.py for roofline.traffic
Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming
read, so it is doubled; WRITE_SIZE is taken as is.  Other access widths are
uncalibrated (the guide says so): the K1r/K2/K4 byte loads make `fetch_bytes`
an estimate, exact only up to that factor.
Usage: tools/pmc_summary.py [gpurun_out/prof] [round]"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "prof")
rnd = sys.argv[2] if len(sys.argv) > 2 else "r02"
out = os.path.join(ROOT, "profiles")
os.makedirs(out, exist_ok=True)


def per_kernel(path):
    """{kernel: {counter: mean value per launch}}"""
    agg = {}
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("snappy_amd::", "")
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


for w in sorted(os.listdir(src)):
    d = os.path.join(src, w)
    bench = os.path.join(d, "bench.json")
    if not os.path.exists(bench):
        continue
    lines = [l for l in open(bench) if l.startswith("{")]
    if not lines:
        continue
    line = json.loads(lines[-1])
    shutil.copyfile(bench, os.path.join(out, f"{rnd}_{w}_bench.json"))
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copyfile(stats, os.path.join(out, f"{rnd}_{w}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(d, "fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(d, "write", "run_counter_collection.csv"))
    sq = per_kernel(os.path.join(d, "sq", "run_counter_collection.csv"))
    for k, cs in per_kernel(os.path.join(d, "sq2", "run_counter_collection.csv")).items():
        sq.setdefault(k, {}).update({c: v for c, v in cs.items() if c != "SQ_WAVES"})
    n = line["config"]["bytes_per_gpu"]
    # bench.py matches a summary to its line by workload and launch size
    res = {"label": w, "workload": line["config"].get("workload_name", w), "bytes_per_gpu": n,
           "launch_bytes": line["config"].get("launch_bytes", n), "round": rnd,
           "note": "per launch; FETCH_SIZE KiB x1024 x2 (gfx950 half-count correction), WRITE_SIZE KiB x1024; "
                   "SQ_* as rocprofv3 reports them (SQ_WAVE_CYCLES/SQ_BUSY_CYCLES in quad-cycles per the guide)",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write) | set(sq)):
        if not k.startswith("k"):
            continue
        f = fetch.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 * 2
        wr = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        e = {"fetch_bytes": round(f), "write_bytes": round(wr), "hbm_bytes": round(f + wr)}
        for c, v in sorted(sq.get(k, {}).items()):
            e[c] = round(v)
        if e.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
                if c in e:
                    e[c + "_per_wave"] = round(e[c] / e["SQ_WAVES"], 1)
            # busy fractions: the counters are quad-cycles summed over
            # waves, so a per-SIMD fraction is waves-per-SIMD x per-wave count / per-wave
            # SQ_WAVE_CYCLES; waves per SIMD from the kernel's occupancy
            occ = {"k1r_match_units": 3, "k1r_match_units64": 3, "k4_decompress_units": 8, "k2_emit_units": 6}.get(k)
            wc = e.get("SQ_WAVE_CYCLES", 0) / e["SQ_WAVES"]
            if occ and wc:
                frac = {}
                for c, name in (("SQ_ACTIVE_INST_VALU", "simd_valu_active"), ("SQ_ACTIVE_INST_SCA", "simd_salu_active"),
                                ("SQ_ACTIVE_INST_LDS", "simd_lds_inst_active")):
                    if c in e:
                        frac[name] = round(occ * e[c] / e["SQ_WAVES"] / wc, 3)
                for c, name in (("SQ_WAIT_ANY", "wave_waitcnt_parked"), ("SQ_WAIT_INST_ANY", "wave_issue_stalled"),
                                ("SQ_ACTIVE_INST_ANY", "wave_issuing"), ("SQ_WAIT_INST_LDS", "wave_lds_issue_stalled")):
                    if c in e:
                        frac[name] = round(e[c] / e["SQ_WAVES"] / wc, 3)
                frac["waves_per_simd"] = occ
                frac["wave_cycles_per_wave"] = round(4 * wc)
                e["busy"] = frac
        res["kernels"][k] = e
    for name in (f"{rnd}_{w}_pmc.json", f"pmc_{w}.json"):
        json.dump(res, open(os.path.join(out, name), "w"), indent=1)
    # the bench line ran before these passes (it read the previous pmc_<W>.json):
    # give its roofline the traffic measured now on the same code and workload
    k = line.get("roofline", {}).get("kernel")
    if k in res["kernels"]:
        line["roofline"]["traffic"] = res["kernels"][k]["hbm_bytes"]
        line["roofline"]["traffic_source"] = f"profiles/{rnd}_{w}_pmc.json"
        with open(os.path.join(out, f"{rnd}_{w}_bench.json"), "w") as f:
            f.write(json.dumps(line) + "\n")
    print(w, json.dumps(res["kernels"], indent=None)[:2000])
