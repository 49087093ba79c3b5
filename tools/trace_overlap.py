#!/usr/bin/env python3
"""Overlap of the exchange with the compute in a rocprofv3 kernel trace
(tools/gpu_session.sh step `tracee2e`: bench.py's end-to-end pipeline over a
1-rank RCCL communicator).  For every kernel family -- RCCL collectives,
K1r, K2/K3, K4, copies -- its queues and streams, launches and busy time; then
how much of the RCCL kernels' time runs while a K1r launch is in flight, and
on which queues.  Usage: tools/trace_overlap.py <run_kernel_trace.csv> [out.json]"""
import csv
import json
import sys


def family(name: str) -> str:
    n = name.lower()
    if "nccl" in n or "rccl" in n:
        return "rccl"
    for k in ("k1r_match_units64", "k1r_match_units", "k2_emit_units", "k3_scan", "k4_decompress", "k5"):
        if k in n:
            return k
    return "other"


def merge(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def overlap(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if hi > lo:
            tot += hi - lo
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    fam = {}
    for r in rows:
        f = family(r["Kernel_Name"])
        d = fam.setdefault(f, {"launches": 0, "queues": set(), "streams": set(), "iv": []})
        d["launches"] += 1
        d["queues"].add(int(r["Queue_Id"]))
        d["streams"].add(int(r.get("Stream_Id") or 0))
        d["iv"].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    res = {"source": sys.argv[1], "families": {}}
    for f, d in sorted(fam.items()):
        m = merge(d["iv"])
        res["families"][f] = {"launches": d["launches"], "queues": sorted(d["queues"]), "streams": sorted(d["streams"]),
                              "busy_ms": round(sum(b - a for a, b in m) / 1e6, 3)}
    if "rccl" in fam and "k1r_match_units" in fam:
        r = merge(fam["rccl"]["iv"])
        k = merge(fam["k1r_match_units"]["iv"])
        ov = overlap(r, k)
        tot = sum(b - a for a, b in r)
        res["rccl_during_k1r_ms"] = round(ov / 1e6, 3)
        res["rccl_total_ms"] = round(tot / 1e6, 3)
        res["rccl_overlap_fraction"] = round(ov / tot, 3) if tot else None
        res["rccl_queues_disjoint_from_k1r"] = not (fam["rccl"]["queues"] & fam["k1r_match_units"]["queues"])
    # every (queue, stream, kernel family) against K1r's launches: at world 1 RCCL's
    # all-gather is a copy kernel on the process group's own stream, so the copy
    # kernels are listed per queue / stream as well
    if "k1r_match_units" in fam:
        k = merge(fam["k1r_match_units"]["iv"])
        per = {}
        for r in rows:
            n = r["Kernel_Name"]
            f = family(n)
            if f == "other":
                f = n.split("(")[0].split("<")[0].replace("void ", "")[:48]
            key = f"q{r['Queue_Id']}/s{r.get('Stream_Id') or 0}/{f}"
            per.setdefault(key, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        res["vs_k1r"] = {}
        for key, iv in sorted(per.items()):
            m = merge(iv)
            tot = sum(b - a for a, b in m)
            res["vs_k1r"][key] = {"launches": len(iv), "busy_ms": round(tot / 1e6, 3),
                                  "during_k1r_ms": round(overlap(m, k) / 1e6, 3)}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
