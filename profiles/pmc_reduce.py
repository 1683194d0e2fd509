#!/usr/bin/env python3
"""Reduce a profiles/run_profile.sh output directory to per-launch HBM bytes.

Reads the two separate PMC passes (FETCH_SIZE, WRITE_SIZE; rocprofv3 counter_collection
CSVs, kB per dispatch) and the kernel-trace stats, and prints one JSON object per
kernel of the Mult (the fused apply, the partial-sum pass, ...):
  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
("per launch" = per Mult: summed over the instantiations a Mult launches once each, see below).
The factor 2 is the gfx950 correction of MI355X_MICROARCH.md (HBM section: FETCH_SIZE
reports 1/2 of the bytes of wide coalesced streaming reads).  The dominant kernel's
entry is what bench.py reports as roofline.traffic (copied to profiles/pmc_<tag>_n1_<layout>.json).
"""
import csv
import glob
import json
import os
import sys

KERNELS = {"apply": "k_apply_tpe", "apply_line": "k_apply_line", "apply_brick": "k_apply_brick", "diag_tpe": "k_diag_tpe", "pcg_step": "k_pcg_step", "sum_partials": "k_sum_partials", "apply_wpe": "k_apply_wpe"}


# A kernel key may cover several instantiations launched once each per Mult (the p >= 3 brick
# kernel's two-colour schedule: the first colour's launch, then the second's with FUSE): the
# figures per Mult are the sums over the instantiations of their per-dispatch averages.


def counters(d, name):
    """key -> [per-Mult value (sum over instantiations of the per-dispatch mean), dispatches]."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name:
                continue
            for key, pat in KERNELS.items():
                if pat in r["Kernel_Name"]:
                    per.setdefault(key, {}).setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: [sum(sum(v) / len(v) for v in names.values()), sum(len(v) for v in names.values()), len(names)]
            for k, names in per.items()}


def stats(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            for key, pat in KERNELS.items():
                if pat in r["Name"]:
                    per.setdefault(key, []).append(r)
    out = {}
    for key, rows in per.items():
        out[key] = {"calls": min(int(r["Calls"]) for r in rows), "avg_ns": sum(float(r["AverageNs"]) for r in rows),
                    "min_ns": sum(float(r["MinNs"]) for r in rows), "max_ns": sum(float(r["MaxNs"]) for r in rows),
                    "launches_per_mult": len(rows)}
    return out


def main(root):
    fetch = counters(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(root, "write"), "WRITE_SIZE")
    st = stats(os.path.join(root, "trace"))
    bench = {}
    try:
        bench = json.loads(open(os.path.join(root, "bench_trace.json")).read().strip().splitlines()[-1])
    except Exception:
        pass
    res = {"bench_under_trace": {k: bench.get(k) for k in ("value", "ms_per_step", "config")},
           "roofline_under_trace": bench.get("roofline"),
           "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 B (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md)",
           "kernels": {}}
    for key in KERNELS:
        if key not in fetch and key not in st:
            continue
        f = fetch.get(key)
        w = write.get(key)
        fk = f[0] if f else None
        wk = w[0] if w else None
        e = {"FETCH_SIZE_kB_avg": fk, "WRITE_SIZE_kB_avg": wk, "dispatches": [f[1] if f else 0, w[1] if w else 0],
             "instantiations": f[2] if f else None, "trace": st.get(key)}
        if fk is not None and wk is not None:
            e["hbm_bytes_per_launch"] = (2.0 * fk + wk) * 1024.0
            if st.get(key):
                e["hbm_GBs"] = e["hbm_bytes_per_launch"] / (st[key]["avg_ns"] * 1e-9) / 1e9
        res["kernels"][key] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
