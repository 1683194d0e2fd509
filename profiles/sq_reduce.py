#!/usr/bin/env python3
"""Reduce a rocprofv3 --pmc counter CSV (any counters) to per-kernel averages per dispatch.
Usage: python3 profiles/sq_reduce.py <dir containing */run_counter_collection.csv>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            k = k.split("<")[0].split("::")[-1]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {"vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]),
                       "lds": int(r["LDS_Block_Size"]), "grid": int(r["Grid_Size"]),
                       "wg": int(r["Workgroup_Size"])}
    out = {}
    for k, cs in acc.items():
        if not k.startswith("k_"):
            continue
        o = {c: sum(v) / len(v) for c, v in cs.items()}
        o["dispatches"] = max(len(v) for v in cs.values())
        wc = o.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in o:
                    o[c + "_frac"] = o[c] / wc
        o.update(meta[k])
        out[k] = o
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
