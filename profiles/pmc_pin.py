#!/usr/bin/env python3
"""Pin a reduced profile (profiles/pmc_reduce.py output) as the traffic figure bench.py
reports: profiles/pmc_<workload>_n1_<layout>.json = the dominant kernel's per-launch HBM bytes
(separate FETCH_SIZE / WRITE_SIZE passes) plus its second (partial-sum) pass.
Usage: python3 profiles/pmc_pin.py <prof_dir> <workload> <kernel_key> > profiles/pmc_<workload>_n1_<layout>.json
(<layout> = the bench line's config.qdata_layout: affine | blocked | native)"""
import json
import os
import sys


def main(prof_dir, workload, key):
    s = json.load(open(os.path.join(prof_dir, "pmc_summary.json")))
    k = s["kernels"][key]
    alg = (s.get("roofline_under_trace") or {}).get("algorithmic_bytes_per_launch")
    out = {
        "kernel": key,
        "workload": workload,
        "FETCH_SIZE_kB_avg": k["FETCH_SIZE_kB_avg"],
        "WRITE_SIZE_kB_avg": k["WRITE_SIZE_kB_avg"],
        "dispatches": k["dispatches"],
        "trace_avg_ns": (k.get("trace") or {}).get("avg_ns"),
        "correction": s["correction"] + "; the halving is calibrated for 4, 8 and 16 B/lane reads and for "
                                        "one-lane-per-128-B-line gathers, WRITE_SIZE exact for 8 and 16 B/lane "
                                        "stores (profiles/r2_fetch_calibration.json)",
        "commit": os.environ.get("COMMIT"),
        "date": os.environ.get("PIN_DATE"),
        "hbm_bytes_per_launch": k["hbm_bytes_per_launch"],
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": k["hbm_bytes_per_launch"] / alg if alg else None,
        "second_pass": s["kernels"].get("sum_partials"),
        "source": f"{os.environ.get('PIN_SCRIPT', 'profiles/collect_r3.sh')} {workload} (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate "
                  "passes) -> profiles/pmc_reduce.py -> profiles/pmc_pin.py",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
