#!/usr/bin/env python3
"""Reduce the fetch_calib counter passes: per calibration kernel, FETCH_SIZE / WRITE_SIZE bytes
(kB x 1024) against the bytes it is known to move, and its streaming rate (kernel trace).
fetch_calib dispatches, in order: memset (hipMemset of the 1 GiB buffer), evict, rd16, evict, rd8, evict, rd4, evict, rdl8, evict, wr8,
evict, wr16 (evict = a 512 MiB wr8 stream that pushes the buffer out of the Infinity Cache)."""
import csv
import glob
import json
import os
import sys

ORDER = ["memset", "evict", "rd16", "evict", "rd8", "evict", "rd4", "evict", "rdl8", "evict", "wr8", "evict", "wr16"]


def per_dispatch(d, counter):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                k = int(r["Dispatch_Id"])
                acc[k] = acc.get(k, 0.0) + float(r["Counter_Value"])
    return [acc[k] * 1024 for k in sorted(acc)]


def durations(d):
    ts = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ts.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return [t for _, t in sorted(ts)]


def main(d):
    known = json.load(open(os.path.join(d, "known.json")))
    fetch = per_dispatch(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(d, "write"), "WRITE_SIZE")
    dur = durations(os.path.join(d, "trace"))
    assert len(fetch) == len(write) == len(ORDER), (len(fetch), len(write))
    kb = {"rd16": known["bytes"], "rd8": known["bytes"], "rd4": known["bytes"], "rdl8": known["rdl8_lines"] * 128,
          "wr8": known["bytes"], "wr16": known["bytes"], "evict": known["bytes"] // 2, "memset": known["bytes"]}
    out = {"source": "profiles/calib/run_calib.sh: fetch_calib.hip under separate rocprofv3 --pmc FETCH_SIZE and "
                     "--pmc WRITE_SIZE passes; 1 GiB buffer, every byte touched once; kB counters x 1024",
           "note": "rdl8 reads 8 B of every 128-B line: known_B counts whole lines",
           "dispatches": []}
    for i, name in enumerate(ORDER):
        o = {"kernel": name, "known_B": kb[name], "FETCH_B": fetch[i], "WRITE_B": write[i]}
        if name.startswith("rd"):
            o["known_over_FETCH"] = kb[name] / max(fetch[i], 1.0)
        else:
            o["known_over_WRITE"] = kb[name] / max(write[i], 1.0)
        if i < len(dur):
            o["us"] = dur[i] / 1e3
            o["GBs"] = kb[name] / dur[i]
        out["dispatches"].append(o)
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
