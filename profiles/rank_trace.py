#!/usr/bin/env python3
"""Reduce a rocprofv3 kernel trace of bench.py --loopback N (profiles/rank_trace.sh): per kernel
name and grid size, the number of dispatches and the median duration.  With N subdomains the
interior apply kernels appear as N grid sizes (one per member) of ~30+ dispatches each.
Usage: python3 profiles/rank_trace.py <trace dir> <N>"""
import csv
import re
import glob
import statistics
import sys


def main(d, n):
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not files:
        raise SystemExit(f"no kernel trace under {d}")
    groups = {}
    seq = []
    for row in csv.DictReader(open(files[0])):
        m = re.search(r"(k_[a-z0-9_]+?)(?:ILi|I|\(|<|$)", row["Kernel_Name"])
        name = m.group(1) if m else row["Kernel_Name"]
        grid = int(row.get("Grid_Size_X") or row.get("Grid_Size") or 0)
        dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        groups.setdefault((name, grid), []).append(dur)
        seq.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), name, grid))
    print(f"N={n}")
    for (name, grid), v in sorted(groups.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
        if len(v) < 20 or not name.startswith(("k_apply", "k_sum")):
            continue
        print(f"  {name:24s} grid {grid:9d}  dispatches {len(v):5d}  median {statistics.median(v) / 1e3:8.1f} us")


def last_mult(d, n):
    """The apply / sum dispatches of the last timed Mult (before bench's STREAM reference),
    in start order, relative to the first: a rank's kernels alone once the members' work is
    serialised on the stream."""
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    seq = []
    for row in csv.DictReader(open(files[0])):
        m = re.search(r"(k_[a-z0-9_]+?)(?:ILi|I|\(|<|$)", row["Kernel_Name"])
        seq.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), m.group(1) if m else row["Kernel_Name"][:24],
                    int(row.get("Grid_Size_X") or 0)))
    seq.sort()
    cut = next(i for i, r in enumerate(seq) if r[2] == "k_stream_copy")
    mult = [r for r in seq[:cut] if r[2].startswith(("k_apply", "k_sum"))][-(3 * n if n > 1 else 2):]
    t0 = mult[0][0]
    print(f"  last Mult, N={n}: start..end us (duration) kernel grid")
    for s_, e_, name, grid in mult:
        print(f"    {(s_ - t0) / 1e3:8.1f} .. {(e_ - t0) / 1e3:8.1f}  ({(e_ - s_) / 1e3:6.1f})  {name:18s} {grid}")
    print(f"    Mult span {(mult[-1][1] - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
    last_mult(sys.argv[1], int(sys.argv[2]))

