#!/usr/bin/env python3
"""Timeline of the last replayed member Mult in a rocprofv3 kernel trace of
bench.py --loopback N --member R (profiles/member_trace.sh): the apply / sum / copy dispatches of
the final graph replay, start..end relative to the first, plus the median per kernel name.
Usage: python3 profiles/member_trace.py <trace dir> [kernels per Mult]"""
import csv
import glob
import re
import statistics
import sys


def main(d, per):
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not files:
        raise SystemExit(f"no kernel trace under {d}")
    seq = []
    for row in csv.DictReader(open(files[0])):
        m = re.search(r"(k_[a-z0-9_]+?)(?:ILi|I|\(|<|$)", row["Kernel_Name"])
        name = m.group(1) if m else row["Kernel_Name"][:28]
        seq.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), name,
                    int(row.get("Grid_Size_X") or row.get("Grid_Size") or 0)))
    seq.sort()
    seq = [r for r in seq if r[2].startswith(("k_apply", "k_sum", "k_gather"))]
    groups = {}
    for s_, e_, n, g in seq:
        groups.setdefault((n, g), []).append(e_ - s_)
    for (n, g), v in sorted(groups.items()):
        if len(v) >= 10:
            print(f"  {n:22s} grid {g:9d} dispatches {len(v):5d} median {statistics.median(v) / 1e3:7.1f} us")
    last = seq[-per:]
    t0 = last[0][0]
    print("  last Mult: start..end us (duration) kernel grid")
    for s_, e_, n, g in last:
        print(f"    {(s_ - t0) / 1e3:7.1f} .. {(e_ - t0) / 1e3:7.1f} ({(e_ - s_) / 1e3:6.1f})  {n:20s} {g}")
    print(f"    span {(max(r[1] for r in last) - t0) / 1e3:.1f} us; gap to the previous Mult's last kernel "
          f"{(t0 - seq[-per - 1][1]) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
