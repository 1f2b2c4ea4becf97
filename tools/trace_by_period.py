#!/usr/bin/env python3
"""Step-kernel durations by episode period from a rocprofv3 kernel trace (p_kernel_trace.csv): the
period of each step launch is counted from the last reset launch before it; prints the median duration
per period and per period mod 4 (the drawn-demand table's hand-over steps are t % 4 == 0).

    python tools/trace_by_period.py TRACE_CSV [STEP_KERNEL_SUBSTRING]
"""
import csv
import sys
from collections import defaultdict
from statistics import median


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "imenv_step"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    t = None
    by_t, by_m = defaultdict(list), defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if "imenv_reset_kernel" in name:
            t = 0
        elif key in name and t is not None:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            by_t[t].append(d)
            by_m[t % 4].append(d)
            t += 1
    for tt in sorted(by_t):
        print("t=%2d n=%3d median %.3f us" % (tt, len(by_t[tt]), median(by_t[tt])))
    for m in sorted(by_m):
        print("t%%4=%d n=%3d median %.3f us" % (m, len(by_m[m]), median(by_m[m])))


if __name__ == "__main__":
    main()
