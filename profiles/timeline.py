#!/usr/bin/env python3
"""One pipeline step's dispatch sequence from a rocprofv3 kernel trace: duration and the idle gap before each
dispatch (host round trips show up as gaps), plus per-step totals.  A step starts at k_minmax.
Usage: timeline.py OUT_DIR [step index]"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    r = sorted(csv.DictReader(open(f)), key=lambda x: int(x["Start_Timestamp"]))
    names = [x["Kernel_Name"].split("(")[0].replace("void ", "") for x in r]
    starts = [i for i, n in enumerate(names) if n == "ad::k_minmax"]
    i0, i1 = starts[k], starts[k + 1]
    busy = gaps = 0.0
    for i in range(i0, i1):
        dur = (int(r[i]["End_Timestamp"]) - int(r[i]["Start_Timestamp"])) / 1e3
        gap = (int(r[i]["Start_Timestamp"]) - int(r[i - 1]["End_Timestamp"])) / 1e3
        busy += dur
        gaps += max(gap, 0.0) if i > i0 else 0.0
        print("%7.1f %6.1f  %s" % (dur, gap, names[i][:110]))
    print("dispatches %d  busy %.1f us  gaps %.1f us  step %.1f us"
          % (i1 - i0, busy, gaps, (int(r[i1]["Start_Timestamp"]) - int(r[i0]["Start_Timestamp"])) / 1e3))


if __name__ == "__main__":
    main()
