"""Per-launch durations of a kernel from a rocprofv3 --kernel-trace CSV (diagnostic):
    python tools/launch_hist.py <kernel_trace.csv> [kernel substring] [period]
Prints percentiles and the mean duration by launch index modulo `period` (default 20: the reference's
random goal changes fire when an env's time is a multiple of 5 s = 20 steps)."""
import csv
import sys

import numpy as np


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "cn_step_kernel"
    period = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if name in r.get("Kernel_Name", ""):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    d = np.array([(b - a) / 1e3 for a, b in rows])
    gaps = np.array([(rows[k + 1][0] - rows[k][1]) / 1e3 for k in range(len(rows) - 1)])
    print("%d launches of *%s*: mean %.2f us, p10 %.2f, p50 %.2f, p90 %.2f, p99 %.2f, max %.2f; gap mean %.2f us"
          % (len(d), name, d.mean(), *np.percentile(d, [10, 50, 90, 99]), d.max(), gaps.mean() if len(gaps) else 0))
    m = [d[k::period].mean() for k in range(period)]
    print("mean by launch index mod %d: %s" % (period, " ".join("%.1f" % x for x in m)))
    hist, edges = np.histogram(d, bins=12)
    for h, e0, e1 in zip(hist, edges[:-1], edges[1:]):
        print("  %7.1f-%7.1f us %6d %s" % (e0, e1, h, "#" * int(60 * h / max(hist.max(), 1))))


if __name__ == "__main__":
    main()
