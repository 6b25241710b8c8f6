"""Per-(kernel, grid) durations from a rocprofv3 ``--kernel-trace --output-format csv`` run.

usage: python tools/trace_summary.py <run_kernel_trace.csv> [top] [last]

``--stats`` averages every dispatch of a kernel, so the bench's small parity
and secondary launches dilute the timed batch.  Grouping by grid size
separates the 262144-frame headline launches; their average is the figure to
compare with bench.py's ``roofline.kernel_ms`` (HIP events on the launch stream).  Since round 4 the bench's timed
steps overlap on two streams (a dispatch's start-to-end then includes the other stream's kernel) and a clock-settle
phase precedes them; ``roofline.kernel_ms`` is timed over the 10 single-stream launches right after the timed
region, so ``last_avg_us`` -- the average of each group's last ``last`` (default 10) dispatches in start order -- is
the figure that must agree with it.
"""
from __future__ import annotations

import collections
import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    by = collections.defaultdict(list)
    for r in rows:
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        by[(r["Kernel_Name"].split("(")[0], grid)].append((t0, (t1 - t0) / 1e3))
    print(f"{'kernel':58s} {'grid':>9s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'total_us':>10s} "
          f"{'last_avg_us':>11s}")
    for (name, grid), tv in sorted(by.items(), key=lambda kv: -sum(d for _, d in kv[1]))[:top]:
        v = [d for _, d in sorted(tv)]
        tail = v[-last:]
        print(f"{name[:58]:58s} {grid:9d} {len(v):6d} {sum(v) / len(v):9.2f} {min(v):9.2f} {sum(v):10.1f} "
              f"{sum(tail) / len(tail):11.2f}")


if __name__ == "__main__":
    main()
