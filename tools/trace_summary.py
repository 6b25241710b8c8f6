"""Per-(kernel, grid) durations from a rocprofv3 ``--kernel-trace --output-format csv`` run.

usage: python tools/trace_summary.py <run_kernel_trace.csv> [top]

``--stats`` averages every dispatch of a kernel, so the bench's small parity
and secondary launches dilute the timed batch.  Grouping by grid size
separates the 262144-frame headline launches; their average is the figure to
compare with bench.py's ``roofline.kernel_ms`` (HIP events on the launch stream).
"""
from __future__ import annotations

import collections
import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    by = collections.defaultdict(list)
    for r in rows:
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        by[(r["Kernel_Name"].split("(")[0], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':58s} {'grid':>9s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'total_us':>10s}")
    for (name, grid), v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{name[:58]:58s} {grid:9d} {len(v):6d} {sum(v) / len(v):9.2f} {min(v):9.2f} {sum(v):10.1f}")


if __name__ == "__main__":
    main()
