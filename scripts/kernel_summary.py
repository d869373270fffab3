#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` (top-N kernels by total time)."""
import csv
import sys


def main(path: str, top: int = 30) -> None:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time: {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
    print(f"{'total_ms':>9} {'pct':>6} {'calls':>7} {'avg_us':>9}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} {float(r['Percentage']):6.2f} {r['Calls']:>7} "
              f"{float(r['AverageNs']) / 1e3:9.2f}  {r['Name'][:100]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
