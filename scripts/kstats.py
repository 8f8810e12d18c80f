#!/usr/bin/env python3
"""Per-kernel launches and average durations from a rocprofv3 --kernel-trace --stats directory:
scripts/kstats.py <dir> — one line per kernel (torch's own kernels skipped), busiest first."""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    f = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True) + glob.glob(d + "/run_kernel_stats.csv")
    rows = [r for r in csv.DictReader(open(f[0])) if "at::native" not in r["Name"]]
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]) if "TotalDurationNs" in r else 0)
    for r in rows:
        print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>4} {float(r['AverageNs']) / 1e3:9.1f} us")


if __name__ == "__main__":
    main()
