"""Per-step kernel timeline (start offset, gap since the previous kernel, duration) from a rocprofv3
kernel trace: python3 scripts/timeline.py <dir with run_kernel_trace.csv> [first-kernel-substring]"""
import csv
import glob
import sys

d = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_boundaries"
f = glob.glob(d + "/**/run_kernel_trace.csv", recursive=True) + glob.glob(d + "/run_kernel_trace.csv")
rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = prev = int(rows[a]["Start_Timestamp"])
busy = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:6.1f} {r['Kernel_Name'][:70]}")
    prev = e
print(f"step {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
