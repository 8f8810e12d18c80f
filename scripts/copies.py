"""Copies and fills of one C4 step from a rocprofv3 --memory-copy-trace + --kernel-trace run:
python3 scripts/copies.py <dir> -> per copy: offset, direction, bytes (between two k_boundaries starts)"""
import csv
import glob
import sys

d = sys.argv[1]
kf = glob.glob(d + "/**/run_kernel_trace.csv", recursive=True)[0]
mf = glob.glob(d + "/**/run_memory_copy_trace.csv", recursive=True)
ks = sorted(csv.DictReader(open(kf)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(ks) if "k_boundaries" in r["Kernel_Name"]]
t0, t1 = int(ks[idx[-2]]["Start_Timestamp"]), int(ks[idx[-1]]["Start_Timestamp"])
print("kernel-trace copies/fills in the step:")
for r in ks[idx[-2]:idx[-1]]:
    if "rocclr" in r["Kernel_Name"]:
        print(f"  {(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} us {r['Kernel_Name'][:40]}")
if mf:
    ms = sorted(csv.DictReader(open(mf[0])), key=lambda r: int(r["Start_Timestamp"]))
    print("memory-copy trace in the step:", list(ms[0].keys()) if ms else [])
    for r in ms:
        s = int(r["Start_Timestamp"])
        if t0 <= s < t1:
            print(f"  {(s - t0) / 1e3:8.1f} us {r.get('Direction', '?'):>20} {r.get('Bytes', r.get('Size', '?'))}")
