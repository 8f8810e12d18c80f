"""Per-kernel average durations from a rocprofv3 database (ROCm 7.2's default output): usage
python3 scripts/dbstats.py <dir-with-.db> — one line per kernel, launches and average microseconds."""
import collections
import glob
import sqlite3
import sys

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True) + glob.glob(sys.argv[1] + "/*.db")
c = sqlite3.connect(db[0])
names = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kd = next(t for t in names if t.startswith("rocpd_kernel_dispatch"))
ks = next(t for t in names if t.startswith("rocpd_info_kernel_symbol"))
sym = {r[0]: r[1] for r in c.execute(f"select id, kernel_name from {ks}")}
d = collections.defaultdict(list)
for kid, s, e in c.execute(f"select kernel_id, start, end from {kd}"):
    d[sym.get(kid, str(kid))].append((e - s) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if "at::native" in k:
        continue
    print(f"{k.split('(')[0][:70]:70s} {len(v):5d} {sum(v) / len(v):9.1f} us")
