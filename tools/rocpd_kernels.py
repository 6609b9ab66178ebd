"""Per-kernel dispatch count and mean duration from a rocprofv3 results database (rocpd sqlite)."""
import collections
import glob
import sqlite3
import sys

f = sys.argv[1] if sys.argv[1].endswith(".db") else glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(f)
sfx = [r[0] for r in c.execute("select name from sqlite_master where type='table' and name like 'rocpd_kernel_dispatch%'")][0]
sfx = sfx[len("rocpd_kernel_dispatch"):]
q = (f"select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch{sfx} d "
     f"join rocpd_info_kernel_symbol{sfx} s on d.kernel_id = s.id")
agg = collections.defaultdict(list)
for n, a, b in c.execute(q):
    agg[n].append((b - a) / 1e6)
for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print(f"{n[:80]:80s} n={len(v):3d} mean={sum(v) / len(v):8.3f} ms median={sorted(v)[len(v) // 2]:8.3f}")
