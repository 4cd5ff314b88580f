"""Per-kernel durations from a rocprofv3 run_results.db (kernels view): mean us, count, name."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
d = collections.defaultdict(list)
for n, s, e in c.execute(f"select {name}, start, end from kernels"):
    d[n].append((e - s) / 1e3)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1]))[: int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{sum(v) / len(v):10.1f} us x{len(v):4d}  {k[:110]}")
