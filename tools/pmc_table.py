"""Per-kernel averages of the PMC counters in a rocprofv3 rocpd database."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
filt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = c.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection").fetchall()
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for name, cn, v, d in rows:
    if filt in name:
        agg[name.split("(")[0][-60:]][cn].append(v)
for k, d in agg.items():
    print(k)
    print("   " + "  ".join(f"{cn}={sum(v) / len(v):.4g}" for cn, v in sorted(d.items())))
