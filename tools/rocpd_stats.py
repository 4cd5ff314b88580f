"""Per-kernel duration summary from a rocprofv3 rocpd database (run_results.db)."""
import sqlite3
import sys


def stats(path, top=25):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(
        f"select {name}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
        f"from kernels group by {name} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = ["Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage"]
    for r in rows[:top] if top else rows:
        out.append(f'"{r[0][:110]}",{r[1]},{r[2]},{r[3]:.1f},{r[4]},{r[5]},{100.0 * r[2] / tot:.2f}')
    return "\n".join(out)


if __name__ == "__main__":
    print(stats(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25))
