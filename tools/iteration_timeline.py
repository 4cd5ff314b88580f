"""One off-policy iteration of the bench from a rocprofv3 kernel trace (run_kernel_trace.csv):
the dispatches between two consecutive optimizer kernels in the middle of the last epoch, with
start / end / duration in us relative to the first optimizer kernel.
Usage: python tools/iteration_timeline.py <run_kernel_trace.csv> [iteration index from the end]"""
import csv
import sys


def main(path, back=10):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]
           or "rmsprop_kernel" in r["Kernel_Name"]]
    if len(opt) < back + 2:
        raise SystemExit("not enough iterations in the trace")
    a, b = opt[-back - 1], opt[-back]
    t0 = int(rows[a]["Start_Timestamp"])
    print("# one off-policy iteration (us from the optimizer kernel that starts it)")
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:100]}")
    print(f"# iteration: {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
