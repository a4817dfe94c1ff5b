"""Average duration of one kernel over a bench run's TIMED steps from a rocprofv3 kernel trace (the stats CSV averages
every launch, warm-up steps and their first touches included):

    python tools/rocprof_timed_avg.py profiles/r05zc_kernel_trace_x6.csv "conv1d_x6_kernel<6, 2, 2, 8, 3, false, 1, false, true>" 36
(the last N launches of that kernel: timed steps x launches per step)"""
import csv
import sys


def main():
    path, name, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    print(f"{len(d)} launches, mean {sum(d) / len(d):.4f} ms; last {n}: mean {sum(d[-n:]) / n:.4f} ms")


if __name__ == "__main__":
    main()
