"""Average duration of a kernel's back-to-back launch runs in a rocprofv3 kernel trace: the bench's roofline phase
launches the dominant pass K times in a row inside one event pair (pemp_prof_enable("edge_step@K")), so the runs
of >= K consecutive launches of that kernel are exactly the launches the line's `roofline.avg_launch_us` times.

usage: python tools/trace_kernel_runs.py <run_kernel_trace.csv> <kernel-substring> [K=8]
"""
import csv
import statistics
import sys


def main(path, pat, k=8):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], []
    for r in rows:
        if pat in r["Kernel_Name"]:
            cur.append(r)
            continue
        if len(cur) >= k:
            runs.append(cur)
        cur = []
    if len(cur) >= k:
        runs.append(cur)
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for run in runs for r in run]
    alld = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if pat in r["Kernel_Name"]]
    print(f"trace `{path}`, kernel `{pat}`")
    print(f"- runs of >= {k} back-to-back launches: {len(runs)} runs, {len(d)} launches, "
          f"mean {statistics.mean(d):.2f} us, median {statistics.median(d):.2f} us")
    print(f"- every launch of the kernel in the run (all phases, incl. other batch shapes): {len(alld)}, "
          f"median {statistics.median(alld):.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 8)
