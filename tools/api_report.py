"""Host-side HIP API cost per call from a rocprofv3 --hip-runtime-trace CSV (GPU box).

usage: python tools/api_report.py gpurun_out/<dir>/run_hip_api_trace.csv
Prints per API function: calls, mean and total host microseconds, sorted by total."""
import collections
import csv
import sys


def main(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("| API | calls | mean us | total ms |")
    print("|---|---:|---:|---:|")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:25]:
        print(f"| {k} | {len(v)} | {sum(v) / len(v):.2f} | {sum(v) / 1e3:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
