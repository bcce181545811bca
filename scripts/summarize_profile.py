"""Summarise a rocprofv3 ``*_kernel_stats.csv`` as per-step kernel time (top N)."""
import csv
import sys


def main(path, steps, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total GPU kernel time {tot / 1e6:.1f} ms over {steps} steps -> {tot / 1e6 / steps:.2f} ms/step")
    print(f"{'ms/step':>8} {'calls/step':>10} {'avg us':>8}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} {int(r['Calls']) / steps:10.1f} "
              f"{float(r['AverageNs']) / 1e3:8.1f}  {r['Name'][:100]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 30)
