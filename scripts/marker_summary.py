"""Summarise a ``rocprofv3 --marker-trace`` CSV (the roctx ranges of ``IIT_PROFILE=1``): per range name, the
count, total and mean host-side duration -- which phases of the training loop the wall-clock goes to."""
import csv
import sys
from collections import defaultdict


def main(path: str) -> None:
    tot, cnt = defaultdict(float), defaultdict(int)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Function") or row.get("Name") or row.get("Operation") or "?"
            try:
                dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6  # ns -> ms
            except (KeyError, ValueError):
                continue
            tot[name] += dur
            cnt[name] += 1
    print(f"{'range':32s} {'count':>7s} {'total ms':>10s} {'mean ms':>9s}")
    for name in sorted(tot, key=tot.get, reverse=True):
        print(f"{name[:32]:32s} {cnt[name]:7d} {tot[name]:10.1f} {tot[name] / cnt[name]:9.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
