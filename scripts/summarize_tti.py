"""One line per scripts/time_to_iia.py JSON record in a log (other lines echoed, truncated)."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        print(line.strip()[:200])
        continue
    r = json.loads(line)
    print(r["model"], r["engine"], r["dtype"], "graphs" if r["graphs"] else "eager", r["steady_s_per_epoch"], r["final"])
