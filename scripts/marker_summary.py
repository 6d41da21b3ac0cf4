"""Summarise rocprofv3 --marker-trace output: total / mean duration per roctx range name.

Usage: python scripts/marker_summary.py TRACE_DIR OUT.csv
"""

import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main() -> None:
    src, out = sys.argv[1], sys.argv[2]
    tot: dict[str, float] = defaultdict(float)
    cnt: dict[str, int] = defaultdict(int)
    for path in glob.glob(os.path.join(src, "**", "*marker_api_trace.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                name = r.get("Message") or r.get("Marker_Message") or r.get("Function") or ""
                name = re.sub(r"\d+", "#", name)  # "step 12 rows 0:33" -> "step # rows #:#"
                try:
                    dt = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                except (KeyError, ValueError):
                    continue
                tot[name] += dt
                cnt[name] += 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["range", "count", "total_ms", "mean_ms"])
        for k in sorted(tot, key=lambda k: -tot[k]):
            w.writerow([k, cnt[k], f"{tot[k] / 1e6:.3f}", f"{tot[k] / 1e6 / cnt[k]:.3f}"])
    print(f"wrote {out}: {len(tot)} ranges")


if __name__ == "__main__":
    main()
