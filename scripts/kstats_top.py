"""Print the top kernels of a rocprofv3 kernel_stats.csv: share, calls, mean time, short name."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.1f} ms")
for r in rows[:n]:
    name = r["Name"]
    name = name[name.find("::") + 2:] if "::" in name else name
    name = name[: name.find("(")] if "(" in name else name
    print(f"{float(r['Percentage']):6.2f} {int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:9.1f}us  {name[:100]}")
