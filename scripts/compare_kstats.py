"""Per-kernel comparison of two rocprofv3 kernel_stats.csv files, per round:
    python scripts/compare_kstats.py A.csv rounds_A B.csv rounds_B scale
prints, for each kernel (template arguments kept), A's ms per round × scale (the share B would
take if the kernel's time scaled with the work), B's ms per round, and B / (A × scale): the
kernels whose time does not shrink with a smaller cohort lead (ratio >> 1)."""
import csv
import sys


def load(path, rounds):
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0] if not name.startswith("at::") else name[:60]
        out[name] = out.get(name, 0.0) + float(r["TotalDurationNs"]) / 1e6 / rounds
    return out


def main():
    a = load(sys.argv[1], float(sys.argv[2]))
    b = load(sys.argv[3], float(sys.argv[4]))
    s = float(sys.argv[5])
    ta, tb = sum(a.values()) * s, sum(b.values())
    print(f"total: A x {s} = {ta:.1f} ms/round, B = {tb:.1f} ms/round, ratio {tb / ta:.3f}")
    rows = sorted(set(a) | set(b), key=lambda k: -(b.get(k, 0) - a.get(k, 0) * s))
    print(f"{'A*s ms':>9} {'B ms':>9} {'B-A*s':>8} {'ratio':>6}  kernel")
    for k in rows:
        x, y = a.get(k, 0) * s, b.get(k, 0)
        print(f"{x:9.2f} {y:9.2f} {y - x:8.2f} {y / x if x else float('inf'):6.2f}  {k[:110]}")


if __name__ == "__main__":
    main()
