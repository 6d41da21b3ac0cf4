"""Fold rocprofv3 `--pmc` per-dispatch CSVs into one per-kernel summary (profiles/*.csv).

Usage: python scripts/pmc_summary.py OUT.csv PASS_DIR [PASS_DIR ...]

Each PASS_DIR is a `rocprofv3 --pmc ... --kernel-trace --stats --output-format csv -d PASS_DIR`
output. Counter values are summed per kernel name over all its dispatches; the kernel time comes
from the pass's kernel trace. Derived columns (gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots"
and "DVFS give-back"):

- clock_ghz        = GRBM_GUI_ACTIVE / 16 / kernel time. Per-dispatch GRBM_GUI_ACTIVE on this
                     image (ROCm 7.2, gfx950) accumulates 16 instances: GRBM/t reads 37-39 per ns on
                     long dispatches, i.e. 2.3-2.45 GHz over 16 (over 8 it would be an impossible 4.7)
- mfma_util        = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMD x 256 CU x kernel time x clock)
                     (busy cycles of all MFMA pipes over the cycles of the dispatch; the split-bf16
                     fp32 kernels issue 3 MFMAs per useful product, so useful work is 1/3 of it)
- lds_conflict_pct = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
- hbm_gb_s         = (TCC_EA0_RDREQ + TCC_EA0_WRREQ) x 64 B / kernel time; a lower bound: a wide
                     coalesced read is tallied at half its bytes on gfx950
"""

from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def _rows(pattern: str):
    for path in glob.glob(pattern, recursive=True):
        with open(path, newline="") as f:
            yield from csv.DictReader(f)


def _short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return name[:160]


def fold(pass_dirs: list[str]):
    counters: dict[str, dict[str, float]] = defaultdict(lambda: defaultdict(float))
    time_ns: dict[str, float] = defaultdict(float)
    calls: dict[str, int] = defaultdict(int)
    for d in pass_dirs:
        seen_time: dict[str, float] = defaultdict(float)
        seen_calls: dict[str, int] = defaultdict(int)
        for r in _rows(os.path.join(d, "**", "*counter_collection.csv")):
            k = _short(r.get("Kernel_Name", ""))
            counters[k][r["Counter_Name"]] += float(r["Counter_Value"])
        for r in _rows(os.path.join(d, "**", "*kernel_trace.csv")):
            k = _short(r.get("Kernel_Name", ""))
            seen_time[k] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            seen_calls[k] += 1
        for k, v in seen_time.items():  # every pass runs the same program: keep the first
            if k not in time_ns:
                time_ns[k], calls[k] = v, seen_calls[k]
    return counters, time_ns, calls


def main() -> None:
    out, dirs = sys.argv[1], sys.argv[2:]
    counters, time_ns, calls = fold(dirs)
    total = sum(time_ns.values()) or 1.0
    names = sorted(set(time_ns) | set(counters), key=lambda k: -time_ns.get(k, 0.0))
    cols = sorted({c for v in counters.values() for c in v})
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "time_ms", "pct_time", "clock_ghz", "mfma_util", "lds_conflict_pct",
                    "hbm_gb_s_lower"] + cols)
        for k in names:
            c = counters.get(k, {})
            t = time_ns.get(k, 0.0)
            grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
            clock = grbm / 16 / t if t and grbm else None
            mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
            util = mfma / (4 * 256 * t * clock) if mfma is not None and clock else None
            lds = c.get("SQ_LDS_IDX_ACTIVE")
            conf = 100.0 * c["SQ_LDS_BANK_CONFLICT"] / lds if lds and "SQ_LDS_BANK_CONFLICT" in c else None
            req = c.get("TCC_EA0_RDREQ_sum", 0.0) + c.get("TCC_EA0_WRREQ_sum", 0.0)
            hbm = req * 64 / t if t and req else None  # bytes/ns = GB/s

            def f3(x):
                return "" if x is None else f"{x:.4g}"

            w.writerow([k, calls.get(k, 0), f"{t / 1e6:.3f}", f"{100 * t / total:.2f}", f3(clock), f3(util), f3(conf),
                        f3(hbm)] + [f"{c.get(x, 0):.0f}" for x in cols])
    print(f"wrote {out}: {len(names)} kernels")


if __name__ == "__main__":
    main()
