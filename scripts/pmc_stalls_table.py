"""Table of scripts/pmc_agg.py output (one --pmc pass with the stall counters): per kernel the
share of run time, MFMA-busy fraction of the CU-cycles and the wave-cycle split."""
import ast
import sys

rows = []
for line in open(sys.argv[1]):
    i = line.rfind(" {")
    if i < 0:
        continue
    head, d = line[:i], ast.literal_eval(line[i + 1:])
    name, calls = head.rsplit(" ", 1)
    ns = sum(v for k, v in d.items() if k.startswith("ns_"))
    rows.append((name, int(calls), ns, d))
tot = sum(r[2] for r in rows) or 1
print(f"{'%time':>6} {'ms':>8} {'mfma':>6} {'wait':>6} {'issue':>6} {'lds':>6} {'active':>6}  kernel")
for name, calls, ns, d in sorted(rows, key=lambda r: -r[2])[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    gui = d.get("GRBM_GUI_ACTIVE", 0) or 1
    # MFMA busy per CU-cycle: SQ_VALU_MFMA_BUSY_CYCLES summed over SIMDs / (GUI cycles x 256 CUs x 4 SIMDs)
    mf = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui / 16 * 256 * 4)  # (GRBM_GUI_ACTIVE counts 16 instances)
    f = lambda k: d.get(k, 0) / wc
    nm = name.replace("void ", "").replace("(anonymous namespace)::", "")[:90]
    print(f"{100 * ns / tot:6.2f} {ns / 1e6:8.1f} {mf:6.3f} {f('SQ_WAIT_ANY'):6.3f} {f('SQ_WAIT_INST_ANY'):6.3f} "
          f"{f('SQ_WAIT_INST_LDS'):6.3f} {f('SQ_ACTIVE_INST_ANY'):6.3f}  {nm}")
