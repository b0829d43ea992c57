"""Summarise rocprofv3 --pmc passes (scripts/pmc_session.sh) per kernel.

usage: python scripts/pmc_summary.py gpurun_out/pmc [workload ...]

For each workload and kernel: dispatch count and the per-dispatch mean of
every counter collected, plus derived ratios:
  mfma_cyc/simd = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs * 256 CUs): matrix-core
                busy cycles of one SIMD; divided by the kernel's duration in
                shader cycles (kernel trace x 2.4 GHz) it is the MFMA
                utilisation
  lds_conflict= SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  l2_hit      = TCC_HIT / (TCC_HIT + TCC_MISS)
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on waitcnt/barrier)
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

CUS = 256


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("gelim::", "")
    depth, out = 0, []
    for ch in name:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:44]


def load(root: Path, wl: str):
    # kernel -> counter -> list of per-dispatch values
    vals = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for f in sorted(root.glob(f"{wl}_p*/**/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            did = r.get("Dispatch_Id", r.get("Correlation_Id", "0"))
            vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add((f.parent.name, did))
    return vals, calls


def main() -> None:
    root = Path(sys.argv[1])
    wls = sys.argv[2:] or sorted({p.name.split("_p")[0] for p in root.glob("*_p*") if p.is_dir()})
    for wl in wls:
        vals, calls = load(root, wl)
        if not vals:
            continue
        print(f"== {wl}")
        for k in sorted(vals, key=lambda k: -vals[k].get("SQ_WAVE_CYCLES", 0)):
            v = vals[k]
            passes = {p for p, _ in calls[k]}
            nd = max(1, len(calls[k]) // max(1, len(passes)))
            m = {c: x / nd for c, x in v.items()}
            der = []
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                der.append(f"mfma_cyc/simd={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * CUS):.4g}")
            if m.get("SQ_LDS_IDX_ACTIVE"):
                der.append(f"lds_conflict={m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:.3f}")
            h, mi = m.get("TCC_HIT_sum", m.get("TCC_HIT")), m.get("TCC_MISS_sum", m.get("TCC_MISS"))
            if h is not None and mi is not None and h + mi > 0:
                der.append(f"l2_hit={h / (h + mi):.3f}")
            if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m:
                der.append(f"wait_frac={m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
            print(f"  {k:44s} dispatches/pass={nd:5d}  " + "  ".join(der))
            print("      " + "  ".join(f"{c}={x:.4g}" for c, x in sorted(m.items())))


if __name__ == "__main__":
    main()
