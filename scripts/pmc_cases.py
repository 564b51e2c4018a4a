"""Summarise scripts/pmc_multitile.sh: HBM bytes per launch of the apply kernel
(the largest-grid k_gf_apply* dispatches) for each (case, mode), with the gfx950
corrections of MI355X_MICROARCH.md (read bytes = 2 * FETCH_SIZE KiB, write bytes =
WRITE_SIZE KiB).  One JSON line per (case, mode).

    python scripts/pmc_cases.py [gpurun_out]
"""
import csv
import json
import statistics
import sys
from pathlib import Path


def median_value(d):
    rows = [r for r in csv.DictReader(open(d / "run_counter_collection.csv")) if "k_gf_apply" in r["Kernel_Name"]]
    if not rows:
        return None, None
    g = max(int(r["Grid_Size"]) for r in rows)
    sel = [r for r in rows if int(r["Grid_Size"]) == g]
    return statistics.median(float(r["Counter_Value"]) for r in sel), sel[0]["Kernel_Name"]


def main():
    out = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
    for d in sorted(out.glob("pmcmt_*_FETCH_SIZE")):
        key = d.name[len("pmcmt_"):-len("_FETCH_SIZE")]
        case, mode = key.split("_", 1)
        f, name = median_value(d)
        w, _ = median_value(out / f"pmcmt_{key}_WRITE_SIZE")
        if f is None or w is None:
            continue
        print(json.dumps({"case": case, "mode": mode, "kernel": name, "read_bytes": 2 * f * 1024,
                          "write_bytes": w * 1024}))


if __name__ == "__main__":
    main()
