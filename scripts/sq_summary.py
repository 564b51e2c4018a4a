"""Summarise scripts/pmc_sq.sh (rocprofv3 shader-counter passes) into
profiles/r01_sq_summary.json: per case, the counters of the largest k_gf_apply
launch, and the derived rates used in DESIGN.md section 4 (VALU instructions per
second, effective clock from GRBM_GUI_ACTIVE / 8 XCDs, waiting share)."""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main(src=None):
    src = Path(src) if src else ROOT / "gpurun_out"
    out = {}
    for case in ("clay104", "clay42"):
        ctr = defaultdict(list)
        for f in sorted(glob.glob(str(src / f"sq_{case}_*" / "run_counter_collection.csv"))) + \
                sorted(glob.glob(str(src / f"sq_{case}_*.csv"))):
            rows = [r for r in csv.DictReader(open(f)) if "k_gf_apply" in r["Kernel_Name"]]
            if not rows:
                continue
            grid = max(int(r["Grid_Size"]) for r in rows)
            # the repair launch (NT loads for the single-tile headline map)
            for r in rows:
                if int(r["Grid_Size"]) == grid or (case == "clay42" and "true, true" in r["Kernel_Name"]):
                    if case == "clay42" and "true, true" not in r["Kernel_Name"]:
                        continue
                    ctr[r["Counter_Name"]].append((float(r["Counter_Value"]),
                                                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9,
                                                   r["Kernel_Name"][:60], int(r["Grid_Size"])))
        if not ctr:
            continue
        d = {k: v[-1][0] for k, v in ctr.items()}
        t = ctr["SQ_INSTS_VALU"][-1][1]
        d["kernel"] = ctr["SQ_INSTS_VALU"][-1][2]
        d["grid"] = ctr["SQ_INSTS_VALU"][-1][3]
        d["launch_s_profiled"] = t
        d["valu_wave_instr_per_s"] = d["SQ_INSTS_VALU"] / t
        d["effective_clock_GHz"] = d["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
        d["wait_inst_any_over_wave_cycles"] = d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]
        d["valu_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        d["scalar_cache_hit_rate"] = d.get("SQC_DCACHE_HITS", 0) / max(1.0, d.get("SQC_DCACHE_REQ", 1))
        out[case] = d
    (ROOT / "profiles" / "r01_sq_summary.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
