"""Summarise scripts/pmc_sq_ab.sh: per tag (A/B), the shader counters of the bench's
kernel (rows of the instance named in meta.json, at its most frequent grid), per wave."""
import csv, glob, json, statistics, sys
from collections import Counter
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]


def main(src=None, wl="clay104"):
    src = Path(src) if src else ROOT / "gpurun_out"
    out = {}
    for tag in ("A", "B"):
        vals = {}
        for d in sorted(glob.glob(str(src / f"sqab_{wl}_{tag}_*"))):
            if not Path(d).is_dir():
                continue
            meta = json.loads((Path(d) / "meta.json").read_text())
            f = glob.glob(str(Path(d) / "**" / "*counter_collection.csv"), recursive=True)[0]
            rows = [r for r in csv.DictReader(open(f)) if meta["kernel"] in r["Kernel_Name"]]
            grid = Counter(r["Grid_Size"] for r in rows).most_common(1)[0][0]
            for r in rows:
                if r["Grid_Size"] == grid:
                    vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            vals["kernel"] = meta["kernel"]
            vals["bench_launch_ms"] = meta["avg_launch_ms"]
        d = {k: (statistics.median(v) if isinstance(v, list) else v) for k, v in vals.items()}
        w = d.get("SQ_WAVES", 1)
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM", "SQ_WAVE_CYCLES",
                  "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_INST_CYCLES_SALU"):
            if k in d:
                d[k + "_per_wave"] = d[k] / w
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d and "algorithmic_bytes_per_launch" in meta:
            hbm = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024  # gfx950 FETCH_SIZE half-count
            d["hbm_over_algorithmic"] = hbm / meta["algorithmic_bytes_per_launch"]
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        out[tag] = d
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
