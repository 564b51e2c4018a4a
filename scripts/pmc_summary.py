"""Summarise the rocprofv3 PMC passes of scripts/pmc.sh into
profiles/pmc_traffic.json (read by bench.py as roofline.traffic, only while the
kernel family's sources still hash to the value recorded per workload) and a per-workload counter table.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts
exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so
read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B stores
(bytes = WRITE_SIZE * 1024).  Values are per launch of the bench's kernel over
its resident pool: rows whose kernel name carries the instance the bench
reported (meta.json) and whose grid is that kernel's most frequent grid (the
pool launches, not the encode that builds the pool)."""
import csv
import glob
import json
import statistics
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def rows_for(d: Path, kernel: str):
    f = glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit("no counter file under %s" % d)
    rows = [r for r in csv.DictReader(open(f[0])) if kernel in r["Kernel_Name"]]
    if not rows:
        raise SystemExit("no %s rows in %s" % (kernel, f[0]))
    grid = Counter(r["Grid_Size"] for r in rows).most_common(1)[0][0]
    return [r for r in rows if r["Grid_Size"] == grid]


def counter(rows, name):
    v = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == name]
    return statistics.median(v) if v else None


def main(src=None, out_table="profiles/r02_pmc_workloads.json"):
    src = Path(src) if src else ROOT / "gpurun_out"
    old = ROOT / "profiles" / "pmc_traffic.json"
    traffic = json.loads(old.read_text()).get("workloads", {}) if old.exists() else {}
    old_t = ROOT / out_table
    table = json.loads(old_t.read_text()).get("workloads", {}) if old_t.exists() else {}
    for meta_f in sorted(glob.glob(str(src / "pmc_*_0" / "meta.json")), key=lambda f: ("_c" in f, f)):
        d0 = Path(meta_f).parent
        w = json.loads(Path(meta_f).read_text())
        name, kernel = w["workload"], w["kernel"]
        base = str(d0)[:-2]
        fetch = counter(rows_for(Path(base + "_0"), kernel), "FETCH_SIZE")
        write = counter(rows_for(Path(base + "_1"), kernel), "WRITE_SIZE")
        rd, wr = 2 * fetch * 1024, write * 1024
        algo = w["algorithmic_bytes_per_launch"]
        algo_wr = w["pool_stripes"] * w["write_bytes_per_unit"]
        shape = w.get("launch_shape") or kernel
        entry = {
            "kernel": kernel, "launch_shape": shape, "tune": w.get("tune", []), "pool_stripes": w["pool_stripes"],
            "kernel_source_hash": w["kernel_source_hash"],
            "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
            "algorithmic_bytes_per_launch": algo, "traffic_over_algorithmic": (rd + wr) / algo,
            "read_over_algorithmic_read": rd / (algo - algo_wr),
            "write_over_algorithmic_write": wr / algo_wr if algo_wr else None,
        }
        # one profile per full launch shape (the selection's candidates); the workload's own
        # fields are the shape its default (untuned) run launches
        by_shape = dict(traffic.get(name, {}).get("by_shape", {}))
        by_shape[shape] = entry
        if not w.get("tune") or name not in traffic:
            traffic[name] = dict(entry)
        else:
            traffic[name] = dict(traffic[name])
        traffic[name]["by_shape"] = by_shape
        t = dict(entry)
        sq_dir = Path(base + "_2")
        if sq_dir.exists():
            rows = rows_for(sq_dir, kernel)
            c = {n: counter(rows, n) for n in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES",
                                                "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                                "GRBM_GUI_ACTIVE")}
            dur = statistics.median((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in rows)
            t.update(c)
            t["launch_s_profiled"] = dur
            t["valu_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
            t["valu_wave_instr_per_s"] = c["SQ_INSTS_VALU"] / dur
            t["wait_inst_any_over_wave_cycles"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
            t["active_valu_over_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
            t["effective_clock_GHz"] = c["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9  # GRBM sums the 8 XCDs
        t["bench_avg_launch_ms"] = w["avg_launch_ms"]
        table[name if not w.get("tune") else "%s [%s]" % (name, shape)] = t
    # workloads not re-profiled in this run keep their entries (and their own hashes)
    out = {"correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of 16-B/lane streaming reads); "
                         "write = WRITE_SIZE x 1024",
           "workloads": traffic}
    (ROOT / "profiles" / "pmc_traffic.json").write_text(json.dumps(out, indent=1) + "\n")
    (ROOT / out_table).write_text(json.dumps({"workloads": table}, indent=1) + "\n")
    print(json.dumps(table, indent=1))


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
