"""profiles/<tag>_clock_drift.json: the sustained pass's shader clock per quarter, two ways.
  1. in-kernel (unprofiled bench line): Σ Δs_memtime ÷ Σ Δs_memrealtime × 100 MHz over every
     workgroup of each launch (the guide's DVFS item 6 method), from the line's `sustained`;
  2. counters (tools/profile.sh's `clock` pass, rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES):
     GRBM_GUI_ACTIVE ÷ 8 XCDs ÷ the dispatch's wall time, per frame-kernel dispatch of the
     sustained pass (the last 200 of the C3 grid). Under --pmc the dispatches run one at a time
     and this quotient reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md, DVFS
     give-back), so it is compared quarter against quarter, not with the unprofiled figure.
usage: python tools/clock_drift.py <bench json line file> <clock pass dir> <out json>"""
import csv
import glob
import json
import os
import statistics
import sys


def bench_line(path):
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            return json.loads(ln)
    raise SystemExit(f"no bench line in {path}")


def pmc_dispatches(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    disp = {}
    for r in csv.DictReader(open(f[0])):
        if "cg_frame_kernel" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"grid": int(r["Grid_Size"]), "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def main():
    line = bench_line(sys.argv[1])
    out = {"in_kernel": None, "counters": None}
    s = line.get("sustained")
    if s:
        out["in_kernel"] = {
            "method": "Σ Δs_memtime ÷ Σ Δs_memrealtime × 100 MHz over every workgroup of each launch (unprofiled)",
            "quarters_mhz": [round(q["shader_clock_mhz"], 1) for q in s["quarters"]],
            "quarters_ms_per_step": [round(q["ms_per_step"], 5) for q in s["quarters"]],
            "timed_region_mhz": round(line["roofline"].get("shader_clock_mhz", 0.0), 1),
            "change_last_vs_first": s.get("shader_clock_change_last_vs_first"),
            "finding": s.get("finding"),
        }
    ds = pmc_dispatches(sys.argv[2])
    grid = statistics.mode(d["grid"] for d in ds)
    c3 = [d for d in ds if d["grid"] == grid]
    sus = c3[-200:]
    q = []
    for i in range(4):
        part = sus[i * len(sus) // 4:(i + 1) * len(sus) // 4]
        mhz = [d["GRBM_GUI_ACTIVE"] / 8.0 / d["ns"] * 1e3 for d in part if d["ns"] > 0 and "GRBM_GUI_ACTIVE" in d]
        busy = [d["SQ_BUSY_CYCLES"] / d["ns"] for d in part if d["ns"] > 0 and "SQ_BUSY_CYCLES" in d]
        q.append({"dispatches": len(part), "grbm_mhz_median": round(statistics.median(mhz), 1) if mhz else None,
                  "sq_busy_per_ns_median": round(statistics.median(busy), 3) if busy else None,
                  "dispatch_us_median": round(statistics.median(d["ns"] for d in part) / 1e3, 2)})
    out["counters"] = {
        "method": "GRBM_GUI_ACTIVE / 8 / dispatch wall, per cg_frame_kernel dispatch of the sustained pass "
                  "(rocprofv3 --pmc serialises dispatches; reads high below ~0.3 ms: quarter vs quarter only)",
        "dispatches_c3": len(c3), "quarters": q,
        "change_last_vs_first": (q[-1]["grbm_mhz_median"] / q[0]["grbm_mhz_median"] - 1.0)
        if q[0]["grbm_mhz_median"] and q[-1]["grbm_mhz_median"] else None,
    }
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out)[:600])


if __name__ == "__main__":
    main()
