"""Copy the rocprofv3 CSVs of tools/profile.sh into profiles/ (named per round) and derive
the per-launch HBM traffic (FETCH_SIZE x2 on gfx950 + WRITE_SIZE, MI355X_MICROARCH.md) and
the SQ issue/wait breakdown of cg_frame_kernel."""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof")
RND = sys.argv[1] if len(sys.argv) > 1 else "r1"
DST = os.path.join(ROOT, "profiles")
KERNEL = "cg_frame_kernel<128, 1, 0>("   # the batch instantiation (pipeline, xyzi16)


def one(pattern):
    got = sorted(glob.glob(os.path.join(SRC, "**", pattern), recursive=True))
    if not got:
        raise SystemExit(f"missing {pattern} under {SRC}")
    return got[0]


def counters(path):
    """{counter: [per-dispatch value]} for the pipeline kernel (values summed per dispatch)."""
    per = {}
    for row in csv.DictReader(open(path)):
        if KERNEL not in row["Kernel_Name"]:
            continue
        key = (row["Counter_Name"], row["Dispatch_Id"])
        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for (name, _), v in sorted(per.items()):
        out.setdefault(name, []).append(v)
    return out


os.makedirs(DST, exist_ok=True)
shutil.copy(one("stats/**/run_kernel_stats.csv"), os.path.join(DST, f"{RND}_kernel_stats.csv"))
shutil.copy(one("stats/**/run_kernel_trace.csv"), os.path.join(DST, f"{RND}_kernel_trace.csv"))
fetch_csv, write_csv, sq_csv = (one(f"{n}/**/run_counter_collection.csv") for n in ("fetch", "write", "sq"))
shutil.copy(fetch_csv, os.path.join(DST, f"{RND}_pmc_fetch_size.csv"))
shutil.copy(write_csv, os.path.join(DST, f"{RND}_pmc_write_size.csv"))
shutil.copy(sq_csv, os.path.join(DST, f"{RND}_pmc_sq.csv"))

F = 256
fetch = statistics.median(counters(fetch_csv)["FETCH_SIZE"])      # KB per dispatch
write = statistics.median(counters(write_csv)["WRITE_SIZE"])
hbm = (2 * fetch + write) * 1024
json.dump({"kernel": "cg_frame_kernel<128,1,0> (pipeline, xyzi16)", "frames_per_launch": F,
           "fetch_size_kb_per_launch": fetch, "write_size_kb_per_launch": write,
           "correction": "FETCH_SIZE x2 for wide coalesced streaming reads on gfx950 "
                         "(MI355X_MICROARCH.md, HBM); WRITE_SIZE as reported",
           "hbm_bytes_per_launch": hbm, "hbm_bytes_per_frame": hbm / F,
           "command": "tools/profile.sh: rocprofv3 --pmc FETCH_SIZE (then --pmc WRITE_SIZE) -- "
                      "python3 bench.py --no-cpu --steps 5 --warmup 2 --streams 1"},
          open(os.path.join(DST, f"{RND}_traffic.json"), "w"), indent=1)
sq = {k: statistics.median(v) for k, v in counters(sq_csv).items()}
waves = 256 * 8
wc = sq["SQ_WAVE_CYCLES"]
json.dump({"kernel": "cg_frame_kernel<128,1,0>", "waves_per_launch": waves,
           "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / waves,
           "valu_insts_per_point": sq["SQ_INSTS_VALU"] / waves / 128,
           "lds_insts_per_wave": sq["SQ_INSTS_LDS"] / waves,
           "vmem_rd_insts_per_wave": sq["SQ_INSTS_VMEM_RD"] / waves,
           "wave_time_fraction": {"active": sq["SQ_ACTIVE_INST_ANY"] / wc, "waiting": sq["SQ_WAIT_ANY"] / wc,
                                  "issue_stalled": sq["SQ_WAIT_INST_ANY"] / wc,
                                  "valu_active": sq["SQ_ACTIVE_INST_VALU"] / wc},
           "raw_per_dispatch": sq,
           "command": "tools/profile.sh: rocprofv3 --pmc <8 SQ counters> -- python3 bench.py --no-cpu "
                      "--steps 5 --warmup 2 --streams 1"},
          open(os.path.join(DST, f"{RND}_sq_counters.json"), "w"), indent=1)
stats = list(csv.DictReader(open(os.path.join(DST, f"{RND}_kernel_stats.csv"))))
for r in stats:
    if KERNEL in r["Name"]:
        print("rocprof average ns:", r["AverageNs"], "calls", r["Calls"])
print("hbm bytes per frame:", hbm / F)
print(json.dumps(json.load(open(os.path.join(DST, f"{RND}_sq_counters.json")))["wave_time_fraction"]))

# timing check: the bench's in-kernel launch span vs rocprofv3's kernel trace over the same
# timed launches: dispatches [warmup, warmup + steps) of the stats run (the warmup steps come
# first; the untimed event pass and the later legs follow the timed region)
trace = [r for r in csv.DictReader(open(os.path.join(DST, f"{RND}_kernel_trace.csv"))) if KERNEL in r["Kernel_Name"]]
dur_us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in trace]
bench = [json.loads(x) for x in open(os.path.join(SRC, "stats.log")) if x.startswith("{")][0]
steps = bench["steps"]
roof = bench["roofline"]
warm = bench["warmup"]
timed = statistics.mean(dur_us[warm:warm + steps])
# (the HIP events of the bench's untimed pass, the next `steps` dispatches after the timed
# region, against rocprofv3's figure for those same launches)
ev_pass = statistics.mean(dur_us[warm + steps:warm + 2 * steps])
json.dump({"kernel": KERNEL, "launches_traced": len(dur_us), "timed_launches": steps,
           "rocprof_avg_us_timed": timed, "rocprof_avg_us_event_pass": ev_pass,
           "rocprof_avg_us_all": statistics.mean(dur_us),
           "bench_avg_kernel_us": roof["avg_kernel_ms"] * 1e3, "bench_source": roof.get("avg_kernel_ms_source"),
           "bench_avg_launch_us_events": roof.get("avg_launch_ms_events", float("nan")) * 1e3,
           "relative_difference": roof["avg_kernel_ms"] * 1e3 / timed - 1.0,
           "events_vs_rocprof_same_launches": roof.get("avg_launch_ms_events", float("nan")) * 1e3 / ev_pass - 1.0,
           "bench_value_under_rocprof": bench["value"],
           "command": "tools/profile.sh step 1: rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu"},
          open(os.path.join(DST, f"{RND}_timing_check.json"), "w"), indent=1)
print(open(os.path.join(DST, f"{RND}_timing_check.json")).read())
