"""Summarise a scripts/profile.sh run into profiles/: the rocprofv3 kernel stats of the bench's
dominant kernel, its per-launch HBM traffic from the PMC passes, and profiles/traffic.json (read
by bench.py for roofline.traffic).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of wide coalesced reads (128-B requests tallied at 64 B), so
read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE * 1024 is exact for full-line stores.
Usage: python scripts/summarize_profile.py gpurun_out/prof_r01 r01
"""
import csv
import json
import os
import re
import shutil
import sys

KERNEL = "k_sgns_o2"  # matches k_sgns_o2 and k_sgns_o2_ring


def main(src, tag, kernel=KERNEL):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, "%s_kernel_stats.csv" % tag))
    row = [r for r in csv.DictReader(open(stats)) if kernel in r["Name"]][0]
    # the timed launches only: profile.sh runs bench.py with one warm-up launch first, and a
    # launch early in training updates (writes) more rows than a later one (C5: 2.87 s / 5.9e12 B
    # written for the warm-up launch vs 2.06 s / 2.1e12 B for the last, r06_c5), so averages that
    # include it do not describe the launches bench.py times
    skip = int(os.environ.get("SKIP_LAUNCHES", "1"))
    trace = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv")))
             if kernel in r["Kernel_Name"]]
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace]
    timed = durs[skip:] if len(durs) > skip else durs
    avg_ms = sum(timed) / len(timed)
    pmc = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for r in csv.DictReader(open(os.path.join(src, "pmc_" + c,
                                                            "run_counter_collection.csv")))
                if kernel in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        allv = [float(r["Counter_Value"]) for r in rows]
        vals = allv[skip:] if len(allv) > skip else allv
        pmc[c] = sum(vals) / len(vals)
        pmc[c + "_launches"] = len(vals)
        pmc[c + "_per_launch_all"] = allv
    read_b = 2 * pmc["FETCH_SIZE"] * 1024
    write_b = pmc["WRITE_SIZE"] * 1024
    bench = json.load(open(os.path.join(src, "trace_bench.json")))
    cfg = bench["config"]
    pairs = bench["roofline"].get("pairs_per_launch", cfg["pairs_per_step_per_gpu"])
    alg = bench["roofline"]["bytes_per_pair"] * pairs  # SURVEY.md §8d model (7,168 B at C3)
    alg_skip = bench["roofline"].get("bytes_per_pair_skip_adjusted",
                                     bench["roofline"]["bytes_per_pair"]) * pairs
    m = re.search(r"d=(\d+), negative=(\d+)", cfg["workload"])
    dim, neg = int(m.group(1)), int(m.group(2))
    ml = re.search(r"lr=([0-9.eE+-]+)", cfg["workload"])
    traffic = {"kernel": row["Name"], "tag": tag,
               "walks_per_launch": cfg.get("walks_per_launch", cfg["walks_per_step_per_gpu"]),
               "dim": dim, "negative": neg, "lr": float(ml.group(1)) if ml else None,
               "negative_table": cfg.get("negative_table", "uint32"),
               "hbm_bytes_per_launch": read_b + write_b,
               "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
               "algorithmic_bytes_per_launch": alg,
               "algorithmic_skip_adjusted_bytes_per_launch": alg_skip,
               "pairs_per_launch": pairs,
               "rocprof_avg_kernel_ms": avg_ms,
               "rocprof_launch_ms_all": durs, "timed_launches_from": skip,
               "rocprof_stats_avg_kernel_ms_all_launches": float(row["AverageNs"]) / 1e6,
               "bench_event_avg_kernel_ms": bench["roofline"]["avg_kernel_ms"],
               "actual_hbm_GBps": (read_b + write_b) / avg_ms / 1e6,
               "raw": pmc}
    if cfg["workload"].startswith("configs[2]/C3"):  # the default bench line reads this one
        json.dump(traffic, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    if cfg["workload"].startswith("configs[4]/C5"):  # ... and its C5-shard row this one
        json.dump(traffic, open(os.path.join(dst, "traffic_c5.json"), "w"), indent=1)
    json.dump(traffic, open(os.path.join(dst, "%s_traffic.json" % tag), "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
