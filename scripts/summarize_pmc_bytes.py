"""Summarise scripts/pmc_bytes.sh runs (TCC_EA0_RDREQ by request size, TCC_EA0_WRREQ) into
profiles/r02_traffic_calibration.json: for the traffic probe (scripts/traffic_probe.hip: known
byte counts in the O2 kernel's access patterns) the measured bytes / known bytes, and for the O2
kernel its exact fabric read bytes (sum of requests x their size) and write bytes, next to the
FETCH_SIZE/WRITE_SIZE figure scripts/summarize_profile.py derives (2 x FETCH_SIZE x 1024).

    python scripts/summarize_pmc_bytes.py gpurun_out/pmcb_probe gpurun_out/pmcb_bench \
        gpurun_out/probe_r02 profiles/traffic.json
"""
import collections
import csv
import json
import os
import sys


def load(d):
    res = collections.defaultdict(dict)
    for i in range(3):
        for r in csv.DictReader(open(os.path.join(d, "pass%d" % i, "run_counter_collection.csv"))):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            res[k].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out = {}
    for k, cs in res.items():
        v = {c.replace("TCC_EA0_", "").replace("_sum", ""): sum(x) / len(x) for c, x in cs.items()}
        v["read_bytes"] = v.get("RDREQ_128B", 0) * 128 + v.get("RDREQ_64B", 0) * 64 + \
            v.get("RDREQ_32B", 0) * 32
        v["write_bytes"] = v.get("WRREQ_64B", 0) * 64 + (v.get("WRREQ", 0) - v.get("WRREQ_64B", 0)) * 32
        out[k] = v
    return out


def main(probe_dir, bench_dir, probe_fs_dir, traffic_json):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    known = json.load(open(os.path.join(probe_dir, "pass0.out")))
    probe = load(probe_dir)
    cal = {}
    for k, kn in known.items():
        if not isinstance(kn, dict):
            continue
        m = probe[k]
        cal[k] = {"known": kn, "measured_read_bytes": m["read_bytes"],
                  "measured_write_bytes": m["write_bytes"], "RDREQ_128B": m.get("RDREQ_128B"),
                  "RDREQ_64B": m.get("RDREQ_64B"), "RDREQ_32B": m.get("RDREQ_32B"),
                  "WRREQ_64B": m.get("WRREQ_64B")}
        if "read" in kn:
            cal[k]["read_ratio"] = m["read_bytes"] / kn["read"]
        if "write" in kn:
            cal[k]["write_ratio"] = m["write_bytes"] / kn["write"]
        if "accesses" in kn:
            cal[k]["read_bytes_per_access"] = m["read_bytes"] / kn["accesses"]
    # FETCH_SIZE / WRITE_SIZE of the same probe kernels (scripts/probe_traffic.sh)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(probe_fs_dir, "pmc_" + c, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            if k in cal:
                cal[k][c + "_KiB"] = sum(v) / len(v)
    bench = load(bench_dir)
    o2 = [k for k in bench if "k_sgns_o2" in k][0]
    t = json.load(open(traffic_json))
    out = {
        "what": "FETCH_SIZE/WRITE_SIZE calibration on known byte counts in the O2 kernel's access "
                "patterns (scripts/traffic_probe.hip), and the O2 kernel's exact fabric bytes from "
                "request-size counters (scripts/pmc_bytes.sh)",
        "finding": "every read request of these patterns is a 128-B request (TCC_EA0_RDREQ_128B = "
                   "RDREQ): 512-B row gathers with dword-per-lane loads, streaming 16-B loads AND "
                   "4-B scattered table reads alike; FETCH_SIZE tallies each at 64 B, so read bytes "
                   "= 2 x FETCH_SIZE x 1024 for the whole O2 kernel (rows and negative-table draws); "
                   "stores and float atomics are 64-B write requests, WRITE_SIZE x 1024 exact",
        "probe": cal,
        "o2_kernel": {"name": o2, "exact_read_bytes": bench[o2]["read_bytes"],
                      "exact_write_bytes": bench[o2]["write_bytes"],
                      "exact_total_bytes": bench[o2]["read_bytes"] + bench[o2]["write_bytes"],
                      "counters": {k: v for k, v in bench[o2].items()
                                   if k not in ("read_bytes", "write_bytes")},
                      "fetch_write_size_total_bytes": t["hbm_bytes_per_launch"],
                      "fetch_write_size_source": os.path.basename(traffic_json)},
    }
    json.dump(out, open(os.path.join(root, "profiles", "r02_traffic_calibration.json"), "w"),
              indent=1)
    print(json.dumps(out["o2_kernel"], indent=1))
    for k, v in cal.items():
        print(k, {x: v[x] for x in v if x.endswith("ratio") or x.endswith("per_access")})


if __name__ == "__main__":
    main(*sys.argv[1:5])
