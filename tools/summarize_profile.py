#!/usr/bin/env python3
"""Summarize a tools/profile.sh run (rocprofv3 kernel trace + PMC passes) into
profiles/<tag>_summary.json (and, for the default cfg2 bench kernel,
profiles/traffic.json).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports
half the bytes of wide coalesced reads on gfx950, so it is doubled;
WRITE_SIZE (KB) is exact for 16-B streaming stores.  Counters come from
separate --pmc passes (never combined with trace domains).

    tools/summarize_profile.py <tag> [--kernel SUBSTRING] [--no-traffic]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="block_sums", help="substring of the kernel name to summarize")
    ap.add_argument("--no-traffic", action="store_true", help="do not rewrite profiles/traffic.json")
    ap.add_argument("--outdir", default="profiles")
    ap.add_argument("--timed", type=int, default=0,
                    help="the bench's timed launches are the last N dispatches: report their mean too")
    ap.add_argument("--traffic-key", default=None,
                    help="also write the HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE) to profiles/traffic.json "
                         "under this key (cfg4 / cfg5 / filesums lines)")
    ap.add_argument("--roll-cus", type=int, default=224,
                    help="CUs the roll's workgroups occupy (cfg3 batch: all but RSG_CONFIRM_CUS = 32 of 256)")
    a = ap.parse_args()
    tag, kernel, outdir = a.tag, a.kernel, a.outdir
    src = f"gpurun_out/prof_{tag}"

    def rows(path):
        return [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]

    stats = list(csv.DictReader(open(glob.glob(f"{src}/trace/*kernel_stats.csv")[0])))
    trace = [r for r in csv.DictReader(open(glob.glob(f"{src}/trace/*kernel_trace.csv")[0]))]
    counters = defaultdict(list)
    for f in glob.glob(f"{src}/pmc_*/*counter_collection.csv"):
        for r in rows(f):
            counters[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in counters.items()}
    mine = sorted((r for r in trace if kernel in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in mine]
    steady = sorted(durs)[len(durs) // 4: 3 * len(durs) // 4] if len(durs) >= 8 else durs
    out = {
        "tag": tag,
        "kernel_filter": kernel,
        "kernel_stats": [{k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs")} for r in stats],
        "dispatches": len(durs),
        "us_mean": round(sum(durs) / max(len(durs), 1), 2),
        "us_interquartile_mean": round(sum(steady) / max(len(steady), 1), 2),
        **({"timed_launches": a.timed, "timed_launches_us_mean": round(sum(durs[-a.timed:]) / a.timed, 2)}
           if a.timed and len(durs) >= a.timed else {}),
        "pmc_mean_per_dispatch": {k: round(v, 1) for k, v in sorted(avg.items())},
    }
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = avg["FETCH_SIZE"] * 1024 * 2  # gfx950: FETCH_SIZE reads half of wide coalesced reads
        write = avg["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = {"fetch_corrected": int(fetch), "write": int(write), "total": int(fetch + write),
                                       "note": "FETCH_SIZE*2 (gfx950 wide-read correction) + WRITE_SIZE, KB->B"}
    if "GRBM_GUI_ACTIVE" in avg and durs:
        out["effective_clock_ghz"] = round(avg["GRBM_GUI_ACTIVE"] / 8 / (out["us_mean"] * 1e3), 3)
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_BUSY_CYCLES" in avg:
        out["note_units"] = "SQ_* wave/active counters count quad-cycles (MI355X_MICROARCH.md constants table)"
    os.makedirs(outdir, exist_ok=True)
    json.dump(out, open(f"{outdir}/{tag}_summary.json", "w"), indent=1)
    def merge(name, upd):
        path = f"{outdir}/{name}"
        cur = json.load(open(path)) if os.path.exists(path) else {}
        cur.update(upd)
        json.dump(cur, open(path, "w"), indent=1)

    if "hbm_bytes_per_launch" in out and a.traffic_key:
        merge("traffic.json", {a.traffic_key: out["hbm_bytes_per_launch"]["total"],
                               a.traffic_key + "_source": f"profiles/{tag}_summary.json: FETCH_SIZE x 2 + WRITE_SIZE "
                                                         "per launch (rocprofv3 --pmc passes of the bench workload)"})
    elif "hbm_bytes_per_launch" in out and kernel == "block_sums" and not a.no_traffic:
        merge("traffic.json", {"block_sums_kernel_cfg2_bytes_per_launch": out["hbm_bytes_per_launch"]["total"],
                               "source": f"profiles/{tag}_summary.json"})
    if "roll" in kernel and not a.no_traffic:
        if "FETCH_SIZE" in avg:
            merge("traffic.json", {"roll_packed_kernel_cfg3_bytes_per_launch": int(avg["FETCH_SIZE"] * 1024 * 2),
                                   "roll_packed_kernel_cfg3_source": f"profiles/{tag}_summary.json: FETCH_SIZE x 2 "
                                   "(the gfx950 correction) per roll launch over a 1 GiB cfg3 source"})
        if "SQ_INSTS_VALU" in avg:
            merge("counters.json", {"roll_packed_kernel_cfg3": {
                "valu_wave_insts_per_launch": int(avg["SQ_INSTS_VALU"]),
                "salu_insts_per_launch": int(avg.get("SQ_INSTS_SALU", 0)),
                "branch_insts_per_launch": int(avg.get("SQ_INSTS_BRANCH", 0)),
                "lds_bank_conflict_frac": round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"], 4)
                if avg.get("SQ_LDS_IDX_ACTIVE") else None,
                "clock_ghz": out.get("effective_clock_ghz") or 2.4,
                "roll_cus": a.roll_cus,
                "kernel_us_mean": out["us_mean"],
                "source": f"profiles/{tag}_summary.json (rocprofv3 --pmc passes of bench.py --workload cfg3)"}})
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
