"""Digest rocprofv3 CSVs into profiles/pmc_summary.json (per-launch numbers).

FETCH_SIZE on gfx950 reads exactly half of the bytes of a wide coalesced
streaming read (MI355X_MICROARCH.md, HBM section: FETCH_SIZE = TCC_EA0_RDREQ x
64 B while the requests are 128 B), and is in KiB: corrected HBM read bytes =
FETCH_SIZE x 1024 x 2.
usage: python tools/pmc_summary.py <pmc_fetch csv> <pmc_lds csv> <kernel_stats csv> <out json>
"""
import csv
import json
import sys

KERNELS = {"k_chunks": "k_chunks<", "k_combine": "k_combine<", "k_entries": "k_entries((",
           "k_plan_count": "k_plan_count", "k_plan_scan": "k_plan_scan"}


def per_kernel(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        for short, pat in KERNELS.items():
            if pat in r["Kernel_Name"]:
                agg.setdefault(short, {}).setdefault(r["Counter_Name"], []).append(
                    float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main(fetch_csv, lds_csv, stats_csv, out):
    res = {}
    fetch = per_kernel(fetch_csv)
    lds = per_kernel(lds_csv) if lds_csv != "-" else {}
    for k in set(fetch) | set(lds):
        e = {}
        if "FETCH_SIZE" in fetch.get(k, {}):
            kib = fetch[k]["FETCH_SIZE"]
            e["FETCH_SIZE_kib_per_launch"] = kib
            e["hbm_read_bytes_per_launch_corrected"] = int(kib * 1024 * 2)
        for c, v in lds.get(k, {}).items():
            e[c] = v
        if "SQ_LDS_BANK_CONFLICT" in e and e.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = e["SQ_LDS_BANK_CONFLICT"] / e["SQ_LDS_IDX_ACTIVE"]
        res[k] = e
    if stats_csv != "-":
        for r in csv.DictReader(open(stats_csv)):
            for short, pat in KERNELS.items():
                if pat in r["Name"]:
                    res.setdefault(short, {})["rocprof_avg_ns"] = float(r["AverageNs"])
                    res[short]["rocprof_calls"] = int(r["Calls"])
    res["_note"] = ("per-launch averages; hbm_read_bytes_per_launch_corrected = FETCH_SIZE(KiB) "
                    "x 1024 x 2 (gfx950 half-count correction, MI355X_MICROARCH.md HBM section)")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:5])
