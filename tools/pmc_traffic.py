"""Digest one rocprofv3 --pmc FETCH_SIZE pass into profiles/pmc/<key>.json, the
file bench.py reads as `roofline.traffic` for exactly that workload.

    python tools/pmc_traffic.py <counter_collection.csv> <key> <kernels> <algo_bytes> <last> [source]

kernels: comma-separated substrings of the kernel names that make up one step
of the workload (e.g. "k_chunks<" or "k_entries_tiny,k_entries(("); the
traffic of a step is the sum over them of their average FETCH_SIZE per
dispatch over the last `last` dispatches of each (the bench's timed steps:
set-up launches of the same kernel, e.g. the object fill's empty k_chunks,
are excluded).  FETCH_SIZE is in KiB and, on gfx950, counts half the bytes of wide
coalesced streaming reads (MI355X_MICROARCH.md, HBM section): corrected HBM
read bytes = FETCH_SIZE x 1024 x 2.
"""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(csv_path, key, kernels, algo_bytes, last, source=None):
    pats = [k for k in kernels.split(",") if k]
    per = {p: [] for p in pats}
    for r in csv.DictReader(open(csv_path)):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        for p in pats:
            if p in r["Kernel_Name"]:
                per[p].append(float(r["Counter_Value"]))
                break
    per = {p: v[-int(last):] for p, v in per.items()}
    missing = [p for p, v in per.items() if not v]
    if missing:
        sys.exit(f"no FETCH_SIZE rows for {missing} in {csv_path}")
    kib = {p: sum(v) / len(v) for p, v in per.items()}
    corrected = int(round(sum(kib.values()) * 1024 * 2))
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"],
                              capture_output=True, text=True).stdout.strip()
    except OSError:
        head = None
    out = {
        "workload": key,
        "kernels": pats,
        "dispatches": {p: len(v) for p, v in per.items()},
        "FETCH_SIZE_kib_per_dispatch": kib,
        "hbm_read_bytes_per_launch": corrected,
        "algorithmic_bytes_per_launch": int(algo_bytes),
        "traffic_over_algorithmic": round(corrected / int(algo_bytes), 5),
        "correction": "FETCH_SIZE(KiB) x 1024 x 2 (gfx950 half count, MI355X_MICROARCH.md HBM section)",
        "source_csv": source or os.path.relpath(csv_path, ROOT),
        "tree": head,
    }
    os.makedirs(os.path.join(ROOT, "profiles", "pmc"), exist_ok=True)
    path = os.path.join(ROOT, "profiles", "pmc", key + ".json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:7])
