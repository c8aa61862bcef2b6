"""Merge the corrected HBM read bytes per step of a multi-kernel path into
profiles/pmc_summary.json.

A step of the entries path is several launches (binning + k_entries_tiny +
k_entries); this sums FETCH_SIZE per launch over the
named scan kernels. Same correction as tools/pmc_summary.py:
FETCH_SIZE (KiB) x 1024 x 2 (MI355X_MICROARCH.md, HBM section).
usage: python tools/pmc_step_traffic.py <pmc csv> <key> <kernel substring>...
"""
import csv
import json
import os
import sys


def main(path, key, pats):
    per = {p: [] for p in pats}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        for p in pats:
            if p in r["Kernel_Name"]:
                per[p].append(float(r["Counter_Value"]))
    kib = {p: sum(v) / len(v) for p, v in per.items() if v}
    total = int(round(sum(kib.values()) * 1024 * 2))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_summary.json")
    d = json.load(open(out))
    d[key] = {"kernels": sorted(kib), "FETCH_SIZE_kib_per_step": kib,
              "hbm_read_bytes_per_launch_corrected": total}
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
    print(key, total)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
