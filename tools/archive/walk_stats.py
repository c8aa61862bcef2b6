"""Walk-kernel averages (us) from rocprofv3 kernel_stats CSVs: walk_stats.py <dir>..."""
import csv
import re
import sys

KS = ["k_walk_sync", "k_walk_parts", "k_walk_fix", "k_walk_emit", "k_walk_copy", "k_seg_walk"]
for d in sys.argv[1:]:
    avg = {}
    for r in csv.DictReader(open(f"{d}/t_kernel_stats.csv")):
        for k in KS:
            if re.search(r"\b" + k + r"\b", r["Name"]):
                avg[k] = float(r["AverageNs"]) / 1e3
    print(d, " ".join(f"{k.replace('k_walk_', '')}={avg.get(k, 0):.0f}" for k in KS),
          "walk=%.0f" % sum(avg.get(k, 0) for k in KS[:5]))
