"""Per-kernel averages (us) from rocprofv3 kernel_stats CSVs: kstats.py <pattern,...> <dir>..."""
import csv
import sys

pats = sys.argv[1].split(",")
for d in sys.argv[2:]:
    avg = {}
    for r in csv.DictReader(open(f"{d}/t_kernel_stats.csv")):
        for k in pats:
            if k in r["Name"]:
                avg[k] = avg.get(k, 0) + float(r["AverageNs"]) / 1e3
    print(d, " ".join(f"{k}={avg.get(k, 0):.1f}" for k in pats))
