"""Per-kernel PMC sums (per dispatch) from rocprofv3 counter_collection.csv files under a directory."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            k = k.split("(")[0][:40]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    print("==", d)
    for k, c in agg.items():
        n = len(disp[k])
        print(f"  {k:40s} dispatches={n}", " ".join(f"{m}={v / n:.4g}" for m, v in sorted(c.items())))
