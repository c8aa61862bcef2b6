"""Per-kernel average durations from a rocprofv3 kernel_trace.csv (skips the first 2 launches of each)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
st = collections.defaultdict(list)
for r in rows:
    st[r["Kernel_Name"][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in st.items():
    w = v[2:] or v
    print(f"{k:50s} n={len(v):3d} avg={sum(w) / len(w):9.1f}us")
