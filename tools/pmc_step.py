"""Per-kernel HBM traffic of one replay step from rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes (tools/gpu_r06_pmc_step.sh): the last `steps` dispatches of
each kernel are the timed steps (set-up launches of the same kernel, e.g. the
fill's stamp scan, come first).  FETCH_SIZE x 2 (the gfx950 half count of
wide reads, MI355X_MICROARCH.md HBM section); WRITE_SIZE as counted.

    python tools/pmc_step.py gpurun_out/r06/pmc_step v64 3 4294967296"""
import collections
import csv
import glob
import sys

d, tag, steps, seg_bytes = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
tot = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = collections.defaultdict(list)
    for f in glob.glob(f"{d}/{tag}_{c}/**/*counter_collection.csv", recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            if r["Counter_Name"] == c:
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                per[k].append(float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1))
    # kernels of the step run at least `steps` times; the fill's run once
    tot[c] = {k: sum(v[-steps:]) / steps for k, v in per.items() if k.startswith("k_") and len(v) >= steps}
ks = sorted(set(tot["FETCH_SIZE"]) | set(tot["WRITE_SIZE"]), key=lambda k: -tot["FETCH_SIZE"].get(k, 0))
print(f"{tag}: per step, GB (FETCH_SIZE x 2 | WRITE_SIZE)")
fr = wr = 0
for k in ks:
    a, b = tot["FETCH_SIZE"].get(k, 0) / 1e9, tot["WRITE_SIZE"].get(k, 0) / 1e9
    fr += a
    wr += b
    if a + b > 0.001:
        print(f"  {k:28s} read {a:7.3f}  write {b:7.3f}")
print(f"  total read {fr:.3f} GB + write {wr:.3f} GB = {(fr + wr) / (seg_bytes / 1e9):.2f}x the {seg_bytes / 1e9:.2f} GB of segments")
