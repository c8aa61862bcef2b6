"""Summarise tools/gpu_ab.sh output: per case, the median step time, value and
scan-kernel roofline fraction of every variant, and its ratio to base.

    python tools/ab_summary.py gpurun_out/ab1
"""
import glob
import json
import os
import statistics
import sys


def main(d):
    cases = open(os.path.join(d, "cases.txt")).read().strip().split(";")
    runs = {}
    for p in sorted(glob.glob(os.path.join(d, "*_*.jsonl"))):
        name = os.path.basename(p)[:-len(".jsonl")]
        v, i = name.rsplit("_", 1)
        lines = [json.loads(x) for x in open(p) if x.strip().startswith("{")]
        runs.setdefault(int(i), {})[v] = lines
    for i in sorted(runs):
        print(f"case {i}: {cases[i] if i < len(cases) else '?'}")
        base = None
        for v in ["base"] + sorted(k for k in runs[i] if k != "base"):
            if v not in runs[i]:
                continue
            ls = runs[i][v]
            ms = statistics.median(x["ms_per_step"] for x in ls)
            fr = [x.get("roofline", {}).get("frac") for x in ls]
            fr = statistics.median(f for f in fr if f is not None) if any(f is not None for f in fr) else None
            val = statistics.median(x["value"] for x in ls)
            if v == "base":
                base = ms
            rel = f"{base / ms:.3f}x" if base else ""
            print(f"  {v:14s} n={len(ls)} step {ms:.4f} ms  value {val:.1f}  frac {fr}  {rel}")


if __name__ == "__main__":
    main(sys.argv[1])
