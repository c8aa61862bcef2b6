"""Per-kernel statistics from a rocprofv3 SQLite output (run_results.db):
kernel-trace averages, and with --pmc the per-dispatch counter averages.

    python tools/rocpd_stats.py <run_results.db> [name-substring ...]
"""
import sqlite3
import sys
from collections import defaultdict


def main(db, pats):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    dur = defaultdict(list)
    for n, s, e in c.execute(f"select {name}, start, end from kernels"):
        dur[n].append(e - s)
    tot = sum(sum(v) for v in dur.values())
    rows = sorted(dur.items(), key=lambda kv: -sum(kv[1]))
    for n, v in rows:
        if pats and not any(p in n for p in pats):
            continue
        print(f"{n[:60]:60s} calls={len(v):4d} avg_us={sum(v) / len(v) / 1e3:10.2f} "
              f"pct={100 * sum(v) / tot:5.1f}")
    ccols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    if not ccols or "counter_value" not in ccols:
        return
    cname = "kernel_name" if "kernel_name" in ccols else "name"
    vals = defaultdict(lambda: defaultdict(list))
    for n, cn, cv in c.execute(f"select {cname}, counter_name, counter_value from counters_collection"):
        vals[n][cn].append(cv)
    for n, d in vals.items():
        if pats and not any(p in n for p in pats):
            continue
        print(n[:60], " ".join(f"{k}={sum(v) / len(v):.4g}" for k, v in sorted(d.items())))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
