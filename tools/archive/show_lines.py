"""Print the main fields of bench.py JSON lines: python tools/show_lines.py files..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:   # a failed run
        print(f"{f}: {e}")
        continue
    r = d.get("roofline") or {}
    print(f"{f.split('/')[-1]:24s} {d['value']:>9} {d['unit']:5s} ms {d['ms_per_step']:<8} frac {r.get('frac')} "
          f"kern_ms {r.get('scan_ms_per_step', '')} ok {d.get('all_segments_verified', d.get('bit_exact', ''))}")
