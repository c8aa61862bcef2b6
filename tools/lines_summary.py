"""One line per bench JSON file: value, step, roofline fraction, CPU baseline.

    python tools/lines_summary.py gpurun_out/r03lines/*.json
"""
import json
import sys


def main(paths):
    for p in paths:
        try:
            with open(p) as f:
                d = json.loads(f.read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError) as e:
            print(f"{p}: unreadable ({e})")
            continue
        r = d.get("roofline") or {}
        c = d.get("cpu_baseline") or {}
        ok = c.get("bit_exact_vs_gpu", c.get("all_verified"))
        if d.get("bit_exact") is not None:
            ok = f"{ok}/{d.get('bit_exact')}"
        print(f"{p}: {d.get('value')} {d.get('unit')} step {d.get('ms_per_step')} ms "
              f"frac {r.get('frac')} kernel {r.get('avg_kernel_ms')} ms traffic {r.get('traffic')} | "
              f"cpu {c.get('value')} {c.get('kind')} x{c.get('cores')} exact {ok}"
              + (f" rescues {d['bin_rescues']}" if "bin_rescues" in d else ""))


if __name__ == "__main__":
    main(sys.argv[1:])
