"""Turn the FETCH_SIZE passes of tools/final_pmc.sh into profiles/pmc/<key>.json
(the files bench.py reads as roofline.traffic): for each run, the traffic key
and the algorithmic bytes come from that run's own bench line, the kernel from
its roofline, and the last `steps` dispatches are the timed ones.

    python tools/final_pmc_digest.py gpurun_out/pmc [profiles/rNN/pmc]

The counter CSVs are copied next to the JSON sources (second argument) so the
digests cite files that are committed.
"""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {"k_chunks": "k_chunks<", "k_entries": "k_entries(",
          "object verify": "k_entries(,k_walk_copyv<8192u>,k_walk_copyv<12288u>"}


def main(out, keep):
    os.makedirs(keep, exist_ok=True)
    for js in sorted(glob.glob(os.path.join(out, "*.json"))):
        name = os.path.basename(js)[:-5]
        lines = [json.loads(x) for x in open(js) if x.startswith("{")]
        csvs = glob.glob(os.path.join(out, name, "**", "*counter_collection.csv"), recursive=True)
        if not lines or not csvs:
            print(f"{name}: no line or no counter CSV, skipped")
            continue
        line = lines[-1]
        rf = line["roofline"]
        kern = next(v for k, v in KERNEL.items() if rf["kernel"].startswith(k))
        dst = os.path.join(keep, f"fetch_{name}.csv")
        shutil.copyfile(csvs[0], dst)
        subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), dst,
                               rf["traffic_key"], kern, str(rf["algorithmic_bytes_per_launch"]),
                               str(line["steps"]), os.path.relpath(dst, ROOT)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "pmc", "csv"))
