"""Per-kernel register / LDS / spill summary of the device library (hipcc
-Rpass-analysis=kernel-resource-usage), for checking that a kernel change
kept its occupancy.

    python tools/resource_usage.py [-DMACRO=1 ...] [--filter k_entries]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ramcloud_amd", "csrc", "ramcrc_device.hip")


def main(argv):
    defines = [a for a in argv if a.startswith("-D")]
    filt = None
    if "--filter" in argv:
        filt = argv[argv.index("--filter") + 1]
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
               "-fconstexpr-steps=1000000000", "-fPIC", "-I" + os.path.join(ROOT, "include"),
               "-I" + os.path.dirname(SRC), "-c", SRC, "-o", os.path.join(td, "d.o"),
               "-Rpass-analysis=kernel-resource-usage"] + defines
        p = subprocess.run(cmd, capture_output=True, text=True, cwd=td)
    if p.returncode:
        sys.stderr.write(p.stderr[-4000:])
        return p.returncode
    rows, cur = [], None
    for line in p.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
        if not m:
            continue
        s = m.group(1).strip()
        if s.startswith("Function Name:"):
            name = s.split(":", 1)[1].strip()
            dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            cur = {"name": re.sub(r"\(anonymous namespace\)::", "", dm)}
            rows.append(cur)
        elif cur is not None and ":" in s:
            k, v = s.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        if filt and filt not in r["name"]:
            continue
        print(f"{r['name'][:70]:70s} vgpr={r.get('VGPRs','?'):>4s} agpr={r.get('AGPRs','?'):>3s} "
              f"sgpr={r.get('SGPRs','?'):>3s} spill_v={r.get('VGPRs Spill','?')} "
              f"spill_s={r.get('SGPRs Spill','?')} lds={r.get('LDS Size [bytes/block]','?')} "
              f"occ={r.get('Occupancy [waves/SIMD]','?')}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
