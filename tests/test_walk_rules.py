"""The parallel walk's first-hop filter (ramcloud_amd/csrc/walk_rules.h) is a
superset of the exact plausibility rule for every header byte and top length
byte, on both sides of the capacity cut-offs it uses (host build of the same
header the kernels include)."""
import os
import subprocess

from conftest import ROOT


def test_first_hop_filter_is_superset(tmp_path):
    exe = tmp_path / "walk_rules_test"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Werror",
                           "-I" + os.path.join(ROOT, "ramcloud_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "walk_rules_test.cc"), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    fields = dict(kv.split("=") for kv in out.stdout.split())
    assert int(fields["violations"]) == 0
    assert int(fields["checked"]) > 10_000_000
    # the filter passes every exact survivor and not many more
    assert int(fields["exact"]) <= int(fields["filter"]) < 2 * int(fields["exact"]) + 1000
