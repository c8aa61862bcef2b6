"""The multi-GPU recovery shard's layout and step orchestration
(ramcloud_amd/csrc/shard_plan.h -- the code ramcrc_shard_segments and k_unpad
run on every rank) on the CPU: ranges, owners and gather slots for nseg
0..4100 x N 1..8, and whole steps at N 1..8 in both process models with host
stand-ins for the scan, the streams and the RCCL all-gather, including a rank
whose scan fails (it must still join the collective).  Host build of the same
header the library includes."""
import os
import subprocess

from conftest import ROOT


def test_shard_plan_host(tmp_path):
    exe = tmp_path / "shard_plan_test"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-pthread",
                           "-I" + os.path.join(ROOT, "ramcloud_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "shard_plan_test.cc"), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    fields = dict(kv.split("=") for kv in out.stdout.split())
    assert int(fields["failures"]) == 0
    assert int(fields["layout_checked"]) > 60_000_000
    assert int(fields["steps_checked"]) > 1_000_000
