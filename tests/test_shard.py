"""The C-ABI multi-GPU shard entry (ramcrc_shard_*, include/ramcrc.h) and its
C++ wrapper Crc32CShard (include/ramcloud/Crc32CBatch.h), driven from a
hipcc-built host program as a RAMCloud backup process would
(src/BackupMasterRecovery.cc:743-809): argument validation on the CPU; on the
GPU, every visible GPU one rank, CRCs bit-exact against the oracle."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def _build(ramcrc, tmp_path):
    exe = tmp_path / "shard_test"
    libdir = os.path.dirname(ramcrc.lib_path())
    subprocess.check_call([
        "/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-O2", "-Wall", "-Werror",
        "-I" + os.path.join(ROOT, "include", "ramcloud"),
        "-I" + os.path.join(ROOT, "include"),
        os.path.join(ROOT, "tests", "cpp", "shard_test.cc"),
        "-L" + libdir, "-lramcrc", "-Wl,-rpath," + libdir, "-o", str(exe)])
    return exe


def test_shard_args(ramcrc, tmp_path):
    exe = _build(ramcrc, tmp_path)
    out = subprocess.run([str(exe), "args"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "failures=0" in out.stdout


def test_shard_range_matches_python(ramcrc):
    from ramcloud_amd.recovery_scan import shard_range
    for n in (0, 1, 7, 11, 2048, 2049):
        for w in (1, 2, 3, 4, 8):
            for r in range(w):
                assert ramcrc.shard_range(n, w, r) == shard_range(n, r, w)


def test_shard_unique_id_is_128_bytes(ramcrc):
    a, b = ramcrc.shard_unique_id(), ramcrc.shard_unique_id()
    assert len(a) == 128 and len(b) == 128


@pytest.mark.gpu
@pytest.mark.parametrize("nseg,seg_bytes", [(48, 8 << 20), (7, 3 << 20)])
def test_shard_gpu_vs_oracle(ramcrc, oracle_mod, tmp_path, nseg, seg_bytes):
    from ramcloud_amd import workloads
    exe = _build(ramcrc, tmp_path)
    out = subprocess.run([str(exe), "gpu", str(nseg), str(seg_bytes)], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    got = {}
    for line in out.stdout.splitlines():
        if line.startswith("crc "):
            _, i, h = line.split()
            got[int(i)] = int(h, 16)
    assert sorted(got) == list(range(nseg))
    host = np.concatenate([workloads.splitmix_bytes_np(workloads.SEGMENT_SEED + i, seg_bytes)
                           for i in range(nseg)])
    want = oracle_mod.segments(host, seg_bytes, nseg, threads=8)
    assert [got[i] for i in range(nseg)] == [int(x) for x in want]


@pytest.mark.gpu
def test_shard_python_binding(ramcrc, oracle_mod):
    """ramcrc.Shard on one GPU (ncclCommInitAll of device 0), results in the
    shard's buffers and in caller tensors, odd segment count."""
    import torch
    from ramcloud_amd import workloads
    seg, nseg = 1 << 20, 13
    d = torch.empty(nseg * seg, dtype=torch.uint8, device="cuda")
    workloads.splitmix_fill_segments(d, seg, workloads.SEGMENT_SEED)
    want = oracle_mod.segments(d.cpu().numpy(), seg, nseg, threads=8)
    sh = ramcrc.Shard(devices=[0])
    try:
        sh.segments([d], seg, nseg)
        sh.sync()
        assert np.array_equal(sh.results(nseg), want)
        out = torch.zeros(nseg, dtype=torch.int32, device="cuda")
        sh.segments([d], seg, nseg, outs=[out])
        sh.sync()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    finally:
        sh.close()
