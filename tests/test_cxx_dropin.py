"""Compile and run tests/cpp/crc32c_test.cc: the drop-in include/ramcloud/Crc32C.h
used exactly as RAMCloud's callers and src/Crc32CTest.cc use the reference class."""
import os
import subprocess

import pytest

from conftest import ROOT


def test_cxx_dropin(golden, ramcrc, tmp_path):
    vec = tmp_path / "vectors.txt"
    with open(vec, "w") as f:
        f.write("INPUT " + bytes(golden["crc32c_test"]["input"]).hex() + "\n")
        for c in golden["crc32c_test"]["crcByLength"]:
            f.write(f"CRC {c:08x}\n")
        for c in golden["segment_certificates"] + golden["object_checksums"] + golden["tombstone_checksums"]:
            data = c.get("stream", c.get("bytes"))
            f.write(f"GOLDEN {data} {c['checksum']:08x}\n")
    exe = tmp_path / "crc32c_test"
    libdir = os.path.dirname(ramcrc.lib_path())
    cmd = ["g++", "-std=c++11", "-O2", "-Wall", "-Werror",
           "-I" + os.path.join(ROOT, "tests", "cpp"),
           "-I" + os.path.join(ROOT, "include", "ramcloud"),
           "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "crc32c_test.cc"),
           os.path.join(ROOT, "ramcloud_amd", "dropin", "Crc32C.cc"),
           "-L" + libdir, "-lramcrc", "-Wl,-rpath," + libdir, "-o", str(exe)]
    subprocess.check_call(cmd)
    out = subprocess.run([str(exe), str(vec)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "failures=0" in out.stdout


def _build_batch_test(ramcrc, tmp_path):
    exe = tmp_path / "batch_test"
    libdir = os.path.dirname(ramcrc.lib_path())
    subprocess.check_call([
        "g++", "-std=c++11", "-O2", "-Wall", "-Werror",
        "-I" + os.path.join(ROOT, "tests", "cpp"),
        "-I" + os.path.join(ROOT, "include", "ramcloud"),
        "-I" + os.path.join(ROOT, "include"),
        os.path.join(ROOT, "tests", "cpp", "batch_test.cc"),
        os.path.join(ROOT, "ramcloud_amd", "dropin", "Crc32C.cc"),
        "-L" + libdir, "-lramcrc", "-Wl,-rpath," + libdir, "-o", str(exe)])
    return exe


def test_cxx_batch_wrapper_without_gpu(ramcrc, tmp_path):
    """Crc32CBatch compiles against the C ABI alone and reports a missing GPU
    as an exception (never a crash); skipped where a GPU is visible."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_cxx_batch_wrapper_gpu")
    exe = _build_batch_test(ramcrc, tmp_path)
    out = subprocess.run([str(exe), "nodev"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "exception" in out.stdout


@pytest.mark.gpu
def test_cxx_batch_wrapper_gpu(ramcrc, tmp_path):
    exe = _build_batch_test(ramcrc, tmp_path)
    out = subprocess.run([str(exe), "gpu"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout


def _build_replay_test(ramcrc, tmp_path):
    exe = tmp_path / "replay_test"
    libdir = os.path.dirname(ramcrc.lib_path())
    subprocess.check_call([
        "/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-O2", "-Wall", "-Werror",
        "-I" + os.path.join(ROOT, "tests", "cpp"),
        "-I" + os.path.join(ROOT, "include", "ramcloud"),
        "-I" + os.path.join(ROOT, "include"),
        os.path.join(ROOT, "tests", "cpp", "replay_test.cc"),
        os.path.join(ROOT, "ramcloud_amd", "dropin", "Crc32C.cc"),
        "-L" + libdir, "-lramcrc", "-Wl,-rpath," + libdir, "-o", str(exe)])
    return exe


def test_cxx_replay_wrapper_builds(ramcrc, tmp_path):
    """Crc32CBatch::deviceReplayVerify compiles into a host program (hipcc,
    for hipMalloc) against the C ABI."""
    assert _build_replay_test(ramcrc, tmp_path).exists()


@pytest.mark.gpu
def test_cxx_replay_wrapper_gpu(ramcrc, tmp_path):
    """The C++ replay wrapper on the device: a damaged object counted, a wrong
    certificate flagged, entries walked in both segments."""
    exe = _build_replay_test(ramcrc, tmp_path)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout
