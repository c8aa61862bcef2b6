"""The drop-in Crc32C.h against the reference's own caller headers and
structures:

  * compile probe: include/ramcloud/Crc32C.h with the reference's src/Buffer.h,
    Minimal.h, Tub.h and LogMetadata.h (the latter's own #include "Crc32C.h"
    resolves to the drop-in through the shared include guard, as when the
    drop-in replaces src/Crc32C.h), the Buffer overloads instantiated against
    the real Buffer::Iterator, under EXPOSE_PRIVATES -- build container only,
    nothing from the reference is copied;
  * BackupReplicaMetadata (src/BackupMasterRecovery.h:517-628): 64 packed
    42-byte records sealed through the drop-in, every seal recomputed by the
    oracle over bytes [0, 38), single-bit damage caught; the SegmentCertificate
    streams of src/SegmentTest.cc:159,369,373 give the golden checksums."""
import os
import subprocess

import pytest

from conftest import ROOT

REF_SRC = "/root/reference/src"


def _cmd(ramcrc, src, out, extra):
    libdir = os.path.dirname(ramcrc.lib_path())
    # the drop-in's directory first: it must shadow the reference's src/Crc32C.h
    return (["g++", "-std=c++11", "-O2", "-Wall", "-Werror",
             "-I" + os.path.join(ROOT, "include", "ramcloud"), "-I" + os.path.join(ROOT, "include")]
            + extra +
            ([] if out is None else [src, os.path.join(ROOT, "ramcloud_amd", "dropin", "Crc32C.cc"),
                                     "-L" + libdir, "-lramcrc", "-Wl,-rpath," + libdir, "-o", out]))


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference headers only in the build container")
def test_dropin_compiles_against_reference_headers(ramcrc):
    src = os.path.join(ROOT, "tests", "cpp", "replica_metadata_test.cc")
    for defs in (["-DREF_HEADERS", "-DPROBE_BUFFER", "-DEXPOSE_PRIVATES"],
                 ["-DREF_HEADERS", "-DPROBE_BUFFER"]):
        cmd = ["g++", "-std=c++11", "-fsyntax-only", "-Wall", "-Werror"] + defs + [
            "-I" + os.path.join(ROOT, "include", "ramcloud"), "-I" + os.path.join(ROOT, "include"),
            "-I" + REF_SRC, src]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]


def _run(ramcrc, tmp_path, extra):
    exe = str(tmp_path / "replica_metadata_test")
    src = os.path.join(ROOT, "tests", "cpp", "replica_metadata_test.cc")
    subprocess.check_call(_cmd(ramcrc, src, exe, extra))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout


def _check_output(out, oracle_mod, golden):
    metas = certs = 0
    gold = {c.get("stream"): c["checksum"] for c in golden["segment_certificates"]}
    for line in out.splitlines():
        parts = line.split()
        if parts[0] == "meta":
            rec = bytes.fromhex(parts[1])
            assert len(rec) == 42
            ck = int(parts[2], 16)
            assert oracle_mod.crc32c(rec[:38]) == ck
            assert int.from_bytes(rec[38:], "little") == ck
            metas += 1
        elif parts[0] == "cert":
            stream = bytes.fromhex(parts[1]) if len(parts) == 4 else b""
            length, ck = int(parts[-2]), int(parts[-1], 16)
            full = stream + length.to_bytes(4, "little")
            assert ck == oracle_mod.crc32c(full)
            assert gold[full.hex()] == ck   # the SegmentTest golden for this stream
            certs += 1
    assert metas == 64 and certs == 3
    assert "failures=0" in out
    return gold


def test_replica_metadata_seal(ramcrc, oracle_mod, golden, tmp_path):
    """With the repo's Buffer test double (tests/cpp/Buffer.h): runs anywhere."""
    _check_output(_run(ramcrc, tmp_path, ["-I" + os.path.join(ROOT, "tests", "cpp")]),
                  oracle_mod, golden)


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference headers only in the build container")
def test_replica_metadata_seal_reference_certificate(ramcrc, oracle_mod, golden, tmp_path):
    """Same, with the reference's own SegmentCertificate class (src/LogMetadata.h:85-128)."""
    _check_output(_run(ramcrc, tmp_path, ["-DREF_HEADERS", "-I" + REF_SRC]), oracle_mod, golden)


def test_segment_certificate_goldens(golden, oracle_mod):
    """The certificate streams above are the reference's SegmentTest goldens."""
    vals = {c["checksum"] for c in golden["segment_certificates"]}
    assert {0x48674BC7, 0x87A632E2, 0x62F2F7F6} <= vals
