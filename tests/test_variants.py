"""The A/B variant table (ramcloud_amd/variants.py) and the RAMCRC_LIB guard:
every variant moves a knob that exists in the sources away from its default,
and no variant -- nor any library loaded through RAMCRC_LIB -- names a knob
that gave wrong results (build.UNSAFE_DEFINES).  CPU only."""
import glob
import os
import re

import pytest

from ramcloud_amd import build, ramcrc
from ramcloud_amd.variants import VARIANTS

CSRC = os.path.join(os.path.dirname(build.__file__), "csrc")


def _sources():
    return "".join(open(f).read() for f in glob.glob(os.path.join(CSRC, "*")) if os.path.isfile(f))


def test_variant_knobs_exist_and_move():
    src = _sources()
    defaults = dict(re.findall(r"#ifndef (RAMCRC_\w+)\n(?://[^\n]*\n)*#define \1 (\S+)", src))
    for name, defs in VARIANTS.items():
        assert defs, name
        for d in defs:
            k, v = d.split("=")
            assert k in defaults, f"{name}: {k} is not a knob of the sources"
            assert defaults[k] != v, f"{name}: {d} is the default"


def test_no_unsafe_variant_and_build_refuses():
    for name, defs in VARIANTS.items():
        assert not build.unsafe_defines(defs), name
    with pytest.raises(ValueError):
        build._compile("/nonexistent/lib.so", ("RAMCRC_PROBE_FOLD=1",))


def test_build_info_defines_parsed():
    assert ramcrc.build_defines("ramcrc gfx950 src_sha=0123 part_shift=16 defines=none") == []
    info = "ramcrc gfx950 src_sha=0123 defines=RAMCRC_PU=3,RAMCRC_WALK_DEBUG=1"
    assert ramcrc.build_defines(info) == ["RAMCRC_PU=3", "RAMCRC_WALK_DEBUG=1"]
    assert build.unsafe_defines(ramcrc.build_defines(info)) == ["RAMCRC_WALK_DEBUG=1"]


def test_product_library_reports_no_defines():
    if not os.path.exists(build.LIB):
        pytest.skip("library not built")
    blob = open(build.LIB, "rb").read()
    assert b" defines=none" in blob
