import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "crc32c_golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def golden_base(golden, oracle_mod):
    r = golden["random"]
    return oracle_mod.splitmix_bytes(r["seed"], r["base_len"])


@pytest.fixture(scope="session")
def ramcrc():
    from ramcloud_amd import build, ramcrc as rc
    build.build()
    rc.lib()
    return rc
