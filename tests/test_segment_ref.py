"""The oracle's restatement of Segment::checkMetadataIntegrity
(src/Segment.cc:758-800) against the reference's own walk scenarios:
src/SegmentTest.cc:598-620 (payload scribble OK, metadata scribble "bad
checksum"), :622-648 (a 1 GiB entry with head = 1: "run off past expected
length", then "past allocated segment size"), at both segment sizes the test
is instantiated with, and src/SegmentIteratorTest.cc:44-186 (buffer and
empty-segment certificates, records found by isDone / next / getType /
getLength).  The expected outcomes are the reference tests' own; the GPU
walkers run the same fixture in tests/test_gpu_segment_ref.py."""
import pytest

import segment_ref

CASES = segment_ref.load()["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_walk_matches_reference_expectation(case, oracle_mod):
    seg = segment_ref.build(case, oracle_mod)
    flags, ck, n, table = oracle_mod.check_metadata(seg, case["cert"][0], case["cert"][1],
                                                    capacity=case["capacity"],
                                                    table_cap=case["capacity"] + 1)
    assert flags == segment_ref.flag_value(case["expect"]), (flags, case["expect"])
    if case["expect"] == "OK":
        assert ck == case["cert"][1]
    if "records" in case:
        assert segment_ref.records_of(table) == case["records"]
        assert n == len(case["records"])


def test_fixture_covers_every_outcome():
    seen = {c["expect"] for c in CASES}
    assert seen == {"OK", "BAD_CHECKSUM", "PAST_LENGTH", "PAST_CAPACITY"}
    caps = {c["capacity"] for c in CASES if c["cite"].startswith("src/SegmentTest.cc")}
    assert caps == {8 << 20, 66560}
