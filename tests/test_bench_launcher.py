"""bench.py's multi-rank contract on the CPU: `python bench.py --gpus 2` starts
its own two ranks (no external launcher), shards the config-4 recovery batch
of RecoverSegmentBenchmark-shaped segments, gathers the CRCs (gloo here,
RCCL on the GPU box) and prints one JSON line with n_gpus 2 and strong
scaling; the gathered CRCs equal the oracle's.  A launcher whose WORLD_SIZE
disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

import numpy as np

from conftest import ROOT


def _json_line(stdout):
    lines = [x for x in stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_spawns_ranks_and_gathers(oracle_mod, ramcrc):
    from ramcloud_amd import segments, workloads
    nseg, seg, vlen = 9, 64 * 1024, 1024
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--host-dry-run", "--nseg-total", str(nseg), "--seg-kib", "64",
                          "--value-len", str(vlen), "--steps", "2", "--warmup", "1"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = _json_line(out.stdout)
    assert line["n_gpus"] == 2
    assert line["scaling"] == "strong"
    assert line["dry_run"] is True
    assert line["config"]["parallelism"] == "shard2"
    per = segments.objects_per_segment(seg, vlen)
    want = []
    for i in range(nseg):
        s = workloads.splitmix_bytes_np(workloads.SEGMENT_SEED + i, seg)
        ramcrc.segment_fill_objects(s, vlen, first_key=i * per)
        want.append(oracle_mod.crc32c(s))
    assert line["crcs"] == want
    # the reference CPU baseline rides on the N > 1 line too (rank 0, whole batch)
    cpu = line["cpu_baseline"]
    assert cpu["bit_exact_vs_gpu"] is True and cpu["cores"] >= 1 and cpu["value"] > 0
    assert cpu["kind"] in ("reference", "port")


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--host-dry-run"], capture_output=True, text=True, timeout=120,
                         env=env, cwd=ROOT)
    assert out.returncode == 2
    assert "WORLD_SIZE" in out.stderr


def test_host_cpu_info_and_threads():
    sys.path.insert(0, ROOT)
    import bench
    info = bench.host_cpu_info()
    assert info["physical_cores"] >= 1 and info["logical"] >= info["physical_cores"] // 2
    t = bench.baseline_threads(info)
    assert 1 <= t <= info["physical_cores"]
    q = info["cgroup_cpu_quota"]
    if q:
        assert t <= max(1, int(q))
    fake = dict(info, physical_cores=128, affinity=256, cgroup_cpu_quota=16.0)
    assert bench.baseline_threads(fake) == 16
    fake = dict(info, physical_cores=128, affinity=256, cgroup_cpu_quota=None)
    assert bench.baseline_threads(fake) == 128


def test_traffic_lookup_is_per_workload(tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    assert bench.traffic_for("no_such_workload") == (None, None)
    r = bench.roofline("k_chunks", 8 << 30, 1.25, "no_such_workload")
    assert r["traffic"] is None and r["traffic_source"] is None
    assert abs(r["achieved"] - (8 << 30) / 1.25e-3 / 1e9) < 0.1
