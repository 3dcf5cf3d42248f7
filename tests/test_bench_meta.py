"""bench.py's extra JSON objects read committed profiles: the files it names
must exist and carry the fields it reports (a wrong path silently drops
`c2_end_to_end` or `roofline.traffic` from the round's bench line)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_c2_reference_profile_present():
    c2 = bench.c2_reference()
    assert c2 is not None, "profiles/<e2e>.json named by bench.c2_reference() is missing or malformed"
    assert c2["csv_byte_identical"] is True
    assert c2["genomes"] == 2000 and c2["reference_wall_s"] > c2["ours_wall_s"] > 0
    assert os.path.exists(os.path.join(ROOT, c2["source"]))


def test_pmc_traffic_profile_present():
    t = bench.traffic_from_profiles(10000, 100, 1)
    assert t is not None and 1e9 < t < 1e11  # HBM bytes per k_rows_pl launch at 10k
    assert bench.traffic_from_profiles(2000, 100, 1) is None  # other shapes: not measured


def test_host_info_fields():
    h = bench.host_info(16)
    assert set(h) == {"cpu_model", "nproc", "affinity_cpus", "usable_cpus", "cgroup_cpu_quota", "threads_used"}
    assert h["threads_used"] == 16


def _run_bench(*args, env=None):
    import subprocess

    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=e, timeout=120)


def test_bench_spawns_its_own_ranks():
    """`python bench.py --gpus N` without a launcher starts N rank processes
    itself (before any GPU call): N distinct RANKs, each with WORLD_SIZE = N,
    one rendezvous address on 127.0.0.1."""
    import json

    r = _run_bench("--gpus", "3", "--launch-dry-run")
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1, 2]
    assert {x["world_size"] for x in lines} == {3}
    assert sorted(x["local_rank"] for x in lines) == [0, 1, 2]
    assert len({x["master"] for x in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")


def test_bench_refuses_world_size_mismatch():
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero instead of
    measuring a different number of GPUs."""
    r = _run_bench("--gpus", "8", "--launch-dry-run", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_bench_single_rank_dry_run():
    import json

    r = _run_bench("--launch-dry-run")
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip())["world_size"] == 1
