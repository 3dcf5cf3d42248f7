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
    assert set(h) == {"cpu_model", "nproc", "usable_cpus", "threads_used"} and h["threads_used"] == 16
