"""bench.py's host logic (no GPU): the PMC traffic figure is reported only for the library
build -- or a build of the same sources -- it was measured on."""
import json

import bench


def _db(tmp_path, entry):
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"c2_key": entry}))
    return str(p)


def test_traffic_for_matching_build(tmp_path):
    p = _db(tmp_path, {"hbm_bytes_per_launch": 123, "build_id": "b1", "source_id": "s1"})
    assert bench.traffic_for(p, "c2_key", "b1", "other") == (123, "b1")
    # a rebuild of the same sources (hipcc output differs byte for byte)
    assert bench.traffic_for(p, "c2_key", "b2", "s1") == (123, "b1")


def test_traffic_for_stale_or_missing(tmp_path):
    p = _db(tmp_path, {"hbm_bytes_per_launch": 123, "build_id": "b1", "source_id": "s1"})
    assert bench.traffic_for(p, "c2_key", "b2", "s2") == (None, "b1")
    assert bench.traffic_for(p, "other_key", "b1", "s1") == (None, None)
    assert bench.traffic_for(str(tmp_path / "absent.json"), "c2_key", "b1", "s1") == (None, None)


def test_committed_traffic_is_stamped():
    """Every committed entry names the build and sources it was measured on."""
    with open(bench.os.path.join(bench.ROOT, "profiles", "pmc_traffic.json")) as f:
        db = json.load(f)
    for key in ("c2_n16384_d0.001_float64_alg1_w1", "c4_n65536_d0.005_float64_alg3_w1",
                "c5_n262144_d0.001_float64_alg2_w1"):
        assert db[key]["build_id"] and db[key]["source_id"], key
        assert db[key]["hbm_bytes_per_launch"] > 0
