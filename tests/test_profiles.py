"""The committed measurement record is reproducible: profiles/counters.json
(read by bench.py for roofline.traffic / lds_hit) is what tools/counters.py
computes from the committed rocprofv3 PMC CSVs it names."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DB = os.path.join(ROOT, "profiles", "counters.json")


def _records():
    return sorted(json.load(open(DB)).items()) if os.path.exists(DB) else []


@pytest.mark.parametrize("key,rec", _records(), ids=lambda x: x if isinstance(x, str) else "")
def test_counters_json_reproducible_from_committed_csvs(key, rec, tmp_path):
    srcs = [os.path.join(ROOT, s) for s in rec["sources"]]
    assert all(os.path.exists(s) for s in srcs), "a source CSV of the record is not committed"
    # run the committed script on a copy of the tree's profiles dir
    work = tmp_path / "repo"
    (work / "profiles").mkdir(parents=True)
    (work / "tools").mkdir()
    script = os.path.join(ROOT, "tools", "counters.py")
    (work / "tools" / "counters.py").write_text(open(script).read())
    subprocess.run([sys.executable, str(work / "tools" / "counters.py"), key, str(int(rec["frames_per_launch"]))] + srcs,
                   check=True, capture_output=True, cwd=ROOT)
    got = json.load(open(work / "profiles" / "counters.json"))[key]
    for k, kr in rec["kernels"].items():
        for field in ("traffic", "lds_hit", "fetch", "write"):
            if field in kr:
                assert got["kernels"][k][field] == pytest.approx(kr[field], rel=1e-12), (k, field)
    # the x2 FETCH_SIZE correction is calibrated on the pre-pass: its reads are the int32 symbols
    assert rec["pre_calibration"] == pytest.approx(1.0, abs=0.01)
