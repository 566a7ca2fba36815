"""The committed GPU test record must belong to the kernel sources in the tree (CPU test).

scripts/gpu_record.py runs `pytest -m gpu` and smoke() on an MI355X and writes
profiles/<tag>_gpu_tests.json stamped with the kernel-source hash the library was built from. A
kernel edit without a new GPU run makes the newest record stale, and this test fails: the record can
no longer vouch for the bit-exactness of the kernels that ship.
"""
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _newest_record():
    recs = glob.glob(os.path.join(ROOT, "profiles", "r*_gpu_tests.json"))
    assert recs, "no profiles/r*_gpu_tests.json GPU test record committed"
    # newest by round, then by the record's own UTC stamp (file mtimes do not survive a checkout)
    key = lambda p: (int(re.match(r"r(\d+)", os.path.basename(p)).group(1)),  # noqa: E731
                     json.load(open(p)).get("utc", ""))
    return max(recs, key=key)


def test_newest_gpu_record_matches_kernel_sources(spt):
    path = _newest_record()
    rec = json.load(open(path))
    tree = spt.kernel_sources_sha16()
    assert rec["kernel_sources_sha16"] == tree, (
        f"{os.path.basename(path)} tested kernel sources {rec['kernel_sources_sha16']}, the tree has "
        f"{tree}: run scripts/gpu_record.py on the GPU again")
    assert rec["libspt_build_sources_sha16"] == tree, "the library that ran was built from other sources"


def test_newest_gpu_record_is_green():
    rec = json.load(open(_newest_record()))
    py = rec["pytest"]
    assert py["exit"] == 0 and py["failed"] == 0 and py["error"] == 0, py
    assert py["passed"] >= 150, py
    assert rec["smoke"]["exit"] == 0, rec["smoke"]
    assert rec["libspt_mapped"] == {"pytest": True, "smoke": True}, rec["libspt_mapped"]
    assert re.fullmatch(r"[0-9a-f]{40}", rec["git_head"]), rec["git_head"]
