"""The committed GPU test record (profiles/<tag>_gpu_tests.json): run `pytest -m gpu` once and
smoke() once on the GPU box, and stamp the outcome with the build that ran.

usage (on the GPU box, from the repo root; SPT_GIT_HEAD = the commit under test, passed by the caller
because .git does not travel):  python scripts/gpu_record.py TAG
Writes gpurun_out/<TAG>_gpu_tests.json (copied to profiles/ by hand) with: git head, the tree's
kernel_sources_sha16, the hash embedded in the libspt.so that ran (spt_build_sources_sha16), the
library's sha256, collected/passed counts, every test's outcome, and the in-tree .so files the pytest
and smoke processes had mapped (/proc/self/maps). tests/test_gpu_record.py fails on CPU when the
newest record names kernel sources other than the tree's.
Exit status: pytest's (or smoke's) when either fails, else 0.
"""
import hashlib
import importlib
import json
import os
import subprocess
import sys
import time
import xml.etree.ElementTree as ET

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sha256(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def junit_outcomes(path):
    out = {}
    for tc in ET.parse(path).getroot().iter("testcase"):
        name = f"{tc.get('classname')}::{tc.get('name')}"
        kind = "passed"
        for child in tc:
            if child.tag in ("failure", "error"):
                kind = "failed" if child.tag == "failure" else "error"
            elif child.tag == "skipped":
                kind = "skipped"
        out[name] = kind
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r06"
    gout = os.path.join(ROOT, "gpurun_out")
    os.makedirs(gout, exist_ok=True)
    junit = os.path.join(gout, f"{tag}_junit_gpu.xml")
    maps_pytest = os.path.join(gout, f"{tag}_maps_pytest.txt")
    maps_smoke = os.path.join(gout, f"{tag}_maps_smoke.txt")
    env = dict(os.environ, SPT_MAPS_OUT=maps_pytest)
    t0 = time.time()
    with open(os.path.join(gout, f"{tag}_pytest_gpu.log"), "w") as log:
        rc_py = subprocess.call(
            ["timeout", "-k", "10", "600", sys.executable, "-u", "-m", "pytest", "tests", "-m", "gpu",
             "-q", "--timeout", "120", "--timeout-method", "thread", f"--junitxml={junit}"],
            cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT)
    t_py = time.time() - t0
    rc_sm = None
    smoke_tail = ""
    if rc_py == 0:
        code = ("import __graft_entry__ as g; g.smoke()\n"
                "libs = sorted({l.split()[-1] for l in open('/proc/self/maps') "
                f"if l.rstrip().endswith('.so') and {ROOT!r} in l}})\n"
                f"open({maps_smoke!r}, 'w').write('\\n'.join(libs) + '\\n')\n")
        p = subprocess.run(["timeout", "-k", "10", "300", sys.executable, "-c", code], cwd=ROOT,
                           capture_output=True, text=True)
        rc_sm, smoke_tail = p.returncode, (p.stdout + p.stderr).strip().splitlines()[-3:]
    spt = importlib.import_module("small-pathtracer_amd")
    lib = spt.LIB_PATH
    outcomes = junit_outcomes(junit) if os.path.exists(junit) else {}
    counts = {k: sum(1 for v in outcomes.values() if v == k) for k in ("passed", "failed", "error", "skipped")}
    read = lambda p: open(p).read().split() if os.path.exists(p) else []  # noqa: E731
    rec = {
        "tag": tag,
        "git_head": os.environ.get("SPT_GIT_HEAD", "unknown"),
        "git_dirty": os.environ.get("SPT_GIT_DIRTY", "unknown"),
        "kernel_sources_sha16": spt.kernel_sources_sha16(),
        "libspt_build_sources_sha16": spt.build_sources_sha16(),
        "libspt_sha256": sha256(lib),
        "pytest": {"command": "pytest tests -m gpu -q --timeout 120 --timeout-method thread",
                   "exit": rc_py, "seconds": round(t_py, 1), "collected": len(outcomes), **counts},
        "smoke": {"exit": rc_sm, "tail": smoke_tail},
        "maps_pytest": read(maps_pytest),
        "maps_smoke": read(maps_smoke),
        "libspt_mapped": {"pytest": any(p.endswith("/libspt.so") for p in read(maps_pytest)),
                          "smoke": any(p.endswith("/libspt.so") for p in read(maps_smoke))},
        "outcomes": outcomes,
        "host": os.uname().nodename,
        "utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
    }
    with open(os.path.join(gout, f"{tag}_gpu_tests.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: rec[k] for k in ("git_head", "kernel_sources_sha16",
                                          "libspt_build_sources_sha16", "pytest", "smoke",
                                          "libspt_mapped")}))
    sys.exit(rc_py or (rc_sm or 0))


if __name__ == "__main__":
    main()
