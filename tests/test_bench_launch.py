"""bench.py --gpus N without a launcher spawns its own N ranks: the rank
environment each child sees, exit-status propagation, and the launch timeout. CPU only: the
hidden --probe-env flag makes each child report its environment and exit before any GPU work."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, extra_env=None, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=timeout)


def lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_spawns_n_ranks_with_rank_environment():
    r = run(["--gpus", "3", "--probe-env"])
    assert r.returncode == 0, r.stderr
    # rank 0's JSON is the parent's stdout; the other ranks' output goes to stderr
    (d0,) = lines(r.stdout)
    assert d0["RANK"] == "0"
    got = sorted(lines(r.stdout) + lines(r.stderr), key=lambda d: int(d["RANK"]))
    assert [d["RANK"] for d in got] == ["0", "1", "2"]
    assert [d["LOCAL_RANK"] for d in got] == ["0", "1", "2"]
    assert {d["WORLD_SIZE"] for d in got} == {"3"}
    assert {d["MASTER_ADDR"] for d in got} == {"127.0.0.1"}
    assert len({d["MASTER_PORT"] for d in got}) == 1 and int(got[0]["MASTER_PORT"]) > 0
    assert {d["SPT_BENCH_SPAWNED"] for d in got} == {"1"}


def test_one_gpu_does_not_spawn():
    r = run(["--gpus", "1", "--probe-env"])
    assert r.returncode == 0, r.stderr
    (d,) = lines(r.stdout)
    assert d["RANK"] is None and d["SPT_BENCH_SPAWNED"] is None


def test_external_launcher_is_respected():
    # WORLD_SIZE already set (torch.distributed.run): bench.py is one rank and spawns nothing
    r = run(["--gpus", "2", "--probe-env"], {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"})
    assert r.returncode == 0, r.stderr
    (d,) = lines(r.stdout)
    assert d["RANK"] == "1" and d["SPT_BENCH_SPAWNED"] is None


def test_failing_rank_status_propagates():
    r = run(["--gpus", "2", "--probe-env"], {"SPT_PROBE_FAIL_RANK": "1", "SPT_PROBE_EXIT": "7"})
    assert r.returncode == 7
    assert "rank 1 exited with status 7" in r.stderr


def test_hung_rank_is_ended_at_the_launch_timeout():
    t0 = time.monotonic()
    r = run(["--gpus", "2", "--probe-env", "--launch-timeout", "4"], {"SPT_PROBE_HANG_RANK": "0"})
    assert r.returncode == 124, (r.returncode, r.stderr)
    assert time.monotonic() - t0 < 60
    assert "ending them (status 124)" in r.stderr


def test_eight_spawned_ranks_forward_exactly_one_json_line():
    """The driver's 8-GPU form without a launcher (`bench.py --gpus 8`): eight probe ranks start with
    RANK 0..7 and one MASTER_PORT, and the parent's stdout holds exactly one JSON line (rank 0's);
    the other seven ranks' lines go to stderr."""
    r = run(["--gpus", "8", "--probe-env"])
    assert r.returncode == 0, r.stderr
    out = lines(r.stdout)
    assert len(out) == 1 and out[0]["RANK"] == "0" and out[0]["WORLD_SIZE"] == "8"
    assert [x for x in r.stdout.splitlines() if x.strip()] == [r.stdout.strip()]
    got = sorted(out + lines(r.stderr), key=lambda d: int(d["RANK"]))
    assert [d["RANK"] for d in got] == [str(i) for i in range(8)]
    assert len({d["MASTER_PORT"] for d in got}) == 1
