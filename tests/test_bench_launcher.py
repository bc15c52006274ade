"""bench.py's N-rank launcher on the CPU: `python3 bench.py --gpus N`
with no RANK in the environment -- the form the driver uses for N = 1 -- spawns its own N
ranks (gloo here, RCCL on the GPU node), and the shards + result gathers give the N = 1
outputs. The `dist-selftest` workload runs the launcher, the round-robin shards of
acquisition.m:47-80's PRNs and trackingCT.m:22-528's channels and dist.py's gathers on host
arrays only, so no GPU is needed."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(n, extra_env=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                           "--workload", "dist-selftest"], env=env, capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT)


def _line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # one JSON line, from rank 0 only
    return json.loads(lines[0])


def test_spawned_ranks_equal_one_rank():
    one = _line(_run(1))
    assert one["n_gpus"] == 1 and one["rccl_world"] == 1 and not one["spawned"]
    for n in (2, 3):
        many = _line(_run(n))
        assert many["spawned"] and many["n_gpus"] == n and many["rccl_world"] == n
        assert many["backend"] == "gloo"
        assert many["digest"] == one["digest"] and many["acquired"] == one["acquired"]
        assert sum(many["config"]["prns_per_rank"]) == 32
        assert sum(many["config"]["channels_per_rank"]) == 8


def test_failing_rank_fails_the_job():
    p = _run(2, {"BENCH_SELFTEST_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert "rank 1 exited" in p.stderr


def test_terminating_the_launcher_stops_the_ranks(tmp_path):
    """SIGTERM to the parent (a driver's time limit) reaches the spawned ranks: none is left
    running on its GPU (BENCH_SELFTEST_SLEEP keeps the ranks busy)."""
    import signal
    import time
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["BENCH_SELFTEST_SLEEP"] = "60"
    env["BENCH_SELFTEST_PIDFILE"] = str(tmp_path / "pids")
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload",
                          "dist-selftest"], env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    deadline = time.time() + 60
    while time.time() < deadline and len((tmp_path / "pids").read_text().split() if (tmp_path / "pids").exists() else []) < 2:
        time.sleep(0.2)
    pids = [int(x) for x in (tmp_path / "pids").read_text().split()]
    assert len(pids) == 2
    p.send_signal(signal.SIGTERM)
    p.wait(timeout=60)
    assert p.returncode != 0
    time.sleep(1.0)
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, pid
