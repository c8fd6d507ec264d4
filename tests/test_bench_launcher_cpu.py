"""CPU: bench.py's own rank launcher (`python bench.py --gpus N` with no external launcher)
gives every child the torch.distributed.run environment, forwards rank 0's JSON line, and
stops the job when one rank fails (gloo stand-in for the GPU ranks)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tests", "_launch_probe.py")

_DRIVER = """
import sys
sys.path.insert(0, {root!r})
import bench
sys.exit(bench.launch_ranks({n}, {argv!r}, script={probe!r}))
"""


def _run(n, argv, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    code = _DRIVER.format(root=ROOT, n=n, argv=list(argv), probe=PROBE)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout, env=env)


def test_rank_environments():
    import bench
    envs = bench.rank_environments(4, {"X": "1"}, 29511)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
               and e["X"] == "1" for e in envs)


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_runs_n_ranks(n):
    r = _run(n, ["--gpus", str(n), "--steps", "3"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout        # only rank 0's line on stdout
    ln = lines[0]
    assert ln["rank"] == 0 and ln["world"] == n and ln["gpus"] == n and ln["steps"] == 3
    assert ln["sum"] == n * (n + 1) / 2     # every rank joined the same group
    assert ln["master"].startswith("127.0.0.1:")
    others = [json.loads(x) for x in r.stderr.splitlines() if x.startswith("{")]
    assert sorted(o["local_rank"] for o in others) == list(range(1, n))


def test_launcher_propagates_a_rank_failure():
    r = _run(2, ["--gpus", "2", "--fail-rank", "1"], timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode != 0 and "must agree" in r.stderr
