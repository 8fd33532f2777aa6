"""bench.py's own rank launcher (`python bench.py --gpus N` without
torch.distributed.run): the children's environment, rank 0's line as the only
stdout, and a failing rank's status propagated.  CPU only: the
--launch-dry-run ranks return before anything touches a GPU."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None, timeout=120):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("n", [2, 4])
def test_children_get_the_torchrun_environment(n):
    p = run(["--gpus", str(n), "--launch-dry-run"])
    assert p.returncode == 0, p.stderr
    out = [json.loads(x) for x in p.stdout.splitlines() if x.strip()]
    assert len(out) == 1 and out[0]["rank"] == 0  # only rank 0's line on stdout
    lines = [json.loads(x) for x in p.stderr.splitlines() if x.startswith("{")]
    ranks = {d["rank"]: d for d in out + lines}
    assert sorted(ranks) == list(range(n))
    ports = {d["env"]["MASTER_PORT"] for d in ranks.values()}
    pids = {d["pid"] for d in ranks.values()}
    assert len(ports) == 1 and len(pids) == n  # one rendezvous, one process per rank
    for r, d in ranks.items():
        e = d["env"]
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == (str(r), str(r), str(n))
        assert e["MASTER_ADDR"] == "127.0.0.1"
        assert int(e["GPU_MAX_HW_QUEUES"]) <= 32
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_a_failing_rank_fails_the_job():
    p = run(["--gpus", "3", "--launch-dry-run", "--dry-run-fail-rank", "1"])
    assert p.returncode == 5
    assert "rank 1 exited with status 5" in p.stderr


def test_a_hung_rank_is_ended_after_another_fails():
    t0 = time.monotonic()
    p = run(["--gpus", "3", "--launch-dry-run", "--dry-run-fail-rank", "2", "--dry-run-hang-rank", "1"],
            env_extra={"BENCH_LAUNCH_GRACE_S": "1"}, timeout=60)
    assert p.returncode == 5
    assert "terminating rank 1" in p.stderr
    assert time.monotonic() - t0 < 30  # not the hung rank's 600 s


def test_one_gpu_does_not_launch():
    """--gpus 1 runs in this process (no launcher): the dry-run flag reports rank 0."""
    p = run(["--gpus", "1", "--launch-dry-run"])
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout.strip())
    assert d["rank"] == 0 and d["env"]["WORLD_SIZE"] is None


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    with open(f"/proc/{pid}/stat") as f:  # (a zombie is gone for our purpose)
        return f.read().split(") ")[1][0] != "Z"


def _start_with_hung_rank():
    """The launcher with rank 1 hung (rank 0 done): returns (launcher, rank 1 pid)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", "--launch-dry-run", "--dry-run-hang-rank", "1"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    for line in p.stderr:
        if line.startswith("{"):
            d = json.loads(line)
            if d["rank"] == 1:
                return p, d["pid"]
    raise AssertionError("rank 1 never reported")


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGKILL"])
def test_a_stopped_launcher_takes_its_ranks_along(sig):
    """A driver's time limit stops the launcher: SIGTERM -> it ends its ranks
    itself; SIGKILL (no handler runs) -> the kernel's parent-death signal."""
    import signal

    p, pid1 = _start_with_hung_rank()
    try:
        assert _alive(pid1)
        p.send_signal(getattr(signal, sig))
        p.wait(timeout=30)
        t_end = time.monotonic() + 20
        while _alive(pid1) and time.monotonic() < t_end:
            time.sleep(0.1)
        assert not _alive(pid1), f"rank 1 (pid {pid1}) outlived its launcher"
    finally:
        if p.poll() is None:
            p.kill()
        if _alive(pid1):
            os.kill(pid1, 9)
