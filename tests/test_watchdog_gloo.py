"""The N > 1 bench's watchdog on the CPU (gloo, world size 2).

bench.py guards every blocking wait of a rank (its launches, the gather of
its packed share, the barriers) with rtgo.watchdog.Watchdog: a wait that has
not completed within --watchdog seconds prints the rank, step and partition
and ends the process with status 3, instead of hanging the job.  Here the
gather is bench.py --host-gather's transport (rtgo.watchdog.host_gather over
gloo); one rank withholding its share must make the other's watchdog fire,
and a normal gather must not."""
import os
import socket
import subprocess
import sys
import time

from conftest import PKG, ROOT

WORKER = r"""
import os, sys, time
sys.path[:0] = [ROOT, PKG]
import torch, torch.distributed as dist
from rtgo.watchdog import Watchdog, host_gather
rank, world, withhold = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
dist.init_process_group("gloo", rank=rank, world_size=world)
wd = Watchdog(2.0, rank)
share = torch.full((4096,), rank + 1, dtype=torch.uint8)
if rank == withhold:
    time.sleep(30)  # never joins the gather
    sys.exit(0)
with wd.guard("timed launch", step="launch 0: steps of seeds 1..16", partition="balanced, 12 of 475 tiles on rank %d" % rank):
    parts = host_gather(dist, share, rank, world)
if rank == 0:
    assert [int(p[0]) for p in parts] == list(range(1, world + 1)), parts
print("gathered", rank, flush=True)
dist.destroy_process_group()
""".replace("ROOT", repr(ROOT)).replace("PKG", repr(PKG))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(withhold):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    procs = [subprocess.Popen([sys.executable, "-c", WORKER, str(r), "2", str(withhold)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    return procs


def test_watchdog_fires_when_a_rank_withholds_its_share():
    procs = _run(withhold=1)
    t0 = time.monotonic()
    try:
        out, err = procs[0].communicate(timeout=60)
        took = time.monotonic() - t0
    finally:
        procs[1].kill()  # the withholding rank (still sleeping)
        procs[1].communicate()
    assert procs[0].returncode == 3, (procs[0].returncode, err[-2000:])
    assert "rank 0: watchdog: timed launch did not complete within 2 s" in err, err[-2000:]
    assert "launch 0: steps of seeds 1..16" in err and "balanced, 12 of 475 tiles on rank 0" in err
    assert "gathered" not in out
    assert took < 45, took


def test_watchdog_stays_quiet_when_every_rank_gathers():
    procs = _run(withhold=-1)
    for p in procs:
        out, err = p.communicate(timeout=60)
        assert p.returncode == 0, err[-2000:]
        assert "gathered" in out and "watchdog" not in err
