"""GPU, world_size 2 through a REAL process group: fresh rank processes
(tests/mp_gpu_worker.py, gloo, both on cuda:0) run shard.sharded_refmerge and
gossip.sharded_round with their actual all-reduce / all-gather sequences and
check each rank's output against the oracle (oc_refmerge) and the pyref round
simulation -- not against another GPU path."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_two_fresh_ranks_match_oracle(world):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mp_gpu_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=100)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (rc, out) in enumerate(outs):
        assert rc == 0, f"rank {r} failed:\n{out[-4000:]}"
        assert f"RANK {r} OK sharded_refmerge sharded_round sharded_set_merge_local(lww,orset)" in out, out[-2000:]
