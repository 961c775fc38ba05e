"""The N > 1 bench line, end to end: bench.py under torch.distributed.run
with two gloo ranks sharing cuda:0 (the driver's 8-GPU runs use nccl, one
GPU per rank; the code path after init is the same).  The line must carry
the self-checks of DESIGN.md section 6.5: every rank's [Q | b_i] replica
fingerprint equal, rank 0's one-GPU replay of the rotation order bit-equal to
the two-rank result, the RMSE gap to an N = 1 run, the exchange time."""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("exchange", ["rotate", "delta"])
def test_bench_two_ranks_checks_itself(exchange):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus",
           "2", "--backend", "gloo", "--workload", "small", "--steps", "2", "--warmup", "1",
           "--exchange", exchange]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=540)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["exchange"] == exchange
    m = d["multi_gpu"]
    assert m["replicas_agree"] and len(set(m["replica_fingerprints"])) == 1
    assert abs(m["n1"]["rmse_gap_vs_n1"]) < 0.05
    assert d["phases"]["exchange_ms_per_epoch"] > 0
    if exchange == "rotate":
        assert m["replay"]["bit_equal"]
        assert d["phases"]["ring_pass_ms_per_epoch"] > 0
    assert d["roofline"]["frac"] > 0
