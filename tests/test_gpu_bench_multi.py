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
        # the delta exchange measured in the same job, nested
        de = d["delta_exchange"]
        assert de["exchange"] == "delta" and de["value"] > 0
        assert de["multi_gpu"]["replicas_agree"]
    else:
        assert "delta_exchange" not in d
    assert d["roofline"]["frac"] > 0
    # the default line: FP64 (the reference's arithmetic) at top level, the
    # FP32 perf layout nested with its own checks
    assert d["dtype"] == "f64"
    f = d["fp32_layout"]
    assert f["dtype"] == "f32" and f["value"] > 0 and f["multi_gpu"]["replicas_agree"]
    if exchange == "rotate":
        assert f["multi_gpu"]["replay"]["bit_equal"]


@pytest.mark.timeout(600)
def test_bench_c4_shape_eight_ranks_rotate():
    """configs[3] (C4) at its real shape: 1M x 100K, 100M ratings, rank 64,
    user-sharded over 8 ranks -- here 8 gloo ranks sharing cuda:0 with
    per-stratum launches (MF_STRATA_PERSISTENT=0: eight processes share the
    CUs, so a persistent grid cannot count on co-residency; same bits).  The
    line's own checks must hold at this shape (FP64, the headline's dtype):
    the eight replicas agree, rank
    0's one-GPU replay of the 8-rank rotation order is bit-equal, and the
    RMSE after 2 epochs is within 1e-3 of the N = 1 schedule's."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus",
           "8", "--backend", "gloo", "--workload", "c3", "--steps", "1", "--warmup", "1",
           "--dtype", "float64"]
    env = dict(os.environ, MF_STRATA_PERSISTENT="0")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=540, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["nnz"] == 100_000_000 and d["dtype"] == "f64"
    assert d["config"]["exchange"] == "rotate"
    m = d["multi_gpu"]
    assert m["replicas_agree"] and len(set(m["replica_fingerprints"])) == 1
    assert m["replay"]["bit_equal"]
    assert abs(m["n1"]["rmse_gap_vs_n1"]) < 1e-3
