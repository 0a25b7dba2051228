"""Real multi-process runs of the product's multi-GPU driver on the box's one GPU: 2 and 3 ranks
(torch.distributed.run, gloo — RCCL needs one GPU per rank, the driver's 8-GPU run is not ours
to launch), each a separate process through libghs_mst.so, checked against the oracle."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,scale", [(2, 16), (3, 14)])
def test_ranks_in_separate_processes_match_oracle(world, scale, tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path / "verdict.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "gpu_workers", "dist_ranks.py"), str(out), str(scale)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    v = json.loads(out.read_text())
    assert v == {"world": world, "m": v["m"], "flags_match_oracle": True, "totals_match_oracle": True,
                 "ranks_agree": True, "collected_match_oracle": True}


def test_setup_failure_fails_every_rank(tmp_path):
    """One rank's setup fails (ghs_config_t.fault_rank): every rank raises from the constructor's
    setup agreement — the failing one with its own error, the others GHS_E_STATE — and nothing
    waits in a collective (the subprocess would time out)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_ghs_implementation_amd import _native
    out = tmp_path / "verdict.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "gpu_workers", "dist_ranks.py"), str(out), "12", "fault"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    v = json.loads(out.read_text())
    assert v == {"world": 3, "codes": [_native.GHS_E_STATE, _native.GHS_E_NOMEM, _native.GHS_E_STATE]}


def test_bench_two_ranks_sharing_the_gpu(tmp_path):
    """bench.py's N > 1 leg (gloo, both ranks on the one GPU, R-MAT s16): the line names the loop
    that ran and its MSF matches a one-GPU solve of the same graph edge for edge."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--scale", "16",
           "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["loop"] == "run_rounds"
    assert line["parity"]["match"] is True, line["parity"]
