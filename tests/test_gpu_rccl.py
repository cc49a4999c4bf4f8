"""The RCCL transport with real separate processes (MI355X, one card).

Two torchrun ranks share the box's one GPU; `scripts/rccl_ranks.py` gives each rank its own
NCCL_HOSTID so RCCL accepts them (they talk through its socket transport instead of xGMI). This runs
the product multi-GPU path end to end -- ncclCommInitRank, the ncclSend/ncclRecv halo groups, the
ncclAllGather reductions, and (overlap=1) the comm stream -- and compares the gathered fields with the
undecomposed run and with the oracle (same tolerances as test_gpu_multirank.py).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

_PORT = [29611]


def _launch(tmp_path, decomp, overlap, steps=1, walls=0, mesh="10,8,6"):
    n = 1
    for d in decomp.split(","):
        n *= int(d)
    out = tmp_path / f"rccl_{decomp.replace(',', '')}_{overlap}_{steps}_{walls}.json"
    port = _PORT[0]; _PORT[0] += 1
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "scripts", "rccl_ranks.py"), "--decomp", decomp, "--overlap", str(overlap),
           "--steps", str(steps), "--walls", str(walls), "--mesh", mesh, "--out", str(out)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    return json.loads(out.read_text())


@pytest.mark.parametrize("overlap", [0, 1])
def test_rccl_two_ranks_match_single_domain_and_oracle(tmp_path, overlap):
    r = _launch(tmp_path, "2,1,1", overlap)
    assert len(set(r["p_iters_per_rank"])) == 1, r      # every rank took the same convergence decisions
    for n, e in r["vs_single_domain"].items():
        assert e < 1e-9, (n, e, r)
    for n, e in r["vs_oracle"].items():
        assert e < 1e-9, ("oracle", n, e, r)


def test_rccl_four_ranks_walls_two_steps(tmp_path):
    r = _launch(tmp_path, "2,2,1", 1, steps=2, walls=1, mesh="8,8,4")
    assert len(set(r["p_iters_per_rank"])) == 1, r
    for n, e in r["vs_single_domain"].items():
        assert e < 1e-9, (n, e, r)


def test_rccl_eight_ranks_config5_layout(tmp_path):
    """BASELINE config 5's decomposition (2x2x2 blocks, 8 ranks, processorCyclic wrap-around) at a small
    mesh: eight RCCL processes vs the single-domain run and the oracle. (The full 256^3 = 16.8M-cell run
    of the same script is scripts/rccl_config5.sh, recorded in profiles/.)"""
    r = _launch(tmp_path, "2,2,2", 0, mesh="16,16,16")
    assert r["world"] == 8 and len(set(r["p_iters_per_rank"])) == 1, r
    for n, e in r["vs_single_domain"].items():
        assert e < 1e-9, (n, e, r)
    for n, e in r["vs_oracle"].items():
        assert e < 1e-9, ("oracle", n, e, r)
