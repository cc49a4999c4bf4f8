"""bench.py's own multi-rank launcher: `python3 bench.py --gpus N` started without a torchrun environment
spawns its N ranks (one process per GPU, torch.distributed.run on 127.0.0.1) and rank 0 prints the line.

CPU: the launcher and the decomposition with --dry-run (gloo, no GPU touched). GPU: the real 2-rank bench
on the box's one card (DFMI_RCCL_SPLIT_HOSTS=1: RCCL over sockets), a functional check of the line, not a
scaling number."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(args, timeout, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout      # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("n_gpus,layout", [(2, "2x1x1"), (4, "2x2x1")])
def test_bench_spawns_its_ranks_dry_run(n_gpus, layout):
    d = _run(["--gpus", str(n_gpus), "--n", "16", "--dry-run"], 240, {"DFMI_RCCL_SPLIT_HOSTS": "1"})
    assert d["n_gpus"] == n_gpus and d["scaling"] == "weak"
    assert layout in d["config"]["parallelism"]
    assert d["config"]["cells_total"] == n_gpus * 16 ** 3
    assert sorted(e["rank"] for e in d["ranks"]) == list(range(n_gpus))
    assert sorted(e["local_rank"] for e in d["ranks"]) == list(range(n_gpus))
    assert all(e["proc_faces"] > 0 for e in d["ranks"])   # every block has processor patches


def test_bench_single_gpu_dry_run_stays_in_process():
    d = _run(["--gpus", "1", "--n", "8", "--dry-run"], 120)
    assert d["n_gpus"] == 1 and d["config"]["parallelism"] == "single"


@pytest.mark.gpu
def test_bench_two_ranks_on_one_card():
    """the same command the driver runs for N = 2, on one GPU: both ranks step the decomposed box over RCCL"""
    d = _run(["--gpus", "2", "--n", "16", "--steps", "3", "--warmup", "1", "--roof-steps", "1", "--alt-steps", "0",
              "--no-cpu", "--no-flame"], 280, {"DFMI_RCCL_SPLIT_HOSTS": "1"})
    assert d["n_gpus"] == 2 and "2x1x1" in d["config"]["parallelism"]
    assert d["finite"] and d["value"] > 0
    assert d["ms_per_step_median"] > 0
    assert "comm" in d and d["comm"]["points"]
