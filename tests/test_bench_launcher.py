"""CPU: bench.py's multi-rank launcher end to end under gloo (``--backend gloo --proxy``): --gpus N
starts N ranks itself (torch.distributed.run as a child process), every rank takes its LPT share of
the configs[3] job, the timed region is bracketed by barriers and max-reduced, and the finished
stand-in waveforms travel by the gather-v.  The proxy line is plumbing only, never a measurement."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO


def _run(*argv, timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks_with_configs3_default(n):
    rec = _run("--gpus", str(n), "--backend", "gloo", "--proxy", "--steps", "2", "--warmup", "1")
    assert rec["proxy"] is True
    assert rec["n_gpus"] == n and rec["world_size_seen"] == n
    # N > 1 defaults to configs[3]: 64 sentences per rank, L ~ U{60..160} (seed 3)
    assert rec["config"]["sentences_per_gpu"] == 64 and rec["config"]["sentences_total"] == 64 * n
    assert rec["config"]["lengths"] == "uniform"
    sys.path.insert(0, REPO)
    from conftest import load_pkg
    w = load_pkg("weights")
    lens = w.synthetic_lengths(64 * n, 3)
    assert rec["config"]["frames_per_step"] == sum(2 * int(L) + 22 for L in lens)
    # the line carries its own single-GPU point of the same per-rank workload (rank 0's share)
    sh = load_pkg("sharding")
    costs = [2 * int(L) + 22 for L in lens]
    share0 = sh.lpt_partition(costs, n, capacity=64)[0]
    ref = rec["scaling_ref_1rank"]
    assert ref["frames_per_step"] == sum(costs[i] for i in share0)
    assert ref["value"] > 0 and ref["ms_per_step"] > 0
    assert abs(rec["efficiency"] - rec["value"] / (n * ref["value"])) < 1e-9 * rec["efficiency"]
    assert "configs3_share_1rank" not in rec


def test_launcher_single_rank_default_is_configs1():
    rec = _run("--gpus", "1", "--backend", "gloo", "--proxy", "--steps", "2", "--warmup", "0")
    assert rec["n_gpus"] == 1 and rec["world_size_seen"] == 1
    assert rec["config"]["sentences_per_gpu"] == 1 and rec["config"]["lengths"] == "fixed"
    assert rec["config"]["frames_per_step"] == 222  # L = 100 -> 2L + 22
    # ... plus the N=8 line's per-rank workload on this one GPU: rank 0's share of configs[3]
    from conftest import load_pkg
    sh = load_pkg("sharding")
    lens = load_pkg("weights").synthetic_lengths(512, 3)
    costs = [2 * int(L) + 22 for L in lens]
    share0 = sh.lpt_partition(costs, 8, capacity=64)[0]
    share = rec["configs3_share_1rank"]
    assert share["sentences"] == 64 and share["frames_per_step"] == sum(costs[i] for i in share0)
    assert "scaling_ref_1rank" not in rec and "efficiency" not in rec


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--proxy", "--backend", "gloo"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=REPO)
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)
