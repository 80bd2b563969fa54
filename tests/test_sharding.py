"""Multi-rank sentence sharding on CPU: LPT partition and the gloo world_size>1
gather-v of waveforms + global int16 peak normalisation, against a single-process restatement of
Synthesizer.tts's join (server/synthesizer.py:157-161, utils/audio.py:56-58)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_pkg

sharding = load_pkg("sharding")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_wav(i, L):
    """Stand-in for sentence i's waveform: 275 * (2L+21) samples, deterministic."""
    n = 275 * (2 * L + 21)
    return np.random.Generator(np.random.PCG64(i)).standard_normal(n) * (0.1 + 0.01 * i)


def test_lpt_partition_balanced_and_complete():
    rng = np.random.Generator(np.random.PCG64(3))
    L = rng.integers(60, 161, size=512)
    costs = [sharding.sentence_cost(int(x), 1000) for x in L]
    parts = sharding.lpt_partition(costs, 8)
    assert sorted(i for p in parts for i in p) == list(range(512))
    assert all(len(p) == 64 for p in parts)
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)  # LPT bound
    assert max(loads) / (sum(costs) / 8) < 1.01
    assert parts == sharding.lpt_partition(costs, 8)  # deterministic on every rank


def test_lpt_partition_edge_cases():
    assert sharding.lpt_partition([], 4) == [[], [], [], []]
    assert sharding.lpt_partition([5], 3) == [[0], [], []]
    assert sharding.lpt_partition([3, 3, 3, 3], 2) == [[0, 2], [1, 3]]
    with pytest.raises(ValueError):
        sharding.lpt_partition([1, 2, 3], 2, capacity=1)
    # capacity binds before load balance
    parts = sharding.lpt_partition([100, 1, 1, 1], 2, capacity=2)
    assert sorted(map(len, parts)) == [2, 2]
    assert sharding.sentence_cost(100, 1000) == 222
    assert sharding.sentence_cost(600, 1000) == 1000
    assert sharding.sentence_cost(10, 1000, forward_attn_mask=False) == 1020


def _worker(rank, world, port, lens, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        costs = [sharding.sentence_cost(L, 1000) for L in lens]
        parts = sharding.lpt_partition(costs, world)
        mine = parts[rank]
        wavs = [torch.from_numpy(_fake_wav(i, lens[i])) for i in mine]
        peak = sharding.global_peak(wavs)
        allw = sharding.gather_waveforms(wavs, mine, len(lens))
        if rank == 0:
            pcm = sharding.join_int16(allw, peak)
            np.savez(out_path, pcm=pcm, peak=peak, n=[len(w) for w in allw])
        else:
            assert allw is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nsent", [(2, 7), (3, 2), (2, 1)])
def test_gloo_gather_matches_single_process(world, nsent):
    lens = [int(x) for x in np.random.Generator(np.random.PCG64(nsent)).integers(3, 30, size=nsent)]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r0.npz")
        mp.spawn(_worker, args=(world, _free_port(), lens, out), nprocs=world, join=True)
        z = np.load(out)
        ref_w = [_fake_wav(i, L) for i, L in enumerate(lens)]
        assert list(z["n"]) == [len(w) for w in ref_w]
        ref_peak = max(np.abs(w).max() for w in ref_w)
        assert float(z["peak"]) == ref_peak
        # single-process Synthesizer.tts join: sentences + 10 000 zeros, one global peak
        y = np.concatenate([np.concatenate([w, np.zeros(10000)]) for w in ref_w])
        ref_pcm = (y * (32767 / max(0.01, np.max(np.abs(y))))).astype(np.int16)
        np.testing.assert_array_equal(z["pcm"], ref_pcm)
