"""Sentence sharding across GPUs: one process per GPU, sentences are independent.

The reference synthesises a request's sentences one after another in one process
(server/synthesizer.py:128-161).  Here a request's sentences are dealt to ranks by
longest-processing-time (LPT) greedy on their decoder cost, every rank synthesises its share as
one batch with no data-path collective, and only the finished waveforms travel: an all_gather of
per-sentence sample counts, then a gather-v of the float64 samples to rank 0 (point-to-point
send/recv, so over xGMI every peer uses its own link), and an all_reduce(MAX) of |y| for the global
int16 peak normalisation of save_wav (utils/audio.py:56-58).

Device-agnostic: the same code runs over RCCL on MI355X and over gloo on CPU (tests).
"""
from __future__ import annotations

import heapq
import math

import numpy as np
import torch
import torch.distributed as dist

SENTENCE_GAP = 10000  # zeros between sentences (server/synthesizer.py:158)


def sentence_cost(L: int, max_steps: int, forward_attn_mask: bool = True) -> int:
    """Cost model for the partition: decoder steps ~ 2L+22 under the forward-attention mask (the
    alignment advances about one id per two frames before the stop rule fires,
    layers/tacotron2.py:256-277), otherwise the max_steps cap (+20)."""
    return min(2 * L + 22, max_steps) if forward_attn_mask else max_steps + 20


def lpt_partition(costs, world: int, capacity: int | None = None):
    """Longest-processing-time greedy: sentences sorted by cost (descending, index ascending on
    ties) go to the rank with the least load so far (lowest rank on ties); a rank holding
    ``capacity`` sentences takes no more.  Returns per-rank index lists, each in ascending order."""
    n = len(costs)
    if capacity is None:
        capacity = math.ceil(n / world) if n else 0
    if capacity * world < n:
        raise ValueError(f"{n} sentences do not fit {world} ranks x capacity {capacity}")
    order = sorted(range(n), key=lambda i: (-costs[i], i))
    heap = [(0, r) for r in range(world)]
    parts = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        while len(parts[r]) >= capacity:  # full ranks leave the heap for good
            load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + costs[i], r))
    return [sorted(p) for p in parts]


def gather_waveforms(wavs, indices, n_total: int, group=None, dst: int = 0):
    """Gather-v of variable-length 1-D waveforms to ``dst``.

    wavs: this rank's waveforms (1-D tensors on the communication device), indices: their global
    sentence indices.  Returns the list of all n_total waveforms in global order on ``dst``
    (tensors on the same device) and None elsewhere.  Collectives: one all_gather of int64
    [count, total samples] headers, one all_gather of the per-sentence (index, length) table,
    then one send per non-empty rank into dst."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = wavs[0].device if len(wavs) else torch.device("cpu")
    if not len(wavs):
        dev = _comm_device(group)
    cnt = torch.tensor([len(wavs), sum(int(w.numel()) for w in wavs)], dtype=torch.int64, device=dev)
    hdr = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(hdr, cnt, group=group)
    counts = [int(h[0]) for h in hdr]
    cmax = max(counts) if counts else 0
    rows = [[int(i), int(w.numel())] for i, w in zip(indices, wavs)]
    rows += [[-1, -1]] * (max(cmax, 1) - len(rows))
    table = torch.tensor(rows, dtype=torch.int64).to(dev)
    tables = [torch.empty_like(table) for _ in range(world)]
    dist.all_gather(tables, table, group=group)
    dtype = wavs[0].dtype if len(wavs) else torch.float64
    if rank != dst:
        if len(wavs):
            op = dist.P2POp(dist.isend, torch.cat([w.reshape(-1) for w in wavs]), _global(dst, group), group)
            for req in dist.batch_isend_irecv([op]):
                req.wait()
        return None
    # every peer's receive is posted at once (one group: over xGMI each peer streams on its own
    # link concurrently), then waited on together
    bufs = {}
    ops = []
    for r in range(world):
        if r != rank and counts[r] > 0:
            bufs[r] = torch.empty(int(hdr[r][1]), dtype=dtype, device=dev)
            ops.append(dist.P2POp(dist.irecv, bufs[r], _global(r, group), group))
    for req in (dist.batch_isend_irecv(ops) if ops else []):
        req.wait()
    out = [None] * n_total
    for r in range(world):
        tab = tables[r][:counts[r]].cpu().tolist()
        if r == rank:
            buf = torch.cat([w.reshape(-1) for w in wavs]) if len(wavs) else torch.empty(0, dtype=dtype, device=dev)
        else:
            if counts[r] == 0:
                continue
            buf = bufs[r]
        off = 0
        for i, n in tab:
            out[i] = buf[off:off + n]
            off += n
    missing = [i for i, w in enumerate(out) if w is None]
    if missing:
        raise RuntimeError(f"gather_waveforms: sentences {missing[:8]} were not produced by any rank")
    return out


def global_peak(wavs, group=None) -> float:
    """max |y| over every rank's sentences (all_reduce MAX of one scalar)."""
    dev = wavs[0].device if len(wavs) else _comm_device(group)
    m = torch.zeros(1, dtype=torch.float64, device=dev)
    for w in wavs:
        if w.numel():
            m = torch.maximum(m, w.abs().max().to(torch.float64).reshape(1))
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    return float(m.item())


def join_int16(wavs, peak: float | None = None) -> np.ndarray:
    """Synthesizer.tts's output (server/synthesizer.py:157-161 + save_wav): sentences in order, each
    followed by 10 000 zeros, peak-normalised to int16 over the whole request."""
    parts = []
    for w in wavs:
        parts.append(np.asarray(w.cpu().numpy() if torch.is_tensor(w) else w, dtype=np.float64))
        parts.append(np.zeros(SENTENCE_GAP))
    y = np.concatenate(parts) if parts else np.zeros(0)
    if peak is None:
        peak = float(np.max(np.abs(y))) if y.size else 0.0
    return (y * (32767 / max(0.01, peak))).astype(np.int16)


def synthesize_sharded(model, ap, ids_list, group=None, seed=0, max_batch=None):
    """Synthesizer.tts over all ranks: LPT shard, local batched synthesis, gather-v to rank 0.

    Returns (int16 waveform with 10 000-sample gaps on rank 0 / None elsewhere, info); on rank 0
    ``info["wavs"]`` holds every sentence's float64 waveform (device tensors, global order).
    Initial Griffin-Lim phases come from the device generator seeded with ``seed + rank``, sentence
    b of the rank's batch (its ``partition`` list, ascending) at generator row b."""
    from .synthesis import synthesize_batch

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mask = bool(getattr(model, "flags", {}).get("forward_attn_mask", True))
    costs = [sentence_cost(len(x), model.decoder.max_decoder_steps, mask) for x in ids_list]
    cap = max_batch or math.ceil(len(ids_list) / world)
    parts = lpt_partition(costs, world, cap)
    mine = parts[rank]
    wavs = []
    info = {"partition": parts, "frames": []}
    if mine:
        out, inf = synthesize_batch(model, ap, [ids_list[i] for i in mine], seed=seed + rank, phase="device",
                                    keep_outputs=True)
        wav_dev = inf["wav_dev"]
        wavs = [wav_dev[k, :n] for k, n in enumerate(inf["samples"])]
        info["frames"] = inf["frames"]
        info["gl_iterations"] = inf["gl_iterations"]
        info["mel_post"] = inf["mel_post"]  # this rank's batch, padded [B, Tmax, 80] (batch order = partition)
    peak = global_peak(wavs, group)
    allw = gather_waveforms(wavs, mine, len(ids_list), group)
    if rank != 0:
        return None, info
    info["wavs"] = allw
    return join_int16(allw, peak), info


def _comm_device(group):
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _global(r, group):
    return r if group is None else dist.get_global_rank(group, r)
