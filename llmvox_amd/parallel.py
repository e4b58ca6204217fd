"""Stream sharding over the GPUs of one node.

Utterance streams are independent: stream g runs on rank g // streams_per_rank, weights are
replicated, the AR/codec math needs no exchange. The path's only exchange — the text plans
coming from the LLM host rank and the PCM going back to it — is one scatter and one gather
over torch.distributed (RCCL over xGMI on MI355X; gloo in the CPU tests).
"""
from __future__ import annotations

from typing import List, Optional

import torch


def shard_of(stream: int, streams_per_rank: int) -> int:
    return stream // streams_per_rank


def scatter_plans(full: Optional[torch.Tensor], streams_per_rank: int, n_pos: int, device, dist=None,
                  rank: int = 0) -> torch.Tensor:
    """Rank 0 holds the [world*S, n_pos] int32 text-id plans; every rank receives its [S, n_pos]."""
    if dist is None:
        return full[:streams_per_rank].contiguous().to(device)
    mine = torch.empty(streams_per_rank, n_pos, dtype=torch.int32, device=device)
    chunks = list(full.to(device).split(streams_per_rank)) if rank == 0 else None
    dist.scatter(mine, chunks, src=0)
    return mine


def gather_pcm(pcm: torch.Tensor, dist=None, rank: int = 0, world: int = 1) -> Optional[List[torch.Tensor]]:
    """Every rank's [S, samples] float32 PCM to rank 0 (None elsewhere)."""
    if dist is None:
        return [pcm]
    out = [torch.empty_like(pcm) for _ in range(world)] if rank == 0 else None
    dist.gather(pcm, out, dst=0)
    return out


def scatter_texts(texts: Optional[List[str]], streams_per_rank: int, device, dist=None, rank: int = 0,
                  world: int = 1) -> List[str]:
    """Rank 0 holds the world*S request texts (the LLM host side); every rank receives its S. The
    text travels as UTF-8 code units in an int32 tensor (RCCL moves device tensors): the longest
    length is broadcast first, then one scatter of [S, 1 + longest] (length in column 0)."""
    if dist is None:
        return list(texts[:streams_per_rank])
    S = streams_per_rank
    enc = [t.encode("utf-8") for t in texts] if rank == 0 else None
    meta = torch.tensor([max(len(e) for e in enc) if rank == 0 else 0], dtype=torch.int64, device=device)
    dist.broadcast(meta, src=0)
    L = int(meta.item())
    mine = torch.zeros(S, L + 1, dtype=torch.int32, device=device)
    chunks = None
    if rank == 0:
        full = torch.zeros(world * S, L + 1, dtype=torch.int32)
        for i, e in enumerate(enc):
            full[i, 0] = len(e)
            if e:
                full[i, 1:1 + len(e)] = torch.tensor(list(e), dtype=torch.int32)
        chunks = list(full.to(device).split(S))
    dist.scatter(mine, chunks, src=0)
    h = mine.cpu()
    return [bytes(h[i, 1:1 + int(h[i, 0])].to(torch.uint8).tolist()).decode("utf-8") for i in range(S)]


def gather_bytes(items: List[bytes], device, dist=None, rank: int = 0, world: int = 1) -> Optional[List[List[bytes]]]:
    """Every rank's per-stream byte strings (the f32le PCM of its streams, variable length) to rank 0,
    as [rank][stream] (None elsewhere): the sizes first (one int64 per stream), then each rank's
    concatenation padded to the longest one (its length from an all-reduce MAX), one gather."""
    if dist is None:
        return [list(items)]
    sizes = torch.tensor([len(x) for x in items], dtype=torch.int64, device=device)
    all_sizes = [torch.empty_like(sizes) for _ in range(world)] if rank == 0 else None
    dist.gather(sizes, all_sizes, dst=0)
    payload = b"".join(items)
    tot = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    dist.all_reduce(tot, op=dist.ReduceOp.MAX)
    n = (int(tot.item()) + 3) // 4  # whole int32 words
    buf = torch.zeros(max(n, 1), dtype=torch.int32)
    if payload:
        buf.view(torch.uint8)[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
    buf = buf.to(device)
    outs = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, outs, dst=0)
    if rank != 0:
        return None
    res = []
    for r in range(world):
        raw = outs[r].cpu().view(torch.uint8).numpy().tobytes()
        off, lst = 0, []
        for z in all_sizes[r].cpu().tolist():
            lst.append(raw[off:off + z])
            off += z
        res.append(lst)
    return res
