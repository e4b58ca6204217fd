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
