"""Stream sharding over the GPUs of one node.

Utterance streams are independent: stream g runs on rank g // streams_per_rank, weights are
replicated, the AR/codec math needs no exchange. The path's only exchange — the text plans
coming from the LLM host rank and the PCM going back to it — is one scatter and one gather
over torch.distributed (RCCL over xGMI on MI355X; gloo in the CPU tests).
"""
from __future__ import annotations

import time
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


def gather_pcm(pcm: torch.Tensor, dist=None, rank: int = 0, world: int = 1, async_op: bool = False):
    """Every rank's [S, samples] float32 PCM to rank 0 (None elsewhere). async_op: returns (outputs,
    work) with the collective in flight (work None when the backend ran it synchronously)."""
    if dist is None:
        return ([pcm], None) if async_op else [pcm]
    out = [torch.empty_like(pcm) for _ in range(world)] if rank == 0 else None
    if not async_op:
        dist.gather(pcm, out, dst=0)
        return out
    work = dist.gather(pcm, out, dst=0, async_op=True) if getattr(dist, "supports_async", True) else \
        dist.gather(pcm, out, dst=0)
    return out, work


class ChunkGather:
    """The PCM gather of the overlapped multi-GPU schedule (bench.run_chunks at N > 1; reference: the
    replicas' PCM reaching the client, streaming_server.py:357-376,428-469). A chunk's PCM is gathered
    to rank 0 only once the host has seen its codec event (``issue``), on a stream of its own (``stream``:
    neither the decode stream nor the codec stream ever waits on the collective, and no queue parks on
    another queue's event), asynchronously; ``wait(key)`` (host-side completion poll) runs before the
    chunk's PCM buffer is written again. ``keep``: rank 0 keeps every gathered chunk (tests)."""

    def __init__(self, dist, rank: int, world: int, stream=None, keep: bool = False):
        self.dist, self.rank, self.world, self.stream = dist, rank, world, stream
        self.work = {}
        self.seq = 0
        self.keep = keep
        self.gathered: List[List[torch.Tensor]] = []

    def issue(self, key, pcm: torch.Tensor):
        self.wait(key)
        if self.stream is not None:
            with torch.cuda.stream(self.stream):
                out, work = gather_pcm(pcm, self.dist, self.rank, self.world, async_op=True)
        else:
            out, work = gather_pcm(pcm, self.dist, self.rank, self.world, async_op=True)
        self.seq += 1
        self.work[key] = (work, out, self.seq)

    def wait(self, key):
        w = self.work.pop(key, None)
        if w is None:
            return
        work, out, _ = w
        if work is not None:
            while not work.is_completed():  # host poll: nothing is enqueued on any stream
                time.sleep(20e-6)
        if self.keep and out is not None:
            self.gathered.append([o.detach().cpu() for o in out])

    def drain(self):
        for key in sorted(self.work, key=lambda k: self.work[k][2]):  # in issue order
            self.wait(key)


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
