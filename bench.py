#!/usr/bin/env python3
"""LLMVoX streaming-TTS hot path on MI355X — the driver's benchmark.

Default workload (BASELINE.json configs[2], the largest single-GPU configuration): "30M LLMVoX
bf16, 1xMI355X, 32 concurrent streams batched decode + vocoder". One bench STEP = one 256-token
chunk of 32 utterance streams: 256 batched greedy AR decode steps of the speech-token GPT (B = 32
rows per step) + the WavTokenizer decode of the 32 x 256 codes (one batched codec call, 2,621,440
PCM samples at 24 kHz) + the PCM copy to the host. Each stream speaks utterances of --utterance
1024 tokens (N = 1024 per stream): four consecutive steps continue one utterance
(KV positions 0..1023), then the stream starts its next utterance (a new sentence, its KV slot
reset, as the reference resets it at every end of audio, streaming_server.py:406-417);
--utterance 0 keeps one utterance per stream for the whole run. Synthetic input: stream 0's first
utterance is the config's 64-char sentence, every other one a seeded random 64-char sentence
(ByT5 ids, then PAD); seeded synthetic weights at the reference init
scales (no checkpoints offline). p50 first-chunk latency is measured separately on one stream of
the same engine through the service scheduler (FusedScheduler), from the first text word enqueued
to the first 3,200-sample (10-token) dump as bytes on the host.

Multi-GPU: ``--gpus N`` runs one process per GPU. Under torch.distributed.run (WORLD_SIZE set, it
must equal N) each rank is one such process; without it bench.py spawns the N ranks itself (before
any GPU call) on 127.0.0.1. Each rank runs its own streams (independent utterance streams: weak
scaling); rank 0 scatters the text-id plans and gathers the PCM over RCCL (the path's only
exchange, BASELINE north_star).

--config selects the other BASELINE.json workloads (per GPU; weak scaling over --gpus):
  1  1 stream, 256-token chunks (configs[1])
  2  32 streams batched, 256-token chunks (configs[2], default)
  3  the service path: FusedScheduler replica streams (replica index = stream % 2, initial dump
     10 / 160, x3 growth to 1280) over one utterance of --utt-tokens 2048 per step; every dump is
     decoded as its own codec call and delivered as f32le bytes on the host (configs[3])
  4  8 streams, fp8 (e4m3fn) KV cache + fp8 codec weights, KV reset every --reset-every chunks
     (a new sentence), 256-token chunks (configs[4])

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SENTENCE = "The quick brown fox jumps over the lazy dog near the river bank."
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (8.0 TB/s spec)


def sentence_ids(text):
    from llmvox_amd.tokenizer import ByteTokenizer
    tok = ByteTokenizer()
    ids = []
    for w in text.split(" "):
        t = tok(w.strip())["input_ids"]
        if w.endswith("."):
            t = t + [385]
        ids += t
    return ids


def random_sentence(rng):
    letters = "abcdefghijklmnopqrstuvwxyz "
    s = "".join(rng.choice(list(letters), size=63))
    s = " ".join(w for w in s.split(" ") if w) or "a"
    return (s[:63]).strip() + "."


def plan_for(ids, start, n, pad=384):
    out = np.full(n, pad, dtype=np.int32)
    seg = ids[start:start + n]
    out[:len(seg)] = seg
    return out


# ---------------------------------------------------------------------------------------
def attn_splits(B, wbytes):
    """KV splits per (row, head) of the decode attention at this B (ar_kernels.hip launch_op /
    attn_ns_max): 16 on the B <= 2 GEMV path; bf16 weights at B >= 5: one (round 3); otherwise
    (bf16 at 3 <= B <= 4, the fp32 batched path at 3 <= B <= 64) halved until splits x 8 heads x B
    <= 256 blocks. One split: the attention writes the normalised operand rows itself and no split
    partials exist."""
    if B < 3 or B > 64:
        return 16
    if wbytes == 2 and B >= 5:  # (5 <= B <= 8: one split of 8-wave blocks)
        return 1
    ns = 16
    while ns > 1 and ns * 8 * B > 256:
        ns //= 2
    return ns


def kernel_bytes(which, B, t, wbytes, kvbytes):
    """Algorithmic HBM bytes of one launch of op `which` (weights streamed once + KV + the
    activations it must read and write), as the batched path at this B moves them. Split-KV partials
    (8 heads x ns x (96 + 2) fp32 per row) are charged only when the attention runs more than one
    split (attn_splits)."""
    D, F, V = 768, 3072, 4096
    act = 4 * B
    mfma = wbytes == 2 and 3 <= B <= 64
    ns = attn_splits(B, wbytes)
    parts = act * 8 * ns * 98 if ns > 1 else 0           # split-KV partials written / read once
    rows_bf16 = 2 * D * B                                  # one bf16 operand row set
    # the batched path's LayerNorm ahead of c_attn (layers >= 1) and lm_head folds the previous mlp
    # c_proj's four K-slice partials into x: x and the four partial rows read, x written back and the
    # bf16 operand rows written (ar_rows_kernel<4>, part of those probes); at B <= 8 the GEMM
    # prologue reads x and the partials itself (nothing written)
    fold = (6 * act * D + rows_bf16 if B > 8 else 5 * act * D) if mfma else 0
    if which == 0:
        return 3 * D * D * wbytes + (rows_bf16 if mfma else act * D) + act * D + 2 * D * kvbytes * B + fold
    if which == 1:
        kv = 2 * t * D * kvbytes * B
        return kv + act * D + (rows_bf16 if (mfma and ns == 1) else parts)
    if which == 2:  # (+ the merge kernel when ns > 1) x read + written, bf16 copy for c_fc
        merge = (parts + 2 * rows_bf16) if (mfma and ns > 1) else parts
        return D * D * wbytes + (rows_bf16 if (mfma and ns == 1) else merge) + 2 * act * D + \
            (rows_bf16 if mfma else 0)
    if which == 3:
        return F * D * wbytes + ((rows_bf16 + 2 * F * B) if mfma else act * (D + F))
    if which == 4:  # mfma: four K-slice partials (fp32) out
        return D * F * wbytes + ((2 * F * B + 4 * act * D) if mfma else act * (F + 2 * D))
    if which == 5:
        return V * D * wbytes + ((rows_bf16 if mfma else act * D) + act * V) + fold
    raise ValueError(which)


def step_bytes(B, t, wbytes, kvbytes):
    """Algorithmic HBM bytes of one whole decode step of B rows at KV position t:
    every GEMM weight once (62.9 MB bf16) + the K/V history of 4 layers read + the new key / value
    written, per row."""
    D, F, V, L = 768, 3072, 4096, 4
    weights = (L * (3 * D * D + D * D + 2 * F * D) + V * D) * wbytes
    return weights + L * B * (2 * t * D * kvbytes + 2 * D * kvbytes)


KNAMES = {0: "ar_gemv c_attn", 1: "ar_attn (split-KV decode)", 2: "ar_gemv c_proj(+merge)",
          3: "ar_gemv c_fc(+gelu)", 4: "ar_gemv mlp.c_proj", 5: "ar_gemv lm_head"}
KCALLS = {0: 4, 1: 4, 2: 4, 3: 4, 4: 4, 5: 1}


def pmc_key(dtype, kv_dtype, B, pos):
    """Key of a probe workload in profiles/pmc_traffic.json (tools/pmc_traffic.py KEY argument):
    weight dtype, KV dtype, batch rows and the KV position the probe ran at."""
    return f"{dtype}/kv{kv_dtype}/B{B}/P{pos}"


def pmc_traffic(key, kernel):
    """HBM bytes per launch of a probed kernel from the committed PMC passes over the SAME probe
    workload (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), or None when no pass
    was collected at this key: traffic is never paired with a different position or batch."""
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        return json.load(open(pmc)).get(f"{key}:{kernel}")
    except (OSError, ValueError):
        return None


def pmc_codec(key):
    """MFMA busy cycles / GRBM active cycles of the codec's large GEMM (gemm_glds_kernel, gemm_bf16_kernel) from a
    committed rocprofv3 pass over the same codec call (profiles/pmc_codec.json, tools/pmc_codec.py)."""
    pmc = os.path.join(ROOT, "profiles", "pmc_codec.json")
    try:
        return json.load(open(pmc)).get(key)
    except (OSError, ValueError):
        return None


def cpu_threads():
    """Threads for the CPU baseline: this process's physical cores — the CPUs it may run on
    (sched_getaffinity), one per physical core (SMT siblings dropped), capped by the cgroup CPU
    quota (a GPU box grants each GPU's jobs a share of the host, e.g. 16 CPUs)."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    cores = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                cores.add(f.read().strip().split(",")[0].split("-")[0])
        except OSError:
            cores.add(str(c))
    n, why = len(cores), f"{len(cores)} physical cores of {len(cpus)} CPUs in the affinity mask"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
            if quota < n:
                n, why = quota, why + f", cgroup CPU quota {quota}"
    except (OSError, ValueError):
        pass
    return n, why


def probe_kernels(eng, slots, t, wbytes, kvbytes, iters=200, rounds=3):
    """Average launch time of each op's kernel(s) at KV position t, HIP events on the stream the
    kernels run on. The library replays each op's `iters` launches as one HIP graph, as the
    decode step is replayed (launched one by one from the host, 3-5 us kernels measured the
    host's launch rate too: the same kernel read 3.3-5.8 us from box to box). One untimed pass
    captures the graphs and warms clocks and caches; the lowest of `rounds` timed passes is kept.
    An op fused into the previous one (mlp c_proj inside the fused MLP at small B) has no kernel
    of its own: its bytes are charged to the fused kernel."""
    from llmvox_amd._lib import LvxError
    for k in KNAMES:
        try:
            eng.probe_kernel(k, slots, iters)
        except LvxError as e:
            if e.code != -2:
                raise
    best = None
    for _ in range(rounds):
        r = _probe_pass(eng, slots, t, wbytes, kvbytes, iters)
        if best is None:
            best = r
        else:
            for k, v in r.items():
                if v["avg_us"] < best[k]["avg_us"]:
                    best[k] = v
    return best


def _probe_pass(eng, slots, t, wbytes, kvbytes, iters):
    from llmvox_amd._lib import LvxError
    res = {}
    s = torch.cuda.current_stream(eng.device)
    B = slots.numel()
    for k in KNAMES:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        try:
            eng.probe_kernel(k, slots, iters)
        except LvxError as e:
            if e.code != -2:  # LVX_E_STATE: fused into the previous op at this B
                raise
            res[k - 1]["name"] = "ar_mlp fused (c_fc+gelu+c_proj)"
            res[k - 1]["bytes"] += kernel_bytes(k, B, t, wbytes, kvbytes)
            res[k - 1]["gbs"] = res[k - 1]["bytes"] / (res[k - 1]["avg_us"] * 1e-6) / 1e9
            continue
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        by = kernel_bytes(k, B, t, wbytes, kvbytes)
        res[k] = {"name": KNAMES[k], "avg_us": us, "bytes": by, "gbs": by / (us * 1e-6) / 1e9,
                  "share_us_per_step": us * KCALLS[k]}
    return res


# ---------------------------------------------------------------------------------------
def dump_schedule(n_tokens, first, max_dump=1280):
    """The reference's dump sizes (streaming_server.py:357-422): first, x3 growth capped at
    max_dump, the remainder flushed at the end of the utterance."""
    out, ds, left = [], first, n_tokens
    while left > 0:
        out.append(min(ds, left))
        left -= out[-1]
        ds = min(ds * 3, max_dump)
    return out


def cpu_baseline(n_chunks, chunk, min_seconds=10.0, max_seconds=30.0, schedule=None):
    """The reference CPU eager path (oracle restatement: fp32, B=1, O(t) history/KV cats),
    on this host's cores, on the same chunked workload; whole utterances are repeated until
    at least ``min_seconds`` of CPU work is timed (bounded by ``max_seconds``)."""
    from llmvox_amd import weights as LW
    from oracle import reference_cpu as R
    threads, why = cpu_threads()
    torch.set_num_threads(threads)
    gw, cw, tt = LW.synthetic_all(1234)
    W, Wc = R.to_torch(gw), R.to_torch(cw)
    table = torch.from_numpy(tt)
    cb = Wc[R.CODEBOOK_KEY]
    ids = sentence_ids(SENTENCE)
    schedule = schedule or [chunk] * n_chunks
    starts = np.concatenate([[0], np.cumsum(schedule)]).astype(int).tolist()
    t0 = time.perf_counter()
    done, passes = 0, 0
    rates = []  # tokens/s of each whole pass (utterance)
    with torch.inference_mode():
        while time.perf_counter() - t0 < min_seconds:
            hist, kv, prev = None, None, None
            passes += 1
            tp, dp = time.perf_counter(), done
            for c in range(len(schedule)):
                toks = []
                for i in range(starts[c], starts[c + 1]):
                    tid = ids[i] if i < len(ids) else 384
                    te = table[tid].view(1, 1, -1)
                    se = torch.zeros(1, 1, 512) if i == 0 else cb[prev].view(1, 1, -1)
                    x = R.build_input(te, se)
                    hist = x if hist is None else torch.cat([hist, x], dim=1)
                    logits, kv = R.gpt_forward(W, hist, kv)
                    prev = R.greedy_token(logits)
                    toks.append(prev)
                pcm = R.decode_codes(Wc, torch.tensor([toks]))
                _ = pcm.numpy().astype("float32").tobytes()
                done += len(toks)
                if time.perf_counter() - t0 > max_seconds:
                    break
            else:
                rates.append((done - dp) / (time.perf_counter() - tp))
            if time.perf_counter() - t0 > max_seconds:
                break
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": done / dt, "unit": "speech tokens/s", "cores": threads, "kind": "port",
            "passes": passes, "pass_min": round(min(rates), 1) if rates else None,
            "pass_max": round(max(rates), 1) if rates else None,
            "sample": f"{done} tokens: fp32 AR steps + one codec decode per dump of {schedule[:8]} tokens, "
                      f"over {passes} utterance(s) of {sum(schedule)} positions, 1 stream, oracle/reference_cpu.py, "
                      f"{dt:.1f} s on {cpu}, torch threads {threads} ({why})"}


class _HostCollectives:
    """torch.distributed facade for the gloo rehearsal: device tensors go through host copies
    (synchronously: no async_op)."""
    supports_async = False

    def __init__(self, d):
        self.d = d
        self.ReduceOp = d.ReduceOp

    def __getattr__(self, k):
        return getattr(self.d, k)

    def _host(self, t):
        return None if t is None else t.cpu()

    def scatter(self, out, chunks, src=0):
        o = out.cpu()
        self.d.scatter(o, [c.cpu() for c in chunks] if chunks is not None else None, src=src)
        out.copy_(o)

    def gather(self, t, out, dst=0):
        o = [x.cpu() for x in out] if out is not None else None
        self.d.gather(t.cpu(), o, dst=dst)
        if out is not None:
            for x, y in zip(out, o):
                x.copy_(y)

    def all_reduce(self, t, op=None):
        h = t.cpu()
        self.d.all_reduce(h, op=op)
        t.copy_(h)

    def broadcast(self, t, src=0):
        h = t.cpu()
        self.d.broadcast(h, src=src)
        t.copy_(h)


# ---------------------------------------------------------------------------------------
def run_config3(args, eng, world, rank, local, dist):
    """configs[3]: the service path. Every GPU runs --streams replica streams through
    FusedScheduler (streaming.py: the reference's audio_generator_sync semantics, continuous
    batching, one HIP-graph replay per decode step, one codec call per dump, f32le bytes on the
    host). Stream g uses replica index g % 2 (initial dump 10 / 160, x3 to 1280,
    streaming_server.py:357-422). One step = one utterance of --utt-tokens tokens per stream; the
    utterance's tail below the dump size is flushed (the reference flushes it at end-of-audio)."""
    from llmvox_amd.parallel import gather_bytes, scatter_texts
    from llmvox_amd.streaming import FusedScheduler
    dev = eng.device
    S, N, K, Wm = args.streams, args.utt_tokens, args.steps, args.warmup
    # the service's schedule (round 5): chunk c + 1's decode queued before chunk c is
    # read back, chunk c's codec on a second stream, each dump delivered when its codec call ends
    # (round 4's overlap delivered a chunk late: p50 first chunk 3.9-4.0 vs 1.33-1.36 ms);
    # --serial-codec: the serial scheduler
    so = dict(kv.split("=") for kv in filter(None, args.sched.split(",")))
    sched = FusedScheduler(eng, max_chunk=int(so.get("mc", 256)), to_bytes=True, overlap=args.codec_overlap,
                           tail=int(so.get("tail", 8)), codec_stream=so.get("cs", "1") != "0")
    rng = np.random.default_rng(1234)  # rank 0 draws every rank's request texts
    pcm_bytes = [0]

    class FirstBytes:  # a stream's sink: when its first PCM bytes were delivered
        t = None

        def put(self, item):
            if self.t is None and isinstance(item, bytes):
                self.t = time.perf_counter()

    def utterance():
        streams = []
        t0 = time.perf_counter()  # first text word enqueued (p50 first-chunk latency starts here)
        # the path's inbound exchange: rank 0 (the LLM host side) scatters the world*S request texts
        texts = ([SENTENCE if g == 0 else random_sentence(rng) for g in range(world * S)] if rank == 0 else None)
        mine = scatter_texts(texts, S, dev, dist, rank, world)
        for s in range(S):
            g = rank * S + s
            st = sched.open_stream(index=g % 2, dump_size=10 if g % 2 == 0 else 160, sink=FirstBytes())
            for w in mine[s].split(" "):
                st.feed(w)
            streams.append(st)
        while min(len(st.tokens) for st in streams) < N:
            if sched.run_chunk() == 0:
                raise RuntimeError("scheduler went idle before the utterance ended")
        sched.flush()
        first = (min(st.sink.t for st in streams if st.sink.t is not None) - t0) * 1e3
        tails = {}  # the tail below the current dump size: flushed as one last dump (end of audio)
        rest = [st for st in streams if st.m.speech_outputs]
        for L in sorted({len(st.m.speech_outputs) for st in rest}):
            grp = [st for st in rest if len(st.m.speech_outputs) == L]
            codes = torch.tensor([st.m.speech_outputs for st in grp], dtype=torch.int32, device=dev)
            for st, row in zip(grp, eng.decode_codes(codes).cpu().numpy()):
                tails[st] = row.astype("float32").tobytes()
                st.m.speech_outputs = []
        # the outbound exchange: every stream's f32le bytes (its dumps in order + the tail) to rank 0
        out = [b"".join(x for x in st.events if isinstance(x, bytes)) + tails.get(st, b"") for st in streams]
        got = gather_bytes(out, dev, dist, rank, world)
        if rank == 0:
            pcm_bytes[0] += sum(len(x) for r in got for x in r)
        n_tok = sum(len(st.tokens) for st in streams)
        for st in streams:
            sched.close_stream(st)
        return n_tok, first

    for _ in range(Wm):
        utterance()
    pcm_bytes[0] = 0
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    toks, firsts = 0, []
    for _ in range(K):
        n, f = utterance()
        toks += n
        firsts.append(f)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    eng.check_errors()
    if dist is not None:
        t_dt = torch.tensor([dt], dtype=torch.float64, device=dev)
        t_tok = torch.tensor([toks], dtype=torch.float64, device=dev)
        dist.all_reduce(t_dt, op=dist.ReduceOp.MAX)
        dist.all_reduce(t_tok, op=dist.ReduceOp.SUM)
        dt, toks = float(t_dt.item()), int(t_tok.item())
    value = toks / dt
    sched.close()

    kern, rl = None, None
    if not args.no_probe:
        slots = torch.arange(S, dtype=torch.int32, device=dev)
        for s in range(S):
            eng.set_slot(s, N - 1, 0)
        wb = 2 if args.dtype == "bf16" else 4
        kb = {"bf16": 2, "fp8": 1, "fp32": 4}[args.kv_dtype or args.dtype]
        kern = probe_kernels(eng, slots, N, wb, kb)
        dom = max(kern.values(), key=lambda r: r["share_us_per_step"])
        rl = {"bound": "hbm", "kernel": dom["name"], "achieved": round(dom["gbs"], 1), "peak": HBM_PEAK_GBS,
              "unit": "GB/s", "frac": round(dom["gbs"] / HBM_PEAK_GBS, 4), "traffic": None,
              "bytes_per_launch": dom["bytes"], "avg_us": round(dom["avg_us"], 3), "kv_positions": N}
        rl["pmc_key"] = pmc_key(args.dtype, args.kv_dtype or args.dtype, S, N)
        rl["traffic"] = pmc_traffic(rl["pmc_key"], dom["name"])
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the CPU baseline: N = 1 runs only
        cpu = cpu_baseline(0, 0, schedule=dump_schedule(N, 10))
    if rank == 0:
        out = {
            "metric": "speech tokens/sec (+ 24kHz audio samples/sec = 320 x tokens/s; p50 first-chunk latency)",
            "value": round(value, 1), "unit": "speech tokens/s", "n_gpus": world, "steps": K, "warmup": Wm,
            "ms_per_step": round(dt / K * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (config sentence + seeded random sentences -> ByT5 ids, seeded synthetic weights)",
            "config": {"workload": f"configs[3]: FusedScheduler service path, {S} replica stream(s)/GPU "
                                   f"(initial dump 10/160, x3 to 1280), {N} tokens per utterance, "
                                   "one codec call per dump, f32le bytes on the host",
                       "codec_schedule": ("FusedScheduler overlap: chunk c + 1's decode queued before chunk c is "
                                          "read back, chunk c's codec on a second stream, each dump delivered when "
                                          "its codec ends" if args.codec_overlap else "serial FusedScheduler"),
                       "streams_per_gpu": S, "utterance_tokens": N, "dump_schedule_replica0": dump_schedule(N, 10),
                       "dump_schedule_replica1": dump_schedule(N, 160),
                       "parallelism": (f"streams sharded over {world} GPU(s); rank 0 scatters the request texts and "
                                       f"gathers every stream's PCM bytes (sizes first) over {dist.get_backend()}"
                                       if dist is not None else "one GPU, no process group (no collective runs)")},
            "pcm_bytes_gathered_rank0": pcm_bytes[0],
            "audio_samples_per_s": round(320 * value, 1),
            "realtime_factor_per_stream": round(value / (world * S) / 75.0, 1),
            "p50_first_chunk_latency_ms": round(statistics.median(firsts), 3),
            "dist": ({"backend": dist.get_backend(), "world_size": dist.get_world_size()} if dist is not None
                     else {"backend": None, "world_size": 1}),
            "roofline": rl, "kv_dtype": args.kv_dtype or args.dtype,
            "codec_weights": args.codec_dtype or args.dtype, "cpu_baseline": cpu,
            "kernels": {v["name"]: {"avg_us": round(v["avg_us"], 2), "GB/s": round(v["gbs"], 1)}
                        for v in kern.values()} if kern else None,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


# ---------------------------------------------------------------------------------------
def spawn_ranks(n):
    """--gpus N without torch.distributed.run: one child process per GPU (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR 127.0.0.1 / a free MASTER_PORT), started before this process has
    touched the GPU. Returns the first failing rank's exit code (the others are then terminated),
    else 0."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in procs:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def rehearse(args, world, rank):
    """--rehearse: the multi-rank skeleton of the bench on the CPU (gloo, no GPU): plan scatter from
    rank 0, the PCM gather to rank 0, barriers and the max-over-ranks clock. Used by
    tests/test_bench_launcher.py for the launcher path. The gather runs both ways the bench runs it:
    once per chunk after a stand-in 'decode' (the serial schedule), and paced as in the overlapped
    schedule (run_chunks at N > 1: ChunkGather.issue once the chunk's 'codec' is done, asynchronously,
    two PCM buffers, ChunkGather.wait before a buffer is written again); rank 0 checks that both give
    every rank's chunks exactly as a single rank would compute them."""
    import torch.distributed as dist
    from llmvox_amd.parallel import ChunkGather, gather_pcm, scatter_plans
    dist.init_process_group("gloo")
    S, n_pos = args.streams, args.chunk
    K = 5
    plans = None
    if rank == 0:
        rng = np.random.default_rng(1234)
        plans = torch.from_numpy(np.stack([plan_for(sentence_ids(SENTENCE if g == 0 else random_sentence(rng)), 0, n_pos)
                                           for g in range(world * S)]))
    dist.barrier()
    t0 = time.perf_counter()
    mine = scatter_plans(plans, S, n_pos, "cpu", dist, rank)

    def decode(c):  # stand-in codec output of chunk c: a function of this rank's plans and c
        return (mine.float() * (c + 1) + c).repeat_interleave(4, dim=1)

    serial = [gather_pcm(decode(c), dist, rank, world) for c in range(K)]
    gather = ChunkGather(dist, rank, world, keep=True)
    bufs = [None, None]
    for c in range(K):  # the overlapped schedule's order: issue c - 1 after c's 'codec' was queued
        i = c & 1
        gather.wait(i)           # the buffer's previous gather has read it
        bufs[i] = decode(c)      # chunk c's 'codec' into buffer i
        if c >= 1:
            gather.issue((c - 1) & 1, bufs[(c - 1) & 1])
    gather.issue((K - 1) & 1, bufs[(K - 1) & 1])
    gather.drain()
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    if rank == 0:
        full = plans.float()
        expect = [(full * (c + 1) + c).repeat_interleave(4, dim=1) for c in range(K)]
        ok = all(torch.equal(torch.cat(serial[c]), expect[c]) for c in range(K))
        ok_paced = len(gather.gathered) == K and all(torch.equal(torch.cat(gather.gathered[c]), expect[c])
                                                     for c in range(K))
        print(json.dumps({"rehearsal": True, "dist": {"backend": dist.get_backend(), "world_size": dist.get_world_size()},
                          "n_gpus": world, "streams_per_rank": S, "gathered_equals_scattered": bool(ok),
                          "paced_gather_equals_single_rank": bool(ok_paced), "chunks": K,
                          "max_over_ranks_s": float(dt.item())}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def first_chunk_latency(eng, reps=12, overlap=True):
    """p50 first-chunk latency: one fresh stream through the service scheduler
    (FusedScheduler: tokenisation, text-id plan upload, 10 fused decode steps, the codec call, PCM
    to the host as f32le bytes), timed from the moment the sentence's words are enqueued to the
    first 3,200-sample dump on the host; first two runs (graph capture, warm-up) dropped."""
    from llmvox_amd.streaming import FusedScheduler
    sched = FusedScheduler(eng, max_chunk=256, max_rows=1, overlap=overlap)
    lat = []

    class FirstBytes:  # the stream's sink: the moment its first PCM bytes are delivered (with the
        t = None       # overlap, by the delivery thread while the scheduler waits for the next chunk)

        def put(self, item):
            if self.t is None and isinstance(item, bytes):
                self.t = time.perf_counter()

    for r in range(reps):
        torch.cuda.synchronize()
        fb = FirstBytes()
        t0 = time.perf_counter()
        st = sched.open_stream(index=0, dump_size=10, sink=fb)
        for w in SENTENCE.split(" "):
            st.feed(w)
        while fb.t is None:
            if sched.run_chunk() == 0:
                raise RuntimeError("scheduler idle before the first dump")
        t1 = fb.t
        assert len(st.events[0]) == 3200 * 4
        sched.close_stream(st)
        sched.flush()
        if r >= 2:
            lat.append((t1 - t0) * 1e3)
    sched.close()
    return statistics.median(lat)


def first_chunk_latency_loaded(eng, busy=31, reps=34, max_chunk=32, seed=99, overlap=True):
    """p50 first-chunk latency UNDER LOAD (reference: a replica's first chunk is
    produced while the other replica decodes, streaming_server.py:357-376): a fresh stream joins a
    FusedScheduler that is already decoding `busy` streams (continuous batching, chunks of up to
    `max_chunk` steps, the service's default, llmvox_amd/server.py). A scheduler thread runs the
    chunks and admits queued requests between chunks, as a service loop does; the request is enqueued
    at a random moment of the chunk in flight. Timed from the enqueue of the sentence's words to its
    first 3,200-sample dump as f32le bytes on the host (the in-flight chunk's remainder, the 10-step
    chunk it joins at B = busy + 1, that chunk's codec calls and the PCM copy included); the first
    two of `reps` dropped (graph capture at the new batch sizes). Returns (p50, p90, max, joins) in ms
    (the tail over >= 30 joins, not the median alone)."""
    import queue
    import threading
    from llmvox_amd.streaming import FusedScheduler
    inbox = queue.Queue()

    def admit():  # queued requests / closes, between chunks or (overlap) while the scheduler waits
        while True:
            try:
                op, arg = inbox.get_nowait()
            except queue.Empty:
                return
            if op == "open":
                sink = arg[1]
                st = sched.open_stream(index=0, dump_size=10, sink=sink)
                for w in arg[0]:
                    st.feed(w)
                sink.stream = st
            else:
                sched.close_stream(arg)

    def waiter(ev):  # as the service's waiter: admissions land while the device works
        ev.synchronize()
        admit()

    sched = FusedScheduler(eng, max_chunk=max_chunk, to_bytes=True, overlap=overlap, waiter=waiter)
    rng = np.random.default_rng(seed)
    words = lambda n: " ".join(random_sentence(rng) for _ in range(n)).split(" ")
    for i in range(busy):  # replica streams as the service opens them (dump 10 / 160, x3 to 1280)
        st = sched.open_stream(index=i % 2, dump_size=10 if i % 2 == 0 else 160)
        for w in words(24):
            st.feed(w)
    done = threading.Event()
    errors = []
    busy_streams = list(sched.streams)

    cur = torch.cuda.current_stream(eng.device)  # (torch's current stream is per thread)

    def loop():
        try:
            torch.cuda.set_stream(cur)  # the graph-replay stream of the timed run
            while not done.is_set():
                admit()
                for st in busy_streams:  # keep the load: top up the text of busy streams running dry
                    if st.m.next_text_id() is None:
                        for w in words(8):
                            st.feed(w)
                if sched.run_chunk() == 0:
                    time.sleep(1e-4)
        except BaseException as e:  # surfaced by the caller
            errors.append(e)

    torch.cuda.synchronize()
    th = threading.Thread(target=loop, name="bench-sched", daemon=True)
    th.start()
    lat = []
    try:
        time.sleep(0.05)  # the busy streams are decoding
        for r in range(reps):
            time.sleep(float(rng.uniform(0.0, 0.008)))  # a random phase of the chunk in flight
            sink = queue.Queue()
            t0 = time.perf_counter()
            inbox.put(("open", (SENTENCE.split(" "), sink)))
            while True:
                try:
                    ev = sink.get(timeout=30)
                except queue.Empty:
                    raise RuntimeError(f"no first chunk within 30 s ({errors!r})")
                if isinstance(ev, bytes):
                    break
            t1 = time.perf_counter()
            assert len(ev) == 3200 * 4
            inbox.put(("close", sink.stream))
            if r >= 2:
                lat.append((t1 - t0) * 1e3)
    finally:
        done.set()
        th.join(timeout=60)
    if errors:
        raise errors[0]
    sched.flush()
    torch.cuda.synchronize()
    for st in list(sched.streams):
        sched.close_stream(st)
    sched.close()
    q = sorted(lat)
    p90 = q[min(len(q) - 1, int(math.ceil(0.9 * len(q))) - 1)]  # nearest-rank
    return statistics.median(lat), p90, max(lat), len(lat)


def run_chunks(eng, mine, S, chunk, K, Wm, reset_every=0, dist=None, rank=0, world=1, codec_overlap=False,
               seconds=0.0, window_s=10.0, record=None, gathered=None):
    """W untimed then K timed bench steps (one step = `chunk` fused decode steps for the S streams,
    the batched codec decode of their codes, the PCM to the host; the PCM gathered to rank 0 when
    distributed). With reset_every R, step c is chunk c % R of utterance c // R: the streams' KV
    slots are reset at every utterance start and `mine` holds the utterances' text plans back to
    back ([S][n_utterances * R * chunk]). Returns (seconds, last token buffer, codec stream, token
    buffers, PCM buffers). seconds > 0 (steady-state mode): chunks run until that much wall time has
    passed instead of K (the plans are cycled), with a device sync every window_s seconds to record
    the rate of each window (run_chunks.windows, run_chunks.k_done). record (a list, tests only): every
    chunk's tokens and PCM, copied on the codec stream before its buffers are reused
    (tests/test_gpu_bench_schedule.py holds the overlapped schedule to the serial one with it).
    gathered (a list, tests only): on rank 0, what the async gather delivered for each timed chunk, as
    [rank][S, samples] host tensors in issue order (tests/test_gpu_rccl.py)."""
    from llmvox_amd.parallel import ChunkGather, gather_pcm
    from llmvox_amd.streams import side_stream
    n_plan_chunks = mine.shape[1] // chunk
    dev = eng.device
    slots = torch.arange(S, dtype=torch.int32, device=dev)
    text_plan = torch.empty(S, chunk, dtype=torch.int32, device=dev)
    rowstep = torch.zeros(S, dtype=torch.int32, device=dev)
    tok_plan = torch.zeros(S, chunk, dtype=torch.int32, device=dev)
    pcm = torch.empty(S, 320 * chunk, dtype=torch.float32, device=dev)
    pcm_host = torch.empty(S, 320 * chunk, dtype=torch.float32, pin_memory=True)
    # codec_overlap (the default since round 4): the codec of chunk c runs on a second stream beside
    # the AR of chunk c + 1, paced by the host so that neither queue ever waits on the other's event
    # (the loop below). With the waits enqueued ahead (rounds 1-4 up to here: the codec queue blocked
    # on the AR's event for a whole chunk) every AR dispatch took ~1 us longer and the overlap lost
    # (195.6k vs 228.1k tok/s; CU-partitioned streams 186-198k); paced: configs[2] 234.8-235.5k vs
    # 228.1-228.3k, configs[1] 13.40-13.44k vs 12.90-12.96k, configs[4] 79.4k vs 76.7-77.0k, the
    # fp32 parity line 143.8k vs 142.6k (profiles/r04/codec_overlap_ab.txt). --serial-codec: the
    # codec after the AR on one stream. tok_plan / pcm are double-buffered for the overlap.
    # (a side stream checked to run beside the decode stream: llmvox_amd/streams.py)
    codec_stream = side_stream(dev, [None]) if codec_overlap else torch.cuda.current_stream(dev)
    tok_bufs = [tok_plan, torch.zeros_like(tok_plan)]
    pcm_bufs = [pcm, torch.empty_like(pcm)]
    ev_ar = [torch.cuda.Event(), torch.cuda.Event()]
    ev_codec = [torch.cuda.Event(), torch.cuda.Event()]
    # the PCM's copy to the host stays on the codec stream: on a stream of its own (so the next chunk's
    # AR would not queue behind it) it measured 192-193k vs 227-229k tok/s, the AR step 157-158 vs
    # 131-132 us (round 4, alternating A/B on one box, profiles/r04/copy_stream_ab.txt): with a second
    # stream in use every one of the step's 26 dependent dispatches took ~1 us longer
    copy_stream = codec_stream
    ev_copy = [torch.cuda.Event(), torch.cuda.Event()]
    # N > 1 with the overlap: chunk c's PCM gather to rank 0 is issued only once
    # the host has seen chunk c's codec event, on a communicator stream of its own, asynchronously,
    # and waited for (host poll) before the PCM buffer is written again: neither the decode nor the
    # codec queue ever holds the collective (round 4 put it on the codec stream, and N > 1 fell back
    # to the serial schedule)
    gather = (ChunkGather(dist, rank, world, side_stream(dev, [None, codec_stream]), keep=gathered is not None)
              if (dist is not None and codec_overlap) else None)
    gpending = [False, False]

    def gather_done(i):  # (host) the chunk in buffer i has finished its codec: send its PCM
        if gather is not None and gpending[i]:
            ev_codec[i].synchronize()
            gather.issue(i, pcm_bufs[i])
            gpending[i] = False
    # per-chunk AR time (the decode steps alone), timing events on the decode stream around
    # ar_steps: read after the timed region for the whole-step roofline (no host sync inside it)
    ar_t = []

    timing = None

    def run_chunk(c):
        ar_part(c)
        codec_part(c)

    def ar_part(c):
        i = c & 1
        main = torch.cuda.current_stream(dev)
        if codec_overlap:
            ev_codec[i].synchronize()  # (host) tok_bufs[i] is free again: no cross-queue wait enqueued
        else:
            main.wait_event(ev_codec[i])  # tok_bufs[i] is free again (its decode has read it)
        col = (c % n_plan_chunks) * chunk  # chunk c of the back-to-back utterance plans (cycled)
        if reset_every and c % reset_every == 0:  # a new utterance: KV slots reset (a new sentence)
            for s_ in range(S):
                eng.reset_slot(s_)
        text_plan.copy_(mine[:, col:col + chunk])
        rowstep.zero_()
        if timing is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(main)
        eng.ar_steps(chunk, slots, text_plan, rowstep, tok_bufs[i])
        ev_ar[i].record(main)
        if timing is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(main)
            timing.append((e0, e1))
        gather_done(i)  # chunk c - 2's PCM (its codec has ended: synchronised above)

    def codec_part(c):
        i = c & 1
        if codec_overlap:
            ev_ar[i].synchronize()  # (host) the chunk's tokens are there: the codec queue never blocks
        if gather is not None:
            gather.wait(i)  # chunk c - 2's gather has read pcm_bufs[i]
        with torch.cuda.stream(codec_stream):
            if not codec_overlap:
                codec_stream.wait_event(ev_ar[i])
            codec_stream.wait_event(ev_copy[i])
            eng.decode_codes(tok_bufs[i], 0, out=pcm_bufs[i])
            if dist is not None and gather is None:
                gather_pcm(pcm_bufs[i], dist, rank, world)  # PCM back to rank 0 (outbound exchange)
            gpending[i] = gather is not None
            if record is not None and timing is not None:  # (timed chunks only)
                record.append((tok_bufs[i].clone(), pcm_bufs[i].clone()))
            ev_codec[i].record(codec_stream)
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_event(ev_codec[i])
            pcm_host.copy_(pcm_bufs[i], non_blocking=True)
            ev_copy[i].record(copy_stream)

    def reset_all():
        for s in range(S):
            eng.reset_slot(s)

    # setup: capture the decode graphs for both token buffers (untimed), warmup, reset
    reset_all()
    for i in range(2):
        rowstep.zero_()
        text_plan.copy_(mine[:, :chunk])
        eng.ar_steps(17, slots, text_plan, rowstep, tok_bufs[i])
        eng.decode_codes(tok_bufs[i], 0, out=pcm_bufs[i])
    torch.cuda.synchronize()
    reset_all()
    for c in range(Wm):
        run_chunk(c)
    if gather is not None:
        for i in range(2):
            gather_done(i)
        gather.drain()
    torch.cuda.synchronize()
    eng.check_errors()
    reset_all()
    torch.cuda.synchronize()
    if gather is not None:
        gather.gathered.clear()  # (tests) the warm-up chunks' gathers

    # timed region: K chunks, barrier + synchronize on both sides
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    timing = ar_t
    t0 = time.perf_counter()
    run_chunks.windows = []
    if seconds > 0:  # steady state: whole utterances until `seconds` have passed, windows of window_s
        c, wc, wt = 0, 0, t0
        if codec_overlap:
            ar_part(0)
        while True:
            if codec_overlap:  # (the overlapped loop below: the AR of c + 1 queued unless c is the last)
                last = time.perf_counter() - t0 >= seconds and (not reset_every or (c + 1) % reset_every == 0)
                if not last:
                    ar_part(c + 1)
                codec_part(c)
            else:
                run_chunk(c)
            c += 1
            now = time.perf_counter()
            done = last if codec_overlap else (now - t0 >= seconds and (not reset_every or c % reset_every == 0))  # whole utterances
            if now - wt >= window_s or done:
                torch.cuda.synchronize()
                now = time.perf_counter()
                run_chunks.windows.append({"chunks": c - wc, "seconds": round(now - wt, 3),
                                           "tokens_per_s": round((c - wc) * S * chunk / (now - wt), 1)})
                wc, wt = c, now
                if done:
                    break
        K = c
    elif codec_overlap:
        # the codec of chunk c on its own stream beside the AR of chunk c + 1, paced by the host: the
        # AR of c + 1 is queued before the AR of c ends, and the codec of c only once that AR has ended,
        # so neither queue ever holds a wait on the other's event (a queue blocked on another queue's
        # signal slowed every dispatch of the AR chain by ~1 us: profiles/r04/codec_overlap_ab.txt)
        ar_part(0)
        for c in range(K):
            if c + 1 < K:
                ar_part(c + 1)
            codec_part(c)
    else:
        for c in range(K):
            run_chunk(c)
    if gather is not None:  # the last chunks' gathers (inside the timed region)
        for c in range(K - 2, K):
            if c >= 0:
                gather_done(c & 1)
        gather.drain()
    run_chunks.k_done = K
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    eng.check_errors()
    if gathered is not None and gather is not None:
        gathered.extend(gather.gathered)
    run_chunks.ar_ms = [a.elapsed_time(b) for a, b in ar_t]
    return dt, tok_bufs[(K - 1) & 1], codec_stream, tok_bufs, pcm_bufs


def parity_mode_line(S, chunk, K=4, Wm=1, codec_overlap=False, utt_chunks=4):
    """The fp32 parity mode (weights, KV and codec in fp32: bit-exact ids against the reference,
    tests/test_gpu_parity.py, test_gpu_f32b.py) on the headline's workload: K chunks of 1,024-token
    utterances per stream (utt_chunks chunks each, the KV slots reset at every utterance start: KV
    positions 0..1,023, as configs[2]'s utterances; VERDICT r03 item 2: round 3 ran K = 2, positions
    0..511 only), after Wm warm-up steps. K is the headline's own chunk count (round 5; rounds 3-4
    ran 4 chunks against the headline's 20, so the last chunk's codec, which no next chunk hides,
    weighed 1/4 of a step here and 1/20 there)."""
    from llmvox_amd.engine import build_engine
    utt = utt_chunks * chunk
    n_utt = -(-max(K, Wm) // utt_chunks)
    eng = build_engine(torch.cuda.current_device(), "fp32", "fp32", max_streams=S, max_positions=utt + 1,
                       max_codec_frames=S * chunk)
    try:
        rng = np.random.default_rng(1234)
        plans = np.zeros((S, n_utt * utt), dtype=np.int32)
        for g in range(S):
            for u in range(n_utt):
                ids = sentence_ids(SENTENCE if (g == 0 and u == 0) else random_sentence(rng))
                plans[g, u * utt:(u + 1) * utt] = plan_for(ids, 0, utt)
        mine = torch.from_numpy(plans).to(eng.device)
        dt, _, _, _, _ = run_chunks(eng, mine, S, chunk, K, Wm, utt_chunks, codec_overlap=codec_overlap)
        return {"value": round(S * K * chunk / dt, 1), "unit": "speech tokens/s", "ms_per_step": round(dt / K * 1e3, 3),
                "steps": K, "warmup": Wm, "dtype": "fp32", "kv_dtype": "fp32", "codec_weights": "fp32",
                "ar_gemm": "exact fp32 products (v_mfma_f32_16x16x4_f32), fp32 accumulate: ids bit-exact",
                "codec_gemm": ("bf16x3 split products (hi.hi + lo.hi + hi.lo on v_mfma_f32_16x16x32_bf16, "
                               "fp32 accumulate) in the >= 192-tile GEMMs, exact fp32 elsewhere; PCM within "
                               "2e-4 / RMS 1e-5 of the reference (tests/test_gpu_parity.py)"),
                "streams": S, "kv_positions": f"0..{min(K, utt_chunks) * chunk - 1}",
                "utterances": f"{K / utt_chunks:g} per stream ({utt_chunks} chunks each)",
                "ar_ms_per_chunk": round(sum(run_chunks.ar_ms) / K, 3)}
    finally:
        eng.close()


def main():
    import faulthandler
    faulthandler.enable()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--streams", type=int, default=0, help="streams per GPU (default: the config's: 1 / 32 / 1 / 8)")
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--kv-dtype", default=None, choices=["bf16", "fp32", "fp8"],
                    help="KV cache dtype (default: --dtype); fp8 = OCP e4m3fn (configs[4])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--no-parity-line", action="store_true", help="skip the fp32 parity-mode line")
    ap.add_argument("--no-loaded-latency", action="store_true",
                    help="skip the first-chunk latency of a stream joining a busy scheduler")
    ap.add_argument("--probe-pos", type=int, default=0,
                    help="KV position of the roofline probe (default: the run's mean position, steps * chunk / 2)")
    ap.add_argument("--codec-overlap", action="store_true",
                    help="(default) the codec on a second HIP stream beside the next chunk's AR, host-paced")
    ap.add_argument("--serial-codec", action="store_true",
                    help="the codec after each chunk's AR on the same stream (no overlap)")
    ap.add_argument("--graph-stream", action="store_true", help="(default) kept for old command lines")
    ap.add_argument("--sched", default="",
                    help="configs[3] FusedScheduler knobs: tail=N (steps after the planning event), mc=N (max chunk), cs=0 "
                         "(the codec on the decode stream: 2 processes sharing one card, DESIGN 4)")
    ap.add_argument("--null-stream", action="store_true",
                    help="run on torch's default (null) stream: the decode steps are launched kernel by kernel")
    ap.add_argument("--no-graphs", action="store_true",
                    help="never replay graphs (steps and kernel probes launched kernel by kernel)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the multi-rank path on one GPU (collectives on host copies)")
    ap.add_argument("--no-dist-world1", dest="dist_world1", action="store_false",
                    help="at N = 1, no process group (by default N = 1 creates a one-rank RCCL group and runs the "
                         "scatter / async gather path of N > 1: the same code the N-GPU lines time)")
    ap.add_argument("--dist-world1", dest="dist_world1", action="store_true", help="(default) kept for old command lines")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4],
                    help="BASELINE.json workload (2: default, 32 streams; 1: one stream; 3: scheduler replicas; 4: fp8)")
    ap.add_argument("--codec-dtype", default=None, choices=["fp8"], help="fp8 codec weights (configs[4])")
    ap.add_argument("--utt-tokens", type=int, default=2048, help="configs[3]: tokens per utterance (one step)")
    ap.add_argument("--utterance", type=int, default=1024,
                    help="configs[1]/[2]/[4]: tokens per utterance (SURVEY 8(d) N = 1024; a multiple of --chunk): "
                         "KV reset and a new sentence at every utterance start; 0 = one utterance for the whole run")
    ap.add_argument("--seconds", type=float, default=0.0,
                    help="steady-state mode: run whole utterances for this many seconds instead of --steps "
                         "(configs[4]: continuous sentences with a KV reset per sentence), rate per 10 s window")
    ap.add_argument("--opt", default="",
                    help="library options for A/B runs, name=value[,name=value] (lvx_set_option; default: production)")
    ap.add_argument("--rehearse", action="store_true",
                    help="CPU-only rehearsal of the multi-rank skeleton (gloo; tests/test_bench_launcher.py)")
    ap.set_defaults(dist_world1=True)
    args = ap.parse_args()
    args.codec_overlap = not args.serial_codec
    if args.streams == 0:
        args.streams = {1: 1, 2: 32, 3: 1, 4: 8}[args.config]
    if args.config == 4:
        args.kv_dtype = args.kv_dtype or "fp8"
        args.codec_dtype = args.codec_dtype or "fp8"

    # one process per GPU: under torch.distributed.run WORLD_SIZE is set (and must equal --gpus);
    # without it, --gpus N > 1 spawns the N ranks here, before anything touches the GPU
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(world_env or 1)
    if world != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
                         "different GPU count than requested\n")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse:
        return rehearse(args, world, rank)
    dist, dist_info = None, None
    if world > 1 or args.dist_world1:
        import torch.distributed as tdist
        if world == 1:
            # a one-rank RCCL group (in-process store, no rendezvous), so that the N = 1 run takes the
            # N > 1 code path: the RCCL text scatter, the async PCM gather on its communicator stream and
            # its completion polls. Round 6, one box: 233.0k / 231.4k tok/s with it,
            # 234.0k without (profiles/r06/dist_world1_ab.txt)
            torch.cuda.set_device(local)
            try:
                tdist.init_process_group("nccl", store=tdist.HashStore(), rank=0, world_size=1,
                                         device_id=torch.device(f"cuda:{local}"))
                dist = tdist
            except Exception as e:  # (reported in the line: dist backend null)
                sys.stderr.write(f"bench.py: no one-rank RCCL group ({e!r}); N = 1 runs without collectives\n")
                dist = None
        elif args.dist_backend == "gloo":  # rehearsal: every rank may share one GPU
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            tdist.init_process_group("gloo")
            dist = _HostCollectives(tdist)
        else:
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
            dist = tdist
        if dist is not None:
            dist_info = {"backend": tdist.get_backend(), "world_size": tdist.get_world_size()}

    from llmvox_amd.engine import build_engine
    S, chunk, K, Wm = args.streams, args.chunk, args.steps, args.warmup
    if max(K, Wm) * chunk > 8192:
        raise SystemExit("steps * chunk must stay within block_size 8192 positions")
    kvd = args.kv_dtype or args.dtype
    eng = build_engine(local, args.dtype, kvd, max_streams=max(S, 1), max_positions=8192,
                       max_codec_frames=max(S * chunk, 1280 * S if args.config == 3 else 0),
                       codec_dtype=args.codec_dtype)
    dev = eng.device
    torch.cuda.set_device(dev)
    for kv in filter(None, args.opt.split(",")):
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    if args.no_graphs:
        eng.set_graphs(False)
    if not args.null_stream:
        # decode steps replayed as HIP graphs need a non-default stream (the legacy null stream,
        # torch's default, cannot be captured; the library launches its steps one by one there).
        # Round 3, alternating A/B on one box (tools/gpu_graph_ab.sh): graphs equal or faster and
        # steadier (configs[2] 224.6 / 224.7k vs 218.7 / 223.7k; configs[1] 12.8 / 13.0k vs 12.2 /
        # 12.9k), and launched steps swing with host load (B = 8: 107-180 vs 99-104 us/step,
        # tools/step_sweep.py): the host no longer paces the step.
        # (round 5: the decode stream at high queue priority, the codec's at the default, measured the
        # same: 234.5 / 235.6 / 235.3k vs 235.4 / 235.7 / 233.7k tok/s, profiles/r05/priority_ab.txt)
        torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    if args.config == 3:
        try:
            return run_config3(args, eng, world, rank, local, dist)
        finally:
            _release(eng)

    # ---- text plans: stream 0 of rank 0 opens with the config sentence; every other utterance is a
    # seeded random sentence; utterances back to back per stream
    if args.utterance and args.utterance % chunk:
        raise SystemExit("--utterance must be a multiple of --chunk")
    reset_every = args.utterance // chunk if args.utterance else 0
    utt = args.utterance or max(K, Wm) * chunk
    n_utt = -(-max(K, Wm) * chunk // utt)
    if args.seconds > 0:
        if not reset_every:
            raise SystemExit("--seconds needs utterances (--utterance > 0): a KV reset per sentence")
        n_utt = max(n_utt, 16)  # a pool of 16 sentences per stream, cycled
    n_pos = n_utt * utt
    plans = np.zeros((world * S, n_pos), dtype=np.int32)
    rng = np.random.default_rng(1234)
    for g in range(world * S):
        for u in range(n_utt):
            ids = sentence_ids(SENTENCE if (g == 0 and u == 0) else random_sentence(rng))
            plans[g, u * utt:(u + 1) * utt] = plan_for(ids, 0, utt)
    from llmvox_amd.parallel import scatter_plans
    # rank 0 scatters the text-id shards over RCCL (the path's inbound exchange)
    mine = scatter_plans(torch.from_numpy(plans), S, n_pos, dev, dist, rank)

    dt, last_tok, codec_stream, tok_bufs, pcm_bufs = run_chunks(
        eng, mine, S, chunk, K, Wm, reset_every, dist, rank, world, args.codec_overlap, seconds=args.seconds)
    windows = list(run_chunks.windows)
    if args.seconds > 0:
        K = run_chunks.k_done
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    total_tokens = world * S * K * chunk
    value = total_tokens / dt
    toks_rank0 = last_tok[0].cpu().numpy()

    p50 = first_chunk_latency(eng, overlap=args.codec_overlap)
    p50_loaded = None
    if args.config in (1, 2, 4) and not args.no_loaded_latency:
        eng.check_errors()
        p50_loaded = first_chunk_latency_loaded(eng, busy=min(31, eng.max_streams - 1), overlap=args.codec_overlap)

    # ---- roofline: dominant kernel class at the run's mean KV position, timed live with HIP
    # events on the compute stream; traffic from a PMC pass over the same probe workload
    rl, kern = None, None
    slots = torch.arange(S, dtype=torch.int32, device=dev)
    if not args.no_probe:
        for s in range(S):
            eng.reset_slot(s)
        span = (min(K, reset_every) if reset_every else K) * chunk  # positions one utterance spans
        ppos = args.probe_pos or max(1, span // 2)
        for s in range(S):
            eng.set_slot(s, ppos - 1, 0)
        wb = 2 if args.dtype == "bf16" else 4
        kb = {"bf16": 2, "fp8": 1, "fp32": 4}[kvd]
        kern = probe_kernels(eng, slots, ppos, wb, kb)
        dom = max(kern.values(), key=lambda r: r["share_us_per_step"])
        key = pmc_key(args.dtype, kvd, S, ppos)
        rl = {"bound": "hbm", "kernel": dom["name"], "achieved": round(dom["gbs"], 1), "peak": HBM_PEAK_GBS,
              "unit": "GB/s", "frac": round(dom["gbs"] / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(key, dom["name"]),
              "bytes_per_launch": dom["bytes"], "avg_us": round(dom["avg_us"], 3), "kv_positions": ppos,
              "pmc_key": key,
              # rocprofv3 --pmc faults under HIP-graph replay (also without this library:
              # tools/pmc_graph_repro.hip, profiles/r04/pmc_repro_*.log), so the counters come from
              # the same command with the steps launched kernel by kernel (--null-stream): the same
              # kernels and grids, per-dispatch bytes
              "traffic_launch_path": "null stream (PMC pass; the timed run replays graphs)"}
        # PMC traffic / algorithmic bytes per probed kernel (a ratio well above 1 = operand re-fetch)
        rl["traffic_ratio"] = {v["name"]: (round(pmc_traffic(key, v["name"]) / v["bytes"], 3)
                                           if pmc_traffic(key, v["name"]) else None) for v in kern.values()}

    # ---- codec: one batched decode of a chunk (S streams x chunk frames), HIP events on the
    # stream it runs on; algorithmic FLOPs per SURVEY 8(d): 125,566,976 + 3,072 L per frame
    torch.cuda.synchronize()
    with torch.cuda.stream(codec_stream):
        eng.decode_codes(tok_bufs[0], 0, out=pcm_bufs[0])
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(codec_stream)
        for _ in range(5):
            eng.decode_codes(tok_bufs[0], 0, out=pcm_bufs[0])
        c1.record(codec_stream)
    c1.synchronize()
    codec_ms = c0.elapsed_time(c1) / 5
    codec_flops = S * chunk * (125_566_976 + 3_072 * chunk)
    codec_peak = 2500.0 if args.dtype == "bf16" else 157.3  # dense bf16 MFMA / exact-f32 MFMA, TFLOP/s
    peak_note = None
    if args.codec_dtype == "fp8":
        # pwconv1 (12 x 2 x 768 x 2,304 = 42,467,328 FLOPs per frame, 33.8 % of the codec) runs W8A8 on
        # the fp8 MFMA (dense 5,000 TFLOP/s); every other FLOP on bf16 MFMA (2,500): the peak is the
        # rate at which the decode's FLOP mix would run with each part at its own peak
        f_pw1 = S * chunk * 42_467_328
        codec_peak = codec_flops / (f_pw1 / 5000.0 + (codec_flops - f_pw1) / 2500.0)
        peak_note = ("FLOP-weighted: pwconv1 at the dense fp8 MFMA peak 5,000 TFLOP/s, the rest at the dense "
                     "bf16 peak 2,500")
    ckey = f"{args.codec_dtype or args.dtype}/F{S * chunk}/L{chunk}"
    codec = {"frames": S * chunk, "avg_ms": round(codec_ms, 3),
             "achieved": round(codec_flops / (codec_ms * 1e-3) / 1e12, 2), "peak": round(codec_peak, 1),
             "unit": "TFLOP/s", "frac": round(codec_flops / (codec_ms * 1e-3) / 1e12 / codec_peak, 4),
             "gemm_mfma_busy": pmc_codec(ckey), "pmc_key": ckey}
    if peak_note:
        codec["peak_note"] = peak_note

    # whole decode step against HBM: algorithmic bytes of every step of the timed chunks (their KV
    # positions) over the measured AR time of those chunks (events around ar_steps in the timed loop)
    wb = 2 if args.dtype == "bf16" else 4
    kb = {"bf16": 2, "fp8": 1, "fp32": 4}[kvd]
    ar_ms = getattr(run_chunks, "ar_ms", [])
    step_rl = None
    if ar_ms:
        tot_b = 0
        for c in range(K):
            p0 = (c % reset_every) * chunk if reset_every else c * chunk
            tot_b += sum(step_bytes(S, p + 1, wb, kb) for p in range(p0, p0 + chunk))
        us = sum(ar_ms) * 1e3 / (K * chunk)
        gbs = tot_b / (K * chunk) / (us * 1e-6) / 1e9
        step_rl = {"bound": "hbm", "bytes_per_step": round(tot_b / (K * chunk)), "us_per_step": round(us, 2),
                   "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                   "ar_ms_per_chunk": round(sum(ar_ms) / K, 3),
                   "note": "all GEMM weights once + 4 layers of K/V history read and the new key/value written, "
                           "per decode step at the timed chunks' positions, over the decode steps' own time"}

    parity = None
    if rank == 0 and world == 1 and not args.no_parity_line and args.dtype == "bf16" and args.config in (1, 2):
        # the headline's chunk count, 1,024-token utterances (positions 0..1,023 as the headline's)
        parity = parity_mode_line(S, chunk, K=K, codec_overlap=args.codec_overlap,
                                  utt_chunks=max(1, min(4, utt // chunk)))
        parity["ratio_to_headline"] = round(parity["value"] / value, 4)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the CPU baseline: N = 1 runs only
        # the same utterance length as the timed run (one stream: the oracle is B = 1)
        cpu = cpu_baseline(min(K, reset_every) if reset_every else K, chunk)

    if rank == 0:
        out = {
            "metric": "speech tokens/sec (+ 24kHz audio samples/sec = 320 x tokens/s; p50 first-chunk latency)",
            "value": round(value, 1),
            "unit": "speech tokens/s",
            "n_gpus": world,
            "steps": K,
            "warmup": Wm,
            "ms_per_step": round(dt / K * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (config 64-char sentence + seeded random 64-char sentences -> ByT5 ids, "
                    "seeded synthetic weights at reference init scales)",
            "config": {"workload": f"configs[{args.config}]: 30M LLMVoX {args.dtype}, "
                                   f"{S} stream(s)/GPU, {chunk}-token chunk, greedy AR + WavTokenizer decode + PCM to host"
                                   + (", fp8 KV + fp8 codec weights" if args.config == 4 else "")
                                   + (f", utterances of {utt} tokens (KV reset + a new sentence per utterance)"
                                      if reset_every else f", one {K * chunk}-token utterance per stream"),
                       "streams_per_gpu": S, "chunk_tokens": chunk, "utterance_tokens": utt,
                       "kv_positions": f"0..{min(K * chunk, utt) - 1}",
                       "parallelism": (f"streams sharded over {world} GPU(s), {dist_info['backend']} scatter text / "
                                       "async gather PCM" if dist_info else
                                       "one GPU, no process group (no collective runs)"),
                       "codec_schedule": ("chunk c's codec on a second stream beside chunk c + 1's AR (host-paced)"
                                          if args.codec_overlap else "codec after each chunk's AR, one stream")},
            "dist": dist_info or {"backend": None, "world_size": 1},
            "audio_samples_per_s": round(320 * value, 1),
            "realtime_factor_per_stream": round(value / (world * S) / 75.0, 1),
            "p50_first_chunk_latency_ms": round(p50, 3),
            "p50_first_chunk_latency_loaded_ms": round(p50_loaded[0], 3) if p50_loaded else None,
            "first_chunk_latency_loaded": ({"p50_ms": round(p50_loaded[0], 3), "p90_ms": round(p50_loaded[1], 3),
                                            "max_ms": round(p50_loaded[2], 3), "joins": p50_loaded[3],
                                            "busy_streams": min(31, eng.max_streams - 1), "max_chunk": 32,
                                            "note": "a fresh stream joining a FusedScheduler already decoding the "
                                                    "busy streams; enqueue -> first 3,200-sample dump on the host"}
                                           if p50_loaded else None),
            "roofline": rl,
            "step_roofline": step_rl,
            "codec_roofline": codec,
            "kv_dtype": kvd,
            "codec_weights": args.codec_dtype or args.dtype,
            "parity_mode_fp32": parity,
            "cpu_baseline": cpu,
            "kernels": {v["name"]: {"avg_us": round(v["avg_us"], 2), "GB/s": round(v["gbs"], 1)}
                        for v in kern.values()} if kern else None,
            "tokens_head": toks_rank0[:8].tolist(),
        }
        if args.seconds > 0:
            rates = [w["tokens_per_s"] for w in windows if w["seconds"] >= 1.0]
            out["steady_state"] = {"seconds": round(dt, 3), "chunks": K, "utterances_per_stream": K // reset_every,
                                   "windows": windows,
                                   "spread": (round((max(rates) - min(rates)) / (sum(rates) / len(rates)), 4)
                                              if rates else None)}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    _release(eng)


def _release(eng):
    """Free the library context (its graphs, streams, device memory) while the HIP runtime is fully
    up: left to the garbage collector at interpreter exit, lvx_destroy can run during the runtime's own
    teardown."""
    torch.cuda.synchronize()
    eng.close()


if __name__ == "__main__":
    if os.environ.get("LVX_PROFILE_DIR"):  # development: a cProfile of each rank's process (host time)
        import cProfile
        import pstats
        d = os.environ["LVX_PROFILE_DIR"]
        os.makedirs(d, exist_ok=True)
        pr = cProfile.Profile()
        try:
            pr.runcall(main)
        finally:
            out = os.path.join(d, f"rank{os.environ.get('RANK', '0')}.txt")
            with open(out, "w") as f:
                pstats.Stats(pr, stream=f).sort_stats("tottime").print_stats(25)
                pstats.Stats(pr, stream=f).sort_stats("cumulative").print_stats(45)
    else:
        main()
