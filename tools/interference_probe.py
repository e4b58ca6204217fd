"""Development probe: how much does the batched codec decode slow the decode steps running beside it?
B = 32 bf16 decode steps (HIP-graph replay on stream A) at positions P0.., alone and with the
32 x 256-frame codec decode enqueued back to back on a second stream C (no cross-stream waits: the
host enqueues both), C either a plain stream or one created with a CU mask (hipExtStreamCreateWithCUMask,
bit i = logical CU i). Prints us per step, the codec's ms per call beside the steps and the step time
lost per ms of codec work.
usage: python tools/interference_probe.py [P0] [mask ...]   mask: all | first:K | stride:K (K of 256 CUs)
  | lowprio (a low-priority plain stream, the steps' stream high) | opt=name=value (an option for the
  codec calls, on a plain stream) | copy:MB (a torch copy of MB megabytes instead
  of the codec) | mm:N (a torch bf16 N x N x N matmul instead of the codec) | mm:MxNxK (an M x K by K x N
  matmul) | split:K (the 32 streams' codec as K calls of 32 / K streams each)
Also printed: the step time lost per codec call (lost per ms x the call's ms beside the steps)."""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
from llmvox_amd.engine import build_engine  # noqa: E402

P0 = int(sys.argv[1]) if len(sys.argv) > 1 else 384
MASKS = sys.argv[2:] or ["all"]
B, N, L = 32, 256, 256
e = build_engine(0, "bf16", "bf16", max_streams=B, max_positions=P0 + N + 2, max_codec_frames=B * L)
dev = e.device
hip = ctypes.CDLL("libamdhip64.so")
n_cu = torch.cuda.get_device_properties(dev).multi_processor_count


def masked_stream(spec):
    if spec == "all" or spec.split(":")[0] in ("opt=", "copy", "mm", "split") or spec.startswith("opt="):
        return torch.cuda.Stream(device=dev)
    if spec == "lowprio":
        return torch.cuda.Stream(device=dev, priority=0)
    kind, k = spec.split(":")
    k = int(k)
    bits = [0] * n_cu
    if kind == "first":
        for i in range(k):
            bits[i] = 1
    else:  # stride: K CUs spread evenly over the logical ids
        for i in range(k):
            bits[(i * n_cu) // k] = 1
    words = (ctypes.c_uint32 * ((n_cu + 31) // 32))()
    for i, b in enumerate(bits):
        if b:
            words[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value, device=dev)


A = torch.cuda.Stream(device=dev, priority=-1 if "lowprio" in MASKS else 0)
plan = torch.full((B, N), 100, dtype=torch.int32, device=dev)
slots = torch.arange(B, dtype=torch.int32, device=dev)
tok = torch.zeros(B, N, dtype=torch.int32, device=dev)
codes = torch.randint(0, 4096, (B, L), dtype=torch.int32, device=dev)
pcm = torch.empty(B, 320 * L, dtype=torch.float32, device=dev)


def ar_run():
    with torch.cuda.stream(A):
        for s in range(B):
            e.set_slot(s, P0, 5)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record(A)
        e.ar_steps(N, slots, plan, rowstep, tok)
        a1.record(A)
    return a0, a1


WORK = {}


def codec_run(C, n, spec="all"):
    with torch.cuda.stream(C):
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if spec.startswith("copy:"):  # ~2 ms of copies per "call"
            mb = int(spec.split(":")[1])
            if spec not in WORK:
                WORK[spec] = (torch.empty(mb << 18, device=dev), torch.empty(mb << 18, device=dev))
            src, dst = WORK[spec]
            reps = max(1, int(2e-3 / (2 * (mb << 20) / 5e12)))
            c0.record(C)
            for _ in range(n * reps):
                dst.copy_(src)
        elif spec.startswith("mm:"):
            dims = [int(x) for x in spec.split(":")[1].split("x")]
            M, N_, K = dims if len(dims) == 3 else dims * 3
            if spec not in WORK:
                WORK[spec] = (torch.randn(M, K, device=dev, dtype=torch.bfloat16), torch.randn(K, N_, device=dev, dtype=torch.bfloat16))
            a, b = WORK[spec]
            reps = max(1, int(2e-3 / (2 * M * N_ * K / 1.0e15)))
            c0.record(C)
            for _ in range(n * reps):
                torch.mm(a, b)
        elif spec.startswith("split:"):
            k = int(spec.split(":")[1])
            g = B // k
            c0.record(C)
            for _ in range(n):
                for j in range(k):
                    e.decode_codes(codes[j * g:(j + 1) * g], 0, out=pcm[j * g:(j + 1) * g])
        else:
            c0.record(C)
            for _ in range(n):
                e.decode_codes(codes, 0, out=pcm)
        c1.record(C)
    return c0, c1


for spec in MASKS:
    C = masked_stream(spec)
    if spec.startswith("opt="):
        _, k, v = spec.split("=")
        e.set_option(k, int(v))
    ar_run()
    codec_run(C, 1, spec)
    torch.cuda.synchronize()
    res = []
    for rep in range(3):
        a0, a1 = ar_run()
        torch.cuda.synchronize()
        alone = a0.elapsed_time(a1) / N * 1e3
        c0, c1 = codec_run(C, 5, spec)
        torch.cuda.synchronize()
        codec_alone = c0.elapsed_time(c1) / 5
        # both together: the steps first (their graph replays queue up), then the codec calls
        a0, a1 = ar_run()
        c0, c1 = codec_run(C, 10, spec)
        torch.cuda.synchronize()
        both_ar = a0.elapsed_time(a1) / N * 1e3
        both_codec = c0.elapsed_time(c1) / 10
        # codec busy inside the steps' window: min(its span, the steps' span)
        overlap_ms = min(c0.elapsed_time(c1), a0.elapsed_time(a1))
        lost = (both_ar - alone) * N / 1e3  # ms of step time lost
        res.append((alone, codec_alone, both_ar, both_codec, lost / overlap_ms))
    res.sort(key=lambda r: r[2])
    a, ca, b, cb, per = res[1]
    print(f"codec stream {spec:10s}: steps alone {a:6.1f} us, beside the codec {b:6.1f} us; codec alone "
          f"{ca:5.2f} ms, beside the steps {cb:5.2f} ms; step time lost per ms of codec {per:5.2f} "
          f"(per call {per * cb:5.2f} ms)", flush=True)
    if spec.startswith("opt="):
        e.set_option(k, 0)
