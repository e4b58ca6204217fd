"""Development probe: the pieces of one default bench step (configs[2]: 32 streams, 256-token chunks,
utterances of 1,024 tokens) timed with HIP events on the stream they run on: the AR chunk (256
fused decode steps), the batched codec decode, the PCM copy to pinned host memory, the KV resets.
usage: python tools/chunk_probe.py [chunks] [max_positions]"""
import sys
import numpy as np
import torch
from llmvox_amd.engine import build_engine

S, chunk = 32, 256
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
mp = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
e = build_engine(0, "bf16", "bf16", max_streams=S, max_positions=mp, max_codec_frames=S * chunk)
dev = e.device
st = torch.cuda.current_stream()
rng = np.random.default_rng(1)
plan_all = torch.from_numpy(rng.integers(3, 380, size=(S, 4 * chunk)).astype(np.int32)).to(dev)
slots = torch.arange(S, dtype=torch.int32, device=dev)
plan = torch.empty(S, chunk, dtype=torch.int32, device=dev)
rowstep = torch.zeros(S, dtype=torch.int32, device=dev)
tok = torch.zeros(S, chunk, dtype=torch.int32, device=dev)
pcm = torch.empty(S, 320 * chunk, dtype=torch.float32, device=dev)
host = torch.empty(S, 320 * chunk, dtype=torch.float32, pin_memory=True)


def ev():
    x = torch.cuda.Event(enable_timing=True)
    x.record(st)
    return x


for s in range(S):
    e.reset_slot(s)
e.ar_steps(17, slots, plan_all[:, :chunk].contiguous(), rowstep, tok)
e.decode_codes(tok, 0, out=pcm)
torch.cuda.synchronize()
rows = []
for c in range(n):
    u = c % 4
    t0 = ev()
    if u == 0:
        for s in range(S):
            e.reset_slot(s)
    t1 = ev()
    plan.copy_(plan_all[:, u * chunk:(u + 1) * chunk])
    rowstep.zero_()
    t2 = ev()
    e.ar_steps(chunk, slots, plan, rowstep, tok)
    t3 = ev()
    e.decode_codes(tok, 0, out=pcm)
    t4 = ev()
    host.copy_(pcm, non_blocking=True)
    t5 = ev()
    rows.append((u, t0, t1, t2, t3, t4, t5))
torch.cuda.synchronize()
print("chunk pos0   reset   plan      AR(ms) us/step  codec(ms)  copy(ms)  total(ms)")
for c, (u, *t) in enumerate(rows):
    d = [t[i].elapsed_time(t[i + 1]) for i in range(5)]
    print(f"{c:5d} {u * chunk:5d} {d[0]:7.3f} {d[1]:6.3f} {d[2]:10.3f} {d[2] / chunk * 1e3:7.1f} {d[3]:9.3f} {d[4]:9.3f} "
          f"{t[0].elapsed_time(t[5]):10.3f}", flush=True)
