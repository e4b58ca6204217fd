"""Development probe: host launch time, single-call latency and back-to-back time of small codec decodes
(the first dumps of a stream: is the decode bound by its kernel launches?). usage: python tools/codec_latency_probe.py"""
import sys, time
import torch
sys.path.insert(0, ".")
from llmvox_amd.engine import build_engine
e = build_engine(0, "bf16", "bf16", max_streams=32, max_positions=64, max_codec_frames=8192)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
for B, L in ((1, 10), (1, 30), (1, 90), (1, 256), (2, 160)):
    codes = torch.randint(0, 4096, (B, L), dtype=torch.int32).to(e.device)
    out = torch.empty(B, 320 * L, device=e.device)
    e.decode_codes(codes, 0, out=out); torch.cuda.synchronize()
    # host launch time of one call (GPU idle before it)
    hs = []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter(); e.decode_codes(codes, 0, out=out); hs.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    # single-call latency (enqueue -> done)
    ls = []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter(); e.decode_codes(codes, 0, out=out); torch.cuda.synchronize(); ls.append(time.perf_counter() - t0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(20): e.decode_codes(codes, 0, out=out)
    b.record(s); b.synchronize()
    print(f"{B}x{L}: host launch {sorted(hs)[5]*1e3:.3f} ms, call latency {sorted(ls)[5]*1e3:.3f} ms, back-to-back {a.elapsed_time(b)/20:.3f} ms", flush=True)
