"""Experiment: two independent AR decode chains (two engines, half the streams each) on two HIP
streams vs one engine with all streams on one stream. us per step for all rows."""
import sys, time
import torch
from llmvox_amd.engine import build_engine

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 2
engs = [build_engine(0, "bf16", "bf16", max_streams=B, max_positions=1024, max_codec_frames=256) for _ in range(nq)]
dev = engs[0].device
streams = [torch.cuda.Stream(device=dev) for _ in range(nq)]


def bufs(b):
    return (torch.arange(b, dtype=torch.int32, device=dev), torch.full((b, 512), 100, dtype=torch.int32, device=dev),
            torch.zeros(b, dtype=torch.int32, device=dev), torch.zeros(b, 512, dtype=torch.int32, device=dev))


def run(parts, nsteps=256, warm=True):
    # parts: list of (engine, stream, rows)
    state = []
    for e, st, b in parts:
        sl, pl, rs, tk = bufs(b)
        for s in range(b):
            e.reset_slot(s)
        state.append((e, st, b, sl, pl, rs, tk))
    torch.cuda.synchronize()
    for e, st, b, sl, pl, rs, tk in state:  # warm to position 256 (and capture graphs)
        with torch.cuda.stream(st):
            e.ar_steps(256, sl, pl, rs, tk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(nsteps // 16):
        for e, st, b, sl, pl, rs, tk in state:
            with torch.cuda.stream(st):
                e.ar_steps(16, sl, pl, rs, tk)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / nsteps * 1e6


one = run([(engs[0], streams[0], B)])
print(f"B={B} one chain: {one:.1f} us/step ({B / one * 1e6:.0f} tok/s)")
for k in range(2, nq + 1):
    per = B // k
    t = run([(engs[i], streams[i], per) for i in range(k)])
    print(f"B={B} {k} chains of {per}: {t:.1f} us/step ({B / t * 1e6:.0f} tok/s)")
t = run([(engs[0], streams[0], B)] + [(engs[i], streams[i], B) for i in range(1, 2)])
print(f"2 chains of {B}: {t:.1f} us/step ({2 * B / t * 1e6:.0f} tok/s)")
