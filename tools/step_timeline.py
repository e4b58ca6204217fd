"""Development probe: in-kernel timeline of one batched decode step (timing build of the library,
`make -C llmvox_amd/csrc timing`). Thread 0 of every block of the batched-step kernels records the
100 MHz real-time counter at entry, after its operands landed and at exit; this prints, per kernel
in step order: blocks, CUs, first/last entry and last exit relative to the step's first entry, the
median entry->operands and operands->exit spans, and the gap from the previous kernel's last exit
to this kernel's first entry (the boundary as the CUs see it).
usage: python tools/step_timeline.py [B] [P0] [graphs 0/1] [opt=value,...]"""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LVX_LIB_PATH", os.path.join(ROOT, "llmvox_amd", "libllmvox_hip_timing.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from llmvox_amd.engine import build_engine  # noqa: E402
from llmvox_amd import _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
P0 = int(sys.argv[2]) if len(sys.argv) > 2 else 512
graphs = int(sys.argv[3]) if len(sys.argv) > 3 else 1
TAGS = {0: "rows", 1: "c_attn", 2: "attn", 3: "c_proj", 4: "c_fc", 5: "mlp_proj", 6: "lm_head", 7: "embed_sel",
        8: "rows_lm"}
NBLK = 1024
lib = _lib.load()
lib.lvx_debug_timeline.restype = ctypes.c_int
lib.lvx_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]

e = build_engine(0, "bf16", os.environ.get("LVX_TL_KV", "bf16"), max_streams=B, max_positions=P0 + 512, max_codec_frames=256)  # LVX_TL_KV=fp8: configs[4]
dev = e.device
for kv in (sys.argv[4].split(",") if len(sys.argv) > 4 else []):
    k, v = kv.split("=")
    e.set_option(k, int(v))
stream = torch.cuda.Stream(device=dev) if graphs else torch.cuda.current_stream(dev)
plan = torch.full((B, 64), 100, dtype=torch.int32, device=dev)
slots = torch.arange(B, dtype=torch.int32, device=dev)
tok = torch.zeros(B, 64, dtype=torch.int32, device=dev)
buf = np.zeros(16 * 4 * NBLK * 4, dtype=np.uint64)
with torch.cuda.stream(stream):
    for rep in range(3):
        for s in range(B):
            e.set_slot(s, P0, 5)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        assert lib.lvx_debug_timeline(None, 0, 1) >= 0
        torch.cuda.synchronize()
        e.ar_steps(16, slots, plan, rowstep, tok)  # the records hold the last step that ran each kernel
        torch.cuda.synchronize()
assert lib.lvx_debug_timeline(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes, 0) > 0
r = buf.reshape(16, 4, NBLK, 4)
rows = []
for tag in range(16):
    for layer in range(4):
        v = r[tag, layer]
        v = v[v[:, 0] != 0]
        if len(v) == 0:
            continue
        t0, t1, t2, hw = (v[:, i].astype(np.int64) for i in range(4))
        cu = set(((h >> 32) & 15, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15) for h in hw.tolist())
        rows.append((int(t0.min()), TAGS.get(tag, str(tag)), layer, len(v), len(cu), t0, t1, t2))
rows.sort(key=lambda x: x[0])
base = rows[0][0]
prev_end = None
print(f"B={B} P0={P0} graphs={graphs}: times in us from the step's first entry (10 ns ticks)")
print(f"{'kernel':10s} L blks CUs  first_in  last_in  last_out   dur  in->ops  ops->out  gap")
tot_gap = 0.0
for first, name, layer, n, ncu, t0, t1, t2 in rows:
    f = (first - base) / 100
    li = (int(t0.max()) - base) / 100
    lo = (int(t2.max()) - base) / 100
    ops = statistics.median(((t1 - t0) / 100).tolist())
    out = statistics.median(((t2 - t1) / 100).tolist())
    gap = (first - prev_end) / 100 if prev_end is not None else 0.0
    tot_gap += gap
    print(f"{name:10s} {layer} {n:4d} {ncu:3d} {f:9.2f} {li:8.2f} {lo:9.2f} {lo - f:6.2f} {ops:7.2f} {out:8.2f} {gap:6.2f}")
    prev_end = int(t2.max())
print(f"step span {(prev_end - base) / 100:.2f} us, sum of gaps {tot_gap:.2f} us over {len(rows)} kernels")
