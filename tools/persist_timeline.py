"""Development probe: task timeline of the persistent decode step (timing build of the library,
`make -C llmvox_amd/csrc timing`). Every task of ar_persist_kernel records (thread 0) the 100 MHz
real-time counter at its start (before its weight loads), when its dependency wait was satisfied,
and after it signalled. Prints per phase: tasks, first start, last wait-done, last end relative to
the step's first start, median wait (start -> wait done) and median work (wait done -> end).
usage: python tools/persist_timeline.py [B] [P0]"""
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
NAMES = ["rows", "c_attn", "attn", "c_proj", "c_fc", "mlp_proj"]
lib = _lib.load()
lib.lvx_debug_persist.restype = ctypes.c_int
lib.lvx_debug_persist.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
e = build_engine(0, "bf16", "bf16", max_streams=B, max_positions=P0 + 512, max_codec_frames=256)
dev = e.device
e.set_option("persist", 1)
e.set_option("pexp", int(os.environ.get("LVX_PEXP", "0")))  # persistent-step A/B bits
plan = torch.full((B, 64), 100, dtype=torch.int32, device=dev)
slots = torch.arange(B, dtype=torch.int32, device=dev)
tok = torch.zeros(B, 64, dtype=torch.int32, device=dev)
buf = np.zeros(8192 * 4, dtype=np.uint64)
stream = torch.cuda.Stream(device=dev)
spans = []
with torch.cuda.stream(stream):
    for rep in range(4):
        for s in range(B):
            e.set_slot(s, P0, 5)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        assert lib.lvx_debug_persist(None, 0, 1) >= 0
        torch.cuda.synchronize()
        e.ar_steps(1, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
assert lib.lvx_debug_persist(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes, 0) > 0
r = buf.reshape(8192, 4).astype(np.int64)
r = r[r[:, 0] != 0]
base = r[:, 0].min()
ph = r[:, 3] >> 32
print(f"B={B} P0={P0}: one persistent step, us from its first task start; {len(r)} tasks")
print(f"{'phase':12s} tasks  first_start  last_waitdone  last_end  med_wait  med_work  max_work")
prev_end = None
for p in sorted(set(ph.tolist())):
    v = r[ph == p]
    l, k = divmod(p, 6)
    name = ("rows_lnf" if p == 24 else "lm_head") if p >= 24 else f"{NAMES[k]}"
    fs = (v[:, 0].min() - base) / 100
    lw = (v[:, 1].max() - base) / 100
    le = (v[:, 2].max() - base) / 100
    wait = statistics.median(((v[:, 1] - v[:, 0]) / 100).tolist())
    work = statistics.median(((v[:, 2] - v[:, 1]) / 100).tolist())
    mwork = ((v[:, 2] - v[:, 1]) / 100).max()
    print(f"{name:9s} L{l if p < 24 else '-'} {len(v):5d} {fs:11.2f} {lw:13.2f} {le:9.2f} {wait:9.2f} {work:9.2f} {mwork:9.2f}")
print(f"step span {(r[:, 2].max() - base) / 100:.2f} us")

# attention tasks of layer 3: wait done -> q barrier (DMA landed) -> LDS tiles -> HBM tiles
lib.lvx_debug_persist_att.restype = ctypes.c_int
lib.lvx_debug_persist_att.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
att = np.zeros(1024 * 4, dtype=np.uint64)
lib.lvx_debug_persist_att(att.ctypes.data_as(ctypes.c_void_p), att.nbytes)
att = att.reshape(1024, 4).astype(np.int64)
v3 = r[(r[:, 3] >> 32) == 20]
wd = {int((x[3] >> 8) & 0xffffff): x[1] for x in v3}
sp = []
for blk, (a0, a1, a2, _) in enumerate(att[:256]):
    if a0 and blk in wd:
        sp.append(((a0 - wd[blk]) / 100, (a1 - a0) / 100, (a2 - a1) / 100))
if sp:
    sp = np.array(sp)
    print("attention L3 (median / max us): wait-done -> q barrier %.2f / %.2f, LDS tiles %.2f / %.2f, HBM tiles %.2f / %.2f"
          % (np.median(sp[:, 0]), sp[:, 0].max(), np.median(sp[:, 1]), sp[:, 1].max(), np.median(sp[:, 2]), sp[:, 2].max()))
