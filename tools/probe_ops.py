"""Per-op probe times (bench.probe_kernels) at B streams, KV position P, for option sets.
usage: python tools/probe_ops.py B P 'opt=v,opt=v' ['opt=v' ...]"""
import sys
import torch
sys.path.insert(0, ".")
from bench import probe_kernels
from llmvox_amd.engine import build_engine

S, P = int(sys.argv[1]), int(sys.argv[2])
e = build_engine(0, "bf16", "bf16", max_streams=S, max_positions=max(1024, P + 1), max_codec_frames=256)
slots = torch.arange(S, dtype=torch.int32, device=e.device)
for spec in sys.argv[3:] or [""]:
    opts = [kv.split("=") for kv in spec.split(",") if kv]
    for k, v in opts:
        e.set_option(k, int(v))
    for s in range(S):
        e.set_slot(s, P - 1, 0)
    r = probe_kernels(e, slots, P, 2, 2)
    tot = sum(v["share_us_per_step"] for v in r.values() if "share_us_per_step" in v)
    print(f"B={S} P={P} [{spec}] step~{tot:.1f} us: " + ", ".join(f"{v['name'].split(' ')[1] if ' ' in v['name'] else v['name']} {v['avg_us']:.2f}" for v in r.values()), flush=True)
    for k, v in opts:
        e.set_option(k, {"bt": 1, "bt_rows": 16, "bt_merge": 0, "mfma_ln": 8, "attn_blocks": 256}.get(k, 0))
