"""Development probe: does a one-rank NCCL (RCCL) process group change the host-side latency of the
one-GPU paths? Times the idle first-chunk latency (bench.first_chunk_latency) and a small
kernel + Event.synchronize round trip before the group exists, with it, and after it is destroyed.
usage: python tools/dist_latency_probe.py [backend nccl|gloo] [calls per phase]"""
import statistics
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from llmvox_amd.engine import build_engine  # noqa: E402


def roundtrip(n=200):
    x = torch.zeros(1024, device="cuda")
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        x.add_(1.0)
        ev = torch.cuda.Event()
        ev.record()
        ev.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(ts)


backend = sys.argv[1] if len(sys.argv) > 1 else "nccl"
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
torch.cuda.set_device(0)
e = build_engine(0, "bf16", "bf16", max_streams=32, max_positions=8192, max_codec_frames=32 * 256)
torch.cuda.set_stream(torch.cuda.Stream(device=e.device))
for phase in ("no group", f"one-rank {backend} group", "group destroyed"):
    if phase.startswith("one-rank"):
        if backend == "nccl":
            dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda:0"))
            t = torch.ones(1, device="cuda")
        else:
            dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)
            t = torch.ones(1)
        dist.all_reduce(t)
        torch.cuda.synchronize()
    elif phase == "group destroyed":
        dist.destroy_process_group()
    rt = roundtrip()
    lat = [bench.first_chunk_latency(e) for _ in range(calls)]
    print(f"{phase:22s} kernel + event sync round trip {rt:7.1f} us; idle first chunk p50 "
          + " / ".join(f"{v:.3f}" for v in lat) + " ms", flush=True)
e.close()
