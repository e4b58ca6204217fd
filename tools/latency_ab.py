"""Development A/B: bench.first_chunk_latency_loaded (31 busy streams, the service's 64-step chunks,
a fresh stream's enqueue -> first dump on the host) with more repetitions than the bench line's 12,
on an engine shaped as the bench's (32 streams, 8,192 positions), graph replay on a side stream.
usage: python tools/latency_ab.py [reps]"""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402
from llmvox_amd.engine import build_engine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 32
e = build_engine(0, "bf16", "bf16", max_streams=32, max_positions=8192, max_codec_frames=32 * 256)
torch.cuda.set_stream(torch.cuda.Stream(device=e.device))
for rep in range(2):
    p50, _, mx, _ = bench.first_chunk_latency_loaded(e, busy=31, reps=reps, seed=99 + rep)
    print(f"loaded first chunk p50 {p50:.2f} ms max {mx:.2f} ms", flush=True)
e.close()
