"""Development A/B: bench.first_chunk_latency_loaded (31 busy streams, the service's 64-step chunks,
a fresh stream's enqueue -> first dump on the host) with more repetitions than the bench line's, on an
engine shaped as the bench's (32 streams, 8,192 positions), graph replay on a side stream.
usage: python tools/latency_ab.py [reps] [mode ...]
modes: "base" (as the bench line), "nodump" (the busy streams never dump: no codec work queued ahead
of the fresh stream's first dump), "mc32" (32-step chunks)."""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402
from llmvox_amd import streaming as S  # noqa: E402
from llmvox_amd.engine import build_engine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 32
modes = sys.argv[2:] or ["base"]
e = build_engine(0, "bf16", "bf16", max_streams=32, max_positions=8192, max_codec_frames=32 * 256)
torch.cuda.set_stream(torch.cuda.Stream(device=e.device))
orig_open = S.FusedScheduler.open_stream
for mode in modes:
    opened = [0]

    def open_stream(self, index=0, dump_size=10, sink=None, **kw):
        opened[0] += 1
        if mode == "nodump" and opened[0] <= 31:  # the busy streams
            dump_size = 1 << 30
        return orig_open(self, index=index, dump_size=dump_size, sink=sink, **kw)

    S.FusedScheduler.open_stream = open_stream
    try:
        for rep in range(3):
            opened[0] = 0
            p50, p90, mx, n = bench.first_chunk_latency_loaded(e, busy=31, reps=reps, seed=99 + rep,
                                                              max_chunk=32 if mode == "mc32" else 64)
            print(f"{mode:7s} loaded first chunk p50 {p50:.2f} ms p90 {p90:.2f} ms max {mx:.2f} ms ({n} joins)",
                  flush=True)
    finally:
        S.FusedScheduler.open_stream = orig_open
e.close()
