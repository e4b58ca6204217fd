"""Development probe: do two torch (HIP) streams of one device run concurrently? With GPU_MAX_HW_QUEUES
(4 by default) hardware queues per process, streams beyond that share queues, and two streams on one
queue execute in order: a codec stream that lands on the decode stream's queue silently loses the
overlap. For streams 1..N of torch's pool, report whether each runs beside stream 0 (an event recorded
on it completes while a ~20 ms spin kernel occupies stream 0).
usage: python tools/stream_queue_probe.py [N]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from llmvox_amd.streams import runs_beside  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device("cuda:0")
base = torch.cuda.Stream(device=dev)
streams = [torch.cuda.Stream(device=dev) for _ in range(n)]
t0 = time.perf_counter()
res = [runs_beside(s, base) for s in streams]
print(f"{(time.perf_counter() - t0) * 1e3:.1f} ms for {n} checks")
print("stream i beside stream 0:", " ".join(f"{i}:{'yes' if r else 'NO'}" for i, r in enumerate(res, 1)))
