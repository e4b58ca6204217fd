"""Development probe: FusedScheduler throughput (the service's scheduler, overlapped) with 32 busy
replica streams at several max_chunk values: tokens consumed per second over a fixed wall time, text
topped up as streams run dry (the same load as bench.first_chunk_latency_loaded, without joins).
usage: python tools/sched_throughput_probe.py [seconds] [max_chunk ...]"""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from llmvox_amd.engine import build_engine  # noqa: E402
from llmvox_amd.streaming import FusedScheduler  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
mcs = [int(v) for v in sys.argv[2:]] or [64, 32]
e = build_engine(0, "bf16", "bf16", max_streams=32, max_positions=8192, max_codec_frames=32 * 256)
torch.cuda.set_stream(torch.cuda.Stream(device=e.device))
rng = np.random.default_rng(5)
words = lambda n: " ".join(bench.random_sentence(rng) for _ in range(n)).split(" ")  # noqa: E731
for rep in range(2):
    for mc in mcs:
        sched = FusedScheduler(e, max_chunk=mc, to_bytes=True, overlap=True)
        sts = []
        for i in range(32):
            st = sched.open_stream(index=i % 2, dump_size=10 if i % 2 == 0 else 160)
            for w in words(24):
                st.feed(w)
            sts.append(st)
        for _ in range(4):  # warm-up (graph capture at this B)
            sched.run_chunk()
        n0 = sum(len(st.tokens) for st in sts)
        launches = []
        orig_launch = sched._launch

        def _launch(ready, plans, n, _o=orig_launch):
            launches.append((n, len(ready)))
            return _o(ready, plans, n)
        sched._launch = _launch
        waits = [0.0]

        def waiter(ev):
            t = time.perf_counter()
            ev.synchronize()
            waits[0] += time.perf_counter() - t
        sched.waiter = waiter
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < secs:
            for st in sts:
                if st.m.next_text_id() is None:
                    for w in words(8):
                        st.feed(w)
            sched.run_chunk()
        sched.flush()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n = sum(len(st.tokens) for st in sts) - n0
        steps = [a for a, _ in launches]
        print(f"max_chunk {mc:3d}: {n / dt:9.1f} tokens/s over {dt:.2f} s ({n} tokens, 32 streams); {len(launches)} chunks, "
              f"mean {np.mean(steps):.1f} steps x {np.mean([b for _, b in launches]):.1f} rows; host waited on the device "
              f"{waits[0]:.2f} s", flush=True)
        for st in list(sched.streams):
            sched.close_stream(st)
        sched.close()
        for s in range(32):
            e.reset_slot(s)
e.close()
