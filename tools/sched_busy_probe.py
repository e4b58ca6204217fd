"""Development probe: how busy is the decode stream in configs[3]'s service loop? Runs bench.py's
configs[3] (FusedScheduler, one stream, utterances of 2,048 tokens, one codec call per dump) with
engine.ar_steps wrapped in timing events, and prints per timed utterance: wall time, the decode
stream's busy time (sum of the ar_steps calls' event spans, each call's span includes any time its
first kernel waited), the gaps between consecutive calls, and the tokens.
usage: python tools/sched_busy_probe.py [utterances]"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402
from llmvox_amd import engine as engine_mod  # noqa: E402

spans = []
orig = engine_mod.Engine.ar_steps


def timed(self, n, *a, **k):
    s = torch.cuda.current_stream(self.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    r = orig(self, n, *a, **k)
    e1.record(s)
    spans.append((e0, e1, n))
    return r


engine_mod.Engine.ar_steps = timed
K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
sys.argv = ["bench.py", "--config", "3", "--steps", str(K), "--warmup", "1", "--no-cpu-baseline", "--no-probe"]
bench.main()
torch.cuda.synchronize()
gaps, busy = [], 0.0
for k, (e0, e1, n) in enumerate(spans):
    busy += e0.elapsed_time(e1)
    if k:
        gaps.append((spans[k - 1][1].elapsed_time(e0), spans[k - 1][2], n))
total = spans[0][0].elapsed_time(spans[-1][1])
idle = sum(g for g, _, _ in gaps)
big = sorted(gaps, reverse=True)[:12]
print(f"ar_steps calls {len(spans)}, first->last {total:.1f} ms, busy {busy:.1f} ms, idle between calls {idle:.2f} ms")
print("largest gaps (ms, steps before, steps after):", [(round(g, 3), a, b) for g, a, b in big])
print("gaps > 0.05 ms:", sum(1 for g, _, _ in gaps if g > 0.05), "of", len(gaps))
