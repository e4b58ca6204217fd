"""Development probe: where a loaded first chunk's time goes (bench.first_chunk_latency_loaded: a fresh
stream joining a FusedScheduler that decodes 31 busy streams). FusedScheduler is wrapped to stamp, per
fresh stream: its admission (open_stream), the launch of the first chunk that carries it (and that
chunk's steps and rows), that chunk's completion on the host, and the delivery of its first dump.
usage: python tools/latency_trace.py [reps] [max_chunk]"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402
from llmvox_amd import streaming as S  # noqa: E402
from llmvox_amd.engine import build_engine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 24
mc = int(sys.argv[2]) if len(sys.argv) > 2 else 64
e = build_engine(0, "bf16", "bf16", max_streams=32, max_positions=8192, max_codec_frames=32 * 256)
torch.cuda.set_stream(torch.cuda.Stream(device=e.device))
F = S.FusedScheduler
orig = {k: getattr(F, k) for k in ("open_stream", "_launch", "_complete", "_deliver")}
rec = {}
count = [0]
log = []


def open_stream(self, *a, **kw):
    st = orig["open_stream"](self, *a, **kw)
    count[0] += 1
    if count[0] > 31:
        rec[st] = {"admit": time.perf_counter()}
    return st


def _launch(self, ready, plans, n):
    t = time.perf_counter()
    r = orig["_launch"](self, ready, plans, n)
    for st, _ in ready:
        if st in rec and "launch" not in rec[st]:
            rec[st].update(launch=t, n=n, rows=len(ready), inflight=len(self.inflight))
    log.append(("launch", t, n, len(ready)))
    return r


def _complete(self, ch):
    t0 = time.perf_counter()
    r = orig["_complete"](self, ch)
    t1 = time.perf_counter()
    for st in ch.ready:
        if st in rec and "complete" not in rec[st]:
            rec[st].update(complete_start=t0, complete=t1)
    log.append(("complete", t0, t1, ch.n))
    return r


def _deliver(self, pcm, order, ready):
    r = orig["_deliver"](self, pcm, order, ready)
    t = time.perf_counter()
    for st in ready:
        if st in rec and "deliver" not in rec[st] and any(isinstance(x, bytes) for x in st.events):
            rec[st]["deliver"] = t
    return r


for k, f in (("open_stream", open_stream), ("_launch", _launch), ("_complete", _complete), ("_deliver", _deliver)):
    setattr(F, k, f)
p50, p90, mx, n = bench.first_chunk_latency_loaded(e, busy=31, reps=reps, seed=99, max_chunk=mc)
print(f"p50 {p50:.2f} p90 {p90:.2f} max {mx:.2f} ms over {n} joins (max_chunk {mc})")
print("per join, ms from admission: first launch carrying it (steps, rows, chunks in flight), host completion of "
      "that chunk, first dump delivered")
for st, r in rec.items():
    a = r["admit"]
    f = lambda k: (r[k] - a) * 1e3 if k in r else float("nan")  # noqa: E731
    print(f"launch {f('launch'):6.2f} (n {r.get('n')}, rows {r.get('rows')}, inflight {r.get('inflight')})  "
          f"complete {f('complete_start'):6.2f}-{f('complete'):6.2f}  deliver {f('deliver'):6.2f}")
e.close()
