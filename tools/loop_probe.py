"""Development probe: bench.py's chunk loop with parts switched off, to locate per-chunk overhead."""
import os, time
import torch
from llmvox_amd.engine import build_engine

S = int(os.environ.get("LP_S", "1"))
e = build_engine(0, "bf16", "bf16", max_streams=S, max_positions=8192, max_codec_frames=S * 256)
dev = e.device
chunk, K = 256, 4
mine = torch.full((S, K * chunk), 100, dtype=torch.int32, device=dev)
slots = torch.arange(S, dtype=torch.int32, device=dev)
text_plan = torch.empty(S, chunk, dtype=torch.int32, device=dev)
rowstep = torch.zeros(S, dtype=torch.int32, device=dev)
tok_bufs = [torch.zeros(S, chunk, dtype=torch.int32, device=dev) for _ in range(2)]
pcm_bufs = [torch.empty(S, 320 * chunk, device=dev) for _ in range(2)]
pcm_host = torch.empty(S, 320 * chunk, pin_memory=True)
codec_stream = torch.cuda.Stream(device=dev)
ev_ar = [torch.cuda.Event(), torch.cuda.Event()]
ev_codec = [torch.cuda.Event(), torch.cuda.Event()]


def run_chunk(c, codec=True, copy=True, overlap=True):
    i = c & 1
    main = torch.cuda.current_stream(dev)
    main.wait_event(ev_codec[i])
    text_plan.copy_(mine[:, c * chunk:(c + 1) * chunk])
    rowstep.zero_()
    e.ar_steps(chunk, slots, text_plan, rowstep, tok_bufs[i])
    ev_ar[i].record(main)
    if not codec:
        return
    st = codec_stream if overlap else main
    with torch.cuda.stream(st):
        st.wait_event(ev_ar[i])
        e.decode_codes(tok_bufs[i], 0, out=pcm_bufs[i])
        if copy:
            pcm_host.copy_(pcm_bufs[i], non_blocking=True)
        ev_codec[i].record(st)


for i in range(2):
    rowstep.zero_(); text_plan.copy_(mine[:, :chunk])
    e.ar_steps(17, slots, text_plan, rowstep, tok_bufs[i]); e.decode_codes(tok_bufs[i], 0, out=pcm_bufs[i])
torch.cuda.synchronize()
ncu = e.device_cus()
configs = [("full (bench)", {}, None), ("no codec", {"codec": False}, None),
           ("codec on main stream", {"overlap": False}, None)]
k = int(os.environ.get("LP_CODEC_CUS", "0"))  # one partition per process (each masked stream takes a HW queue)
if k:
    configs.append((f"partitioned AR {ncu - k} / codec {k} CUs", {}, (e.cu_stream(0, ncu - k), e.cu_stream(ncu - k, k))))
    configs.append((f"codec only partitioned ({k} CUs)", {}, (torch.cuda.current_stream(dev), e.cu_stream(ncu - k, k))))
lo, hi = torch.cuda.Stream.priority_range()
print("stream priority range (low, high):", lo, hi)
configs.append(("priority: AR high, codec low", {}, (torch.cuda.Stream(device=dev, priority=hi),
                                                      torch.cuda.Stream(device=dev, priority=lo))))
configs.append(("AR alone on a torch stream", {"codec": False}, (torch.cuda.Stream(device=dev), None)))
configs.append(("AR alone on a high-priority stream", {"codec": False}, (torch.cuda.Stream(device=dev, priority=hi), None)))
configs.append(("AR alone on an all-CU masked stream", {"codec": False}, (e.cu_stream(0, 0), None)))
only = os.environ.get("LP_ONLY")
if only:
    configs = [c for c in configs if c[0].startswith(only)]
for name, kw, parts in configs:
    ar_st = parts[0] if parts else torch.cuda.current_stream(dev)
    if parts and parts[1] is not None:
        codec_stream = parts[1]
    else:
        codec_stream = torch.cuda.Stream(device=dev)
    best = 1e9
    with torch.cuda.stream(ar_st):
        for rep in range(3):
            for s_ in range(S):
                e.reset_slot(s_)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for c in range(K):
                run_chunk(c, **kw)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
    print(f"S={S} {name:34s}: {best / K:.3f} ms/chunk")
