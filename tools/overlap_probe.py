"""Development probe: how much does a concurrent codec decode slow the B=1 AR chain, and does
confining the codec to a subset of CUs (hipExtStreamCreateWithCUMask) help?"""
import ctypes, time
import torch
from llmvox_amd.engine import build_engine

hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(lo, hi, dev):
    words = [0] * 8
    for cu in range(lo, hi):
        words[cu // 32] |= 1 << (cu % 32)
    arr = (ctypes.c_uint32 * 8)(*words)
    s = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, arr) == 0
    return torch.cuda.ExternalStream(s.value, device=dev)


e = build_engine(0, "bf16", "bf16", max_streams=4, max_positions=4096, max_codec_frames=1024)
dev = e.device
n = 256
plan = torch.full((1, n), 100, dtype=torch.int32, device=dev)
slots = torch.zeros(1, dtype=torch.int32, device=dev)
rowstep = torch.zeros(1, dtype=torch.int32, device=dev)
tok = torch.zeros(1, n, dtype=torch.int32, device=dev)
codes = torch.randint(0, 4096, (1, 256), dtype=torch.int32, device=dev)
pcm = torch.empty(1, 320 * 256, device=dev)


def ar(stream):
    with torch.cuda.stream(stream):
        e.reset_slot(0); rowstep.zero_()
        e.ar_steps(n, slots, plan, rowstep, tok)


def run(main, side, with_codec, reps=5):
    ts = []
    for r in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if with_codec:
            with torch.cuda.stream(side):
                e.decode_codes(codes, 0, out=pcm)
        ar(main)
        main.synchronize()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        ts.append((t1 - t0) * 1e3)
    return min(ts), sorted(ts)[len(ts) // 2]


main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(device=dev)
ar(main); torch.cuda.synchronize()
with torch.cuda.stream(side):
    e.decode_codes(codes, 0, out=pcm)
torch.cuda.synchronize()
print("AR alone            min/med ms: %.3f %.3f" % run(main, side, False))
print("AR + codec (shared) min/med ms: %.3f %.3f" % run(main, side, True))
for lo, hi in ((0, 32), (0, 64), (192, 256)):
    ms = masked_stream(lo, hi, dev)
    with torch.cuda.stream(ms):
        e.decode_codes(codes, 0, out=pcm)
    torch.cuda.synchronize()
    print(f"AR + codec on CUs [{lo},{hi})   min/med ms: %.3f %.3f" % run(main, ms, True))
    mm = masked_stream(hi if lo == 0 else 0, 256 if lo == 0 else lo, dev)
    ar(mm); torch.cuda.synchronize()
    print(f"  + AR on the other CUs       min/med ms: %.3f %.3f" % run(mm, ms, True))
    print(f"  AR alone on the other CUs   min/med ms: %.3f %.3f" % run(mm, ms, False))
# codec alone timings
for lo, hi in ((0, 256), (0, 64)):
    ms = masked_stream(lo, hi, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(ms):
        for _ in range(5):
            e.decode_codes(codes, 0, out=pcm)
    ms.synchronize()
    print(f"codec alone on CUs [{lo},{hi}): %.3f ms" % ((time.perf_counter() - t0) * 1e3 / 5))
