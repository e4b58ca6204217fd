"""Encoder timing (HIP events on the stream lvx_encode runs on): B streams x N samples of audio,
seconds of audio encoded per second, plus the CPU oracle on one stream for comparison.
usage: python tools/encoder_probe.py [reps]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from llmvox_amd import weights as LW  # noqa: E402
from llmvox_amd.encoder import WavEncoder  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
cb = LW.synthetic_codec(1234)[LW.CODEBOOK_KEY]
we = LW.synthetic_encoder(1234)
e = WavEncoder(0, we, cb, max_samples=32 * 24000 * 10)
s = torch.cuda.current_stream()
for B, secs in ((1, 1), (1, 10), (8, 10), (32, 10)):
    N = 24000 * secs
    audio = torch.randn(B, N, device="cuda") * 0.3
    e.encode(audio)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        e.encode(audio)
    b.record(s)
    b.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"encode {B} x {secs} s: {ms:8.2f} ms  {B * secs / ms * 1e3:8.1f} s of audio / s", flush=True)
from oracle import reference_cpu as R  # noqa: E402
We = R.to_torch(LW.encoder_effective(we))
audio = torch.randn(1, 24000) * 0.3
R.encode_infer(We, torch.from_numpy(cb), audio)
t0 = time.perf_counter()
R.encode_infer(We, torch.from_numpy(cb), audio)
dt = time.perf_counter() - t0
print(f"CPU oracle (torch threads {torch.get_num_threads()}): 1 x 1 s in {dt * 1e3:.1f} ms  {1 / dt:.1f} s of audio / s")
