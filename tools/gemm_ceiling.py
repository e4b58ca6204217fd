"""Development probe: what the vendor GEMM (torch.matmul -> hipBLASLt) reaches on the codec's GEMM
shapes at 8,192 frames (M) and at one 256-frame stream, bf16 in / fp32 accumulate, HIP events.
A practical ceiling for codec_kernels.hip's gemm_bf16 (no fused epilogues here).
usage: python tools/gemm_ceiling.py"""
import torch

SHAPES = [("pwconv1", 2304, 768), ("pwconv2", 768, 2304), ("qkv", 2304, 768), ("conv3", 768, 2304),
          ("head", 1282, 768), ("embed7", 768, 3584)]
dev = torch.device("cuda", 0)
for M in (8192, 256):
    for name, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            c = a @ w.t()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 50
        s.record()
        for _ in range(reps):
            c = a @ w.t()
        e.record()
        e.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        print(f"M {M:5d} {name:8s} N {N:4d} K {K:4d}: {us:7.1f} us  {2 * M * N * K / us / 1e6:7.1f} TFLOP/s",
              flush=True)
