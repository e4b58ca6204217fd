"""Golden vectors of the reference's WavTokenizer.encode_infer, produced by the
reference itself: imports /root/reference exactly as make_golden.py does (same stubs, same
synthetic decoder weights), loads the seeded synthetic encoder weights of
llmvox_amd.weights.synthetic_encoder into feature_extractor.encodec.encoder (weight_g / weight_v /
bias / LSTM keys of the reference's state_dict), marks the codebook initialised (a trained
checkpoint has inited = 1; otherwise the first forward would run k-means), and records for seeded
audio:

* the audio itself (inputs), the codes [1, B, T] of encode_infer (features = codebook rows of the
  codes: fixed by the codes);
* the encoder output before quantisation (full for short inputs, RMS + every 7th value otherwise);
* per frame the gap between the best and second-best quantiser score (which codes are robust to
  summation-order rounding).

usage: python tests/golden/make_golden_encoder.py [/root/reference]  -> tests/golden/encoder_golden.npz
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

CASES = ((2, 12000), (1, 6400), (3, 4800), (1, 1000), (1, 300))


def synth_audio(B, N, seed):
    """three sines (100-4000 Hz, 24 kHz) + noise, amplitude ~0.5"""
    rng = np.random.default_rng(seed)
    t = np.arange(N, dtype=np.float64) / 24000.0
    out = np.zeros((B, N), np.float64)
    for b in range(B):
        for _ in range(3):
            f, ph, a = rng.uniform(100, 4000), rng.uniform(0, 2 * np.pi), rng.uniform(0.1, 0.3)
            out[b] += a * np.sin(2 * np.pi * f * t + ph)
        out[b] += 0.05 * rng.standard_normal(N)
    return out.astype(np.float32)


def main(ref_root="/root/reference"):
    import make_golden as mg
    from llmvox_amd import weights as LW
    _, wt, _ = mg.load_reference(ref_root)
    fe = wt.feature_extractor
    we = LW.synthetic_encoder(1234)
    sd = {k[len("feature_extractor."):]: torch.from_numpy(v) for k, v in we.items()}
    missing, unexpected = fe.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert not [m for m in missing if m.startswith("encodec.encoder.")], missing
    vq = fe.encodec.quantizer.vq.layers[0]._codebook
    vq.inited.fill_(1.0)
    fe.eval()
    out = {}
    with torch.inference_mode():
        for i, (B, N) in enumerate(CASES):
            audio = synth_audio(B, N, 100 + i)
            a = torch.from_numpy(audio)
            feats, codes = wt.encode_infer(a, bandwidth_id=torch.tensor([0]))
            emb = fe.encodec.encoder(a.unsqueeze(1))
            x = emb.permute(0, 2, 1).reshape(-1, emb.shape[1])
            e = vq.embed.t()
            dist = -(x.pow(2).sum(1, keepdim=True) - 2 * x @ e + e.pow(2).sum(0, keepdim=True))
            top = torch.topk(dist, 2, dim=-1).values
            assert torch.equal(feats, torch.nn.functional.embedding(codes[0], vq.embed).transpose(1, 2))
            tag = f"{B}x{N}"
            out[f"audio_{tag}"] = audio
            out[f"codes_{tag}"] = codes.numpy().astype(np.int32)
            out[f"gap_{tag}"] = (top[:, 0] - top[:, 1]).numpy().astype(np.float32)
            en = emb.numpy().astype(np.float32)
            if en.size <= 16384:
                out[f"emb_{tag}"] = en
            else:
                out[f"emb_{tag}_rms"] = np.float64(np.sqrt(np.mean(en.astype(np.float64) ** 2)))
                out[f"emb_{tag}_every7"] = en.reshape(-1)[::7].copy()
                out[f"emb_{tag}_shape"] = np.array(en.shape, np.int32)
            print(tag, "T", codes.shape[-1], "codes[:8]", codes.reshape(-1)[:8].tolist(),
                  "min gap", float(out[f"gap_{tag}"].min()), "emb rms", float(np.sqrt(np.mean(en ** 2))))
    np.savez_compressed(os.path.join(HERE, "encoder_golden.npz"), **out)


if __name__ == "__main__":
    main(*sys.argv[1:])
