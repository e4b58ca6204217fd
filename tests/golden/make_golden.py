"""Generate the golden fixtures of the hot path by running the REFERENCE itself.

Run in the build container only (the reference checkout is not on the GPU box):

    python tests/golden/make_golden.py [/root/reference]

It imports the reference's own modules (src/model.py GPT, WavTokenizer's
decoder, streaming_server.audio_generator_sync) with two import stubs for
packages the image lacks (torchaudio, soundfile — used only by classes that
are off the decode path), loads the seeded synthetic weights of
``llmvox_amd.weights`` into them, and records inputs + outputs as small
``.npz`` / ``.json`` files next to this script.  Nothing of the reference's
source is copied; only the numbers it produced.
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import queue
import sys
import threading
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

SENTENCE = "The quick brown fox jumps over the lazy dog near the river bank."


def _install_stubs():
    import transformers  # noqa: F401  (must be imported before the torchaudio stub)
    import importlib.machinery as M
    ta = types.ModuleType("torchaudio")
    ta.__spec__ = M.ModuleSpec("torchaudio", None)
    fn = types.ModuleType("torchaudio.functional")
    fnf = types.ModuleType("torchaudio.functional.functional")
    fnf._hz_to_mel = lambda *a, **k: None
    fnf._mel_to_hz = lambda *a, **k: None
    fn.functional = fnf
    ta.functional = fn
    tr = types.ModuleType("torchaudio.transforms")
    ta.transforms = tr
    sys.modules.update({"torchaudio": ta, "torchaudio.functional": fn,
                        "torchaudio.functional.functional": fnf, "torchaudio.transforms": tr})
    sf = types.ModuleType("soundfile")
    sf.__spec__ = M.ModuleSpec("soundfile", None)
    sys.modules["soundfile"] = sf


def _quiet():
    return contextlib.redirect_stdout(io.StringIO())


def load_reference(ref_root):
    _install_stubs()
    sys.path.insert(0, ref_root)
    sys.path.insert(0, os.path.join(ref_root, "WavTokenizer"))
    from llmvox_amd import weights as LW
    with _quiet():
        from src.model import GPT, GPTConfig
        from decoder.pretrained import WavTokenizer
        gpt = GPT(GPTConfig(n_layer=4, n_head=8, n_embd=768, block_size=8192, bias=False,
                            vocab_size=4096, dropout=0.0, is_train=False))
    gw, cw, tt = LW.synthetic_all(1234)
    sd = {k: torch.from_numpy(v) for k, v in gw.items()}
    missing, unexpected = gpt.load_state_dict(sd, strict=False)
    assert not unexpected and not [m for m in missing if not m.endswith("attn.bias")], (missing, unexpected)
    gpt.eval()
    yaml = os.path.join(ref_root, "WavTokenizer/configs/"
                        "wavtokenizer_smalldata_frame75_3s_nq1_code4096_dim512_kmeans200_attn.yaml")
    with _quiet():
        wt = WavTokenizer.from_hparams0802(yaml)
    csd = {k: torch.from_numpy(v) for k, v in cw.items()}
    missing, unexpected = wt.load_state_dict(csd, strict=False)
    assert not unexpected, unexpected
    dec_missing = [m for m in missing if m.startswith(("backbone.", "head.")) and m != "head.istft.window"]
    assert not dec_missing, dec_missing
    wt.eval()
    embed = torch.nn.Embedding(386, 256)
    embed.weight.data.copy_(torch.from_numpy(tt))
    return gpt, wt, embed


def _pcm_summary(name, p):
    """RMS (float64), 512-sample head and tail, every 64th sample of a PCM vector."""
    p = np.asarray(p, dtype=np.float32)
    return {f"{name}_rms": np.float64(np.sqrt(np.mean(p.astype(np.float64) ** 2))),
            f"{name}_head": p[:512].copy(), f"{name}_tail": p[-512:].copy(), f"{name}_s64": p[::64].copy(),
            f"{name}_len": np.int32(p.size)}


class RefHandler:
    """The ModelHandler members audio_generator_sync touches, backed by the
    reference modules (inference/model_handler.py:45-63)."""

    def __init__(self, gpt, wt, embed, tokenizer):
        self.device = torch.device("cpu")
        self.model = gpt
        self.wavtokenizer = wt
        self.llm_model = embed
        self.tokenizer = tokenizer


class _Stop(Exception):
    pass


def run_reference_scheduler(handler, words, index, dump_size, max_model_calls, timeout=600, record=None):
    """Drive the reference's own audio_generator_sync in a thread and return the
    list of items it put on the audio queue. ``record`` (a list) receives, per model call, the
    (id, top1-top2 margin) the reference's select (softmax -> argmax) makes of its logits."""
    import streaming_server as S
    text_q, audio_q = queue.Queue(), queue.Queue()
    for w in words:
        text_q.put(w)
    real_model = handler.model
    calls = {"n": 0}

    def counted(*a, **k):
        if calls["n"] >= max_model_calls:
            raise _Stop()
        calls["n"] += 1
        out = real_model(*a, **k)
        if record is not None:
            lg = out[0][0, -1]
            t2 = torch.topk(lg, 2).values
            record.append((int(torch.softmax(lg, -1).argmax().item()), float(t2[0] - t2[1])))
        return out

    handler.model = counted
    done = threading.Event()

    def body():
        try:
            with torch.inference_mode():
                S.audio_generator_sync(index, dump_size, handler, text_q, audio_q)
        except _Stop:
            pass
        finally:
            done.set()

    th = threading.Thread(target=body, daemon=True)
    th.start()
    finished = done.wait(timeout)
    handler.model = real_model
    items = []
    while not audio_q.empty():
        items.append(audio_q.get())
    return items, finished, calls["n"]


# ---- scripted fakes for the scheduler-trace fixtures -------------------------

class ScriptModel:
    def __init__(self, script):
        self.script = list(script)
        self.i = 0

    def __call__(self, emb, kvcache=None, targets=None):
        if self.i >= len(self.script):
            raise _Stop()
        tok = self.script[self.i]
        self.i += 1
        logits = torch.zeros(1, 1, 4096)
        logits[0, 0, tok] = 10.0
        return logits, None, (kvcache or []) + [emb.shape[1]]


class FakeWav:
    def codes_to_features(self, codes):
        if codes.dim() == 2:
            codes = codes.unsqueeze(1)
        f = torch.zeros(codes.shape[1], 512, codes.shape[2])
        f[:, 0, :] = codes[0].float()
        return f

    def decode(self, features, bandwidth_id=None):
        return features[:, 0, :].clone()  # [1, L]: the codes, so the dump is readable


class FakeEmbed:
    def __call__(self, ids):
        return torch.zeros(1, ids.shape[1], 256)


SCHED_CASES = [
    # name, words, index, dump, script
    ("eoa_mid", ["Hi", "there."], 0, 10, [5] * 23 + [453] + [7] * 30),
    ("dump_then_eoa", ["one", "two", "three."], 0, 4, [11] * 9 + [453] + [12] * 12),
    ("eoa_exact_dump", ["ab", "cd."], 1, 5, [3] * 4 + [453] + [4] * 10),
    ("end_generation", ["bye<|eot_id|>"], 0, 10, [9] * 6 + [453] + [8] * 5),
    ("mid_word_reset", ["abcdefgh."], 1, 3, [2, 453, 6, 6, 453, 1, 1, 1, 453, 5, 5, 5, 5]),
    ("grow_dumps", ["The", "quick", "brown", "fox."], 0, 2, [21] * 60),
]


def scheduler_traces(tokenizer):
    out = {}
    for name, words, index, dump, script in SCHED_CASES:
        h = RefHandler(ScriptModel(script), FakeWav(), FakeEmbed(), tokenizer)
        with _quiet():
            items, finished, n = run_reference_scheduler(h, words, index, dump, len(script) + 1, timeout=30)
        rec = []
        for it in items:
            if isinstance(it, (bytes, bytearray)):
                rec.append({"audio": np.frombuffer(it, dtype=np.float32).astype(int).tolist()})
            else:
                rec.append({"signal": it})
        out[name] = {"words": words, "index": index, "dump_size": dump, "script": script,
                     "items": rec, "model_calls": h.model.i}
    return out


def main(ref_root="/root/reference"):
    gpt, wt, embed = load_reference(ref_root)
    with _quiet():
        import streaming_server  # noqa: F401
    from oracle.scheduler_cpu import byt5_tokenizer
    tok = byt5_tokenizer()

    # --- a1: tokenisation of the config sentence, word by word (streaming_server.py:288-310)
    words = SENTENCE.split(" ")
    text_ids = []
    for i, w in enumerate(words):
        ids = tok(w.strip())["input_ids"]
        if w.endswith("."):
            ids = ids + [385]
        text_ids += ids

    # --- a2-a11: reference AR loop for one segment, 256 steps (decode loop semantics)
    n_steps = 256
    ids, margins, logits_keep = [], [], {}
    keep = [0, 1, 2, 3, 65, 66, 128, 255]
    hist, kv, prev = None, None, None
    cb = wt.feature_extractor.encodec.quantizer.vq.layers[0].codebook
    with torch.inference_mode(), _quiet():
        for i in range(n_steps):
            tid = text_ids[i] if i < len(text_ids) else 384
            te = embed(torch.tensor([[tid]]))
            se = torch.zeros(1, 1, 512) if i == 0 else \
                wt.codes_to_features(torch.tensor([[prev]])).permute(0, 2, 1)
            x = torch.nn.functional.normalize(torch.cat([te, se], dim=2), p=2, dim=2, eps=1e-8)
            hist = x if hist is None else torch.cat([hist, x], dim=1)
            logits, _, kv = gpt(hist, kvcache=kv)
            prev = int(torch.softmax(logits[:, -1, :], -1).argmax(-1).item())
            t2 = torch.topk(logits[0, -1], 2).values
            ids.append(prev)
            margins.append(float(t2[0] - t2[1]))
            if i in keep:
                logits_keep[i] = logits[0, -1].numpy().copy()
    np.savez_compressed(os.path.join(HERE, "ar_golden.npz"),
                        text_ids=np.array(text_ids, np.int32), ids=np.array(ids, np.int32),
                        margins=np.array(margins, np.float32),
                        logit_steps=np.array(keep, np.int32),
                        logits=np.stack([logits_keep[k] for k in keep]).astype(np.float32),
                        codebook_check=cb[:4, :8].numpy())
    print("AR: ids[:16]", ids[:16], "min margin", min(margins))

    # --- a3, a13-a21: codec decode of seeded codes at several chunk lengths
    rng = np.random.default_rng(7)
    codec = {}
    with torch.inference_mode(), _quiet():
        for L in (1, 2, 10, 30, 90, 160):
            codes = torch.from_numpy(rng.integers(0, 4096, size=(1, L)).astype(np.int64))
            feats = wt.codes_to_features(codes)
            bb = wt.backbone(feats, bandwidth_id=torch.tensor([0]))
            pcm = wt.decode(feats, bandwidth_id=torch.tensor([0]))
            codec[f"codes_{L}"] = codes.numpy().astype(np.int32)
            if L <= 90:
                codec[f"pcm_{L}"] = pcm.numpy().astype(np.float32)
            else:
                p = pcm.numpy()[0]
                codec[f"pcm_{L}_head"] = p[:512].astype(np.float32)
                codec[f"pcm_{L}_tail"] = p[-512:].astype(np.float32)
                codec[f"pcm_{L}_rms"] = np.float64(np.sqrt(np.mean(p.astype(np.float64) ** 2)))
            if L == 10:
                codec["backbone_10"] = bb.numpy().astype(np.float32)
                codec["features_10"] = feats.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "codec_golden.npz"), **codec)
    # the reference's large dumps (streaming_server.py:373-375: 10/160 -> x3 -> 1280):
    # RMS, 512-sample head and tail, and every 64th sample of the PCM
    big = {}
    with torch.inference_mode(), _quiet():
        for L in (270, 480, 810, 1280):
            codes = torch.from_numpy(rng.integers(0, 4096, size=(1, L)).astype(np.int64))
            pcm = wt.decode(wt.codes_to_features(codes), bandwidth_id=torch.tensor([0])).numpy()[0]
            big[f"codes_{L}"] = codes.numpy().astype(np.int32)
            big.update(_pcm_summary(f"pcm_{L}", pcm))
    np.savez_compressed(os.path.join(HERE, "codec_large_golden.npz"), **big)
    print("codec large: rms", {L: float(big[f"pcm_{L}_rms"]) for L in (270, 480, 810, 1280)})
    print("codec: pcm_10 rms", float(np.sqrt(np.mean(codec["pcm_10"] ** 2))))

    # --- end to end: the reference's own audio_generator_sync on the sentence
    h = RefHandler(gpt, wt, embed, tok)
    with _quiet():
        items, finished, n = run_reference_scheduler(h, words, 0, 10, 130 + 1)
    chunks = [np.frombuffer(it, dtype=np.float32) for it in items if isinstance(it, (bytes, bytearray))]
    sizes = [len(c) for c in chunks]
    print("stream chunks", sizes, "model calls", n)
    np.savez_compressed(os.path.join(HERE, "stream_golden.npz"), sizes=np.array(sizes, np.int32),
                        chunk0=chunks[0], chunk1=chunks[1], chunk2=chunks[2],
                        model_calls=np.int32(n))

    # --- the same stream run until replica 0's dumps reach max_dump_size:
    # 10 + 30 + 90 + 270 + 810 + 1280 = 2490 model calls (configs[3]'s dump sizes)
    rec = []
    h = RefHandler(gpt, wt, embed, tok)
    with _quiet():
        items, finished, n = run_reference_scheduler(h, words, 0, 10, 2490, timeout=3600, record=rec)
    chunks = [np.frombuffer(it, dtype=np.float32) for it in items if isinstance(it, (bytes, bytearray))]
    long = {"sizes": np.array([len(c) for c in chunks], np.int32), "model_calls": np.int32(n),
            "ids": np.array([r[0] for r in rec], np.int32), "margins": np.array([r[1] for r in rec], np.float32),
            "text_ids": np.array(text_ids, np.int32)}
    for i, c in enumerate(chunks):
        long.update(_pcm_summary(f"chunk{i}", c))
    # replica 1 (index 1, initial dump 160: 160 + 480 + 1280 = 1920 model calls) on the same text
    rec1 = []
    h = RefHandler(gpt, wt, embed, tok)
    with _quiet():
        items, finished, n1 = run_reference_scheduler(h, words, 1, 160, 1920, timeout=3600, record=rec1)
    chunks = [np.frombuffer(it, dtype=np.float32) for it in items if isinstance(it, (bytes, bytearray))]
    assert [r[0] for r in rec1] == long["ids"][:len(rec1)].tolist()  # the dump policy never feeds back
    long["r1_sizes"] = np.array([len(c) for c in chunks], np.int32)
    long["r1_model_calls"] = np.int32(n1)
    for i, c in enumerate(chunks):
        long.update(_pcm_summary(f"r1_chunk{i}", c))
    np.savez_compressed(os.path.join(HERE, "stream_long_golden.npz"), **long)
    print("long stream chunks", long["sizes"].tolist(), "calls", n, "min margin", float(long["margins"].min()),
          "replica 1 chunks", long["r1_sizes"].tolist())

    # --- scheduler control traces with scripted tokens
    tr = scheduler_traces(tok)
    with open(os.path.join(HERE, "sched_golden.json"), "w") as f:
        json.dump(tr, f, indent=1)
    print("scheduler traces:", {k: len(v["items"]) for k, v in tr.items()})

    # --- text cleaning (streaming_server.py:106-149)
    import streaming_server as SS
    texts = ["  **Hi**  - there #1 & you@x ... 1,000 a/b c\\d 5.", "Step 2. then 3.14 and 2.", "a...b", "x--y",
             "#tag @me & you", "1,234,567 items", "path/to//file", "it's *fine*", "end.<|eot_id|>"]
    with open(os.path.join(HERE, "clean_text_golden.json"), "w") as f:
        json.dump({t: SS.clean_text(t) for t in texts}, f, indent=0)

    # --- tokenizer cases
    cases = ["The", "quick", "bank.", "EOS", "a[PAD]b", "é", "</s>x", "<pad>", " hi ", "<extra_id_0>",
             "x<extra_id_5>y", "<unk>", "a EOS b", "EOSEOS", "", "日本", "it's", "3.14", "tide<|eot_id|>",
             "a </s> b", "[PAD]EOS", "<extra_id_124>", "<extra_id_125>", "x  </s>  y"]
    with open(os.path.join(HERE, "tokenizer_golden.json"), "w") as f:
        json.dump({c: tok(c)["input_ids"] for c in cases}, f, indent=0, ensure_ascii=False)
    sys.stdout.flush()
    os._exit(0)  # the reference's daemon threads may still be blocked on queues


if __name__ == "__main__":
    main(*sys.argv[1:])
