"""Reference logits deep into the KV range the bench runs (bf16 parity pinned only at
positions < 256 while configs[2] decodes positions 0..1023).

Run in the build container only (the reference checkout is not on the GPU box):

    python tests/golden/make_golden_long_logits.py [/root/reference]

Imports the reference's own GPT / WavTokenizer / embedding with the seeded synthetic weights
(make_golden.load_reference), runs its decode loop (the ar_golden loop of make_golden.py, i.e.
streaming_server.py:323-346 for one segment) for 1,024 steps on the config sentence, checks that
its ids are the first 1,024 of stream_long_golden.npz (the reference's own scheduler run), and saves
the logits at positions 511, 767 and 1,023 to ar_long_golden.npz. Only numbers are stored.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402

KEEP = [511, 767, 1023]


def main(ref_root="/root/reference"):
    gpt, wt, embed = MG.load_reference(ref_root)
    long = np.load(os.path.join(HERE, "stream_long_golden.npz"))
    text_ids = long["text_ids"].tolist()
    n = KEEP[-1] + 1
    ids, keep = [], {}
    hist, kv, prev = None, None, None
    with torch.inference_mode(), MG._quiet():
        for i in range(n):
            tid = text_ids[i] if i < len(text_ids) else 384
            te = embed(torch.tensor([[tid]]))
            se = torch.zeros(1, 1, 512) if i == 0 else wt.codes_to_features(torch.tensor([[prev]])).permute(0, 2, 1)
            x = torch.nn.functional.normalize(torch.cat([te, se], dim=2), p=2, dim=2, eps=1e-8)
            hist = x if hist is None else torch.cat([hist, x], dim=1)
            logits, _, kv = gpt(hist, kvcache=kv)
            prev = int(torch.softmax(logits[:, -1, :], -1).argmax(-1).item())
            ids.append(prev)
            if i in KEEP:
                keep[i] = logits[0, -1].numpy().copy()
    assert ids == long["ids"][:n].tolist(), "the decode loop left the reference's own stream"
    np.savez_compressed(os.path.join(HERE, "ar_long_golden.npz"), logit_steps=np.array(KEEP, np.int32),
                        logits=np.stack([keep[k] for k in KEEP]).astype(np.float32),
                        ids=np.array(ids, np.int32))
    print("long logits at", KEEP, "max |logit|", [float(np.abs(keep[k]).max()) for k in KEEP])
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    main(*sys.argv[1:])
