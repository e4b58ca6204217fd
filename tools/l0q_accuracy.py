"""Development check: the teacher-forced test's error measures (tests/test_gpu_teacher_forced.py: max
|logit - reference logit| at the recorded steps, agreement with the reference's ids) for option sets
of the bf16 step, e.g. layer 0's c_attn from the q0 tables (option l0q 1) against the GEMM (l0q 0).
usage: python tools/l0q_accuracy.py [kv dtype] [B] ['opt=v,...' ...]
(defaults: bf16 KV at B = 32 / fp8 KV at B = 16, option sets 'l0q=0' 'l0q=1')"""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import llmvox_amd.engine as E  # noqa: E402
import test_gpu_teacher_forced as T  # noqa: E402

kvd = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else (32 if kvd == "bf16" else 16)
specs = sys.argv[3:] or ["l0q=0", "l0q=1"]
g = np.load(os.path.join(T.GOLDEN, "ar_golden.npz"))
ids, margins, text, keep = g["ids"], g["margins"], g["text_ids"].tolist(), g["logit_steps"].tolist()
build = E.build_engine
for spec in specs:
    opts = [kv.split("=") for kv in spec.split(",") if kv]

    def build_q(*a, _o=opts, **k):
        e = build(*a, **k)
        for name, v in _o:
            e.set_option(name, int(v))
        return e
    E.build_engine = build_q
    allp, kept, rows_ok = T._teacher_forced("bf16", kvd, B, ids, text, keep, 512)
    err = max(float(np.abs(kept[s] - g["logits"][k]).max()) for k, s in enumerate(keep))
    rms = float(np.sqrt(np.mean([np.mean((kept[s] - g["logits"][k]) ** 2) for k, s in enumerate(keep)])))
    print(f"[{spec}] kv={kvd} B={B}: agreement {float((allp[:, 0] == ids).mean()):.4f}, max |dlogit| {err:.4g}, "
          f"rms dlogit {rms:.4g}, rows agree {rows_ok}", flush=True)
