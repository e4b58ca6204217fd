"""Writes the three checkpoints ModelHandler(weights="checkpoint") reads, in the reference's own save
layouts, from the seeded synthetic weights (the real checkpoints are not available offline):

* LLMVoX GPT: src/utils.py:147-153 ``save_checkpoint`` -> {'model', 'optimizer', 'model_args',
  'iter_num', 'config'}; the state dict as torch.compile leaves it (``_orig_mod.`` prefixes) and an
  AdamW state dict after one step (what train.py's optimizer saves);
* WavTokenizer: a Lightning checkpoint {'state_dict', 'epoch', 'global_step',
  'pytorch-lightning_version', 'optimizer_states', 'lr_schedulers'} whose state_dict also holds
  the training-only modules that pretrained.py:101-105 filters out;
* the ByT5 encoder directory (model.safetensors with ``shared.weight`` [384, 256]) that
  model_handler.py:88-105 resizes to 386 rows.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from llmvox_amd import weights as LW


def write_llmvox_ckpt(path, gw, block_size=8192, compiled=True):
    sd = {}
    for i, (k, v) in enumerate(gw.items()):
        t = torch.from_numpy(np.ascontiguousarray(v))
        if k == "transformer.wpe.weight":
            t = t[:block_size].clone()
        sd[("_orig_mod." + k) if compiled else k] = t
    # a real AdamW state after one step over two small parameters
    ps = [torch.nn.Parameter(torch.randn(4, 3)), torch.nn.Parameter(torch.randn(3))]
    opt = torch.optim.AdamW(ps, lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1)
    (ps[0].sum() + ps[1].sum()).backward()
    opt.step()
    model_args = {"n_layer": 4, "n_head": 8, "n_embd": 768, "block_size": block_size, "bias": False,
                  "vocab_size": 4096, "dropout": 0.0}
    config = {"out_dir": "out", "eval_interval": 2000, "batch_size": 8, "learning_rate": 6e-4,
              "max_iters": 600000, "compile": True, "dtype": "bfloat16", "wandb_log": False,
              "checkpoint_filename": "ckpt.pt"}
    torch.save({"model": sd, "optimizer": opt.state_dict(), "model_args": model_args, "iter_num": 1234,
                "config": config}, path)


def write_wavtokenizer_ckpt(path, cw):
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in cw.items()}
    sd["multiperioddisc.discriminators.0.convs.0.weight"] = torch.zeros(32, 1, 5, 1)  # training-only
    sd["melspec_loss.mel_spec.spectrogram.window"] = torch.hann_window(16)
    torch.save({"state_dict": sd, "epoch": 3, "global_step": 1000, "pytorch-lightning_version": "1.8.6",
                "optimizer_states": [{"state": {}, "param_groups": [{"lr": 2e-4, "params": [0, 1]}]}],
                "lr_schedulers": [{"last_epoch": 1000}]}, path)


def write_t5_dir(path, tt):
    from safetensors.numpy import save_file
    os.makedirs(path, exist_ok=True)
    save_file({"shared.weight": np.ascontiguousarray(tt[:384])}, os.path.join(path, "model.safetensors"))


def write_all(root, seed=1234, block_size=8192):
    gw, cw, tt = LW.synthetic_all(seed)
    paths = {"llmvox_checkpoint_path": os.path.join(root, "ckpt_english_tiny.pt"),
             "wav_model_path": os.path.join(root, "wavtokenizer_large_speech_320_24k.ckpt"),
             "encoder_model_path": os.path.join(root, "byt5")}
    write_llmvox_ckpt(paths["llmvox_checkpoint_path"], gw, block_size)
    write_wavtokenizer_ckpt(paths["wav_model_path"], cw)
    write_t5_dir(paths["encoder_model_path"], tt)
    return paths
