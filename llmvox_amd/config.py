"""Static shapes and runtime constants of the LLMVoX streaming-TTS hot path.

Every constant cites where the reference defines it (paths relative to the
reference checkout):

* speech-token GPT:   configs/train_config.py:70-75 (n_layer 4, n_head 8, n_embd 768,
                      block_size 8192, bias False); vocab 4096 from train.py:163.
* text embedding:     inference/model_handler.py:88-105 (ByT5 embed, 384 byte ids +
                      "[PAD]" 384 + "EOS" 385 -> 386 rows, d_model 256).
* codec decoder:      WavTokenizer/configs/wavtokenizer_smalldata_frame75_3s_nq1_code4096_
                      dim512_kmeans200_attn.yaml:39-65.
* streaming policy:   configs/inference_config.py:30-41.
"""
from dataclasses import dataclass, field
from typing import Optional

# ---- speech-token GPT (src/model.py:135-146, configs/train_config.py:70-75) ----
N_LAYER = 4
N_HEAD = 8
N_EMBD = 768
HEAD_DIM = N_EMBD // N_HEAD  # 96
BLOCK_SIZE = 8192
VOCAB = 4096
D_FF = 4 * N_EMBD  # 3072, src/model.py:105
LN_EPS = 1e-5  # src/model.py:38

# ---- input construction (streaming_server.py:325-334) ----
TEXT_DIM = 256
SPEECH_DIM = 512
TEXT_VOCAB = 386
NORM_EPS = 1e-8  # F.normalize eps, streaming_server.py:334

# ---- codec (yaml:39-65, decoder/models.py, decoder/modules.py) ----
CODEBOOK_SIZE = 4096
CODEC_IN = 512
CODEC_DIM = 768
CODEC_FF = 2304
CODEC_LAYERS = 12
ADANORM_N = 4
GN_GROUPS = 32
GN_EPS = 1e-6  # decoder/models.py:16
CODEC_LN_EPS = 1e-6  # decoder/models.py:195, modules.py:72
N_FFT = 1280
HOP = 320
N_BINS = N_FFT // 2 + 1  # 641
SAMPLE_RATE = 24000
ISTFT_PAD = (N_FFT - HOP) // 2  # 480, spectral_ops.py:50
MAG_CLIP = 100.0  # heads.py:57

# ---- streaming / special ids (configs/inference_config.py:30-41) ----
PAD_TOKEN_ID = 384
EOS_TEXT_ID = 385  # streaming_server.py:309
EOA_TOKEN_ID = 453
INITIAL_DUMP_SIZE_1 = 10
INITIAL_DUMP_SIZE_2 = 160
MAX_DUMP_SIZE = 1280
MAX_AUDIO_LENGTH = 8000
EOS_TOKEN = "<|eot_id|>"
# configs/inference_config.py:29 (the LLM text streamer's system prompt, llm_streaming.py)
SYSTEM_PROMPT = ("You are a friendly voicebot that answers questions in a concise way and do not use "
                 "abbreviation.Give short responses")


@dataclass
class InferenceConfig:
    """Runtime config dict of the drop-in (mirrors configs/inference_config.py:4-54).

    Extra keys that the reference does not have:
      weights        "synthetic" (seeded, reference init scales) or "checkpoint".
      weight_dtype   "fp32" (parity mode, the reference runs fp32) or "bf16".
      kv_dtype       "fp32" | "bf16" | "fp8" (OCP e4m3fn KV cache).
      codec_dtype    None (the weight dtype) | "fp8" (e4m3fn codec weights, per-row scales; bf16 mode).
      max_streams    KV slots per device.
      max_positions  KV capacity per slot (<= block_size 8192).
      seed           seed of the synthetic weights.
    """
    wav_config_path: str = ""
    wav_model_path: str = ""
    encoder_model_path: str = ""
    tokenizer_path: str = ""
    llmvox_checkpoint_path: str = ""
    initial_dump_size_1: int = INITIAL_DUMP_SIZE_1
    initial_dump_size_2: int = INITIAL_DUMP_SIZE_2
    max_dump_size: int = MAX_DUMP_SIZE
    max_audio_length: int = MAX_AUDIO_LENGTH
    eos_token: str = EOS_TOKEN
    pad_token_id: int = PAD_TOKEN_ID
    eoa_token_id: int = EOA_TOKEN_ID
    tts_device_1: int = 0
    tts_device_2: int = 0
    weights: str = "synthetic"
    weight_dtype: str = "fp32"
    kv_dtype: str = "fp32"
    codec_dtype: Optional[str] = None
    max_streams: int = 8
    max_positions: int = BLOCK_SIZE
    max_codec_frames: int = MAX_DUMP_SIZE
    seed: int = 1234
    extra: dict = field(default_factory=dict)

    def __getitem__(self, k):  # dict-style access, as the reference uses config["..."]
        return getattr(self, k)

    def get(self, k, default=None):
        return getattr(self, k, default)


def default_config(**overrides) -> dict:
    """Plain dict form (the reference passes a dict to ModelHandler)."""
    cfg = InferenceConfig()
    d = {k: getattr(cfg, k) for k in cfg.__dataclass_fields__ if k != "extra"}
    d.update(overrides)
    return d
