"""llmvox_amd — MI355X-native (gfx950) LLMVoX streaming-TTS hot path.

The speech-token GPT decode step and the WavTokenizer decoder run as hand-written HIP
kernels in ``libllmvox_hip.so`` (C ABI: include/llmvox.h). This package is the host
side: weights, the ``ModelHandler`` drop-in, and the streaming scheduler.
"""
from . import config  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing the package must not need a GPU
    if name == "ModelHandler":
        from .handler import ModelHandler
        return ModelHandler
    if name in ("Engine", "build_engine"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
