"""configs[3]'s dump sizes on the GPU, fp32 parity mode, against the reference's own output.

The reference grows the dump 10 / 160 -> x3 -> 1280 (streaming_server.py:357-376,
configs/inference_config.py:30-33), so real dumps have L in {270, 480, 810, 1280} frames, and the
codec's AttnBlock attends over the whole dump (WavTokenizer/decoder/models.py:107-127: L x L
scores). Fixtures (tests/golden/make_golden.py, from the imported reference):
  * codec_large_golden.npz: PCM of seeded codes at L = 270 / 480 / 810 / 1280 (RMS, 512-sample
    head and tail, every 64th sample);
  * stream_long_golden.npz: the reference's audio_generator_sync on the config sentence run until
    replica 0's dumps reach 1280 (10 + 30 + 90 + 270 + 810 + 1280 = 2490 model calls: ids, margins,
    every chunk's summary) and replica 1's (160 + 480 + 1280 = 1920 calls).
Bars (BASELINE north_star): ids bit-exact; waveform max |diff| < 2e-4 and RMS diff < 1e-5.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
WORDS = "The quick brown fox jumps over the lazy dog near the river bank.".split(" ")


@pytest.fixture(scope="module")
def eng():
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "fp32", "fp32", max_streams=2, max_positions=4096, max_codec_frames=2560)
    yield e
    e.close()


def _check_pcm(pcm, g, name):
    pcm = np.asarray(pcm, dtype=np.float32)
    assert pcm.size == int(g[f"{name}_len"])
    rms = np.sqrt(np.mean(pcm.astype(np.float64) ** 2))
    assert abs(rms - float(g[f"{name}_rms"])) < 1e-5, (name, rms, float(g[f"{name}_rms"]))
    for part, got in (("head", pcm[:512]), ("tail", pcm[-512:]), ("s64", pcm[::64])):
        d = got - g[f"{name}_{part}"]
        assert np.abs(d).max() < 2e-4, (name, part, np.abs(d).max())
        assert np.sqrt(np.mean(d.astype(np.float64) ** 2)) < 1e-5, (name, part)


@pytest.mark.parametrize("L", [270, 480, 810, 1280])
def test_codec_large_dump_matches_reference(eng, L):
    g = np.load(os.path.join(GOLDEN, "codec_large_golden.npz"))
    codes = torch.from_numpy(g[f"codes_{L}"]).to(eng.device)
    pcm = eng.decode_codes(codes).cpu().numpy()[0]
    _check_pcm(pcm, g, f"pcm_{L}")


def test_codec_two_large_dumps_batched(eng):
    """Two 1280-frame dumps in one call (two replicas at max_dump) == the reference per stream."""
    g = np.load(os.path.join(GOLDEN, "codec_large_golden.npz"))
    c = torch.from_numpy(g["codes_1280"])
    codes = torch.cat([c, c.flip(1)], 0).to(eng.device)
    pcm = eng.decode_codes(codes).cpu().numpy()
    _check_pcm(pcm[0], g, "pcm_1280")
    single = eng.decode_codes(codes[1:]).cpu().numpy()[0]
    assert np.abs(pcm[1] - single).max() < 1e-6


def _run_stream(eng, index, dump, n_chunks, max_chunk=256):
    from llmvox_amd.streaming import FusedScheduler
    sch = FusedScheduler(eng, max_chunk=max_chunk)
    st = sch.open_stream(index=index, dump_size=dump)
    for w in WORDS:
        st.feed(w)
    while sum(isinstance(e, bytes) for e in st.events) < n_chunks:
        assert sch.run_chunk() > 0
    sch.flush()
    chunks = [np.frombuffer(e, dtype=np.float32) for e in st.events if isinstance(e, bytes)]
    toks = list(st.tokens)
    sch.close_stream(st)
    return toks, chunks


def test_fused_scheduler_reaches_max_dump_replica0(eng):
    """Replica 0 through its whole dump schedule 10/30/90/270/810/1280 on the fused decode step:
    2,490 ids bit-exact and every chunk (up to the 1,280-frame one) against the reference's stream."""
    g = np.load(os.path.join(GOLDEN, "stream_long_golden.npz"))
    toks, chunks = _run_stream(eng, 0, 10, 6)
    ids = g["ids"]
    mism = np.nonzero(np.asarray(toks[:len(ids)]) != ids)[0]
    assert len(mism) == 0, f"first id mismatch at step {mism[0]} (golden margin {g['margins'][mism[0]]:.3g})"
    assert [len(c) for c in chunks[:6]] == g["sizes"].tolist()
    for i in range(6):
        _check_pcm(chunks[i], g, f"chunk{i}")


def test_fused_scheduler_reaches_max_dump_replica1(eng):
    """Replica 1's schedule 160/480/1280 on the same text (the reference's second queue)."""
    g = np.load(os.path.join(GOLDEN, "stream_long_golden.npz"))
    toks, chunks = _run_stream(eng, 1, 160, 3)
    n1 = int(g["r1_model_calls"])
    assert toks[:n1] == g["ids"][:n1].tolist()
    assert [len(c) for c in chunks[:3]] == g["r1_sizes"].tolist()
    for i in range(3):
        _check_pcm(chunks[i], g, f"r1_chunk{i}")


def test_two_replicas_batched_equal_alone(eng):
    """configs[3]'s pair: replica 0 and replica 1 batched in one scheduler (B = 2 decode steps,
    dumps of different lengths decoded in the same chunk loop) give each replica's solo stream."""
    from llmvox_amd.streaming import FusedScheduler
    g = np.load(os.path.join(GOLDEN, "stream_long_golden.npz"))
    sch = FusedScheduler(eng, max_chunk=256)
    sts = [sch.open_stream(index=0, dump_size=10), sch.open_stream(index=1, dump_size=160)]
    for st in sts:
        for w in WORDS:
            st.feed(w)
    while sum(isinstance(e, bytes) for e in sts[1].events) < 3:
        assert sch.run_chunk() > 0
    sch.flush()
    n1 = int(g["r1_model_calls"])
    for st in sts:
        assert st.tokens[:n1] == g["ids"][:n1].tolist()
    r1 = [np.frombuffer(e, dtype=np.float32) for e in sts[1].events if isinstance(e, bytes)]
    for i in range(3):
        _check_pcm(r1[i], g, f"r1_chunk{i}")
    r0 = [np.frombuffer(e, dtype=np.float32) for e in sts[0].events if isinstance(e, bytes)]
    for i in range(5):  # 10 + 30 + 90 + 270 + 810 = 1200 <= 1920 tokens
        _check_pcm(r0[i], g, f"chunk{i}")
    for st in sts:
        sch.close_stream(st)
