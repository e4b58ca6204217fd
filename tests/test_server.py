"""HTTP layer of the TTS service: request contract and byte framing with a fake service (CPU),
and the real service on the HIP path against the fused scheduler run directly (GPU)."""
import numpy as np
import pytest


class _FakeService:
    def __init__(self):
        self.error = None
        self.sessions = []
        self.texts = []

    def submit(self, text):
        self.texts.append(text)
        return text

    def chunks(self, session):
        for i in range(3):
            yield np.full(320 * (i + 1), i, dtype=np.float32).tobytes()


def test_tts_endpoint_streams_f32le_chunks():
    from fastapi.testclient import TestClient
    from llmvox_amd.server import create_app
    svc = _FakeService()
    client = TestClient(create_app(svc))
    r = client.post("/tts", json={"text": "hello world."})
    assert r.status_code == 200
    assert r.headers["content-type"] == "application/octet-stream"
    pcm = np.frombuffer(r.content, dtype=np.float32)
    assert pcm.size == 320 * 6 and (pcm[:320] == 0).all() and (pcm[-960:] == 2).all()
    assert svc.texts == ["hello world."]
    assert client.post("/tts", json={}).status_code == 422  # TTSRequest requires text
    assert client.get("/health").json()["ok"] is True


@pytest.mark.gpu
def test_tts_service_matches_fused_scheduler():
    """Replica 0 gets the first sentence (and the EOS token routed after the last one), replica 1
    the second. Replica 1's audio would follow replica 0's end-of-audio signal; synthetic weights
    never emit end-of-audio, so the response is replica 0's chunks plus its tail at max_tokens."""
    import torch  # noqa: F401
    from fastapi.testclient import TestClient
    from llmvox_amd.engine import build_engine
    from llmvox_amd.server import TTSService, create_app
    from llmvox_amd.streaming import FusedScheduler
    eng = build_engine(0, "fp32", "fp32", max_streams=8, max_positions=512, max_codec_frames=1280)
    text = "The quick brown fox. Jumps over the dog."
    svc = TTSService(eng, max_chunk=32, max_tokens=200)
    try:
        body = TestClient(create_app(svc)).post("/tts", json={"text": text}).content
    finally:
        svc.shutdown()
    # the same two replica streams through the scheduler directly
    sch = FusedScheduler(eng, max_chunk=32)
    a = sch.open_stream(index=0, dump_size=10)
    b = sch.open_stream(index=1, dump_size=160)
    for w in "The quick brown fox. <|eot_id|>".split():
        a.feed(w)
    for w in "Jumps over the dog.".split():
        b.feed(w)
    while min(len(a.tokens), len(b.tokens)) < 200:
        sch.run_chunk()
    sch.flush()
    ref = []
    for st in (a,):
        chunks = [x for x in st.events if isinstance(x, bytes)]
        ref += chunks
        tail = st.m.speech_outputs
        if tail:
            ref.append(eng.decode_codes(torch.tensor([tail], dtype=torch.int32, device=eng.device))
                       .cpu().numpy()[0].astype("float32").tobytes())
    got = np.frombuffer(body, dtype=np.float32)
    want = np.frombuffer(b"".join(ref), dtype=np.float32)
    assert got.shape == want.shape
    assert np.abs(got - want).max() < 1e-5
