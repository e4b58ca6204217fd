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
    root = client.get("/").json()  # the reference's info endpoint (streaming_server.py:665-672)
    assert root["message"] == "Streaming TTS API" and root["usage"].startswith("POST /tts")
    r = client.options("/tts", headers={"Origin": "http://example.org", "Access-Control-Request-Method": "POST"})
    assert r.status_code == 200 and r.headers["access-control-allow-origin"] in ("*", "http://example.org")
    assert "access-control-allow-origin" not in TestClient(create_app(svc, cors=False)).get(
        "/", headers={"Origin": "http://example.org"}).headers


@pytest.mark.gpu
def test_tts_service_matches_fused_scheduler():
    """Replica 0 gets the first sentence (and the EOS token routed after the last one), replica 1
    the second. Replica 1's audio would follow replica 0's end-of-audio signal; synthetic weights
    never emit end-of-audio, so the response is replica 0's chunks plus its tail at max_tokens
    (each fed stream stops at its own max_tokens)."""
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
    while not (a.m.closed and b.m.closed):  # each stream stops at its own 200th token
        sch.run_chunk()
        for st in (a, b):
            if len(st.tokens) >= 200:
                st.m.closed = True
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


@pytest.fixture(scope="module")
def handler():
    from llmvox_amd.config import default_config
    from llmvox_amd.handler import ModelHandler
    return ModelHandler(default_config(weight_dtype="fp32", kv_dtype="fp32", max_streams=8, max_positions=1024),
                        device_id=0)


@pytest.mark.gpu
def test_one_sentence_without_period_ends_and_service_survives(handler):
    """'hello world' routes every word and the EOS token to replica 0; replica 1 never gets text.
    The request must still end (replica 0 stops at max_tokens), and the service must keep serving."""
    from fastapi.testclient import TestClient
    from llmvox_amd.server import TTSService, create_app
    svc = TTSService(handler.engine, max_chunk=32, max_tokens=96)
    try:
        client = TestClient(create_app(svc))
        for text in ("hello world", "again, no period"):
            r = client.post("/tts", json={"text": text})
            assert r.status_code == 200
            pcm = np.frombuffer(r.content, dtype=np.float32)
            n = pcm.size // 320  # dumps 10 + 30, then the tail: the cap is checked at chunk ends
            assert pcm.size % 320 == 0 and 96 <= n < 96 + 32, n
        assert client.get("/health").json() == {"ok": True, "sessions": 0}
    finally:
        svc.shutdown()


def _segment_tokens(eng, words, n):
    from llmvox_amd.streaming import FusedScheduler
    sch = FusedScheduler(eng, max_chunk=64)
    st = sch.open_stream(index=0, dump_size=10_000)
    for w in words:
        st.feed(w)
    while len(st.tokens) < n:
        assert sch.run_chunk() > 0
    sch.close_stream(st)
    return st.tokens[:n]


class _ScriptedLLM:
    """llm_streaming.StreamModel stand-in: predict() streams fixed pieces (leading spaces, as a
    tokenizer's streamer yields them) with small delays, so words reach the replicas while they
    decode; the prompt must be the request text."""

    def __init__(self, pieces):
        self.pieces = pieces
        self.requests = []

    def predict(self, request):
        import time
        self.requests.append(dict(request))

        def gen():
            for p in self.pieces:
                time.sleep(0.003)
                yield p
        return gen()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["text", "llm"])
def test_tts_two_replica_order_matches_reference_consumers(handler, mode):
    """POST /tts with an end-of-audio id that every segment emits (chosen from the synthetic model's
    own tokens): replica 0's chunks -> its switch signal -> replica 1's chunks -> its switch back ->
    replica 0's EOS segment -> 'end' (streaming_server.py:397-404,428-469). The response body must
    be the byte stream the reference's consumers produce on the same engine: two
    audio_generator_sync threads' queues (the drop-in ModelHandler) read in speaking order."""
    import queue
    from fastapi.testclient import TestClient
    from llmvox_amd import streaming as S
    from llmvox_amd.server import TTSService, create_app
    eng = handler.engine
    text = "The quick brown fox. Jumps over the dog."
    segs = [["The", "quick", "brown", "fox."], ["Jumps", "over", "the", "dog."], ["<|eot_id|>"]]
    toks = [_segment_tokens(eng, w, 160) for w in segs]
    # an id each segment first emits after its text is spoken (first occurrences at >= 30, 30, 3
    # steps: the sentences' text ids are ~22 and 2 long), so each segment ends with its own signal
    first = [{} for _ in toks]
    for f, tk in zip(first, toks):
        for i, t in enumerate(tk):
            f.setdefault(t, i)
    common = [t for t, i in first[0].items() if i >= 30 and first[1].get(t, -1) >= 30 and first[2].get(t, -1) >= 3]
    assert common, "no token that all three segments emit late enough"
    eoa = min(common, key=lambda t: max(first[0][t], first[1][t], first[2][t]))
    cfg = {"eoa_token_id": eoa}
    # the reference-shaped consumers, one replica after the other (each ends at its None word)
    qs_text, qs_audio = [queue.Queue(), queue.Queue()], [queue.Queue(), queue.Queue()]
    routed = S.route_text(text.split() + ["<|eot_id|>"], qs_text)
    assert routed[-1] == "<|eot_id|>"
    for q in qs_text:
        q.put(None)
    for i, dump in ((0, 10), (1, 160)):
        S.audio_generator_sync(i, dump, handler, qs_text[i], qs_audio[i], config=cfg)
    trace = [list(q.queue) for q in qs_audio]
    assert trace[0].count(1) == 1 and trace[0].count("end") == 1 and trace[1].count(0) == 1
    want = b"".join(S.audio_chunks(qs_audio[0], qs_audio[1], timeout=0.01,
                                   stop=lambda: all(q.empty() for q in qs_audio)))
    # mode "llm": the request text is the LLM prompt and the (scripted) reply is spoken, as the
    # reference's /tts does through text_streamer_producer (streaming_server.py:184-248): same
    # routed words, so the same byte stream, although they arrive while the replicas decode
    llm = _ScriptedLLM([" " + w if i else w for i, w in enumerate(text.split())] + ["<|eot_id|>"])
    svc = TTSService(eng, max_chunk=32, max_tokens=4000, eoa_id=eoa, stream_model=llm if mode == "llm" else None)
    try:
        body = TestClient(create_app(svc)).post("/tts", json={"text": "tell me about the fox" if mode == "llm" else text}).content
    finally:
        svc.shutdown()
    if mode == "llm":
        assert llm.requests == [{"system": svc.system_prompt, "prompt": "tell me about the fox"}]
    got, ref = np.frombuffer(body, dtype=np.float32), np.frombuffer(want, dtype=np.float32)
    assert got.shape == ref.shape and got.size > 0
    assert np.abs(got - ref).max() < 1e-5


@pytest.mark.gpu
def test_numeric_error_ends_only_the_request():
    """the B <= 2 fused MLP's range check (error bit 32: a non-finite partial) used to reach
    the service as a device failure, taking every session on the GPU down. It is now raised as
    LvxNumericError naming the rows of that chunk; the service ends those requests and stays in
    service. A NaN planted in one c_fc weight row makes every step's partials non-finite."""
    import numpy as np
    from llmvox_amd import weights as LW
    from llmvox_amd._lib import LvxNumericError
    from llmvox_amd.engine import build_engine
    from llmvox_amd.server import TTSService
    gw, cw, tt = LW.synthetic_all(1234)
    w = np.array(gw["transformer.h.1.mlp.c_fc.weight"], dtype=np.float32, copy=True)
    w[7, 3] = np.nan
    gw["transformer.h.1.mlp.c_fc.weight"] = w
    eng = build_engine(0, "bf16", "bf16", max_streams=4, max_positions=512, max_codec_frames=1280,
                       weights=(gw, cw, tt))
    svc = TTSService(eng, max_chunk=16, max_tokens=64)
    try:
        for _ in range(2):  # the service keeps serving (and failing) requests: the device stays in service
            s = svc.submit("Hello there.")
            with pytest.raises(RuntimeError) as ei:
                b"".join(svc.chunks(s, timeout=0.01))
            assert isinstance(ei.value.__cause__, LvxNumericError), repr(ei.value.__cause__)
            assert svc.error is None and svc.workers[0].error is None
    finally:
        svc.shutdown()
        eng.close()
