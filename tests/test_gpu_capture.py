"""Graph capture beside another thread's event queries (round 6). torch's synchronous collectives record
their completion events on the current stream and the process group's watchdog thread queries them;
HIP refuses a query of an event last recorded in a stream that is capturing. The library captured its
decode graphs on the caller's stream, so a watchdog poll that landed inside a capture aborted the
process and failed the capture (a configs[4] bench line with the one-rank RCCL group, on the GPU box).
A capture stream (lvx_set_capture_stream) takes the capture off the caller's stream; the engine names a
pooled torch stream once an RCCL group exists (one more stream per process otherwise cost two ranks
sharing a GPU 6.5x: profiles/r06/capture_stream_ab.txt)."""
import socket
import threading

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _steps_beside_a_poller(e, B=8, flips=12, poll_events=True):
    """ar_steps on a side stream while another thread polls an event last recorded on that stream;
    every option flip drops the cached graphs (flips x 2 captures). Returns (poll errors, tokens)."""
    dev = e.device
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    plan = torch.full((B, 64), 100, dtype=torch.int32, device=dev)
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    errs, stop = [], threading.Event()
    toks = []
    with torch.cuda.stream(side):
        ev = torch.cuda.Event()
        ev.record(side)

        def poll():
            while not stop.is_set():
                try:
                    ev.query()
                except Exception as x:  # noqa: BLE001 (what the watchdog would have died of)
                    errs.append(repr(x))
                    return

        t = threading.Thread(target=poll if poll_events else stop.wait, daemon=True)
        t.start()
        try:
            for i in range(flips):
                e.set_option("ln_max", 8 if i % 2 == 0 else 7)
                for s in range(B):
                    e.reset_slot(s)
                rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
                tok = torch.zeros(B, 64, dtype=torch.int32, device=dev)
                e.ar_steps(17, slots, plan, rowstep, tok)
                toks.append(tok.cpu().numpy())
            e.check_errors()
        finally:
            stop.set()
            t.join()
            e.set_option("ln_max", 8)
    torch.cuda.current_stream(dev).wait_stream(side)
    return errs, toks


def _engine():
    from llmvox_amd.engine import build_engine
    return build_engine(0, "bf16", "bf16", max_streams=8, max_positions=256, max_codec_frames=64)


def test_capture_stream_beside_event_queries_of_the_callers_stream():
    e = _engine()
    try:
        e.set_capture_stream(torch.cuda.Stream(device=e.device))
        errs, toks = _steps_beside_a_poller(e)
        assert not errs, errs
        for a in toks[2::2]:  # the same option set gives the same tokens every time
            np.testing.assert_array_equal(a, toks[0])
        # captured on the caller's stream (the default; no event queries beside it): the same tokens
        e.set_capture_stream(None)
        e.set_option("ln_max", 7)
        e.set_option("ln_max", 8)
        _, toks2 = _steps_beside_a_poller(e, flips=1, poll_events=False)
        np.testing.assert_array_equal(toks2[0], toks[0])
    finally:
        e.close()


def test_rccl_group_moves_the_capture_off_the_callers_stream():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    e = _engine()
    try:
        x = torch.ones(4, device=e.device)
        dist.all_reduce(x)  # a synchronous collective: its event is recorded on the current stream
        errs, _ = _steps_beside_a_poller(e, flips=4)
        assert not errs, errs
        assert e._capture_stream is not None
        assert e._capture_stream.cuda_stream != torch.cuda.current_stream(e.device).cuda_stream
    finally:
        e.close()
        dist.destroy_process_group()
