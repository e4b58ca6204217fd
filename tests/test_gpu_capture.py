"""Graph capture beside another thread's event queries (round 6). torch's synchronous collectives record
their completion events on the current stream and the process group's watchdog thread queries them;
HIP refuses a query of an event last recorded in a stream that is capturing. The library used to
capture its decode graphs on the caller's stream, so a watchdog poll that landed inside a capture
aborted the process and failed the capture (a configs[4] bench line with the one-rank RCCL group, on
the GPU box). It now captures on a stream of its own and replays on the caller's."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_capture_beside_event_queries_of_the_callers_stream():
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", "bf16", max_streams=8, max_positions=256, max_codec_frames=64)
    dev = e.device
    try:
        B = 8
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        plan = torch.full((B, 64), 100, dtype=torch.int32, device=dev)
        slots = torch.arange(B, dtype=torch.int32, device=dev)
        errs, stop = [], threading.Event()
        with torch.cuda.stream(side):
            ev = torch.cuda.Event()
            ev.record(side)  # an event last recorded on the stream the steps are captured from

            def poll():
                while not stop.is_set():
                    try:
                        ev.query()
                    except Exception as x:  # noqa: BLE001 (what the watchdog would have died of)
                        errs.append(repr(x))
                        return

            t = threading.Thread(target=poll, daemon=True)
            t.start()
            toks = []
            try:
                for i in range(12):  # every option flip drops the cached graphs: 12 x 2 captures
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
        assert not errs, errs
        for a in toks[2::2]:  # the same option set gives the same tokens every time
            np.testing.assert_array_equal(a, toks[0])
    finally:
        e.close()
