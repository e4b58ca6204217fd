"""Child process of tests/test_gpu_exit.py (started by tests/conftest.py before the test session
touches the GPU): an overlapped FusedScheduler with a codec call and its delivery job still in flight,
and the process then exits normally without closing the scheduler or the engine. The exit status must
be 0 (the delivery thread inside Event.synchronize at interpreter finalisation had
aborted the process, 'terminate called without an active exception')."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llmvox_amd import streaming as S
    from llmvox_amd.engine import build_engine
    eng = build_engine(0, "bf16", "bf16", max_streams=4, max_positions=1024, max_codec_frames=4 * 160)
    torch.cuda.set_stream(torch.cuda.Stream())
    sch = S.FusedScheduler(eng, max_chunk=64, overlap=True)
    for i in range(4):
        st = sch.open_stream(index=i % 2, dump_size=10 if i % 2 == 0 else 160)
        for w in "The quick brown fox jumps over the lazy dog near the river bank.".split():
            st.feed(w)
    for _ in range(6):  # chunk c + 1 queued before chunk c completes; its codec and delivery queued
        sch.run_chunk()
    pending = sch.deliverer.pending if sch.deliverer is not None else 0
    print(f"exit_child: {len(sch.inflight)} chunk(s) and {pending} delivery job(s) in flight at exit", flush=True)
    # no sch.close(), no eng.close(): the interpreter's own exit


if __name__ == "__main__":
    main()
