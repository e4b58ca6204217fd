"""FusedScheduler's error paths on CPU stand-in engines:

* a KV-capacity error raised only by a run-ahead row that an end of audio in the chunk before had
  already discarded concerns no live stream: it is dropped, and the stream's items equal the serial
  schedule's (the serial schedule never plans that row);
* a codec call whose error word is set fails only the streams whose dumps it carried: they are named
  in an LvxStreamError and receive nothing more; every other stream's items are delivered, on the
  serial and on the overlapped schedule.
"""
import numpy as np
import pytest
import torch

from llmvox_amd import streaming as S
from llmvox_amd._lib import LvxCapacityError, LvxStreamError
from test_service_multidevice import StateEngine

WORDS = ("some words that keep going for a long while and then some more words until the very end of "
         "this rather long sentence").split()


class ChunkErrEngine(StateEngine):
    """The GPU engine's per-chunk error words: each ar_steps call's capacity flag is its own, read
    back (check_errors) in launch order, as the scheduler takes one word per chunk."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.flags = []

    def ar_steps(self, *a, **kw):
        self.err = False
        super().ar_steps(*a, **kw)
        self.flags.append(self.err)
        self.err = False

    def check_errors(self):
        if self.flags and self.flags.pop(0):
            raise LvxCapacityError(-4, "a stream exceeded its KV capacity (max_positions)")


def _events(st):
    return [("pcm", x.astype(int).tolist()) if isinstance(x, np.ndarray) else ("sig", x) for x in st.events]


def _eoa_then_capacity(overlap):
    # end of audio at position 41 (inside the chunk of positions 40..47); the run-ahead row of the next
    # chunk covers 48..55 and ends exactly at max_positions 56, setting the capacity flag
    eng = ChunkErrEngine(max_streams=2, max_positions=56, eoa=4000)
    sch = S.FusedScheduler(eng, max_chunk=8, to_bytes=False, overlap=overlap)
    st = sch.open_stream(index=0, dump_size=160, eoa_id=4000)
    for w in WORDS:
        st.feed(w)
    for _ in range(40):
        if sch.run_chunk() == 0:
            break
    sch.flush()
    out = (_events(st), list(st.tokens), eng.flags)
    sch.close()
    return out


def test_capacity_error_of_a_discarded_run_ahead_row_is_dropped():
    ev_s, tok_s, _ = _eoa_then_capacity(False)
    ev_o, tok_o, _ = _eoa_then_capacity(True)
    assert ("sig", 0) in ev_s or ("sig", 1) in ev_s or ("sig", "end") in ev_s  # the segment did end
    assert ev_o == ev_s and tok_o == tok_s


class CodecErrEngine(StateEngine):
    """A stand-in with the codec's error word: a decode of `poison_len`-frame dumps sets the
    out-of-range-code bit (4 << 16), taken by take_errors as the real engine's word is."""

    def __init__(self, poison_len=None, **kw):
        super().__init__(**kw)
        self.poison_len = poison_len
        self.codec_bits = 0

    def decode_codes(self, codes, bandwidth_id=0, out=None):
        if self.poison_len is not None and codes.shape[1] == self.poison_len:
            self.codec_bits |= 4 << 16
            self.poison_len = None  # once
        return super().decode_codes(codes, bandwidth_id, out)

    def take_errors(self, which, out):
        out[0] = self.codec_bits
        self.codec_bits = 0


def _codec_run(overlap, poison):
    eng = CodecErrEngine(poison_len=30 if poison else None, max_streams=4, max_positions=4096)
    sch = S.FusedScheduler(eng, max_chunk=16, to_bytes=False, overlap=overlap,
                           stop_rule=lambda st, ntok, pos: ntok >= 300)  # (both runs end at the same point)
    a = sch.open_stream(index=0, dump_size=10)   # dumps of 10, 30, 90, ... frames
    b = sch.open_stream(index=1, dump_size=30)   # its first dump (30 frames) is the poisoned call ...
    c = sch.open_stream(index=0, dump_size=90)   # ... and a's second dump is in a later chunk
    for st in (a, b, c):
        for w in WORDS:
            st.feed(w)
    errors = []
    for _ in range(400):
        try:
            if sch.run_chunk() == 0:
                break
        except LvxStreamError as e:
            errors.append(list(e.streams))
            for st in e.streams:  # the service ends the named streams' requests
                sch.close_stream(st)
    try:
        sch.flush()
    except LvxStreamError as e:
        errors.append(list(e.streams))
    out = {name: (_events(st), len(st.tokens)) for name, st in (("a", a), ("b", b), ("c", c))}
    sch.close()
    return out, errors, (a, b, c)


@pytest.mark.parametrize("overlap", [False, True])
def test_codec_error_fails_only_the_streams_of_its_call(overlap):
    ref, err0, _ = _codec_run(overlap, poison=False)
    got, errs, (a, b, c) = _codec_run(overlap, poison=True)
    assert err0 == []
    # exactly one error, naming b only: the 30-frame call carried b's first dump
    assert len(errs) == 1 and errs[0] == [b]
    # b received nothing at all (its first dump failed; nothing after a hole)
    assert got["b"][0] == []
    # a and c received every item of the run without the failure, in order
    for name in ("a", "c"):
        ev, ev_ref = got[name][0], ref[name][0]
        assert got[name][1] == ref[name][1] > 0  # (both runs to idle: the text is spoken to its end)
        assert ev and ev == ev_ref
