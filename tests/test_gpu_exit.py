"""A process that exits with an overlapped FusedScheduler still holding a chunk and a codec delivery in
flight, without closing it or its engine, exits with status 0 (the b940b4e fix:
the delivery threads are stopped by an atexit hook before the interpreter finalises). The child,
tests/exit_child.py, was started by tests/conftest.py before this session touched the GPU."""
import pytest

pytestmark = pytest.mark.gpu


def test_exit_with_dump_in_flight_is_clean(request):
    proc = getattr(request.config, "lvx_exit_child", None)
    assert proc is not None, "the child was not started (conftest.pytest_collection_finish)"
    try:
        out, _ = proc.communicate(timeout=110)
    except Exception:
        proc.kill()
        proc.communicate()
        raise
    text = out.decode(errors="replace")
    assert "exit_child:" in text, text[-2000:]
    assert proc.returncode == 0, f"rc {proc.returncode}:\n{text[-2000:]}"
    assert "terminate called" not in text and "Fatal Python error" not in text, text[-2000:]
