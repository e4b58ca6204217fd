"""CPU oracle for the LLMVoX streaming-TTS hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``llmvox_amd`` imports this package.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may use it, and only as the checker / the timed CPU baseline.

Parity pinning: the oracle is checked against golden vectors produced by the
reference itself (imported from /root/reference in the build container, see
``tests/golden/make_golden.py``) — token ids bit-exact, PCM within 1e-5.
"""
