"""bench.py's multi-rank launcher on the CPU (gloo, no GPU): `--gpus N` without torch.distributed.run
spawns N ranks itself; under an external launcher WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, cwd=ROOT,
                          capture_output=True, text=True, timeout=240)


def test_gpus2_spawns_two_gloo_ranks():
    r = _run(["--gpus", "2", "--rehearse", "--streams", "3"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1  # rank 0 only
    d = json.loads(line[0])
    assert d["dist"] == {"backend": "gloo", "world_size": 2}
    assert d["n_gpus"] == 2 and d["streams_per_rank"] == 3 and d["gathered_equals_scattered"]
    assert d["paced_gather_equals_single_rank"]  # the overlapped schedule's asynchronous, paced gather


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--rehearse"], env={"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=4" in r.stderr


def test_under_external_launcher():
    """torch.distributed.run sets WORLD_SIZE / RANK itself: bench.py must not spawn again."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(29400 + os.getpid() % 500),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse", "--streams", "2"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["dist"]["world_size"] == 2
