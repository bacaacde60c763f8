"""bench.py's launcher contract, checked without a GPU: a --gpus that
disagrees with the launcher's WORLD_SIZE, or is < 1, exits non-zero before
anything touches a device; the flags parse; legs are validated."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=60)


@pytest.mark.parametrize("gpus,world", [(1, "2"), (2, "4"), (8, "1")])
def test_gpus_world_size_mismatch_exits_nonzero(gpus, world):
    r = _run(["--gpus", str(gpus)], WORLD_SIZE=world)
    assert r.returncode != 0
    assert "disagree" in r.stderr


def test_gpus_below_one_exits_nonzero():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0


def test_unknown_leg_is_refused():
    r = _run(["--legs", "decode,nonsense"])
    assert r.returncode != 0 and "unknown legs" in r.stderr


def test_launcher_forwards_numel_not_n(monkeypatch):
    """launch_ranks rewrites --n (ambiguous for torchrun's parser) to --numel
    and starts the child with the same script and flags."""
    sys.path.insert(0, ROOT)
    import bench

    seen = {}

    class _R:
        returncode = 7

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return _R()

    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--n", "1000", "--steps", "3"])
    monkeypatch.setattr(subprocess, "run", fake_run)
    assert bench.launch_ranks(4) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    tail = cmd[cmd.index(os.path.join(ROOT, "bench.py")):]
    assert tail[1:] == ["--gpus", "4", "--numel", "1000", "--steps", "3"]
    assert seen["env"]["GC_BENCH_LAUNCHED"] == "1"
