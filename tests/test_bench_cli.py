"""bench.py's launch contract, checked without a GPU: under torchrun, a WORLD_SIZE that differs
from --gpus is refused before anything touches the GPU (it used to warn and time one
rank), and the self-launch command is a fresh torch.distributed.run child."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=1" in r.stderr
    assert r.stdout.strip() == ""


def test_self_launch_command(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench

    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    args = bench.parse()
    assert bench.self_launch(args) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["--gpus", "4", "--steps", "3"][-3:]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    json.dumps(cmd)
