"""bench.py --gpus 2 on the one-GPU box (VERDICT r2 "Done" criterion): started WITHOUT a torchrun
environment, the script launches its own 2-rank torch.distributed.run child (gloo: both ranks on
GPU 0), and rank 0 prints one JSON line with n_gpus 2 and a config-5 block.  With --exchange
cabi-ops the step's exchange is the C ABI's own sharded code (crdt_lub_many_multi_sharded,
crdt_vclock_lub_many_sharded) over crdt_ctx_comm_init_ops host callbacks; with --exchange cabi the
RCCL communicator cannot form on one GPU, and every rank falls back to the torch exchange together."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("exchange", ["torch", "cabi-ops", "cabi"])
def test_bench_self_launches_two_ranks(exchange):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--exchange",
           exchange, "--replicas", "65536", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["parity"] == "ok"
    assert out["config"]["replica_merges_per_step"] == 2 * 2 * 65536
    assert out["c5"]["parity"] == "ok" and out["c5"]["config"]["replica_merges_per_step"] == 2 * 65536
    assert out["step_ms"]["min"] <= out["step_ms"]["median"] <= out["step_ms"]["max"]
    if exchange == "cabi-ops":
        assert "crdt_ctx_comm_init_ops" in out["config"]["exchange"]
    if exchange == "cabi":  # RCCL refuses two ranks on one GPU: every rank takes the torch exchange together
        assert "torch" in out["config"]["exchange"]
