"""CPU: bench.py's multi-GPU launch contract.

`bench.py --gpus N` started without a launcher (no WORLD_SIZE) must start
N ranks itself -- one process per GPU through torch.distributed.run on
127.0.0.1 -- before any GPU call, and report n_gpus from the communicator's
rank count.  --dry-run stops each rank after the rendezvous and one gloo
all-reduce (no GPU call), so this runs here."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout   # one JSON line, from rank 0 only
    return json.loads(lines[0])


def test_gpus_2_self_launches_two_ranks():
    out = _run(["--gpus", "2", "--dry-run"])
    assert out["dry_run"] and out["n_gpus"] == 2 and out["ranks_reporting"] == 2


def test_gpus_1_runs_in_process():
    out = _run(["--gpus", "1", "--dry-run"])
    assert out["n_gpus"] == 1 and out["ranks_reporting"] == 1
