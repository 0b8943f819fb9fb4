"""bench.py's multi-GPU launch contract, on the CPU: `--gpus N` without a
launcher's WORLD_SIZE starts torch.distributed.run as a child process (no
exec, nothing touches the GPU first) with N ranks, each seeing its own RANK /
LOCAL_RANK and WORLD_SIZE = N; rank 0's line reaches our stdout."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=timeout)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


def test_gpus_2_spawns_two_ranks():
    rc, lines, err = _run(["--gpus", "2", "--dry-run"])
    assert rc == 0, err[-2000:]
    got = sorted((x["rank"], x["local_rank"], x["world_size"]) for x in lines if x.get("dry_run"))
    assert got == [(0, 0, 2), (1, 1, 2)], (got, err[-2000:])


def test_gpus_1_runs_in_process():
    rc, lines, err = _run(["--dry-run"])
    assert rc == 0, err[-2000:]
    assert [(x["rank"], x["world_size"]) for x in lines] == [(0, 1)]


def test_launcher_env_is_respected():
    """Under a launcher (WORLD_SIZE set) bench.py never spawns again."""
    rc, lines, err = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"})
    assert rc == 0, err[-2000:]
    assert [(x["rank"], x["local_rank"], x["world_size"]) for x in lines] == [(3, 3, 4)]
