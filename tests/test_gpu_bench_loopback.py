"""bench.py's N-rank sequence rehearsed on ONE GPU:
`--loopback 8` runs what `--gpus 8` runs on every rank -- the configs[1]
sharded step, the small-batch sharded points and a reduced configs[3] leg --
as 8 threads over a loopback communicator (mqvs_comm_init_loopback), i.e.
the same mqvs_sharded_search code an RCCL communicator runs
(StorageDistributed.cpp:1057-1060 / MergeTreeBaseSearchManager.cpp:207-297
are what it replaces).  The headline line is printed before the optional
legs, and a leg that fails on one rank is recorded on every rank instead of
losing the line or hanging the others."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--loopback", "8", "--steps", "2", "--warmup", "1", "--n", "2000000", "--nq", "300",
         "--config3-rows", "200000"]


def _run(extra):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL + extra, capture_output=True,
                       text=True, cwd=ROOT, timeout=300)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


def _exact(pt):
    return pt["exact"]["ids_and_dist_bits_equal_on_every_rank"]


def test_loopback_8_runs_the_n_rank_sequence():
    rc, lines, err = _run([])
    assert rc == 0, err[-3000:]
    assert len(lines) == 2, lines  # the headline, then the line with the legs
    head, full = lines
    for x in (head, full):
        assert x["config"]["loopback_virtual_ranks"] == 8
        assert x["exact_check"]["ids_equal"] and x["exact_check"]["dist_bitwise_equal"], x["exact_check"]
        assert x["fast_path_calls"] > 0 and x["redo_calls"] == 0, x
        assert len(x["roofline"]) <= 20
    sb = full["small_batch_sharded"]
    assert [p["nq"] for p in sb] == [1, 16]
    assert all(_exact(p) and p["fast_path_calls"] > 0 for p in sb), sb
    c3 = full["config3_sharded"]
    assert "error" not in c3, c3
    assert c3["rows"] == 8 * 200000 and not c3["full_size"]
    assert [p["nq"] for p in c3["points"]] == [1, 16, 1000]
    assert all(_exact(p) and p["fast_path_calls"] > 0 for p in c3["points"]), c3


def test_loopback_leg_failure_is_collective_and_soft():
    """Rank 3 fails the configs[3] leg (before its first collective): every
    rank records the leg's error, the headline and the other legs stand, rc 0."""
    rc, lines, err = _run(["--inject-leg-failure", "config3:3", "--no-verify"])
    assert rc == 0, err[-3000:]
    assert len(lines) == 2, lines
    head, full = lines
    assert head["value"] > 0 and full["value"] == head["value"]
    assert "injected failure" in full["config3_sharded"]["error"], full["config3_sharded"]
    assert all(_exact(p) for p in full["small_batch_sharded"]), full["small_batch_sharded"]
