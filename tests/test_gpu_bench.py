"""bench.py's multi-GPU launch: `python bench.py --gpus N`
without a launcher starts N rank processes itself, before any GPU call, and
the sharded headline gives the one-GPU joins.  On a one-GPU box the ranks
share the device over the host-staged gloo transport (a rehearsal of the
8-GPU run, not a timing)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--n", "3000", "--L", "20000", "--steps", "1", "--warmup", "0", "--no-cpu", "--no-extras"]


def _bench(args, env=None, timeout=300):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def test_bench_world_mismatch_refused():
    """--gpus N under a launcher whose WORLD_SIZE differs: exit non-zero
    before any GPU work (no GPU needed)."""
    p = _bench(["--gpus", "2"] + SMALL, env={"WORLD_SIZE": "3", "RANK": "0"}, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=3" in p.stderr


@pytest.mark.gpu
def test_bench_gpus2_spawned_same_joins():
    """--gpus 1 pipelined and sequential; --gpus 2 (ranks spawned by bench.py,
    gloo rehearsal on one GPU) in every tree mode: GPU 0's tree beside the
    other ranks' next dist (the default), the dist's row ranges gathered to
    GPU 0 for the single-GPU tree step by step, and the row-sharded tree; the
    same joins as --gpus 1."""
    one = _bench(["--gpus", "1"] + SMALL)
    assert one.returncode == 0, one.stderr[-3000:]
    l1 = json.loads(one.stdout.strip().splitlines()[-1])
    assert l1["n_gpus"] == 1
    # one GPU: the pipelined form (tree beside the next matrix's dist, two LT
    # buffers in turn over warmup + 2 steps) and the sequential one agree
    pipe = _bench(["--gpus", "1"] + SMALL + ["--steps", "2", "--warmup", "1"])
    seq = _bench(["--gpus", "1", "--tree-cus", "0"] + SMALL)
    for p in (pipe, seq):
        assert p.returncode == 0, p.stderr[-3000:]
    lp, ls = (json.loads(p.stdout.strip().splitlines()[-1]) for p in (pipe, seq))
    assert "pipelined" in lp["config"]["parallelism"] and "pipelined" not in ls["config"]["parallelism"]
    assert lp["split"]["joins_sha256"] == ls["split"]["joins_sha256"] == l1["split"]["joins_sha256"]
    # the pipelined stream alternates two alignments (seeds 3, 4): each one's
    # tree is the sequential form's tree of that alignment, and they differ
    seq4 = _bench(["--gpus", "1", "--tree-cus", "0", "--headline-seed", "4"] + SMALL)
    assert seq4.returncode == 0, seq4.stderr[-3000:]
    l4 = json.loads(seq4.stdout.strip().splitlines()[-1])
    by = lp["split"]["joins_sha256_by_alignment"]
    assert by == {"0": [ls["split"]["joins_sha256"]], "1": [l4["split"]["joins_sha256"]]}
    assert by["0"] != by["1"]
    # tree_s is the tree context's device time, not the dist's wall
    assert 0 < lp["split"]["tree_s"] <= lp["split"]["tree_wall_s"] + 1e-3
    for mode in ("gather-pipelined", "gather", "shard"):
        two = _bench(["--gpus", "2", "--shard-transport", "gloo", "--tree-mode", mode] + SMALL)
        assert two.returncode == 0, (mode, two.stderr[-3000:])
        l2 = json.loads(two.stdout.strip().splitlines()[-1])
        assert l2["n_gpus"] == 2
        assert l2["split"]["joins_sha256"] == l1["split"]["joins_sha256"], mode
        assert l2["split"]["joins"] == l1["split"]["joins"] == 2998
