"""bench.py's multi-rank launch (CPU, gloo): ``python bench.py --gpus N`` outside torchrun
starts N ranks itself and the one JSON line on stdout names N; under a launcher whose
WORLD_SIZE differs from --gpus it refuses to run instead of benching the wrong rank count."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        if env is None or k not in env:
            e.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=240, cwd=ROOT)


def test_gpus_2_launches_two_ranks():
    r = _run(["--gpus", "2", "--selftest-launch", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout          # exactly one line on stdout: rank 0's result
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks"] == 2 and d["backend"] == "gloo"


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2", "--selftest-launch"], env={"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_single_rank_selftest():
    r = _run(["--selftest-launch", "--steps", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip())["n_gpus"] == 1


@pytest.mark.gpu
def test_gloo_two_ranks_report_in_step_exchange():
    """`bench.py --gpus 2 --dist-backend gloo` (two ranks on one GPU, the multi-rank logic's
    rehearsal): the line carries the exchange fields as the step ran them — the compute stream's
    waits for the reduce-scatter/all-reduce and for the all-gather, max and min over the ranks —
    and names the path (call by call under gloo)."""
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--dp", "user", "--batch", "8192", "--steps", "12",
              "--warmup", "2", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.strip()][-1])
    assert d["n_gpus"] == 2
    x = d["exchange"]
    assert x["ranks"] == 2 and x["backend"] == "gloo" and x["native_step"] is False
    s = x["in_step"]
    assert s["path"].startswith("call by call") and s["sampled_steps_per_rank"] >= 2
    for k in ("rs_ar_exposed_ms", "ag_exposed_ms"):
        assert s[k]["max"] >= s[k]["min"] >= 0.0, (k, s[k])
    assert s["rs_ar_ms"] is None and s["ag_ms"] is None   # torch's collectives: not observable


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_for_test", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_replay_accounting_counts_only_the_far_rows_in_the_update():
    """The update launch's algorithmic bytes count the catch-up replays it still runs: with the
    replay split (NCF_DEFER_OWED) only rows owing more than that many steps; the build defines
    select the threshold (0: every replay in the update)."""
    import torch
    b = _bench_module()
    assert b.deferred_replay_owed({"defines": ""}) == 4
    assert b.deferred_replay_owed({"defines": "-DNCF_DEFER_OWED=8"}) == 8
    assert b.deferred_replay_owed({"defines": "-DNCF_REPLAY_IN_SCAN=0"}) == 0
    g = torch.Generator().manual_seed(3)
    pool = [(torch.randint(0, 50, (40,), generator=g, dtype=torch.int32),
             torch.randint(0, 20, (40,), generator=g, dtype=torch.int32), None) for _ in range(7)]
    total = b.replayed_rows(pool, 3, 12, 50, 70, items=True)
    far = b.replayed_rows(pool, 3, 12, 50, 70, items=True, far=2)
    assert 0 < far < total
    assert b.replayed_rows(pool, 3, 12, 50, 70, items=True, far=1000) == 0.0
