"""bench.py's N>1 path as the driver launches it: `python3 bench.py --gpus 2 ...` started as a
plain process spawns its own ranks.  On the one-GPU box the two ranks share the
card over gloo (the library's RCCL refuses two ranks on one device), so this runs the N>1 code
path end to end -- rank spawn, DataParallel exchange, max-over-ranks timing, the cross-rank
digest -- and checks the one JSON line rank 0 prints."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra, timeout=400):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--steps", "4", "--warmup", "1", "--cpu-baseline", "0"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 alone prints, once
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_gpus2_spawns_ranks_and_checks_them():
    d = _run([])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["warmup"] == 1
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 2048
    assert d["config"]["dp_exchange"] == "zero/bf16 via torch"
    assert not d["config"]["dp_fallbacks"]
    chk = d["dp_check"]
    assert chk["world"] == 2 and chk["ranks_identical"] is True and chk["finite"] is True
    assert d["value"] > 0 and d["value"] == pytest.approx(2 * 1024 * 5 * 4 / (d["ms_per_step"] * 4e-3), rel=1e-3)


@pytest.mark.gpu
def test_bench_multiview_gpus2_spawns_ranks_and_checks_them():
    d = _run(["--model", "multiview"])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["dp_exchange"] == "torch"
    chk = d["dp_check"]
    assert chk["world"] == 2 and chk["ranks_identical"] is True and chk["finite"] is True
