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
    # the tail's all-reduce rides in the last all-to-all's group once that group passed its self-test
    assert d["config"]["dp_exchange"] == "zero/bf16 tail-in-a2a via torch"
    assert not d["config"]["dp_fallbacks"]
    chk = d["dp_check"]
    assert chk["world"] == 2 and chk["ranks_identical"] is True and chk["finite"] is True
    assert d["value"] > 0 and d["value"] == pytest.approx(2 * 1024 * 5 * 4 / (d["ms_per_step"] * 4e-3), rel=1e-3)
    # self-explaining N > 1 line: the exchange's phases of the last timed step, the communicator
    comm = d["config"]["comm"]
    assert comm["comm_world"] == 2 and comm["comm_rank"] == 0 and "gloo" in comm["transport"]
    ph = d["dp_kernels_ms"]
    for k in ("fwd_bwd", "exchange_before_adam", "adam", "exchange_after_adam"):
        assert ph[k] > 0, (k, ph)
    # the second child: the one-all-reduce exchange on the same two ranks
    alt = d["dp_alt"]
    assert "error" not in alt, alt
    assert alt["dp_exchange"] == "allreduce via torch" and alt["value"] > 0
    assert alt["dp_check"]["ranks_identical"] is True and alt["dp_check"]["world"] == 2
    assert alt["dp_kernels_ms"]["exchange_before_adam"] > 0
    # the third child: the touched-row sparse gradient all-to-all (DataParallel(sparse=True))
    sp = d["dp_alt_sparse"]
    assert "error" not in sp, sp
    assert sp["dp_exchange"] == "zero/bf16 sparse tail-in-a2a via torch" and sp["value"] > 0
    assert sp["dp_check"]["ranks_identical"] is True and sp["dp_check"]["world"] == 2
    assert 0 < sp["dp_sparse"]["rows_sent_frac"] < 1 and sp["dp_sparse"]["steps"] >= 4
    # the fourth child: the peer-store exchange (DataParallel(exchange="peer"), IPC-mapped buffers,
    # one captured graph per region), its ranks bit-identical and no wait timed out
    pe = d["dp_alt_peer"]
    assert "error" not in pe, pe
    assert pe["dp_exchange"] == "zero/bf16 via peer stores" and pe["value"] > 0
    assert pe["dp_launch"] == "one graph per region, collectives captured"
    assert pe["dp_check"]["ranks_identical"] is True and pe["dp_check"]["world"] == 2
    assert pe["peer_status"]["error"] == 0 and pe["peer_status"]["steps"] >= 5, pe["peer_status"]


@pytest.mark.gpu
def test_bench_multiview_gpus2_spawns_ranks_and_checks_them():
    d = _run(["--model", "multiview"])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["dp_exchange"] == "torch"
    chk = d["dp_check"]
    assert chk["world"] == 2 and chk["ranks_identical"] is True and chk["finite"] is True


@pytest.mark.gpu
@pytest.mark.parametrize("comm", ["copy", "peer"])
def test_bench_rehearsal_reports_dp_phases(comm):
    """The captured data-parallel step graph (the one the RCCL ranks time) rehearsed on one GPU with
    its collectives as device copies, or as rank 0 of the peer-store exchange with the peers' buffers
    local: the last step's phase probes are all recorded."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--rehearse-world", "8", "--rehearse-comm", comm,
           "--steps", "4", "--warmup", "2", "--cpu-baseline", "0", "--fp32-line", "0", "--det-line", "0",
           "--fwd-only", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    ph = d["dp_kernels_ms"]
    for k in ("fwd_bwd", "grad_pass", "all_to_all", "tail_allreduce", "adam", "all_gather", "shadow_rebuild"):
        assert k in ph, (k, ph)
    for k in ("fwd_bwd", "grad_pass", "all_to_all", "adam", "all_gather", "shadow_rebuild"):
        assert ph[k] > 0, (k, ph)
    assert d["rehearsal"]["world"] == 8
    if comm == "peer":
        assert d["peer_status"]["error"] == 0 and d["peer_status"]["steps"] >= 6, d["peer_status"]
    # the step's phases fit inside its measured time
    assert sum(v for k, v in ph.items() if k != "source") <= 1.2 * d["ms_per_step"], (ph, d["ms_per_step"])
