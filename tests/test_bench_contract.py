"""bench.py's measurement plumbing on the CPU (no GPU run): the committed profile summaries it
attaches to a line are the ones collected on THAT line's workload, the algorithmic-byte formulas
match DESIGN.md §5, and the committed bench lines keep the driver's JSON contract."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_traffic_lookup_matches_workload():
    t, src = bench.pmc_traffic({"dtype": "bf16", "columns": "zipf", "feed": "device"})
    assert src and set(t) <= {"adam", "spmm_fwd"} and t["adam"] > 0
    d = json.load(open(os.path.join(ROOT, src)))
    assert d["_workload"] == {"dtype": "bf16", "columns": "zipf", "feed": "device"}
    t32, src32 = bench.pmc_traffic({"dtype": "fp32", "columns": "zipf", "feed": "device"})
    assert src32 != src and json.load(open(os.path.join(ROOT, src32)))["_workload"]["dtype"] == "fp32"
    # a workload nobody profiled gets no traffic, never another workload's
    assert bench.pmc_traffic({"dtype": "bf16", "columns": "zipf", "feed": "host"}) == ({}, None)


def test_model_profiles_are_not_taken_for_the_headline():
    mf = bench.mfma_summary("bf16")
    assert mf is not None and "model" not in json.load(open(os.path.join(ROOT, mf["source"])))["_workload"]
    assert not any(k.startswith(("k_gru", "k_rnn")) for k in mf["kernels"])
    v, src = bench.model_profile("traffic", "rnn", "k_gru_bwd_mfma<128, 128, 3>")
    assert v is not None and json.load(open(os.path.join(ROOT, src)))["_workload"]["model"] == "rnn"
    assert bench.model_profile("traffic", "nosuchmodel", "k_rnn_adam") == (None, None)


def test_algorithmic_bytes():
    # SpMM forward: 4(R+1) + NNZ*8 + NNZ*L1*2 + R*L1*4 at the C2 shapes, bf16
    assert bench.spmm_alg_bytes(196608, 6144, 300, 2) == 4 * 6145 + 196608 * 8 + 196608 * 600 + 6144 * 1200
    # fused single-GPU Adam: 24 B per parameter + the gathered [W1; b1] gradient rows + the shadows
    n_params, w1 = 9132040, 30001 * 300
    nnz, R = 197742, 6144
    b = bench.adam_alg_bytes(n_params, True, True, w1, nnz, R, 300, n_params, 0, 1)
    assert 3.5e8 < b < 3.7e8
    shadows = 2 * ((w1 - 300) + 2 * (300 * 300 + 300 * 128))
    assert b == 24 * n_params + 4 * (n_params - w1) + (nnz + R) * (8 + 2 * 300) + shadows
    # fp32 parity mode: dZ1 is stored (and gathered) fp32 (DSSM_BUF_DZ, csrc/plan.hip:602), no shadows
    b32 = bench.adam_alg_bytes(n_params, False, True, w1, nnz, R, 300, n_params, 0, 1)
    assert b32 == 24 * n_params + 4 * (n_params - w1) + (nnz + R) * (8 + 4 * 300)
    assert 4.5e8 < b32 < 4.8e8


@pytest.mark.parametrize("name", ["r02_bench_bf16", "r02_bench_fp32", "r02_bench_rnn", "r02_bench_multiview"])
def test_committed_lines_keep_the_contract(name):
    d = json.loads(open(os.path.join(ROOT, "profiles", name + ".json")).read().strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    r = d["roofline"]
    assert r["bound"] in ("hbm", "mfma") and 0 < r["frac"] < 1
    assert abs(r["achieved"] / r["peak"] - r["frac"]) < 1e-3
    assert abs(r["bytes_per_launch"] / (r["avg_ms"] * 1e-3) / 1e9 - r["achieved"]) <= 1e-3 * r["achieved"] + 0.1
    assert "workload" in d["config"]


def test_gpus_n_spawns_its_own_ranks(monkeypatch, capsys):
    """`bench.py --gpus N` started as a plain process (the driver's verb) launches its N ranks as a
    child torch.distributed.run on 127.0.0.1 with the same arguments, before any GPU call; by default
    a second child then runs the one-all-reduce exchange, and the parent prints ONE line carrying
    the second run's summary as dp_alt."""
    import io
    import json
    import subprocess
    import sys
    seen = []

    class FakeChild:
        def __init__(self, cmd, env=None, stdout=None, text=None, **kw):
            seen.append((cmd, env))
            exch = {1: "zero/bf16 via rccl", 2: "allreduce via rccl", 3: "zero/bf16 sparse via rccl"}.get(
                len(seen), "zero/bf16 via peer stores")
            head = {"value": 1.0, "ms_per_step": 2.0, "steps": 20, "warmup": 5, "unit": "pairs/s",
                    "config": {"dp_exchange": exch}, "dp_kernels_ms": {"adam": 0.05}}
            self.stdout = io.StringIO("progress\n" + json.dumps(head) + "\n") if stdout is not None else None
            self.rc = 7 if stdout is None else 0

        def wait(self):
            return self.rc

        def send_signal(self, sig):
            pass
    monkeypatch.setattr(subprocess, "Popen", FakeChild)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "5", "--dp-alt", "0"])
    args = bench.parse()
    assert args.comm == "rccl"  # strict library RCCL by default: a fallback is never timed
    assert bench.spawn_ranks(args) == 7
    cmd, env = seen[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-8:] == ["--gpus", "8", "--steps", "20", "--warmup", "5", "--dp-alt", "0"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # default: the headline child, then the allreduce / fp32-wire child and the sparse-exchange
    # child; one merged line
    seen.clear()
    capsys.readouterr()
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "5"])
    assert bench.spawn_ranks(bench.parse()) == 0
    assert len(seen) == 4
    off = ["--dp-alt", "0", "--dp-alt-sparse", "0", "--dp-alt-peer", "0"]
    assert seen[0][0][-6:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    assert seen[1][0][-10:] == ["--dp-mode", "allreduce", "--wire", "fp32"] + off
    assert seen[2][0][-8:] == ["--dp-sparse", "1"] + off
    assert seen[3][0][-8:] == ["--dp-exchange", "peer"] + off
    lines = [x for x in capsys.readouterr().out.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["config"]["dp_exchange"] == "zero/bf16 via rccl"
    assert d["dp_alt"]["dp_exchange"] == "allreduce via rccl" and d["dp_alt"]["dp_kernels_ms"] == {"adam": 0.05}
    assert d["dp_alt_sparse"]["dp_exchange"] == "zero/bf16 sparse via rccl"
    assert d["dp_alt_peer"]["dp_exchange"] == "zero/bf16 via peer stores"
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--backend", "gloo"])
    assert bench.parse().comm == "torch"


def test_alternative_leg_time_limit(monkeypatch):
    """An alternative-exchange leg past its wall-clock limit is killed (its own process group) and
    reported, so a stuck alternative never holds back the headline line."""
    import subprocess
    import sys
    import time
    real = subprocess.Popen

    def sleeper(cmd, **kw):  # the rank launcher replaced by a child that never finishes
        return real([sys.executable, "-c", "import time; print('progress', flush=True); time.sleep(120)"], **kw)
    monkeypatch.setattr(subprocess, "Popen", sleeper)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    args = bench.parse()
    t0 = time.perf_counter()
    rc, lines = bench._run_ranks(args, [], capture=True, limit=2.0)
    assert time.perf_counter() - t0 < 30 and rc != 0 and lines == []


def _dp_check_rank(rank, world, port, perturb, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class M:
        n_params = 1000
        params = torch.arange(1024, dtype=torch.float32)
        adam_m = torch.ones(1024)
        adam_v = torch.full((1024,), 0.5)
    m = M()
    if perturb and rank == 1:
        m.adam_v = m.adam_v.clone()
        m.adam_v[999] = float.fromhex("0x1.0000020000000p-1")  # one ulp
    out = bench.dp_check(m, object(), torch.device("cpu"))
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("perturb", [False, True])
def test_dp_check_compares_every_rank(perturb):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    ps = [ctx.Process(target=_dp_check_rank, args=(r, 2, port, perturb, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert outs[0] == outs[1] and outs[0]["world"] == 2 and outs[0]["finite"]
    assert outs[0]["ranks_identical"] is (not perturb)
