#!/usr/bin/env python3
"""Benchmark: DSSM two-tower training step, query-doc pairs/sec (fwd+bwd+Adam).

Workload (BASELINE.json configs[1]): TRIGRAM_D=30000, widths 300/300/128, BS=1024 queries per
GPU, NEG=4, bf16 compute (fp32 master weights and Adam state).  A step = one
sess.run(train_step) of the reference (new_dssm.py:267): forward with batch-stat BN + EMA
update, backward, dense Adam over all 9.13M parameters (+ one RCCL gradient all-reduce when
N > 1).  Pairs per step = BS*(NEG+1) per GPU.  Synthetic batches are generated
on the host and staged in HBM before the timed region; each step just points the plan at the
next staged batch (no copy).

Launch:  python bench.py [--gpus N --steps K --warmup W]
   N>1 as a plain process: bench.py starts its N ranks itself (a child torch.distributed.run on
   127.0.0.1, before any GPU call); or under the launcher directly:
         python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
           --master-port P bench.py --gpus N --steps K --warmup W
   N>1 defaults to the library's RCCL transport, strict (no timed fallback), and ends with a
   cross-rank digest of parameters / Adam state (dp_check in the line).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

D, WIDTHS, BS, NEG = 30000, (300, 300, 128), 1024, 4
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--batches", type=int, default=16,
                    help="distinct staged batches per rank (N=1: one graph holds a step per batch; 16 amortises the "
                         "graph-launch gap and the cycle's one separate rank launch: 183.9 -> 180.6 us/step vs 8)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU port on rank 0")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--parity", type=int, default=1,
                    help="N=1, with --cpu-baseline: one fwd+bwd step per mode (bf16, fp32) on batch 0 against "
                         "the float64 oracle, reported as cpu_baseline.parity_vs_oracle")
    ap.add_argument("--comm", default=None, choices=["auto", "rccl", "torch"],
                    help="N>1 transport: rccl = libdssm.so's own RCCL communicator (the default under the "
                         "nccl backend, strict: a failure raises instead of timing a fallback), torch = "
                         "torch.distributed collectives (the default under gloo), auto = rccl with a "
                         "self-tested torch fallback")
    ap.add_argument("--dp-mode", default="auto", choices=["auto", "zero", "allreduce"],
                    help="N>1 exchange: zero = reduce-scatter + sharded Adam + all-gather "
                         "(default with torch.distributed), allreduce = all-reduce + replicated Adam")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend (gloo: functional rehearsal of N>1 on one GPU)")
    ap.add_argument("--graph", type=int, default=1, help="replay hipGraph-captured steps (0: eager launches)")
    ap.add_argument("--multi-step", type=int, default=1,
                    help="N=1 graph mode: one graph holding a step per staged batch (replayed per cycle)")
    ap.add_argument("--probes", type=int, default=1, help="HIP-event kernel probes in the timed region")
    ap.add_argument("--rehearse-world", type=int, default=1,
                    help="analysis only (N=1): rank 0's share of a W-rank zero/bf16-wire step (the data-"
                         "parallel step graph, chunked gradient pass / Adam / shadow rebuild) with each "
                         "collective replaced per --rehearse-comm")
    ap.add_argument("--rehearse-comm", default="model", choices=["model", "copy", "peer"],
                    help="rehearsal collectives: model = a kernel holding the comm stream for the modelled "
                         "link time (--link-latency-us + bytes sent / --link-gbps); copy = a device copy of "
                         "the same bytes")
    ap.add_argument("--link-gbps", type=float, default=350.0,
                    help="modelled xGMI egress per GPU for --rehearse-comm model (GB/s)")
    ap.add_argument("--link-latency-us", type=float, default=10.0,
                    help="modelled fixed cost per collective for --rehearse-comm model (us)")
    ap.add_argument("--dp-chunks", type=int, default=1,
                    help="N>1 bf16 wire: W1's rows exchanged in this many pieces (1: the parameter wire is "
                         "read by the next step's SpMM directly)")
    ap.add_argument("--model", default="bow", choices=["bow", "rnn", "multiview"],
                    help="bow: the headline BoW DSSM (BASELINE config 2); rnn: the dssm_rnn tower (config 4); "
                         "multiview: multi_view_dssm_v3 (config 5)")
    ap.add_argument("--mv-csc-stream", type=int, default=1,
                    help="multiview, fused optimizer: the CSC transposes on a third stream forked from the step's "
                         "stream (MultiViewDSSM(csc_stream=True)) instead of the item tower's stream")
    ap.add_argument("--feed", default="device", choices=["device", "host"],
                    help="device: batches staged in HBM before the timed region (the headline); host: "
                         "batches streamed from host CSR matrices by the native pinned async feeder "
                         "inside the timed region (PCIe-inclusive rate, N=1)")
    ap.add_argument("--wire", default="auto", choices=["auto", "bf16", "fp32"],
                    help="zero schedule: W1 rows on a bf16 or fp32 wire (auto: bf16 in bf16 mode)")
    ap.add_argument("--columns", default="zipf", choices=["zipf", "uniform"],
                    help="column-id distribution of the synthetic batches (SURVEY 8d: Zipf(1.1) headline, "
                         "uniform variant)")
    ap.add_argument("--fp32-line", type=int, default=1,
                    help="N=1 bf16 headline: also time the fp32 parity mode (the reference's precision, "
                         "new_dssm.py:111-114) over the same K / W in a child process and report it as "
                         "the line's fp32_mode key")
    ap.add_argument("--deterministic", type=int, default=0,
                    help="plan option DETERMINISTIC: run-to-run bit-identical steps (not the headline)")
    ap.add_argument("--fwd32", type=int, default=0,
                    help="bf16 plan option FWD32: the forward at the reference's fp32 precision (fp32 W1 "
                         "gathers, the fp32-parity tiles for layers >= 2), the bf16 backward and optimizer")
    ap.add_argument("--fwd32-line", type=int, default=1,
                    help="N=1 bf16 headline: also time the FWD32 mode (child process) and report it as fwd32_mode")
    ap.add_argument("--det-line", type=int, default=1,
                    help="also time the deterministic mode (child process) and report it beside the line")
    ap.add_argument("--fwd-only", type=int, default=1,
                    help="also time the forward alone (eval mode: EMA-BN forward + cosine + loss, "
                         "new_dssm.py:274-285) over the staged batches, N=1")
    ap.add_argument("--idle-before-warmup", type=float, default=0.0,
                    help="analysis only: seconds of host sleep between the graph builds and the warm-up")
    ap.add_argument("--busy-before-warmup", type=float, default=0.0,
                    help="analysis only: seconds of dense matmul load between the graph builds and the warm-up")
    ap.add_argument("--plan-option", action="append", default=[], metavar="NAME=0|1",
                    help="analysis only: set a schedule option (dssm_plan_set_option, e.g. LAZY_ADAM=0)")
    ap.add_argument("--dp-alt", type=int, default=1,
                    help="N>1 started as a plain process: after the headline ranks exit, run a second N-rank "
                         "child with --dp-mode allreduce --wire fp32 (one fp32 gradient all-reduce + replicated "
                         "Adam) and report its line as dp_alt, so one run measures both exchanges")
    ap.add_argument("--dp-sparse", type=int, default=0,
                    help="N>1 zero/bf16 schedule: the touched-row sparse gradient all-to-all (DataParallel"
                         "(sparse=True): packed touched W1 rows, counts first, the tail all-reduce in the same "
                         "RCCL group; between captured graphs)")
    ap.add_argument("--dp-alt-sparse", type=int, default=1,
                    help="N>1 started as a plain process: also run the --dp-sparse 1 exchange as a third child "
                         "and report it as dp_alt_sparse")
    ap.add_argument("--dp-exchange", default="collective", choices=["collective", "peer"],
                    help="N>1 zero/bf16 schedule: the library's RCCL collectives (default) or the peer-store "
                         "exchange (DataParallel(exchange='peer'): gradient rows stored into the owners' stages "
                         "by the gradient pass, parameters into every rank's wire, epoch flags; DESIGN §6)")
    ap.add_argument("--dp-alt-peer", type=int, default=1,
                    help="N>1 started as a plain process: also run the --dp-exchange peer step as a child and "
                         "report it as dp_alt_peer")
    ap.add_argument("--dp-check", type=int, default=1,
                    help="N>1: after the timed region, gather the sharded optimizer state and compare a "
                         "digest of every rank's parameters / Adam m / v (reported as dp_check)")
    args = ap.parse_args()
    if args.comm is None:  # N>1 default: strict library RCCL on GPUs, so a fallback is never timed
        args.comm = "rccl" if args.backend == "nccl" else "torch"
    return args


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(args, argv, capture: bool, limit: float = None):
    """One child `torch.distributed.run` of args.gpus ranks (127.0.0.1) running this script with
    argv; its non-JSON output is passed through as it arrives (a long run keeps printing progress),
    the JSON line(s) rank 0 prints are returned instead of printed when capture is set.  limit
    (seconds; the alternative-exchange legs): past it the child's own process group (its launcher
    and ranks) is killed and the leg reported as timed out, so a stuck alternative never holds back
    the headline line."""
    import signal
    import subprocess
    import threading
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (the only kind the host driver has)
    env.setdefault("OMP_NUM_THREADS", "1")
    kw = {"start_new_session": True} if limit else {}
    child = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if capture else None, text=True, **kw)

    def forward(sig, _frame):  # the driver's timeout reaches the ranks too
        child.send_signal(sig)
    for sg in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sg, forward)
    timer = None
    if limit:
        def expire():
            try:
                os.killpg(child.pid, signal.SIGKILL)  # the group this Popen started, nothing else
            except (ProcessLookupError, PermissionError):
                pass
        timer = threading.Timer(limit, expire)
        timer.daemon = True
        timer.start()
    lines = []
    if capture:
        for line in child.stdout:
            if line.startswith("{"):
                lines.append(line.strip())
            else:
                sys.stdout.write(line)
                sys.stdout.flush()
    rc = child.wait()
    if timer is not None:
        timer.cancel()
    return rc, lines


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) started as a plain process: launch the N ranks as a child
    `torch.distributed.run` (one process per GPU, rendezvous on 127.0.0.1) with the same
    arguments and return its exit code.  Runs before anything touches the GPU (no HIP call, no
    torch.cuda query), so the parent never holds a device context.  With --dp-alt (default), after
    the headline ranks exit a second child runs the one-all-reduce exchange (--dp-mode allreduce
    --wire fp32) on the same N GPUs, and the parent prints ONE line: the headline's, with the
    alternative's summary under dp_alt."""
    argv = sys.argv[1:]
    alt = args.dp_alt and args.model == "bow" and args.dp_mode != "allreduce"
    alt_sparse = alt and args.dp_alt_sparse and not args.dp_sparse
    alt_peer = alt and args.dp_alt_peer and args.dp_exchange == "collective" and args.gpus <= 8
    t_head = time.perf_counter()
    rc, lines = _run_ranks(args, argv, capture=alt)
    if not alt:
        return rc
    if rc != 0 or not lines:
        for ln in lines:
            print(ln, flush=True)
        return rc or 1
    out = json.loads(lines[-1])
    legs = [("dp_alt", ["--dp-mode", "allreduce", "--wire", "fp32"])]
    if alt_sparse:
        legs.append(("dp_alt_sparse", ["--dp-sparse", "1"]))
    if alt_peer:
        legs.append(("dp_alt_peer", ["--dp-exchange", "peer"]))
    # each alternative leg gets a wall-clock limit from the headline child's own time
    limit = max(180.0, 3.0 * (time.perf_counter() - t_head))
    for key, extra in legs:
        t0 = time.perf_counter()
        arc, alines = _run_ranks(args, argv + extra + ["--dp-alt", "0", "--dp-alt-sparse", "0", "--dp-alt-peer", "0"],
                                 capture=True, limit=limit)
        if arc != 0 or not alines:
            late = time.perf_counter() - t0 >= limit
            out[key] = {"error": f"timed out after {limit:.0f} s" if late else f"exit {arc}, no line"}
            continue
        a = json.loads(alines[-1])
        out[key] = {k: a.get(k) for k in ("value", "unit", "ms_per_step", "steps", "warmup", "final_loss")}
        out[key].update({k: a["config"].get(k) for k in ("dp_exchange", "dp_launch", "comm", "dp_sparse")
                         if k in a.get("config", {})})
        for k in ("dp_kernels_ms", "dp_check", "peer_status"):
            if k in a:
                out[key][k] = a[k]
    print(json.dumps(out), flush=True)
    return 0


def dp_check(model, dp, dev) -> dict:
    """Cross-rank self-check after the timed region: every rank's fp32 parameters, Adam m and v
    (sharded rows gathered first: gather_state) and TF beta powers are hashed; the data-parallel
    step keeps them bit-identical by construction.  EMA shadows are rank-local."""
    import hashlib
    import torch
    import torch.distributed as dist
    if hasattr(dp, "gather_state"):
        dp.gather_state()
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize(dev)
    n = int(getattr(model, "n_params", model.params.numel()))
    h = hashlib.sha256()
    finite = True
    for t in (model.params[:n], model.adam_m[:n], model.adam_v[:n]):
        a = t.detach().cpu().numpy()
        finite = finite and bool(np.isfinite(a).all())
        h.update(a.tobytes())
    if hasattr(model, "beta_powers"):
        h.update(np.asarray(model.beta_powers(), np.float32).tobytes())
    mine = (h.hexdigest(), finite)
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, mine)
    return {"world": len(got), "ranks_identical": all(g[0] == got[0][0] for g in got),
            "finite": all(g[1] for g in got), "digest": got[0][0][:16],
            "what": "sha256 of fp32 params, Adam m, v (+ beta powers) after gather_state, per rank"}


def spmm_alg_bytes(nnz: int, rows: int, n1: int, s_w: int) -> int:
    """indptr + (index, value) per nnz + one gathered W1 row (n1*s_w) per nnz
    + fp32 Z1 output row per input row."""
    return 4 * (rows + 1) + nnz * (4 + 4) + nnz * n1 * s_w + rows * n1 * 4


def adam_alg_bytes(n_params: int, bf16: bool, fused: bool, w1_elems: int, nnz: int, rows: int,
                   n1: int, range_elems: int = None, wire_elems: int = 0, wire_parts: int = 1) -> int:
    """Algorithmic bytes of one k_adam_step launch.

    Every updated element streams p, m, v in and out (24 B).  Its gradient is read as fp32 (4 B),
    except (a) fused single-GPU step: the [W1; b1] rows' gradient is never stored -- the launch
    gathers it from the CSC transpose instead, (index, value) 8 B + one dZ1 row per entry, over
    nnz + rows entries (the ones column gives db1) -- the SpMM-backward bytes of SURVEY §8(d)
    minus its dense dW1 write.  The dZ1 row is stored at the step's dZ element size
    (DSSM_BUF_DZ, csrc/plan.hip:602): bf16 (2 n1 B) in bf16 mode, fp32 (4 n1 B) in fp32 mode;
    (b) data-parallel bf16 wire: the rank's W1 shard reads wire_parts bf16 partial gradients
    (2 B each: one per rank after the all-to-all) and writes a bf16 parameter copy (2 B).  bf16
    mode adds 2 B per weight element written to its shadows (W_l for l >= 2 also transposed: 4 B)."""
    if range_elems is None:
        range_elems = n_params
    b = 24 * range_elems
    if fused:
        dz_bytes = 2 if bf16 else 4
        b += 4 * (n_params - w1_elems) + (nnz + rows) * (8 + dz_bytes * n1)
    else:
        b += 4 * (range_elems - wire_elems) + (2 * wire_parts + 2) * wire_elems
    if bf16:
        sh_w1 = (w1_elems - n1) if fused else 0  # W1's shadow (bias row excluded); wired: from the wire
        sh_rest = sum(2 * WIDTHS[l - 1] * WIDTHS[l] for l in range(1, len(WIDTHS)))
        if not fused and not wire_elems:
            sh_w1 = (w1_elems - n1) * range_elems / max(n_params, 1)  # the shard's share
        b += 2 * (sh_w1 + sh_rest)
    return int(b)


# probe name -> kernel name in the rocprofv3 PMC summary (tools/gpu_pmc.sh + tools/pmc_traffic.py):
# bf16 steps run the SpMM inside k_spmm_scan (merged transpose), fp32 steps as k_spmm_fwd
# (the step kernel's single-GPU variant is k_adam_step<T, false> since round 3; older summaries
# name it k_adam_step<T>)
PMC_KERNELS = {"bf16": {"adam": ("k_adam_step<unsigned short, false>", "k_adam_step<unsigned short>"),
                        "spmm_fwd": ("k_spmm_scan<unsigned short>",)},
               "fp32": {"adam": ("k_adam_step<float, false>", "k_adam_step<float>"),
                        "spmm_fwd": ("k_spmm_fwd<float>",)}}
# the workload a traffic summary without a "_workload" record was collected on (r01: the default
# single-GPU bench line)
DEFAULT_WORKLOAD = {"dtype": "bf16", "columns": "zipf", "feed": "device"}


def pmc_traffic(workload: dict):
    """HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected) from the newest
    committed profiles/r*_traffic.json collected on THIS workload (dtype, column distribution,
    feed); PMC counters cannot be read from inside the timed run.  No matching summary: none."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic*.json")), reverse=True):
        d = json.load(open(f))
        if d.get("_workload", DEFAULT_WORKLOAD) != workload:  # (other rows' files name their model)
            continue
        out = {}
        for probe, names in PMC_KERNELS[workload["dtype"]].items():
            for k in names:
                if k in d:
                    out[probe] = d[k]["hbm_bytes"]
                    break
        return out, os.path.relpath(f, ROOT)
    return {}, None


def model_profile(kind: str, model: str, kernel: str):
    """The newest committed profiles/r*_<kind>_*.json collected on a non-headline row (its
    "_workload" names the bench.py --model) and its record of one kernel: HBM bytes per launch
    ("traffic": tools/pmc_traffic.py) or matrix-core use ("mfma": tools/mfma_util.py)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{kind}_*.json")), reverse=True):
        d = json.load(open(f))
        if d.get("_workload", {}).get("model") == model and kernel in d:
            return d[kernel], os.path.relpath(f, ROOT)
    return None, None


def mfma_summary(dtype: str):
    """Matrix-core use of the MFMA kernels (TFLOP/s vs the dense peak, busy share of the SIMD
    cycles) from the newest committed profiles/r*_mfma*.json of this dtype (tools/mfma_util.py:
    rocprofv3 SQ_INSTS_VALU_MFMA_MOPS_* / SQ_VALU_MFMA_BUSY_CYCLES over kernel-trace durations)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_mfma*.json")), reverse=True):
        d = json.load(open(f))
        if d.get("_workload", {}).get("dtype") != dtype or "model" in d.get("_workload", {}):
            continue
        ks = {k: {x: v[x] for x in ("tflops", "peak_tflops", "frac_of_peak", "mfma_busy", "flops_per_launch")
                  if x in v} for k, v in d.items() if k != "_workload"}
        return {"kernels": ks, "source": os.path.relpath(f, ROOT)}
    return None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(seconds: float):
    """Time the CPU port of the step (oracle/, test infrastructure) on a bounded sample, and the
    NumPy float32 oracle on a shorter one as the secondary number."""
    from oracle import cpu_port
    out = cpu_port.time_steps(D, list(WIDTHS), BS, NEG, budget_s=seconds, scaling=(1, 2, 4, 8, 16))
    if "C/OpenMP" in out.get("sample", ""):
        sec = cpu_port.time_steps(D, list(WIDTHS), BS, NEG, budget_s=min(5.0, seconds / 3), use_c=False)
        out["numpy_oracle"] = {k: sec[k] for k in ("value", "unit", "cores", "sample")}
    return out


def parity_vs_oracle(dev, batch, trained: dict) -> dict:
    """Each mode's measured error against the reference's precision (north star:
    <= 1e-4 relative on the loss and cosine scores).  Part of the cpu_baseline leg -- the one place
    bench.py may call the checker: a fresh plan per mode (bf16 perf mode, bf16 with the fp32-accurate
    forward of plan option FWD32, fp32 parity mode) runs
    ONE training forward + backward on the bench's first staged C2 batch, and the float64 NumPy
    oracle (oracle/dssm_oracle.py, new_dssm.py:117-213) runs the same step on the same parameters.
    Two states: the Glorot init (seed 0, new_dssm.py:118-120) and the bench model's own parameters
    after its timed steps (`trained`).  Reported, not asserted (the tests hold the bars)."""
    import torch
    from oracle import dssm_oracle as O
    from dssm_amd.model import DSSM
    cfg = O.OracleConfig(trigram_d=D, widths=list(WIDTHS), query_bs=BS, neg=NEG)
    states = {"init": O.init_params(cfg, seed=0), "trained": trained}
    out = {"what": "one fwd+bwd step on bench batch 0 vs the float64 oracle: loss |rel|, cos_sim_raw / prob "
                   "max |abs| (cos also / max|cos|), per weight gradient max|err| / max|g| (biases excluded: "
                   "d loss / d b is 0 under batch-stat BN)",
           "batch": {"rows": int(batch.rows), "nnz": int(batch.nnz)}}
    ora = {}
    for sname, p in states.items():
        cache, _ = O.forward(cfg, p, O.make_ema(cfg), batch.as_dict(), True, np.float64)
        ora[sname] = (cache, O.backward(cfg, p, cache, np.float64))
    for mode in ("bf16", "bf16_fwd32", "fp32"):
        dtype = "fp32" if mode == "fp32" else "bf16"
        m = DSSM(D, WIDTHS, BS, NEG, dtype=dtype, init=False, device=dev)
        m.set_fused_w1_adam(False)  # materialise dW1 to read it
        if mode == "bf16_fwd32":
            m.set_option("FWD32", True)
        res = {}
        for sname, p in states.items():
            cache, grads = ora[sname]
            m.load_params(p)
            m.set_batch(batch)
            m.forward(True)
            m.backward()
            torch.cuda.synchronize(dev)
            loss, _ = m.loss_accuracy()
            cos = m.fetch("cos_sim_raw").ravel().astype(np.float64)
            prob = m.fetch("prob").astype(np.float64)
            gg = {k: v.cpu().numpy().astype(np.float64) for k, v in m.named_grads().items()}
            cerr = float(np.abs(cos - cache["cos_sim_raw"]).max())
            res[sname] = {
                "loss": round(float(loss), 7), "loss_oracle": round(float(cache["loss"]), 7),
                "loss_rel_err": float(f"{abs(loss - cache['loss']) / abs(cache['loss']):.3e}"),
                "cos_abs_err": float(f"{cerr:.3e}"),
                "cos_err_over_max": float(f"{cerr / np.abs(cache['cos_sim_raw']).max():.3e}"),
                "prob_abs_err": float(f"{np.abs(prob - cache['prob']).max():.3e}"),
                "grad_err_over_max": {k: float(f"{np.abs(gg[k] - g).max() / max(np.abs(g).max(), 1e-30):.3e}")
                                      for k, g in grads.items() if k.startswith("W")},
            }
        res["meets_1e-4"] = all(r["loss_rel_err"] <= 1e-4 and r["cos_abs_err"] <= 1e-4
                                for k, r in res.items() if k in states)
        out[mode] = res
        del m
        torch.cuda.empty_cache()
    return out


def fp32_mode_line(args) -> dict:
    """The fp32 parity mode (fp32 weights, activations and MFMA 16x16x4 f32) of the same C2
    workload, K timed steps after W warm-up steps, timed by this script in a child process (a
    fresh plan and arenas; the child prints its own line, summarised here)."""
    return child_mode_line(args, ["--dtype", "fp32"])


def deterministic_mode_line(args) -> dict:
    """The same bf16 C2 workload under the plan option DETERMINISTIC (fused statistics summed in a
    fixed order, CSC columns in row order, heavy dW1 rows in item order: run-to-run bit-identical,
    tests/test_gpu_deterministic.py), timed in a child process as fp32_mode_line."""
    return child_mode_line(args, ["--deterministic", "1"])


def child_mode_line(args, extra) -> dict:
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--batches", str(args.batches), "--cpu-baseline", "0",
           "--fwd-only", "0", "--fp32-line", "0", "--det-line", "0", "--fwd32-line", "0",
           "--probes", str(args.probes)] + extra
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not lines:
            return {"error": f"exit {r.returncode}: {r.stderr[-400:]}"}
        d = json.loads(lines[-1])
    except Exception as e:  # reported, never fatal for the headline
        return {"error": repr(e)}
    keep = ("value", "unit", "ms_per_step", "steps", "warmup", "dtype", "roofline", "kernels_ms", "final_loss",
            "schedule")
    return {k: d[k] for k in keep if k in d}


def bench_rnn(args):
    """BASELINE.json config 4 (the reference's dssm_rnn tower, dssm_rnn.py:100-218): word embeddings
    (21,128-token vocabulary, data/vocab.txt's size) -> bidirectional GRU(128) over 32 ids per row ->
    dropout 0.5 -> x20 cosine / softmax, BS=1024, NEG=4; fp32; synthetic ids (uniform, full
    lengths as the reference feeds); one step = forward + BPTT + Adam.  --dtype bf16 (default): the
    MFMA recurrences of csrc/rnn_mfma.hip; fp32: the parity mode.  Not the headline."""
    import torch
    from dssm_amd.rnn import RnnDSSM
    V, E, H, T = 21128, 128, 128, 32
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = RnnDSSM(V, E, H, BS, NEG, T, lr=1e-5, keep_prob=0.5, device=dev, dtype=args.dtype)
    m.init_params(0)
    rng = np.random.Generator(np.random.PCG64(4))
    batches = [rng.integers(1, V, size=(m.R, T)).astype(np.int32) for _ in range(4)]
    staged = []
    for b in batches:  # device-resident ids, swapped in by pointer copy-free assignment
        staged.append(torch.from_numpy(b).to(dev))
    def step(i):
        m.ids = staged[i % len(staged)]
        m.train_step()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    probe = args.dtype == "bf16" and args.probes
    region = None
    if args.graph and args.steps <= 256:
        # the timed region as ONE graph of exactly K steps (each captured step keeps its own dropout
        # mask index); the BPTT probe = two event-record nodes around the LAST step's BPTT launch only
        # (around every step they cost ~11 us/step of node gaps inside the timed region)
        region = torch.cuda.CUDAGraph()
        with torch.cuda.graph(region, stream=stream):
            for i in range(args.steps):
                if probe and i == args.steps - 1:
                    m.lib.dssm_rnn_bf16_probe(1)
                step(args.warmup + i)
        torch.cuda.synchronize()
    elif probe:  # eager: HIP events around every timed BPTT launch, on the stream it runs on
        m.lib.dssm_rnn_bf16_probe(args.steps)
    t0 = time.perf_counter()
    if region is not None:
        region.replay()
    else:
        for i in range(args.steps):
            step(args.warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = {"metric": "query-doc pairs/sec (fwd+bwd), dssm_rnn tower (BASELINE config 4)",
           "value": round(BS * (NEG + 1) * args.steps / el, 1), "unit": "pairs/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
           "data": "synthetic",
           "config": {"workload": "dssm_rnn: vocab 21128, emb 128, BiGRU(128), seq_len 32, dropout 0.5, "
                                  "BS=1024, NEG=4, fwd+BPTT+Adam", "global_batch": BS, "neg": NEG,
                      "parallelism": "dp1", "launch": "hipgraph: one graph of K steps" if region is not None
                      else "eager"},
           "final_loss": round(m.loss(), 3)}
    if probe:
        import ctypes as C
        avg, cnt = C.c_double(), C.c_int()
        m.lib.dssm_rnn_bf16_probe_read(C.byref(avg), C.byref(cnt))
        m.lib.dssm_rnn_bf16_probe(0)
        # BPTT algorithmic bytes: per (direction, step, row, hidden column) the
        # (r, u, c, h_{t-1}) cache read (8 B) and dr, du, dc written (6 B); dx written per input
        # column (2 B); the incoming final-state gradient (fp32)
        R = m.R
        bptt = 2 * T * R * (H * 14 + E * 2) + R * 2 * H * 4
        ms = avg.value
        out["roofline"] = {"bound": "hbm", "achieved": round(bptt / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(bptt / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "traffic": None, "kernel": "k_gru_bwd_mfma", "bytes_per_launch": bptt,
                           "avg_ms": round(ms, 5), "launches": cnt.value}
        t, src = model_profile("traffic", "rnn", "k_gru_bwd_mfma<128, 128, 3>")
        if t is not None:
            out["roofline"].update(traffic=t["hbm_bytes"], traffic_source=src)
        mf = {k: model_profile("mfma", "rnn", k) for k in ("k_gru_fwd_mfma<128, 128, 3>",
                                                          "k_gru_bwd_mfma<128, 128, 3>", "k_rnn_dw")}
        out["mfma"] = {k.split("<")[0]: {x: v[x] for x in ("tflops", "frac_of_peak", "mfma_busy") if x in v}
                       for k, (v, _) in mf.items() if v is not None} or None
    if args.cpu_baseline:
        try:  # the C/OpenMP fp32 restatement (oracle/cpu_c/rnn_cpu.c, test infrastructure) on the host
            from oracle import cpu_c
            host = [b for b in batches]
            out["cpu_baseline"] = cpu_c.rnn_time_steps(V, E, H, BS, NEG, T, m.named(), host, keep=0.5,
                                                       budget_s=min(args.cpu_seconds, 20.0))
            out["cpu_baseline"]["cpu_model"] = cpu_model()
        except Exception as e:
            out["cpu_baseline"] = {"error": repr(e)}
    print(json.dumps(out), flush=True)


def bench_multiview(args):
    """BASELINE.json config 5 (archive/multi_view_dssm_v3.py): user tower + 3 item views (30k-wide
    sparse inputs, FC 300 -> 128, ReLU), in-batch rotated negatives, NEG=4, BS=4096 on one GPU,
    synthetic Zipf trigram rows; the active view cycles 1, 2, 3 over the staged batches.  --dtype
    bf16 (default: the perf mode, bf16 weight shadows / activations / MFMA, fp32 masters and Adam)
    or fp32 (the parity mode, also timed as fp32_mode beside a bf16 line).  One step = forward +
    backward + Adam (user tower + active view).  Not the headline."""
    import torch
    import torch.distributed as dist
    from dssm_amd.data import ZipfColumns, synth_rows
    from dssm_amd.multiview import MultiViewDataParallel, MultiViewDSSM
    B, Dv, L1, L2 = 4096, 30000, 300, 128
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count()) if args.backend == "gloo" else local  # gloo: rehearsal
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:  # config 5 on N GPUs: BS users per rank, gradient all-reduce (weak scaling)
        dist.init_process_group(args.backend, device_id=dev if args.backend == "nccl" else None)
    m = MultiViewDSSM(Dv, [Dv, Dv, Dv], L1, L2, B, NEG, lr=0.05, device=dev, dtype=args.dtype,
                      csc_stream=bool(args.mv_csc_stream))
    m.init_params(0)
    dp = MultiViewDataParallel(m, comm=args.comm) if world > 1 else None
    cols = ZipfColumns(Dv)
    rng = np.random.Generator(np.random.PCG64(7 + rank))
    feeds, host_feeds = [], []
    for b in range(3):
        u = synth_rows(rng, cols, B, 32.0)
        it = synth_rows(rng, cols, B, 32.0)
        m.set_batch(u, it, b + 1)
        feeds.append((dict(m.batch), b + 1))
        host_feeds.append((u, it, b + 1))

    # Adam (user tower + active view, one optimizer launch each) is the dominant kernel: libdssm's
    # dssm_adam_probe records HIP events around each launch on the stream it runs on (inside the
    # captured Adam graphs: event-record nodes timing every replay, read for the latest)
    # hipGraph replay (--graph 1): per staged feed one graph for forward + backward (both towers'
    # streams, fork / join captured) and one for the two Adam launches, so the ~30 host calls of a
    # step (ctypes + stream bookkeeping, about as long as the GPU work) leave the timed loop; the
    # Adam probes bracket the Adam graph's replay on the stream it runs on
    fb_graphs, adam_graphs, region = [], [], None
    stream = torch.cuda.Stream()

    def eager(i):
        m.batch, m.view = dict(feeds[i % 3][0]), feeds[i % 3][1]
        m.forward()
        m.backward()
    with torch.cuda.stream(stream):
        for i in range(max(args.warmup, 3)):
            eager(i)
            if dp is not None:
                dp.exchange()
            m.apply_adam(grad_scale=1.0 / world)
        torch.cuda.synchronize()
        if args.graph and dp is None and args.steps <= 256:
            # one GPU: the whole timed region as ONE graph of exactly K steps (no launch gaps between
            # steps); the Adam probe records the last step's two optimizer launches
            region = torch.cuda.CUDAGraph()
            with torch.cuda.graph(region, stream=stream):
                for i in range(args.steps):
                    j = args.warmup + i
                    m.batch, m.view = dict(feeds[j % 3][0]), feeds[j % 3][1]
                    m.forward()
                    m.backward(join=False)  # fused optimizer: each tower's launch follows on its stream
                    if i == args.steps - 1:
                        m.lib.dssm_adam_probe(2)
                    m.apply_adam(grad_scale=1.0)
        elif args.graph:
            m.lib.dssm_adam_probe(6)  # the 3 Adam graphs' 2 launches each
            for i in range(3):
                m.batch, m.view = dict(feeds[i][0]), feeds[i][1]
                g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g1, stream=stream):
                    m.forward()
                    m.backward()
                with torch.cuda.graph(g2, stream=stream):
                    m.apply_adam(grad_scale=1.0 / world)
                fb_graphs.append(g1)
                adam_graphs.append(g2)

    def step(i):
        if args.graph:
            fb_graphs[i % 3].replay()
            m.view = feeds[i % 3][1]  # the replayed feed's active view: the ranges the exchange sums
        else:
            eager(i)
        if dp is not None:
            dp.exchange()  # between the graphs: RCCL all-reduce of the trained towers' gradients
        if args.graph:
            adam_graphs[i % 3].replay()
        else:
            m.apply_adam(grad_scale=1.0 / world)
    torch.cuda.set_stream(stream)
    if not args.graph:
        m.lib.dssm_adam_probe(2 * args.steps)
    torch.cuda.synchronize()
    if dp is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if region is not None:
        region.replay()
    else:
        for i in range(args.steps):
            step(args.warmup + i)
    torch.cuda.synchronize()
    if dp is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dp is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    import ctypes as C
    avg, cnt = C.c_double(), C.c_int()
    from dssm_amd._lib import check
    check(m.lib.dssm_adam_probe_read(C.byref(avg), C.byref(cnt)), "adam_probe_read")
    adam_ms = avg.value  # per launch
    span_ms = None
    if m.fused_w1_adam and cnt.value >= 2:
        # the two towers' launches run concurrently (two streams): the roofline is over the pair's
        # wall span (latest end - earliest start), each step's pair of recorded launches
        spans = []
        for k in range(cnt.value // 2):
            sp = C.c_double()
            check(m.lib.dssm_adam_probe_span(2 * k, 2, C.byref(sp)), "adam_probe_span")
            spans.append(sp.value)
        span_ms = float(np.mean(spans))
    m.lib.dssm_adam_probe(0)
    tower_params = sum(m.layout[t][1] - m.layout[t][0] for t in ("user", "view1")) / 2
    shadow_elems = (Dv * L1 + L1 * L2) if args.dtype == "bf16" else 0
    if m.fused_w1_adam:
        # one launch per trained tower (dssm_spmm_bwd_w_adam): p, m, v read + written (24 B) per
        # parameter; [W1; b1]'s gradient gathered from the CSC transpose ((index, value) 8 B + one dz1
        # row per entry, nnz + BS entries: the ones column), FC2's split-K partials read (4 B x splits);
        # bf16: + 2 B per weight written to its shadow.  nnz: the staged batches' mean per tower.
        nnz = float(np.mean([int(f[k][0][-1].item()) for f, _ in feeds for k in ("u", "i")]))
        w2 = (L1 + 1) * L2
        splits = max(1, m._splits["u"].value)
        zb = 2 if args.dtype == "bf16" else 4
        adam_bytes = int(24 * tower_params + 4 * splits * w2 + (nnz + B) * (8 + zb * L1) + 2 * shadow_elems)
        adam_kernel = "k_adam_step<unsigned short, false>" if args.dtype == "bf16" else "k_adam_step<float, false>"
    else:
        # p, m, v read + written (24 B) and the fp32 gradient read (4 B) per parameter of the tower; bf16
        # mode: + 2 B per weight written to its shadow, and ONE launch updates both trained towers
        towers_per_launch = 2 if args.dtype == "bf16" else 1
        adam_bytes = int(towers_per_launch * (28 * tower_params + 2 * shadow_elems))
        adam_kernel = "k_adam_flat_shadow" if args.dtype == "bf16" else "k_rnn_adam"
    achieved = (2 * adam_bytes / (span_ms * 1e-3) if span_ms else adam_bytes / (adam_ms * 1e-3)) / 1e9
    out = {"metric": "query-doc pairs/sec (fwd+bwd), multi-view DSSM (BASELINE config 5)",
           "value": round(world * B * (NEG + 1) * args.steps / el, 1), "unit": "pairs/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
           "data": "synthetic",
           "config": {"workload": "multi_view_dssm_v3: user + 3 views (30k sparse -> 300 -> 128), in-batch "
                                  "rotated negatives, BS=4096 per GPU, NEG=4, fwd+bwd+Adam", "global_batch": B * world,
                      "neg": NEG, "parallelism": f"dp{world}",
                      "launch": ("hipgraph: one graph of K steps" if region is not None else "hipgraph") if args.graph else "eager",
                      "dp_exchange": dp.comm if dp is not None else None,
                      "csc_stream": bool(m.csc_stream and m.fused_w1_adam)},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                        "kernel": adam_kernel,
                        "bytes_per_launch": adam_bytes, "avg_ms": round(adam_ms, 5), "launches": cnt.value,
                        **({"pair_span_ms": round(span_ms, 5),
                            "note": "the two towers' launches run concurrently: achieved = 2 x bytes_per_launch "
                                    "/ pair_span_ms"} if span_ms else {})},
           "final_loss": round(m.loss(), 3)}
    t, src = model_profile("traffic", "multiview" if args.dtype == "fp32" else "multiview_bf16",
                           out["roofline"]["kernel"])
    if t is not None:
        out["roofline"].update(traffic=t["hbm_bytes"], traffic_source=src)
    if args.dtype == "bf16" and args.fp32_line and rank == 0 and world == 1:
        out["fp32_mode"] = child_mode_line(args, ["--model", "multiview", "--dtype", "fp32"])
    if dp is not None and args.dp_check:
        out["dp_check"] = dp_check(m, dp, dev)
    if args.cpu_baseline and rank == 0 and world == 1:
        try:  # the NumPy float32 restatement (oracle/, test infrastructure) on the host
            from oracle import cpu_port
            from oracle.multiview_oracle import MvConfig
            cfg = MvConfig(Dv, [Dv, Dv, Dv], L1, L2, B, NEG, lr=0.05)
            host = [(u, it, v, m.rot) for u, it, v in host_feeds]
            out["cpu_baseline"] = cpu_port.time_multiview_steps(cfg, m.named(), host,
                                                                budget_s=min(args.cpu_seconds, 20.0))
            out["cpu_baseline"]["cpu_model"] = cpu_model()
        except Exception as e:
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dp is not None:
        dp.close()
        dist.destroy_process_group()


def fwd_only(model, staged, args, stream):
    """Forward alone, eval mode (on_train=False: EMA-BN, cosine, softmax, loss; new_dssm.py:85-86,
    274-285) over the staged batches, after the training measurement (the step's own forward is
    not separable in time: the training forward also builds the CSC transpose for the backward).
    As the training measurement: the staged batches' forwards captured back to back into ONE graph
    replayed per full cycle (eager launches for a partial cycle, or where capture fails)."""
    import torch
    cycle = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(cycle, stream=stream):
            for ip, ix, vv in staged:
                model.set_batch(indptr=ip, indices=ix, values=vv)
                model.forward(False)
        launch = "hipgraph"
    except Exception:  # capture unsupported: eager launches
        cycle, launch = None, "eager"

    def run(i0, n):
        i = i0
        while i < i0 + n:
            if cycle is not None and i % len(staged) == 0 and i + len(staged) <= i0 + n:
                cycle.replay()
                i += len(staged)
                continue
            ip, ix, vv = staged[i % len(staged)]
            model.set_batch(indptr=ip, indices=ix, values=vv)
            model.forward(False)
            i += 1
    run(0, args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(0, args.steps)  # from batch 0: whole cycles first
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"mode": "eval (EMA-BN) forward + cosine + loss", "launch": launch,
            "ms_per_step": round(1e3 * el / args.steps, 4),
            "value": round(BS * (NEG + 1) * args.steps / el, 1), "unit": "pairs/s"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.model == "rnn":
            raise SystemExit("--model rnn is a single-GPU row (BASELINE config 4)")
        sys.exit(spawn_ranks(args))  # before any GPU call: the ranks are children
    if args.model == "rnn":
        return bench_rnn(args)
    if args.model == "multiview":
        return bench_multiview(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    local = local % max(1, torch.cuda.device_count()) if args.backend == "gloo" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from dssm_amd import _lib
    from dssm_amd.model import DSSM
    from dssm_amd.data import ZipfColumns, synth_batch

    model = DSSM(D, WIDTHS, BS, NEG, dtype=args.dtype, seed=0, device=dev)
    if args.deterministic:
        model.set_option("DETERMINISTIC", True)
    if args.fwd32:
        model.set_option("FWD32", True)
    for opt in args.plan_option:
        name, val = opt.split("=")
        model.set_option(name, bool(int(val)))
    dp = None
    if world > 1:
        from dssm_amd.dist import DataParallel
        dp = DataParallel(model, comm=args.comm, mode=args.dp_mode, wire=args.wire, chunks=args.dp_chunks,
                          sparse=bool(args.dp_sparse), exchange=args.dp_exchange)
    rehearse = args.rehearse_world if world == 1 else 1
    if rehearse > 1:
        # rank 0's kernels of a W-rank bf16-wire step in the data-parallel step graph, each
        # collective replaced by a modelled link time or a device copy (analysis of the N>1 path)
        model.set_fused_w1_adam(False)
        nw = model.dp_wire_size(rehearse, args.dp_chunks)
        wires = [torch.zeros(nw, dtype=torch.bfloat16, device=dev) for _ in range(3)]
        model.set_dp_wire(rehearse, 0, args.dp_chunks, *wires)
        if args.rehearse_comm == "peer":  # rank 0 of the peer-store exchange, the peers' buffers local
            from dssm_amd.dist import RehearsalPeers
            if args.dp_chunks != 1:
                raise SystemExit("--rehearse-comm peer: one wire chunk")
            geo = model.dp_geometry()
            rehearsal_peers = RehearsalPeers(rehearse, nw, geo["n_params"] - geo["extent"], dev)
            model.set_dp_wire(rehearse, 0, 1, wires[0], rehearsal_peers.stage, rehearsal_peers.param_wire)
            a = rehearsal_peers.addr
            model.set_dp_peers(rehearse, a["stage"], a["pwire"], a["tail"], a["flags"])

    cols = ZipfColumns(D, uniform=args.columns == "uniform")
    staged = []
    nnzs = []
    for b in range(args.batches):
        hb = synth_batch(D, BS, NEG, seed=1000 + rank * 100003 + b, cols=cols)
        nnzs.append(hb.nnz)
        staged.append((torch.from_numpy(hb.indptr).to(dev),
                       torch.from_numpy(hb.indices).to(dev),
                       torch.from_numpy(hb.values).to(dev)))
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)  # graph capture needs a non-default stream
    torch.cuda.set_stream(stream)
    probe_ids = (("spmm_fwd", _lib.PROBE_SPMM_FWD), ("adam", _lib.PROBE_ADAM),
                 ("dw1", _lib.PROBE_DW1), ("csc_build", _lib.PROBE_CSC))


    # data parallel on the library's RCCL communicator (or its one-GPU rehearsal): the warm-up and
    # the timed region are each ONE graph of exactly that many whole steps, collectives included
    # (dssm_plan_graph_build_dp_steps; step i+1's rank pass in step i's Adam); longer runs replay a
    # cycle of len(staged) steps plus a partial one.  A capture the runtime refuses falls back to
    # split graphs with host-issued collectives, recorded in the line.
    region_graphs, dp_capture_error = None, None
    dp_events = []  # split-graph data parallel: (phase, start, end) events of the last timed step
    if args.graph and args.feed == "device" and (rehearse > 1 or (dp is not None and dp.capturable)):
        MAX_REGION_STEPS = 256
        comm_mode = 0 if rehearse == 1 else {"copy": 1, "model": 2, "peer": 3}[args.rehearse_comm]

        def dp_graph(batches, probes=False):
            if rehearse == 1:
                return dp.build_region(batches, probes=probes)
            return model.graph_build_dp_steps(batches, 1.0 / rehearse, comm=comm_mode, link_gbps=args.link_gbps,
                                              latency_us=args.link_latency_us, probes=probes)
        try:
            reg, cyc, part = {}, None, {}
            for n in {args.warmup, args.steps} - {0}:
                if n <= MAX_REGION_STEPS:
                    reg[n] = dp_graph([staged[i % len(staged)] for i in range(n)], probes=bool(args.probes))
            if max(args.warmup, args.steps) > MAX_REGION_STEPS:
                cyc = dp_graph(staged, probes=bool(args.probes))
                for r in {args.warmup % len(staged), args.steps % len(staged)} - {0}:
                    part[r] = dp_graph(staged[:r], probes=bool(args.probes))
            region_graphs = (reg, cyc, part)
        except Exception as e:
            if rehearse > 1:
                raise
            dp_capture_error = repr(e)
            print(f"bench: the data-parallel step graph could not be captured ({e}); split graphs instead",
                  file=sys.stderr, flush=True)

    feeder = None
    if args.feed == "host":
        if world > 1 or rehearse > 1 or not args.graph:
            raise SystemExit("--feed host is the N=1 graph-mode measurement")
        # the staged batches re-laid out as the reference's three host CSR matrices; the native
        # feeder assembles each step's combined CSR in pinned memory and copies it on its own
        # stream while the previous step runs; one captured step per feeder slot
        import scipy.sparse as sps
        from dssm_amd.data import csr_rows_slice
        from dssm_amd.feed import Feeder
        hosts = [synth_batch(D, BS, NEG, seed=1000 + b, cols=cols) for b in range(args.batches)]
        mats = []
        for r0, r1 in ((0, BS), (BS, 2 * BS), (2 * BS, BS * (2 + NEG))):
            parts = [csr_rows_slice(h, r0, r1) for h in hosts]
            mats.append(sps.vstack([sps.csr_matrix((p.values, p.indices, p.indptr), shape=(r1 - r0, D))
                                    for p in parts]).tocsr())
        feeder = Feeder(*mats, BS, NEG, max_nnz=model.max_nnz)
        gslots = []
        for slot in range(2):
            feeder.start(slot)
            feeder.next(model)
            gslots.append(model.graph_build(probes=bool(args.probes) and slot == 0))
            feeder.done()
        torch.cuda.synchronize()
        feeder.start(0)
        graphs, adam_graph, cycle, region, probe_graph, split = gslots, None, None, {}, None, False

        def run_steps(i0, n):
            for i in range(i0, i0 + n):
                feeder.next(model, next_batch=(i + 1) % args.batches)
                model.graph_launch(gslots[feeder._cur])
                feeder.done()
    elif region_graphs is not None:
        graphs, adam_graph, probe_graph, split, partial, cycle, region = (None, None, None, True,
                                                                          region_graphs[2], region_graphs[1],
                                                                          region_graphs[0])

        def run_steps(i0, n):
            if n in region:
                model.graph_launch(region[n])
                return
            for _ in range(n // len(staged)):
                model.graph_launch(cycle)
            if n % len(staged):
                model.graph_launch(partial[n % len(staged)])
    elif args.graph and dp is not None:
        # data parallel: per staged batch a captured fwd+bwd graph (and the variant that first
        # rebuilds the shadows from the previous step's all-gathered update), one Adam graph, the
        # exchange's collectives between them (dssm_amd.dist.DataParallel.build_graphs)
        dp.build_graphs(staged, probe_batch=(args.warmup % len(staged)) if args.probes else None)
        graphs, adam_graph, cycle, region, probe_graph, split = None, None, None, {}, None, True

        def run_steps(i0, n):
            for i in range(i0, i0 + n):
                # the timed region's last step: its phases bracketed by events on the stream
                last = bool(args.probes) and i0 == args.warmup and i == i0 + n - 1
                dp.graph_step(i, events=dp_events if last else None)
    elif args.graph:
        # One captured step per staged batch (the batch pointers are baked into the graph).  Timing
        # probes are event nodes inside the graphs (their last replay is read after the timed region).
        graphs = []
        # Probes (graph event-record nodes cost a few us each) ride in batch 0's graph only, so
        # they are sampled once per len(staged) steps inside the timed region.
        split, adam_graph = False, None
        for b, (ip, ix, vv) in enumerate(staged):
            model.set_batch(indptr=ip, indices=ix, values=vv)
            # the probes ride in the graph of the timed region's first step (batch W mod len(staged))
            pr = bool(args.probes) and b == args.warmup % len(staged) and not args.multi_step
            graphs.append(model.graph_build(probes=pr))

        # single GPU: a run of up to MAX_REGION_STEPS steps (the warm-up, the timed region) is ONE
        # multi-step graph of exactly that many steps over the batches in order (one launch, one
        # separate rank launch: a second, partial graph would add its own launch gap and rank
        # launch); longer runs replay a cycle graph of len(staged) steps plus a partial one.
        # Its only probe is the Adam one (the roofline's kernel: two event-record nodes; the eight
        # of the full set cost ~3.7 us/step at K = 20); the secondary probes (transpose, SpMM, dW1)
        # time one untimed replay of a probed cycle after the timed region.
        MAX_REGION_STEPS = 256
        cycle, partial, region, probe_graph = None, {}, {}, None
        if not split and args.multi_step:
            for n in {args.warmup, args.steps} - {0}:
                if n <= MAX_REGION_STEPS:
                    region[n] = model.graph_build_steps([staged[i % len(staged)] for i in range(n)],
                                                        probes="adam" if args.probes else False)
            if region and args.probes:
                probe_graph = model.graph_build_steps(staged, probes=True)
            if max(args.warmup, args.steps) > MAX_REGION_STEPS:
                cycle = model.graph_build_steps(staged, probes=bool(args.probes))
                for r in {args.warmup % len(staged), args.steps % len(staged)} - {0}:
                    partial[r] = model.graph_build_steps(staged[:r], probes=bool(args.probes))

        def run_steps(i0, n):
            if n in region:
                model.graph_launch(region[n])
                return
            if cycle is None:
                for i in range(i0, i0 + n):
                    step(i)
                return
            for _ in range(n // len(staged)):
                model.graph_launch(cycle)
            if n % len(staged):
                model.graph_launch(partial[n % len(staged)])

        def step(i):
            model.graph_launch(graphs[i % len(graphs)])
    else:
        def step(i):
            ip, ix, vv = staged[i % len(staged)]
            model.set_batch(indptr=ip, indices=ix, values=vv)
            model.forward(True)
            model.backward()
            if world > 1:
                dp.exchange_before_adam()
            model.apply_adam(1.0 / max(world, rehearse))
            if dp is not None and dp.mode == "zero":
                dp.exchange_after_adam()
                dp.refresh_shadows()
            elif rehearse > 1:
                model.wire_shadows()

    if not args.graph and feeder is None:
        cycle = None

        def run_steps(i0, n):
            for i in range(i0, i0 + n):
                step(i)
    if args.idle_before_warmup > 0:  # analysis only: host idle time between the graph builds and the warm-up
        time.sleep(args.idle_before_warmup)
    if args.busy_before_warmup > 0:  # analysis only: a dense matmul load right before the warm-up
        xa = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        tb = time.perf_counter()
        while time.perf_counter() - tb < args.busy_before_warmup:
            for _ in range(8):
                xa = (xa @ xa).clamp_(-1, 1)
            torch.cuda.synchronize()
        del xa
    run_steps(0, args.warmup)
    torch.cuda.synchronize()
    if not args.graph and args.probes:
        for _, pid in probe_ids:
            model.probe_enable(pid, args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.warmup, args.steps)
    host_launch = time.perf_counter() - t0  # host time to submit the timed region's launches
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dp is not None and args.graph:
        dp.settle()  # untimed: a last split-graph step's shadow refresh (none after a captured region)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss, acc = model.loss_accuracy()
    check = dp_check(model, dp, dev) if (dp is not None and args.dp_check) else None
    fwd = fwd_only(model, staged, args, stream) if (args.fwd_only and world == 1 and rehearse == 1
                                                   and feeder is None) else None

    dp_kernels = None
    if (world > 1 or rehearse > 1) and args.probes and args.graph and region_graphs is not None:
        # the captured region's last step: its phases' event-record nodes (DSSM_PROBE_DP_*)
        g = region[args.steps] if args.steps in region else (
            cycle if args.steps % len(staged) == 0 else partial[args.steps % len(staged)])
        dp_kernels = {k: round(model.graph_probe_read(g, pid), 5) for k, pid in _lib.DP_PROBES.items()}
        dp_kernels["adam"] = round(model.graph_probe_read(g, _lib.PROBE_ADAM), 5)
        dp_kernels["source"] = "event-record nodes in the captured region's last step"
    elif world > 1 and args.probes and args.graph and dp is not None and dp_events:
        torch.cuda.synchronize()
        dp_kernels = {name: round(a.elapsed_time(b), 5) for name, a, b in dp_events}
        dp_kernels["source"] = "torch.cuda events around the timed region's last step (host-issued exchange)"
    probes = {}
    if args.graph and probe_graph is not None:
        model.graph_launch(probe_graph)  # untimed: the secondary probes' replay
        torch.cuda.synchronize()
    for name, pid in (probe_ids if args.probes else ()):
        if args.graph and region_graphs is not None:
            if name == "adam":  # the data-parallel region: its last step's Adam chunks
                g = region[args.steps] if args.steps in region else (
                    cycle if args.steps % len(staged) == 0 else partial[args.steps % len(staged)])
                probes[name] = model.graph_probe_read(g, pid)
            continue
        if args.graph and dp is not None:  # the timed region's first step's graphs, the Adam graph
            plain, merged_g, adam_g = dp.graph_ids()
            g = adam_g if name == "adam" else (merged_g if merged_g and args.warmup > 0 else plain)[
                args.warmup % len(plain)]
            probes[name] = model.graph_probe_read(g, pid)
            continue
        if args.graph:  # last replay of every staged-batch graph, all inside the timed region
            g = ((region[args.steps] if name == "adam" else probe_graph) if args.steps in region else
                 (cycle if args.steps >= len(staged) else partial[args.steps]) if cycle is not None else
                 (graphs[0] if feeder is not None else graphs[args.warmup % len(graphs)]))
            probes[name] = model.graph_probe_read(g, pid)
        else:
            tot, cnt = model.probe_read(pid)
            probes[name] = tot / max(cnt, 1)  # ms per launch
    ms_per_step = 1e3 * elapsed / args.steps
    pairs = world * BS * (NEG + 1) * args.steps
    value = pairs / elapsed

    # roofline of the dominant HBM-bound kernels (algorithmic bytes / measured avg duration)
    rows = BS * (2 + NEG)
    nnz_avg = int(nnzs[0] if args.graph else np.mean( [nnzs[(args.warmup + i) % len(nnzs)] for i in range(args.steps)]))
    s_w = 2 if args.dtype == "bf16" else 4
    n_params = int(model.n_params)
    w1_elems = (D + 1) * WIDTHS[0]
    fused = world == 1 and rehearse == 1
    wire_elems, range_elems, wire_parts = 0, n_params, 1
    if dp is not None and dp.mode == "zero":
        if dp.wire == "bf16":
            wire_elems = max(0, dp.end - dp.begin)
            range_elems = wire_elems + (n_params - dp.extent)
            wire_parts = world
        else:
            range_elems = max(0, dp.end - dp.begin)
    elif rehearse > 1:
        geo = model.dp_geometry()
        wire_elems = geo["shard_end"] - geo["shard_begin"]
        range_elems = wire_elems + (n_params - geo["extent"])
        wire_parts = rehearse
    kern = {
        "spmm_fwd": (spmm_alg_bytes(nnz_avg, rows, WIDTHS[0], s_w), probes.get("spmm_fwd", 0.0)),
        "adam": (adam_alg_bytes(n_params, args.dtype == "bf16", fused, w1_elems, nnz_avg, rows,
                                WIDTHS[0], range_elems, wire_elems, wire_parts), probes.get("adam", 0.0)),
    }
    # committed PMC summaries profile single-GPU steps (fused Adam) of a named workload
    workload = {"dtype": args.dtype, "columns": args.columns, "feed": args.feed}
    traffic, traffic_src = pmc_traffic(workload) if fused else ({}, None)
    rl = {}
    for k, (byt, ms) in kern.items():
        gbs = byt / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        rl[k] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": byt,
                 "avg_ms": round(ms, 5), "traffic": traffic.get(k),
                 "traffic_source": traffic_src if k in traffic else None}
    dominant = max(kern, key=lambda k: kern[k][1])

    out = {
        "metric": "query-doc pairs/sec (fwd+bwd), TRIGRAM_D=30k NEG=4, 1/2/4/8 MI355X",
        "value": round(value, 1), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
        "config": {"workload": "dssm C2: TRIGRAM_D=30000, widths 300/300/128, NEG=4, "
                               + ("Zipf(1.1)" if args.columns == "zipf" else "uniform-column")
                               + " trigram batches ~32 nnz/row, fwd+bwd+dense Adam",
                   "global_batch": BS * world, "per_gpu_query_bs": BS, "neg": NEG,
                   "trigram_d": D, "widths": list(WIDTHS), "parallelism": f"dp{world}",
                   "avg_nnz_per_step": nnz_avg, "launch": "hipgraph" if args.graph else "eager",
                   "dp_exchange": dp.schedule if dp is not None else None,
                   "dp_fallbacks": dp.fallbacks if dp is not None else None,
                   **({"dp_sparse": {"steps": dp.sparse_stats["steps"],
                                     "rows_sent_frac": round(dp.sparse_stats["rows_sent"]
                                                             / max(1, dp.sparse_stats["rows_dense"]), 4)}}
                      if dp is not None and dp.sparse else {}),
                   "feed": "host CSR -> pinned async H2D (native feeder), PCIe inside the timed region"
                           if feeder is not None else "device-resident staged batches"},
        "roofline": dict(rl[dominant], kernel=dominant),
        "kernels_ms": {k: round(v, 5) for k, v in probes.items()},
        "rooflines": rl,
        "final_loss": round(loss, 5), "final_accuracy": round(acc, 4),
        "schedule": sorted(k for k, v in model.schedule().items() if v),
        "host_launch_ms": round(1e3 * host_launch, 3),
    }
    if args.columns != "zipf":
        out["config"]["columns"] = args.columns
    mf = mfma_summary(args.dtype) if fused else None
    if mf is not None:
        out["mfma"] = mf
    if fwd is not None:
        out["fwd_only"] = fwd
    if rehearse > 1 and dp_kernels is not None:
        out["dp_kernels_ms"] = dp_kernels
    if rehearse > 1:
        out["rehearsal"] = {"world": rehearse, "chunks": args.dp_chunks,
                            "collectives": ({"model": f"modelled: {args.link_latency_us} us + bytes sent / "
                                                      f"{args.link_gbps} GB/s per collective",
                                             "copy": "device copies of the same bytes",
                                             "peer": "peer-store exchange, the peers' buffers local and their "
                                                     "flags raised in advance (no link time)"}[args.rehearse_comm]),
                            "note": "rank 0 of an N-rank bf16-wire step on one GPU; not a headline number"}
    if (dp is not None and dp.peer is not None) or (rehearse > 1 and args.rehearse_comm == "peer"):
        out["peer_status"] = model.peer_status()
        if dp is not None:
            out["peer_status"]["selftest_mismatches"] = dp.peer_selftest
        if out["peer_status"]["error"]:
            raise SystemExit(f"bench: the peer exchange timed out: {out['peer_status']}")
    if dp is not None:
        out["config"]["dp_chunks"] = dp.chunks
        try:
            out["config"]["comm"] = dp.tx.info()
        except Exception as e:  # informational only
            out["config"]["comm"] = {"error": repr(e)}
        if dp_kernels is not None:
            out["dp_kernels_ms"] = dp_kernels
        out["config"]["dp_launch"] = ("one graph per region, collectives captured" if region_graphs is not None
                                      else "split graphs, host-issued collectives" if args.graph else "eager")
        if dp_capture_error:
            out["config"]["dp_capture_error"] = dp_capture_error
        out["dp_check"] = check
    if (args.fp32_line and rank == 0 and world == 1 and rehearse == 1 and args.dtype == "bf16"
            and feeder is None and args.columns == "zipf"):
        out["fp32_mode"] = fp32_mode_line(args)
    if (args.det_line and not args.deterministic and rank == 0 and world == 1 and rehearse == 1
            and args.dtype == "bf16" and feeder is None and args.columns == "zipf"):
        out["deterministic_mode"] = deterministic_mode_line(args)
    if (args.fwd32_line and not args.fwd32 and rank == 0 and world == 1 and rehearse == 1
            and args.dtype == "bf16" and feeder is None and args.columns == "zipf"):
        # the bf16 plan with the forward at the reference's precision (plan option FWD32)
        out["fwd32_mode"] = child_mode_line(args, ["--fwd32", "1"])
    if rank == 0 and world == 1 and args.cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
            out["cpu_baseline"]["cpu_model"] = cpu_model()
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": repr(e)}
        if args.parity and rehearse == 1 and feeder is None and args.columns == "zipf":
            try:  # the checker leg: each mode's error against the float64 oracle on batch 0
                trained = {k: v.detach().cpu().numpy().copy() for k, v in model.named_params().items()}
                b0 = synth_batch(D, BS, NEG, seed=1000 + rank * 100003, cols=cols)
                out["cpu_baseline"]["parity_vs_oracle"] = parity_vs_oracle(dev, b0, trained)
            except Exception as e:
                out["cpu_baseline"]["parity_vs_oracle"] = {"error": repr(e)}
    if feeder is not None:
        feeder.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dp is not None:
        dp.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
