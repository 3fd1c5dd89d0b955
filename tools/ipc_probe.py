"""Diagnostics: can two processes on ONE GPU map each other's device buffers (HIP IPC, dmabuf mode,
HSA_ENABLE_IPC_MODE_LEGACY=0) and see each other's kernel writes?  The precondition of a
peer-store data-parallel exchange tested at world 2 on the one-GPU box.
The parent allocates a buffer, the spawned child maps it through torch's CUDA-tensor IPC, writes
a pattern with a kernel, raises a flag in a second shared buffer; the parent polls the flag from a
kernel-free host loop and checks the pattern.
    python3 tools/ipc_probe.py"""
import os
import sys
import time

import torch
import torch.multiprocessing as mp


def child(buf, flag, q):
    try:
        torch.cuda.set_device(0)
        buf.copy_(torch.arange(buf.numel(), device="cuda", dtype=torch.float32) * 2 + 1)
        torch.cuda.synchronize()
        flag.fill_(1)
        torch.cuda.synchronize()
        q.put(("ok", float(buf[:4].sum().item())))
    except Exception as e:  # noqa: BLE001
        q.put(("error", repr(e)))


def main():
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    ctx = mp.get_context("spawn")
    buf = torch.zeros(1 << 20, device="cuda")
    flag = torch.zeros(1, device="cuda", dtype=torch.int32)
    q = ctx.Queue()
    p = ctx.Process(target=child, args=(buf, flag, q))
    p.start()
    st, v = q.get(timeout=120)
    p.join(60)
    t0 = time.time()
    while int(flag.item()) != 1 and time.time() - t0 < 10:
        time.sleep(0.01)
    want = torch.arange(buf.numel(), device="cuda", dtype=torch.float32) * 2 + 1
    print(f"ipc_probe: child {st} {v}; flag {int(flag.item())}; parent sees the child's writes: "
          f"{bool(torch.equal(buf, want))}", flush=True)
    return 0 if st == "ok" and torch.equal(buf, want) else 1


if __name__ == "__main__":
    sys.exit(main())
