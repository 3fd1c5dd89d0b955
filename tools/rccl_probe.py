"""Probe (GPU box): does the library's RCCL communicator run two ranks on ONE GPU?  Each rank
inits dssm_comm, runs DataParallel's collective self-test through LibTransport and prints the
outcome.  Diagnostics only (multi-GPU runs are the driver's)."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def w(rank, port):
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2,
                            device_id=torch.device("cuda", 0))
    from dssm_amd.dist import DataParallel, LibTransport
    try:
        tx = LibTransport(rank, 2)

        class M:
            params = torch.zeros(1, device="cuda")
        d = DataParallel.__new__(DataParallel)
        d.model, d.world, d.rank = M, 2, rank
        print(rank, "selftest", d._selftest(tx), flush=True)
        tx.destroy()
    except Exception as e:
        print(rank, "failed", repr(e), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(w, args=(29611,), nprocs=2)
