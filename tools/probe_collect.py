"""Diagnostic (N ranks sharing one GPU over gloo): the cost of each step of DistributedMST.collect_mst
on a flags array of the s26 shape — torch.nonzero over the rank's slice, the device-to-host copy,
the gloo gather — to explain the gloo rehearsal's slow collects. Run under torch.distributed.run."""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 1051916369
    flags = (torch.rand(m, device="cuda") < 0.031).to(torch.uint8)
    lo, hi = m * r // w, m * (r + 1) // w
    for it in range(3):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mine = torch.nonzero(flags[lo:hi]).flatten().to(torch.int64) + lo
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        host = mine.to("cpu")
        t2 = time.perf_counter()
        parts = [torch.empty_like(host) for _ in range(w)] if r == 0 else None
        n = torch.tensor([host.numel()])
        ns = [torch.zeros_like(n) for _ in range(w)]
        dist.all_gather(ns, n)
        width = max(int(x.item()) for x in ns)
        pad = torch.full((width,), -1, dtype=torch.int64)
        pad[: host.numel()] = host
        parts = [torch.empty_like(pad) for _ in range(w)] if r == 0 else None
        dist.gather(pad, parts, dst=0)
        t3 = time.perf_counter()
        print(f"rank {r} it {it}: nonzero {1e3 * (t1 - t0):.1f} ms, d2h {1e3 * (t2 - t1):.1f} ms ({host.numel()} eids), "
              f"gather {1e3 * (t3 - t2):.1f} ms", file=sys.stderr, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
