"""The native multi-rank loop (ghs_mst_emulated: N rank threads, in-process collectives) on one
GPU for R-MAT s<scale>, timed by the host (device synced): python tools/emu_native.py 26 8 3"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_ghs_implementation_amd import _native  # noqa: E402
from distributed_ghs_implementation_amd.device import emulated_mst, generate_rmat  # noqa: E402


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    e = generate_rmat(scale, 16, seed=1, wseed=2)
    for r in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # OPT_KEEP_CACHE: the later calls run on the first call's per-rank state (ABI 8 default: freed)
        res, _, flags = emulated_mst(e, world, config=_native.make_config(options=_native.OPT_KEEP_CACHE))
        torch.cuda.synchronize()
        print(f"rep {r} s{scale} x{world} {1e3 * (time.perf_counter() - t0):.2f} ms weight {res.total_weight} "
              f"edges {res.num_mst_edges} reused {res.reused} setup {res.ms_setup:.2f} solve {res.ms_solve:.2f} "
              f"gather {res.ms_gather:.2f} ms (max over ranks)", flush=True)
        del flags


if __name__ == "__main__":
    main()
