"""Where the CSR row derivation's time goes (tools/microbench/csr_rows.hip): each variant streams
the R-MAT s24 canonical list once, k_select-shaped; prints ms per variant (best of --reps)."""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = ["coo_uvw", "csr_vw_only", "csr_window", "csr_heads", "csr_full", "csr_full_trow", "csr_win_fixed",
         "csr_win_next1", "csr_win_next16B"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--grid", type=int, default=2048)
    args = ap.parse_args()
    import torch  # first: the hipcc-built library then binds to torch's HIP runtime (one runtime)
    src = os.path.join(ROOT, "tools", "microbench", "csr_rows.hip")
    so = os.path.join(ROOT, "tools", "microbench", "libcsr_rows.so")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950", "-o", so, src],
                       check=True)
    lib = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    lib.csr_rows_run.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32] + [vp] * 6 + [ctypes.c_int, vp]
    import torch
    from distributed_ghs_implementation_amd.device import generate_rmat
    e = generate_rmat(args.scale, 16, seed=1, wseed=2).with_csr()
    trow = torch.zeros(e.m // 256 + 8, dtype=torch.int32, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for k, name in enumerate(NAMES):
        ts = []
        for r in range(args.reps + 2):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            assert lib.csr_rows_run(k, e.n, e.m, P(e.u), P(e.off), P(e.v), P(e.w), P(trow), P(sink), args.grid,
                                    st) == 0
            b.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(a.elapsed_time(b))
        out[name] = round(min(ts), 4)
    print(json.dumps({"graph": f"rmat-s{args.scale}", "m": e.m, "n": e.n, "grid": args.grid, "ms": out}))


if __name__ == "__main__":
    main()
