import os, sys
sys.path.insert(0, os.getcwd())
import torch
from distributed_ghs_implementation_amd.device import DeviceMST, generate_rmat
s = int(sys.argv[1]) if len(sys.argv) > 1 else 26
e = generate_rmat(s, 16, seed=1, wseed=2)
try:
    r, _ = DeviceMST(e).run()
    print("lib", os.environ.get("GHS_MST_LIB", "tree"), "hv", os.environ.get("GHS_HV"), "s", s, "ok", r.total_weight if hasattr(r, "total_weight") else r)
except Exception as ex:
    print("lib", os.environ.get("GHS_MST_LIB", "tree"), "hv", os.environ.get("GHS_HV"), "s", s, "ERR", ex)
