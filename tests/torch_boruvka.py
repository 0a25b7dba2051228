"""TEST INFRASTRUCTURE ONLY: an independent MSF checker in plain PyTorch for the BASELINE sizes.

The oracle's C Kruskal (oracle/kruskal.c) is the parity anchor, but on one core it needs minutes
for R-MAT s24 (260M edges) and the 16384^2 grid (537M edges). This module recomputes the same
canonical MSF with textbook Boruvka written only in torch tensor ops (scatter_reduce 'amin',
gathers, pointer jumping) — no code shared with the HIP kernels — so the full-size GPU tests
compare the HIP result with an independent computation, bit-exact. It is itself pinned against
the oracle on random tie-heavy graphs by tests/test_oracle.py (CPU tensors).

Key: the canonical strict order (w, eid) (oracle/kruskal.c); with unique keys
the MSF is unique, so Boruvka's result equals Kruskal's edge set.
"""
import torch

_BIAS = 1 << 31


def canonical_keys(w):
    """int64 keys whose signed order is the unsigned order of (w, eid); w holds uint32 bit patterns."""
    m = w.numel()
    ww = w.to(torch.int64) & 0xFFFFFFFF
    return ((ww - _BIAS) << 32) | torch.arange(m, dtype=torch.int64, device=w.device)


def msf_boruvka(n, u, v, w, max_rounds=64):
    """Canonical minimum spanning forest of a canonical edge list (u < v, sorted, unique).

    u, v, w: tensors of equal length holding uint32 bit patterns (any int dtype). Returns a bool
    tensor in_mst[m] on the inputs' device."""
    dev = u.device
    m = u.numel()
    in_mst = torch.zeros(m, dtype=torch.bool, device=dev)
    if m == 0 or n == 0:
        return in_mst
    ar = torch.arange(n, dtype=torch.int64, device=dev)
    comp = ar.clone()
    eu = u.to(torch.int64) & 0xFFFFFFFF
    ev = v.to(torch.int64) & 0xFFFFFFFF
    ek = canonical_keys(w)
    big = torch.iinfo(torch.int64).max
    for _ in range(max_rounds):
        cu = comp[eu]
        cv = comp[ev]
        keep = cu != cv
        if not bool(keep.any()):
            return in_mst
        eu, ev, ek, cu, cv = eu[keep], ev[keep], ek[keep], cu[keep], cv[keep]
        best = torch.full((n,), big, dtype=torch.int64, device=dev)
        best.scatter_reduce_(0, cu, ek, reduce="amin")
        best.scatter_reduce_(0, cv, ek, reduce="amin")
        win_u = best[cu] == ek  # this edge is fragment cu's minimum outgoing edge
        win_v = best[cv] == ek
        chosen = win_u | win_v
        in_mst[(ek[chosen] & 0xFFFFFFFF)] = True
        parent = ar.clone()
        parent[cu[win_u]] = cv[win_u]
        parent[cv[win_v]] = cu[win_v]
        # mutual minimum (both fragments chose the same edge): the smaller id stays the root
        pp = parent[parent]
        parent = torch.where((pp == ar) & (ar < parent), ar, parent)
        while True:  # pointer jumping to the roots
            nxt = parent[parent]
            if torch.equal(nxt, parent):
                break
            parent = nxt
        comp = parent[comp]
    raise RuntimeError("torch Boruvka did not converge")
