#!/usr/bin/env python3
"""Lab timeline of k_rows_ws (needs the lab build: make -C csrc lab; runs with
SMFV_LAB=1 SMFV_WS_ABL=8 SMFV_WS_STAMPS=<file>).  Runs the cop20k surrogate
at K=32 eagerly over rotating copies (cold, like bench.py) and reads the
s_memtime stamps of the last launch: per block and unit, when the compute
waves start (barrier exit) and finish their rows, and when the loader waves
have issued the next unit's DMAs and seen them land.  Prints where each
unit's time goes: compute-bound units (the last compute wave ends after the
last DMA lands) against loader-bound ones, and the average split.

usage: SMFV_LAB=1 SMFV_WS_ABL=8 SMFV_WS_STAMPS=/tmp/st.bin python scripts/lab_stamps.py [K]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch
    import sparsematrixmultiplicationmpi_amd as smfv
    assert os.environ.get("SMFV_LAB") == "1" and os.environ.get("SMFV_WS_ABL") == "8", "lab build, ABL 8"
    path = os.environ["SMFV_WS_STAMPS"]
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    A = smfv.cop20k_surrogate()
    X = smfv.generateLargeFatVector(A.numCols, K)
    copies = []
    for _ in range(12):
        dA = smfv.DeviceCSR(A)
        copies.append((smfv.SpmmPlan(smfv.Variant.ROWWISE, dA, K), torch.from_numpy(X).cuda(),
                       torch.empty((A.numRows, K), dtype=torch.float64, device="cuda")))
    torch.cuda.synchronize()
    for i in range(60):  # warm the clocks; the last launch's stamps are kept
        plan, dX, dY = copies[i % len(copies)]
        plan.run(dX, dY)
    torch.cuda.synchronize()
    U = 32
    st = np.fromfile(path, dtype=np.uint64).astype(np.int64)
    nb = st.size // (16 * U * 2)
    st = st.reshape(nb, 16, U, 2)
    comp, load = st[:, :8], st[:, 8:]
    used = comp[:, 0, :, 0] > 0  # units a block ran
    # (s_memtime counters are per XCD: only differences inside one block are compared)
    print(f"K={K}: {nb} blocks")
    rows = []
    for b in range(nb):
        nu = int(used[b].sum())
        for u in range(nu):
            start = comp[b, :, u, 0].max()  # all compute waves passed the barrier
            cend = comp[b, :, u, 1].max()
            cmin = comp[b, :, u, 1].min()
            nxt = comp[b, :, u + 1, 0].max() if u + 1 < nu else cend
            if u + 1 < nu:
                issued = load[b, :, u, 0].max()
                landed = load[b, :, u, 1].max()
            else:
                issued = landed = start
            rows.append((b, u, start, cend - start, cmin - start, issued - start, landed - start, nxt - start))
    R = np.array(rows, dtype=np.int64)
    mid = (R[:, 1] > 0) & (R[:, 1] < np.array([used[b].sum() for b in R[:, 0]]) - 1)
    M = R[mid]
    comp_bound = M[:, 3] >= M[:, 6]
    print(f"steady units (not first / last of a block): {len(M)}; compute ends last in {comp_bound.mean():.0%}")
    for name, col in (("compute, slowest wave", 3), ("compute, fastest wave", 4), ("DMAs issued", 5),
                      ("DMAs landed", 6), ("unit period (barrier to barrier)", 7)):
        print(f"  {name:34s} mean {M[:, col].mean():8.0f} ticks  median {np.median(M[:, col]):8.0f}")
    # per compute wave: its rows' time in steady units (wave w and w + 4 share a SIMD)
    per_w = []
    for w in range(8):
        d = [comp[b, w, u, 1] - comp[b, :, u, 0].max() for b in range(nb) for u in range(1, int(used[b].sum()) - 1)]
        per_w.append(np.mean(d))
    print("  compute per wave (mean ticks, steady units): " + " ".join(f"w{w}:{v:.0f}" for w, v in enumerate(per_w)))
    first = R[R[:, 1] == 0]
    last = np.array([comp[b, :, int(used[b].sum()) - 1, 1].max() - comp[b, :, int(used[b].sum()) - 1, 0].max()
                     for b in range(nb)])
    print(f"first unit period {np.mean(first[:, 7]):.0f} ticks; last unit's compute {last.mean():.0f} ticks; "
          f"units per block {used.sum(1).mean():.2f}")


if __name__ == "__main__":
    main()
