#!/usr/bin/env python3
"""Sweep row-kernel configurations (SMFV_ROW_CFG="TEAM,H,U"), one process
per configuration (the library reads the variable once).  Each child checks
bit-exactness against the oracle and prints warm / cold median launch time.
Lab tool only (not part of the product or the bench)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
sys.path.insert(0, ROOT)
import numpy as np, torch
import sparsematrixmultiplicationmpi_amd as smfv
from oracle import oracle
from scripts.lab_ablate import timeit
dev = torch.device("cuda", 0)
A = smfv.cop20k_surrogate() if KIND == "cop" else smfv.gen_random_rows(2_000_000, 2_000_000, 16, 2.0, 4096, 42)
X = smfv.generateLargeFatVector(A.numCols, K)
copies = []
for _ in range(6 if KIND == "cop" else 2):
    dA = smfv.DeviceCSR(A, dev)
    copies.append((smfv.SpmmPlan(smfv.Variant.ROWWISE, dA, K), torch.from_numpy(X).to(dev),
                   torch.empty((A.numRows, K), dtype=torch.float64, device=dev)))
p, x, y = copies[0]
p.run(x, y); torch.cuda.synchronize()
ok = None
if KIND == "cop":
    Yref = oracle.spmm("sequential", A.rowPtr, A.colIndices, A.values, X)
    ok = bool(np.array_equal(y.cpu().numpy().view(np.uint64), Yref.view(np.uint64)))
w = timeit(p, x, y); c = timeit(p, x, y, copies=copies)
alg = 12 * A.nnz + 4 * (A.numRows + 1) + 8 * A.numCols * K + 8 * A.numRows * K
print("RESULT " + json.dumps({"cfg": os.environ.get("SMFV_ROW_CFG"), "K": K, "kind": KIND, "exact": ok,
      "warm_us": round(w, 2), "cold_us": round(c, 2), "cold_GBps": round(alg / (c * 1e-6) / 1e9, 1)}))
'''


def main():
    plan = [("cop", 32, c) for c in ("16,1,8", "16,1,16", "8,2,4", "8,2,8", "4,4,4", "4,4,2", "2,8,2",
                                      "8,1,8", "16,2,4")]
    plan += [("cop", 128, c) for c in ("16,4,4", "16,4,2", "32,2,4", "64,1,8", "8,8,2", "16,2,4")]
    if len(sys.argv) > 1:
        plan = [p for p in plan if p[1] == int(sys.argv[1])]
    results = []
    for kind, K, cfg in plan:
        env = dict(os.environ, SMFV_ROW_CFG=cfg)
        code = f"ROOT={ROOT!r}; KIND={kind!r}; K={K}\n" + CHILD
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(f"{cfg} K={K} FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
            if r.returncode not in (0, 1):
                sys.exit(r.returncode)  # a crash: stop using the GPU
            continue
        res = json.loads(line[0][7:])
        results.append(res)
        print(json.dumps(res), flush=True)
    print("ALL " + json.dumps(results))


if __name__ == "__main__":
    main()
