#!/usr/bin/env python3
"""Lab: phase ablation of the tiled kernel (SMFV_TILED_ABLATE = 0 full,
1 stage only, 2 compute only), one process per mode; plus the untiled
kernel for reference.  Not part of the product or the bench."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json
sys.path.insert(0, ROOT)
import torch
import sparsematrixmultiplicationmpi_amd as smfv
from scripts.lab_ablate import variants
dev = torch.device("cuda", 0)
A = smfv.cop20k_surrogate()
w, c = variants(A, 32, dev)
print("RESULT " + json.dumps({"mode": MODE, "warm_us": round(w, 2), "cold_us": round(c, 2)}))
'''
for mode, env in (("full", {"SMFV_TILED_ABLATE": "0"}), ("stage_only", {"SMFV_TILED_ABLATE": "1"}),
                  ("compute_only", {"SMFV_TILED_ABLATE": "2"}), ("untiled", {"LAB_TILES": "off"})):
    r = subprocess.run([sys.executable, "-c", f"ROOT={ROOT!r}; MODE={mode!r}\n" + CHILD],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
    print(line[0][7:] if line else f"{mode} FAILED rc={r.returncode} {r.stderr[-1500:]}", flush=True)
    if r.returncode not in (0, 1):
        sys.exit(r.returncode)
