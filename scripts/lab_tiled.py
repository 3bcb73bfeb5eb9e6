#!/usr/bin/env python3
"""Lab: the tiled kernels (SMFV_TILED_ABLATE = 0 pipelined persistent,
1 one-shot, 2 one-shot stage only, 3 one-shot compute only), one process per
mode; plus the untiled kernel for reference.  Not part of the product or the bench."""
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
for mode, env in (("pipe", {"SMFV_TILED_ABLATE": "0", "LAB_TILES": "force"}),
                  ("pipe_sortindex", {"SMFV_TILED_ABLATE": "0", "SMFV_TILE_SORT": "index", "LAB_TILES": "force"}),
                  ("pipe_contig", {"SMFV_TILED_ABLATE": "0", "SMFV_TILE_ORDER": "0", "LAB_TILES": "force"}),
                  ("pipe_nocompute", {"SMFV_TILED_ABLATE": "5", "LAB_TILES": "force"}),
                  ("pipe_nocompute_contig", {"SMFV_TILED_ABLATE": "5", "SMFV_TILE_ORDER": "0", "LAB_TILES": "force"}),
                  ("pipe_noprefetch", {"SMFV_TILED_ABLATE": "6", "LAB_TILES": "force"}),
                  ("pipe_skeleton", {"SMFV_TILED_ABLATE": "9", "LAB_TILES": "force"}),
                  ("oneshot", {"SMFV_TILED_ABLATE": "1", "LAB_TILES": "force"}),
                  ("untiled", {"LAB_TILES": "off"})):
    r = subprocess.run([sys.executable, "-c", f"ROOT={ROOT!r}; MODE={mode!r}\n" + CHILD],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
    print(line[0][7:] if line else f"{mode} FAILED rc={r.returncode} {r.stderr[-1500:]}", flush=True)
    if r.returncode not in (0, 1):
        sys.exit(r.returncode)
