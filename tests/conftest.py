import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # the native artefacts are built in-tree; build them if this checkout has none
    lib = os.path.join(ROOT, "sparsematrixmultiplicationmpi_amd", "libsmfv.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-j", "8", "-C",
                        os.path.join(ROOT, "sparsematrixmultiplicationmpi_amd", "csrc"), "all"], check=True)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)


def golden_cases():
    import json
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def golden_large_cases():
    """(r4) The fixtures at SURVEY 8(c)'s sizes (tests/golden/make_golden_large.py)."""
    import json
    with open(os.path.join(GOLDEN, "manifest_large.json")) as f:
        return json.load(f)


def load_golden_large(name):
    """A large fixture: the CSR its compact inputs stand for (values k / 7),
    and the reference's result hashes / NonZeroElement XOR masks."""
    import numpy as np
    from sparsematrixmultiplicationmpi_amd import inputs
    g = dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))
    m, n = int(g["m"]), int(g["n"])
    rp = np.zeros(m + 1, np.int32)
    rp[1:] = np.cumsum(g["lens"].astype(np.int64))
    row = np.repeat(np.arange(m, dtype=np.int64), g["lens"].astype(np.int64))
    ci = (row + g["off"].astype(np.int64)).astype(np.int32)
    g["A"] = inputs.SparseMatrix(g["vals"].astype(np.float64) / 7.0, ci, rp, m, n)
    return g


def golden_large_nnz(g, K, p, Y_seq):
    """The reference's NonZeroElement result at p ranks, rebuilt exactly from
    its sequential result (checked against sha_seq by the caller) and the
    fixture's XOR mask."""
    import numpy as np
    y = np.ascontiguousarray(Y_seq, dtype=np.float64).copy().reshape(-1).view(np.uint64)
    idx = g[f"nnzx_idx_k{K}_p{p}"]
    y[idx] ^= g[f"nnzx_xor_k{K}_p{p}"]
    return y.view(np.float64).reshape(Y_seq.shape)


def sha_f64(a):
    import hashlib
    import numpy as np
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def short_rows_band(m, seed, long_every=97):
    """(r5) A pattern for row-pair tiles: rows of 0-7 non-zeros (every
    residue, empty rows included) from a +-12 band, every `long_every`-th row
    30-60 long -- tiles stop at their row count, so the shortest rows ride as
    second rows of teams.  Values uniform in [-1, 1)."""
    import numpy as np
    from sparsematrixmultiplicationmpi_amd import inputs
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 8, m)
    lens[::long_every] = rng.integers(30, 61, lens[::long_every].size)
    cols = []
    for i, L in enumerate(lens):
        lo, hi = max(0, i - 12), min(m, i + 13)
        if L > hi - lo:
            lo, hi = max(0, i - 40), min(m, i + 41)
            L = lens[i] = min(L, hi - lo)
        cols.append(np.sort(rng.choice(np.arange(lo, hi), int(L), replace=False)))
    rp = np.zeros(m + 1, np.int32)
    rp[1:] = np.cumsum(lens)
    ci = np.concatenate(cols).astype(np.int32)
    return inputs.SparseMatrix(rng.uniform(-1, 1, ci.size), ci, rp, m, m)
