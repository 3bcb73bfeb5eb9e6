"""smfv_main: the drop-in for the reference CLI (SC/main.cpp), run under
MPICH with one rank (the GPU box has one GPU).  Checks the argument contract
and the stdout lines SC/scripts/get_csv_all.sh parses."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

import sparsematrixmultiplicationmpi_amd as smfv

MPIEXEC = "/opt/conda/bin/mpiexec"
MAIN = os.path.join(ROOT, "sparsematrixmultiplicationmpi_amd", "smfv_main")


def run_main(args, n=1, timeout=180):
    return subprocess.run([MPIEXEC, "-launcher", "fork", "-n", str(n), MAIN] + args,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_cli_stdout_contract(tmp_path):
    A = smfv.gen_fem27(3000, 14, 14, 0.8, 4)
    mtx = tmp_path / "a.mtx"
    smfv.writeMatrixMarketFile(str(mtx), A, symmetric=True)
    r = run_main(["8", str(mtx)])
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout
    assert "World size: 1" in out
    assert f"Sparse matrix: {mtx}" in out
    assert f"Matrix size: {A.numRows}x{A.numCols}" in out
    assert f"Vector size: {A.numCols}x8" in out
    for name in ("Serial Algo", "Row-wise", "Column-wise", "Non-zero Elements"):
        assert re.search(rf"^{name} Execution time: [0-9.eE+-]+$", out, re.M), name
    for name in ("Row-wise", "Column-wise", "Non-zero Elements"):
        assert f"{name}: Results are the same!" in out  # checked on the device (smfvCompareWithReference)
    # (r2) device-resident input distribution, timed on its own line
    assert re.search(r"^Input distribution time: [0-9.eE+-]+$", out, re.M)
    assert re.search(r"^Plan setup time: [0-9.eE+-]+$", out, re.M)
    # the PETSc block's analogue (SC/main.cpp:352,388 line shapes)
    assert re.search(r"^rocSPARSE Execution time: [0-9.eE+-]+$", out, re.M)
    assert "rocSPARSE: Results are the same!" in out


def test_cli_usage_error():
    if not os.path.exists(MPIEXEC):
        pytest.skip("no MPICH")
    r = run_main(["8"])  # wrong argc -> usage + MPI_Abort (SC/main.cpp:23-30), no GPU touched
    assert r.returncode != 0
    assert "Usage:" in r.stderr
