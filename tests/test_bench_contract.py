"""bench.py's reporting helpers (CPU): the metric string is BASELINE.json's on
the headline config and labels the config that ran elsewhere, the kernel
label follows the plan that ran, and the algorithmic bytes are SURVEY 8(d)'s
formula (94.03 MB per launch on the cop20k_A surrogate at K = 32)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_metric_is_baselines_on_the_headline():
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert bench.metric_for("cop20k_k32", 32, "ROWWISE") == base
    other = bench.metric_for("cop20k_k128", 128, "ROWWISE")
    assert other != base and "K=128" in other
    assert "NONZERO" in bench.metric_for("cop20k_k32", 32, "NONZERO")


def test_algorithmic_bytes_formula():
    # 12 nnz + 4 (m + 1) + 8 n K + 8 m K (CSR once, X once, Y once)
    assert bench.algorithmic_bytes(121192, 121192, 2624346, 32) == 94027228
    assert bench.algorithmic_bytes(10, 20, 7, 3) == 12 * 7 + 4 * 11 + 8 * 20 * 3 + 8 * 10 * 3


def test_kernel_label_follows_the_plan():
    assert bench.kernel_label("ROWWISE", 32, {"tiled": True}) == "k_rows_ws"
    # a one-device NONZERO plan on a re-using pattern runs the tiled kernel
    assert bench.kernel_label("NONZERO", 32, {"tiled": True}) == "k_rows_ws"
    assert bench.kernel_label("NONZERO", 32, {"tiled": False}).startswith("k_merge_flat")
    assert bench.kernel_label("NONZERO", 7, {"tiled": False}).startswith("k_merge ")
    assert bench.kernel_label("ROWWISE", 128, {"tiled": True, "mfma": True}) == "k_rows_mfma"
    assert bench.kernel_label("ROWWISE", 1, {"tiled": False}).startswith("k_spmv_stream")
    assert bench.kernel_label("ROWWISE", 32, {"tiled": False}, 8 * 121192 * 32) == "k_rows_mh<8, 2, 8, true>"


def test_every_config_is_a_baseline_workload():
    kinds = {kind for kind, _, _ in bench.CONFIGS.values()}
    assert {"cop20k", "pow10m", "syn80m"} <= kinds
    assert bench.CONFIGS["cop20k_k32"] == ("cop20k", 32, "ROWWISE")
    assert bench.CONFIGS["pow10m_k32"][2] == "NONZERO"


def test_phase_deadline_prints_a_line_and_exits_4():
    """A multi-GPU phase that never ends (e.g. a hung RCCL call on a first
    8-GPU run) becomes one diagnostic JSON line and exit status 4."""
    import subprocess
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "d = bench.Deadline(0.5, 3, 8, 'm'); d.enter('fast'); d.enter('stuck collective'); "
            "time.sleep(30)") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 4, (r.returncode, r.stderr[-500:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] is None and "stuck collective" in line["error"] and line["rank"] == 3
    # a cancelled deadline never fires
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "d = bench.Deadline(0.3, 0, 1, 'm'); d.enter('x'); d.cancel(); time.sleep(1); print('done')") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "done"
