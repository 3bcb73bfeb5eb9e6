"""bench.py's reporting helpers (CPU): the metric string is BASELINE.json's on
the headline config and labels the config that ran elsewhere, the kernel
label follows the plan that ran, and the algorithmic bytes are SURVEY 8(d)'s
formula (94.03 MB per launch on the cop20k_A surrogate at K = 32)."""
import json
import os
import sys

import pytest

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


def _env_without_world():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    return env


@pytest.mark.parametrize("n", [2, 8])
def test_gpus_n_starts_n_ranks_itself(n):
    """(r5) `python bench.py --gpus N` with no WORLD_SIZE starts
    N ranks as children (torch.distributed.run) instead of timing one GPU;
    --dry-run has them meet over gloo without touching a GPU.  stdout is ONE
    JSON line (rank 0's, re-printed by the parent).  (r6) N = 8 rehearses the
    driver's scaling run's control plane."""
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=_env_without_world(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(out) == 1, r.stdout
    line = json.loads(out[0])
    assert line["dry_run"] and line["n_gpus"] == n
    assert sorted(x["rank"] for x in line["ranks"]) == list(range(n))
    assert len({x["pid"] for x in line["ranks"]}) == n and os.getpid() not in {x["pid"] for x in line["ranks"]}
    assert line["launcher"]["ranks_started"] == n
    # (r6) the N = 2 line carries the CPU/MPI baseline: the
    # reference's kernel under mpiexec, 16 ranks per GPU capped at the CPUs
    # available, timed by rank 0 before any GPU call
    cpu = line["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["unit"] == "GFLOP/s"
    if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "ref_driver")):
        assert cpu["kind"] == "reference"
        assert cpu["cores"] == min(16 * n, len(os.sched_getaffinity(0)))
        assert f"{n}-GPU line" in cpu["note_n_gpus"]


def test_gpus_must_match_world_size():
    """Under a launcher, --gpus N with a different WORLD_SIZE is refused with
    one JSON line and a non-zero status (never a silent 1-GPU line)."""
    import subprocess
    env = _env_without_world()
    env["WORLD_SIZE"] = "3"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] is None and "WORLD_SIZE=3" in line["error"]
