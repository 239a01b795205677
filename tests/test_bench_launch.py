"""bench.py's multi-GPU entry: `python bench.py --gpus N` starts its N ranks itself.

The launching process must never initialise HIP (it starts children, it does not exec after a GPU call),
each rank gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, and a --gpus / world-size mismatch fails."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    return env


def test_launcher_parent_never_imports_torch():
    code = (
        "import runpy, sys\n"
        f"sys.argv = [{BENCH!r}, '--gpus', '3', '--launch-dry-run']\n"
        "try:\n"
        f"    runpy.run_path({BENCH!r}, run_name='__main__')\n"
        "    rc = 0\n"
        "except SystemExit as e:\n"
        "    rc = e.code\n"
        "assert 'torch' not in sys.modules, 'the launching process imported torch'\n"
        "print('PARENT_RC', rc)\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=_env(), capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().splitlines()
    assert lines[-1] == "PARENT_RC 0"
    rank0 = json.loads(lines[0])  # rank 0's line, relayed by the parent
    assert rank0["RANK"] == "0" and rank0["LOCAL_RANK"] == "0" and rank0["WORLD_SIZE"] == "3"
    assert rank0["MASTER_ADDR"] == "127.0.0.1" and int(rank0["MASTER_PORT"]) > 0


def test_failing_rank_ends_the_launch():
    """Rank 1 exits 3 while ranks 0 and 2 block (as ranks waiting in a collective for a dead peer do): the
    launching process stops them and exits non-zero within seconds, naming the rank and its stderr."""
    import time
    env = _env()
    env["DVH_DRY_FAIL"] = "1:3"
    t0 = time.time()
    out = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-dry-run"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=120)
    assert time.time() - t0 < 60
    assert out.returncode == 3, (out.returncode, out.stderr)
    assert "rank 1 exited with 3" in out.stderr
    assert "[dry-run] rank 1 fails with 3" in out.stderr  # the failing rank's stderr tail


def test_world_size_mismatch_exits_nonzero():
    env = _env()
    env["WORLD_SIZE"] = "2"
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4"], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr


@pytest.mark.gpu
def test_two_ranks_strong_scaling_on_one_gpu():
    """Two ranks sharing the box's one GPU (gloo: RCCL refuses two ranks on one device): the fixed job is
    split, rank 0 reports the world size and its half of the job."""
    env = _env()
    env["DVH_DIST_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--workload", "weights", "--scaling", "strong",
                          "--steps", "2", "--warmup", "1", "--no-cpu-baseline"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["n_gpus"] == 2 and res["scaling"] == "strong"
    cfg = res["config"]
    assert cfg["windows_per_step"] == 2 * 1895
    assert abs(cfg["windows_per_step_this_rank"] - 1895) <= 3
