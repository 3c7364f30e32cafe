"""bench.py --gpus N without torchrun: the launcher starts one fresh process per rank with the
torchrun environment, prints nothing itself (rank 0's JSON line is the only stdout line), exits
non-zero when fewer GPUs are visible than ranks requested, ends every rank when one fails, and
never loads torch (no GPU call) in the parent.  The ranks run bench.py's stub worker
(FLACGPU_BENCH_STUB=1: gloo process group, barrier, max over ranks, no GPU), so this runs on CPU."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", **kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_distinct_ranks_one_line(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "3", "--warmup", "1"],
                       env=_env(FLACGPU_BENCH_FAKE_GPUS=str(n), FLACGPU_BENCH_STUB="1"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 3 and d["warmup"] == 1
    ranks = d["ranks"]
    assert sorted(x["rank"] for x in ranks) == list(range(n))
    assert all(x["local_rank"] == x["rank"] for x in ranks)
    assert len({x["pid"] for x in ranks}) == n          # one process per rank
    assert len({x["ppid"] for x in ranks}) == 1         # all children of the one launcher
    assert d["max_over_ranks"] == n - 1


def test_launcher_too_few_gpus_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"],
                       env=_env(FLACGPU_BENCH_FAKE_GPUS="2", FLACGPU_BENCH_STUB="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "2 GPU(s) visible" in r.stderr


def test_launcher_failing_rank_ends_the_run():
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3"],
                       env=_env(FLACGPU_BENCH_FAKE_GPUS="3", FLACGPU_BENCH_STUB="1", FLACGPU_BENCH_STUB_FAIL="1"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 7
    assert r.stdout.strip() == ""
    assert time.time() - t0 < 200  # the other ranks were terminated, not left waiting for rank 1


def test_launcher_parent_never_loads_torch():
    code = ("import sys; sys.argv = ['bench.py', '--gpus', '2']; sys.path.insert(0, %r); import bench; "
            "rc = bench.launch(bench.parse()); assert 'torch' not in sys.modules, 'parent imported torch'; "
            "print('rc', rc, file=sys.stderr)" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT,
                       env=_env(FLACGPU_BENCH_FAKE_GPUS="2", FLACGPU_BENCH_STUB="1"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "rc 0" in r.stderr
    assert len([ln for ln in r.stdout.splitlines() if ln.strip()]) == 1
