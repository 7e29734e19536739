"""bench.py's launcher and launch plan (CPU only): `--gpus N` without a torch.distributed
launcher starts N ranks itself, every rank checks WORLD_SIZE == N, a box with fewer than N
devices fails instead of silently running one GPU, and short runs split into balanced launches."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_plan_launches_balanced():
    assert bench.plan_launches(20, 64) == [20]
    assert bench.plan_launches(100, 64) == [50, 50]
    assert bench.plan_launches(1024, 64) == [64] * 16
    assert bench.plan_launches(65, 64) == [33, 32]
    assert bench.plan_launches(0, 64) == []
    for n in range(1, 300):
        p = bench.plan_launches(n, 64)
        assert sum(p) == n and max(p) <= 64 and max(p) - min(p) <= 1 and len(p) == -(-n // 64)


def test_world_check():
    a = bench.parse(["--gpus", "4"])
    assert bench.world_check(a, {}) == ("spawn", "")
    assert bench.world_check(a, {"WORLD_SIZE": "4"}) == ("run", "")
    act, msg = bench.world_check(a, {"WORLD_SIZE": "2"})
    assert act == "fail" and "WORLD_SIZE=2" in msg
    assert bench.world_check(bench.parse([]), {}) == ("run", "")
    assert bench.world_check(bench.parse(["--gpus", "1"]), {"WORLD_SIZE": "1"}) == ("run", "")


def test_launch_command():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "20"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--master-port=29555" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "20"]


def test_gpus_2_without_devices_fails_loudly():
    """On a box with fewer devices than --gpus (here: none) bench.py exits non-zero with a message."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4"],
                       env=env, capture_output=True, text=True, timeout=120)
    if "GPU(s) visible" not in r.stderr:
        pytest.skip("devices visible")
    assert r.returncode == 2 and "--gpus 2: only" in r.stderr
    assert not r.stdout.strip()  # no bench line from a silent one-GPU run


def test_rank_world_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=3 but --gpus 2" in r.stderr


def test_cpu_baseline_reports_its_spread():
    """The CPU leg reports the frame-time spread, the CPU time the process was actually given and the
    cgroup's throttling over each sample beside the median (the driver's CPU figure
    varied 28 % between boxes with nothing in the line to explain it)."""
    from raytracer_hip import scenes
    sc = scenes.config("C1").resized(64, 48)
    out = bench.cpu_baseline([(sc, None, 0.6), (scenes.reference(32, 32), None, 0.4)], 0.3)
    for e in (out, out["others"]["ref"]):
        p10, p50, p90 = e["frame_ms_p10_p50_p90"]
        assert 0 < p10 <= p50 <= p90 and e["frames"] >= 3
        assert e["cpus_scheduled"] >= 0
        t = e["cgroup_throttled"]
        assert t is None or (t["periods"] >= 0 and t["nr_throttled"] >= 0 and t["throttled_ms"] >= 0)
    assert out["cores"] >= 1 and "frame_ms_p10_p50_p90" in out["sample"]


def test_percentiles_nearest_rank():
    assert bench.percentiles([5, 1, 2, 3, 4]) == [1, 3, 5]
    assert bench.percentiles([7]) == [7, 7, 7]


def test_rank0_tail_solver():
    """bench.solve_rank0_tail (rank 0's measured share): with a uniform cost per row it reproduces the
    closed form h/H = (T/(N-1) - D) / (N T/(N-1) - D), floored to whole bands; rows that cost more than the average
    shrink the tail; a decode above the others' trace share makes rank 0 the compositor (0 rows); a solution at or
    above the uniform share keeps it interleaved (h >= hu)."""
    T, D, H, br = 1136e-6, 36.5e-6, 4320, 8
    for n in (2, 4, 8):
        calls = []

        def probe(rows):
            calls.append(rows)
            return T * rows / H
        h, hu, c = bench.solve_rank0_tail(T, D, H, br, n, probe)
        x = (T / (n - 1) - D) / (n * T / (n - 1) - D)
        assert h == int(x * H // br) * br and h % br == 0 and 0 < h < hu, (n, h, x * H)
        assert hu == (H // n) // br * br and calls[0] == hu and abs(c - T / H) < 1e-15
    h_uniform = bench.solve_rank0_tail(T, D, H, br, 8, lambda rows: T * rows / H)[0]
    h_costly = bench.solve_rank0_tail(T, D, H, br, 8, lambda rows: 1.5 * T * rows / H)[0]
    assert h_costly < h_uniform
    assert bench.solve_rank0_tail(10e-6, 20e-6, 1080, br, 2, lambda rows: 10e-6 * rows / 1080)[0] == 0
    h, hu, _ = bench.solve_rank0_tail(T, 0.0, H, br, 4, lambda rows: 0.5 * T * rows / H)  # a cheap tail, no decode
    assert h >= hu
