"""bench.py's launch contract on CPU (no GPU): `python bench.py --gpus N` without
a launcher starts N ranks itself (a torch.distributed.run child, never an exec
of itself), and the line's n_gpus is the number of ranks that reported; a
launcher with another world size is refused.  The ranks here run the
--launch-check rehearsal (gloo process group, ranks count themselves)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_without_launcher_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--launch-check", "--backend", "gloo"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout   # one line, from rank 0
    assert lines[0]["n_gpus"] == n and lines[0]["world_size"] == n
    # the N-rank line explains itself: every rank's step time, its reduce time, the group
    rk = lines[0]["ranks"]
    assert rk["world_size"] == n and rk["backend"] == "gloo"
    assert len(rk["ms_per_step"]) == n and len(rk["reduce_ms"]) == n
    assert rk["ms_per_step_min"] == min(rk["ms_per_step"]) and rk["ms_per_step_max"] == max(rk["ms_per_step"])
    assert all(0.0 <= x <= y for x, y in zip(rk["reduce_ms"], rk["ms_per_step"]))


def test_build_once_scene_two_ranks(tmp_path):
    """The N-GPU bench compiles the scene once per node: local rank 0 compiles
    and writes the scene cache, rank 1 waits at a gloo barrier and maps it; the
    two descs are byte-identical and the ranks record their scene source, time
    and peak host RSS."""
    r = _run(["--gpus", "2", "--launch-check", "--launch-check-scene", "--backend", "gloo", "--scene-cache-dir",
              str(tmp_path)])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    rk = line["ranks"]
    assert rk["scene_source"] == ["compiled (cache written)", "mapped from the node's scene cache"], rk
    assert line["scene"]["identical_on_every_rank"] and line["scene"]["triangles"] > 1000
    assert len(rk["host_peak_rss_gb"]) == 2 and all(x > 0 for x in rk["host_peak_rss_gb"])
    assert not list(tmp_path.iterdir())     # the cache file is gone once every rank mapped it


def test_single_gpu_runs_in_process():
    r = _run(["--gpus", "1", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["ranks"]["world_size"] == 1 and line["ranks"]["reduce_ms"] is None


def test_roofline_scales_per_unit_counters():
    """Profile counters recorded per unit (render passes, or rays for the primary
    leg) scale to the timed launch; counters without a unit count are not
    applied to another launch shape (a sharded run's 1/N launch)."""
    prof = {"kernels": {"primary_intersect": {"units_per_launch": 2_000_000, "hbm_bytes": 100e6,
                                              "l2_read_bytes": 1e9, "ta_busy": 0.7},
                        "nounits": {"hbm_bytes": 100e6}}}
    full = bench.roofline((prof, "p", True), "primary_intersect", 0.5, 1e9, "k", units=2_000_000)
    eighth = bench.roofline((prof, "p", True), "primary_intersect", 0.5 / 8, 1e9 / 8, "k", units=250_000)
    assert full["traffic"] == 100e6 and eighth["traffic"] == 100e6 / 8
    assert eighth["frac_hbm"] == full["frac_hbm"] and eighth["frac_l2"] == full["frac_l2"]
    none = bench.roofline((prof, "p", True), "nounits", 0.5, 1e9, "k", units=250_000)
    assert none["traffic"] is None and none["frac"] is None and "no units_per_launch" in str(none["profile_matches_binary"])


def test_roofline_of_a_sharded_launch_scales_per_ray():
    """A path-kernel profile of a 1-GPU 8-pass launch carries its traced rays
    (rays_per_launch, tools_pmc_summary.py); rank r of an 8-GPU job traces 1/8
    of the image's rays per pass in its N-pass launch, and its line gets the
    same HBM bytes per ray, so a non-null frac and traffic."""
    prof = {"kernels": {"path_kernel": {"units_per_launch": 8, "rays_per_launch": 150_000_000.0,
                                        "hbm_bytes": 1.77e9, "l2_read_bytes": 2.0e11, "ta_busy": 0.9}}}
    one = bench.roofline((prof, "p", True), "path_kernel", 46.4, 4e11, "k", units=150_000_000.0,
                         unit_key="rays_per_launch")
    rank5 = bench.roofline((prof, "p", True), "path_kernel", 46.4 / 8 * 1.02, 4e11 / 8, "k", units=18_900_000.0,
                           unit_key="rays_per_launch")
    assert rank5["traffic"] is not None and rank5["frac"] is not None
    assert rank5["traffic_per_unit"] == one["traffic_per_unit"] == 1.77e9 / 150_000_000.0
    assert abs(rank5["traffic"] / 18_900_000.0 - one["traffic"] / 150_000_000.0) < 1e-9
    # a profile without rays per launch is not applied by rays
    prof["kernels"]["path_kernel"].pop("rays_per_launch")
    none = bench.roofline((prof, "p", True), "path_kernel", 5.8, 5e10, "k", units=18_900_000.0,
                          unit_key="rays_per_launch")
    assert none["traffic"] is None and "no rays_per_launch" in str(none["profile_matches_binary"])


def test_mismatched_launcher_world_size_fails():
    r = _run(["--gpus", "4", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_launch_groups_near_equal():
    assert bench.launch_groups(20, 8) == [7, 7, 6]
    assert bench.launch_groups(64, 8) == [8] * 8
    assert bench.launch_groups(5, 8) == [5]
    for steps in range(1, 70):
        g = bench.launch_groups(steps, 8)
        assert sum(g) == steps and max(g) - min(g) <= 1 and max(g) <= 8


@pytest.mark.parametrize("rank", [-1, 8])
def test_emulate_rank_outside_the_job_is_refused(rank):
    """--emulate-ranks N --emulate-rank r times rank r's share of an N-GPU job
    (DESIGN §8); a rank outside 0..N-1 is refused before anything touches a GPU."""
    r = _run(["--emulate-ranks", "8", "--emulate-rank", str(rank), "--no-cpu-baseline"], timeout=120)
    assert r.returncode == 2
    assert "outside 0..7" in r.stderr
