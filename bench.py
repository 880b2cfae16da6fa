#!/usr/bin/env python3
"""bench.py — Mrays/s (primary + secondary) of the CudaTracerLib PathTracer hot
path (two-level BVH traversal + Woop intersection driven by the PathTrace<true>
pass loop) on MI355X.

Workload (BASELINE.json metric "Mrays/s (primary+secondary) at 1920x1080,
San-Miguel-scale BVH"): configs[2] = PathTracer on the synthetic ~10M-triangle
scene (seed 0x5EED), 1920x1080, Direct=1, MaxPathLength=50, RRStartDepth=5.

A *step* = one full-image pass-equivalent per GPU: at N GPUs each rank renders
N progressive passes over the 64x64 image tiles it owns (tile_id % N == rank),
so per-GPU work is fixed ("weak" scaling) and the job's image after K steps is
the N*K-spp image, bit-identical to a single-GPU render of the same passes.
After the last step the PixelData framebuffers are summed to rank 0 with one
RCCL reduce over xGMI (inside the timed region).  Rays counted exactly as the
reference's k_getNumRaysTraced (every traceRay incl. NEE shadow rays).

Launch: python bench.py [--gpus N --steps K --warmup W].  For N>1 under
torch.distributed.run (one process per GPU, RCCL backend); started as a plain
`python bench.py --gpus N` the process starts that launcher as a child (before
any GPU call, never an exec of itself) and exits with its status.
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np


KERNEL_NAME = {
    "persistent": "path_kernel_persistent<false,true> + fold_samples_kernel (traversal + shading, path "
                  "regeneration; the bracket covers both, the fold is ~0.03 ms)",
    "megakernel": "path_kernel<false,true> (one thread per pixel path)",
    "wavefront": "wavefront pass (gen/trace/shade/shadow/resolve kernels; timed as one unit)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3, help="1 Cornell, 2 C2 100k, 3 C3 ~10M tris")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-path-length", type=int, default=50)
    ap.add_argument("--rr-start", type=int, default=5)
    ap.add_argument("--shadow-any-hit", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--wpt-passes", type=int, default=3, help="WavefrontPathTracer leg passes (0: skip)")
    ap.add_argument("--closest-shadow-passes", type=int, default=4,
                    help="passes of the leg with the reference's closest-hit Occluded shadow rays (0: skip)")
    ap.add_argument("--prim-passes", type=int, default=16, help="C1 PrimTracer leg passes (0: skip)")
    ap.add_argument("--anim-iters", type=int, default=20, help="animation leg: timed ctl_scene_animate calls (0: skip)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--schedule", default="persistent", choices=["persistent", "megakernel", "wavefront"])
    ap.add_argument("--split-alpha", type=float, default=None, help="BVH reference splitting (default: library's)")
    ap.add_argument("--split-depth", type=int, default=8)
    ap.add_argument("--bins", type=int, default=0, help="SAH bins (0: library default)")
    ap.add_argument("--max-leaf", type=int, default=0, help="max leaf size (0: library default)")
    ap.add_argument("--builder", default="sbvh", choices=["binned", "sbvh"],
                    help="mesh BVH builder: the reference's SBVH (default) or early split clipping + binned SAH")
    ap.add_argument("--sbvh-alpha", type=float, default=1.0e-5, help="SBVH splitAlpha (reference 1e-5)")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="diagnostic: one process renders one rank's share of an N-rank job "
                         "(N passes per step over the tiles with tile %% N == rank), no collective")
    ap.add_argument("--emulate-rank", type=int, default=0,
                    help="the rank whose share --emulate-ranks renders (default 0)")
    ap.add_argument("--binary-passes", type=int, default=8,
                    help="passes of the reference-order leg (CTL_SCENE_BINARY_BVH: the reference's own binary "
                         "visit order, bit-exact to its CPU traversal; 0: skip)")
    ap.add_argument("--steps-per-launch", type=int, default=64,
                    help="steps whose passes go through one ctl_render_passes launch (1: one ctl_render_pass "
                         "launch per pass, the reference's DoPass granularity)")
    ap.add_argument("--one-pass-leg", type=int, default=8,
                    help="passes of the one-launch-per-pass comparison leg (0: skip)")
    ap.add_argument("--bvh", default="wide", choices=["wide", "wideq", "binary"],
                    help="device traversal: 4-wide collapsed BVH (wideq: 64-B quantized nodes), or the reference's "
                         "binary order")
    ap.add_argument("--dopass-leg", type=int, default=8,
                    help="passes of the reference DoPass leg (ctl_scene_update + sampler tables + one "
                         "ctl_render_pass per pass; 0: skip)")
    ap.add_argument("--c5-passes", type=int, default=16,
                    help="C5 (textured scene, full-shading kernel) leg passes (0: skip; skipped when --config 5)")
    ap.add_argument("--ceiling", type=int, default=1,
                    help="measure the HBM-read and dependent node-chain ceilings (libctl_ceiling.so) on rank 0 "
                         "after the timed region and report the path kernel against them (0: skip)")
    ap.add_argument("--launch-check-scene", action="store_true",
                    help="with --launch-check: also rehearse the build-once scene path on a small scene")
    ap.add_argument("--no-build-once", action="store_true",
                    help="every rank compiles the scene (default: local rank 0 compiles, the others map its cache)")
    ap.add_argument("--scene-cache-dir", default="/dev/shm",
                    help="where the build-once scene cache is written (shared by the ranks of a node)")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher rehearsal: the ranks join the process group and count themselves; no GPU, "
                         "no scene (tests/test_bench_launch.py)")
    return ap.parse_args(argv)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, gpus, port):
    """The child command that runs this script once per GPU: torch.distributed.run
    with one process per GPU over 127.0.0.1 (the contract's multi-GPU launch)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch_plan(a, env):
    """What a process started as `bench.py --gpus N` does: "run" (it is a rank, or
    N = 1), "spawn" (no launcher around it and N > 1: start one), or an error
    message (a launcher with a different world size)."""
    world = env.get("WORLD_SIZE")
    if world is None:
        return "spawn" if a.gpus > 1 else "run"
    if int(world) != a.gpus:
        return f"--gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks"
    return "run"


def launch_groups(steps, per_launch):
    """Split `steps` into ceil(steps / per_launch) launches of near-equal size
    (sizes differ by at most one), e.g. 20 at 8 -> 7, 7, 6."""
    if steps <= 0:
        return []
    n = -(-steps // max(1, per_launch))
    base, extra = divmod(steps, n)
    return [base + (1 if i < extra else 0) for i in range(n)]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


PEAK_HBM = 8000.0    # GB/s, MI355X_MICROARCH.md (HBM3E spec)
PEAK_L2 = 34500.0    # GB/s, aggregate L2 rate, MI355X_MICROARCH.md (L2)


def pmc_profile():
    """Newest committed rocprofv3 counter summary (profiles/rNN_pmc.json,
    tools_pmc.sh + tools_pmc_summary.py) and whether it was measured on the
    libctl_trace.so this run loads.  CTL_PMC_PROFILE names another summary
    explicitly (a box-local one, tools/round_measure.sh); nothing outside the
    committed rNN files is picked up by the glob."""
    import glob
    import re
    here = os.path.dirname(os.path.abspath(__file__))
    explicit = os.environ.get("CTL_PMC_PROFILE")
    if explicit:
        files = [explicit]
    else:
        files = [f for f in glob.glob(os.path.join(here, "profiles", "r[0-9][0-9]*_pmc.json"))
                 if re.fullmatch(r"r\d\d(_[a-z0-9]+)?_pmc\.json", os.path.basename(f))]
        files.sort(key=lambda f: os.path.basename(f))
    if not files:
        return None, None, False
    j = json.load(open(files[-1]))
    return j, os.path.relpath(os.path.abspath(files[-1]), here), build_match(j, here)


def roofline(prof, fam, ms, alg_bytes, kernel, units=None, unit_key="units_per_launch"):
    """Roofline of one kernel: physical HBM bytes (PMC counters of the same
    binary) over its live per-launch time against the HBM peak, plus the L2 and
    vector-memory-address-unit fractions that actually bind it.  The
    algorithmic-byte model of SURVEY 8(d) is reported beside it as a model: the
    4-wide tree and the caches serve those bytes, so it is not a fraction of
    any hardware limit.

    units: the work units (render passes) of one timed launch.  A profile that
    records its counters per unit ("per_unit", tools_pmc_summary.py) is scaled
    to this launch shape, so any --steps / launch grouping gets its bytes;
    otherwise the profile's per-launch counters apply as they are.  unit_key
    names the profile's unit count: "units_per_launch" (passes, rays of a
    primary batch) or "rays_per_launch" (rays a path-kernel launch traced, so a
    rank's 1/N-image launch gets the bytes per ray of the 1-GPU profile)."""
    j, path, match = prof
    k = (j or {}).get("kernels", {}).get(fam, {})
    scale = 1.0
    if units is not None and k.get(unit_key):
        scale = units / k[unit_key]
    elif units is not None and k:
        # counters of another launch shape without its unit count cannot be scaled to this one
        k = {}
        match = f"profile has no {unit_key} for " + fam
    hbm = k.get("hbm_bytes")
    hbm = hbm * scale if hbm else hbm
    r = {"bound": "hbm", "achieved": None, "peak": PEAK_HBM, "unit": "GB/s", "frac": None, "traffic": hbm,
         "kernel": kernel, "per_launch_ms": round(ms, 4)}
    if units is not None and k.get(unit_key):
        r["traffic_per_unit"] = k["hbm_bytes"] / k[unit_key] if k.get("hbm_bytes") else None
        r["profile_units_per_launch"] = k[unit_key]
        r["scaled_by"] = unit_key
    if hbm:
        ach = hbm / (ms * 1e-3) / 1e9
        r["achieved"] = round(ach, 2)
        r["frac"] = r["frac_hbm"] = round(ach / PEAK_HBM, 4)
    if k.get("l2_read_bytes"):
        r["frac_l2"] = round(k["l2_read_bytes"] * scale / (ms * 1e-3) / 1e9 / PEAK_L2, 4)
    if k.get("ta_busy") is not None:
        r["frac_ta"] = round(k["ta_busy"], 4)
        # TA_TA_BUSY counts cycles with requests in flight: on the traversal it reads
        # high while the dependent node-fetch chain, not the unit's throughput, binds
        # (probes/ta_probe.hip and the cooperative-fetch experiment)
        r["binding_unit"] = ("latency of the dependent node-fetch chain (TA busy = requests in flight)"
                             if k["ta_busy"] > 0.5 else "latency / issue (no unit above 50 %)")
    for key in ("l2_hit_rate", "ta_cycles_per_vmem_wave_inst", "valu_lane_util"):
        if key in k:
            r[key] = round(k[key], 4)
    if k.get("counters_per_launch", {}).get("SQ_INSTS_VMEM_RD") is not None:
        r["vmem_rd_wave_insts_per_launch"] = round(k["counters_per_launch"]["SQ_INSTS_VMEM_RD"] * scale, 1)
    r["profile"] = path
    r["profile_matches_binary"] = match
    r["alg_model"] = {"bytes_per_launch": int(alg_bytes), "gbs": round(alg_bytes / (ms * 1e-3) / 1e9, 2),
                      "note": "SURVEY 8(d) model: 64 B per inner node, 52 B per triangle test, 108 B per "
                              "instance entry of the reference's binary traversal of the same rays; L2-served, "
                              "not a bound"}
    return r


def measure_ceilings(device, lanes):
    """Measured ceilings of the resources the traversal uses (libctl_ceiling.so,
    csrc/device/ceiling.hip), on this run's GPU after its timed region:
    hbm_read_gbs  STREAM-like read of 8 GiB (best of 10), the practical HBM
                  ceiling SURVEY 8(d) asks for beside the 8 TB/s spec;
    node_chain    lane node steps per second of dependent walks over random
                  128-B nodes, seven 16-B loads per step (the wide node fetch),
                  4 waves per SIMD (the path kernel's occupancy), `lanes` active
                  lanes per wave (its measured VALU lane use), with the nodes
                  L2-resident (2 MiB; the path kernel hits L2 99 %) and spread
                  over 0.54 GB (every step a far fetch), and with all 64 lanes."""
    import ctypes as C
    here = os.path.dirname(os.path.abspath(__file__))
    L = C.CDLL(os.path.join(here, "cudatracerlib_amd", "_lib", "libctl_ceiling.so"))
    L.ctl_ceiling_hbm_read.argtypes = [C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
    L.ctl_ceiling_node_chain.argtypes = [C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(C.c_double)]
    out = {"source": "cudatracerlib_amd/csrc/device/ceiling.hip"}
    o = (C.c_double * 3)()
    if L.ctl_ceiling_hbm_read(device, 8 << 30, 10, o) != 0:
        raise RuntimeError("ctl_ceiling_hbm_read failed")
    out["hbm_read_gbs"] = round(o[0], 1)
    out["hbm_read_gbs_mean"] = round(o[1], 1)
    chain = {}
    for name, nbytes, act, share, steps in (("l2_resident", 2 << 20, lanes, 1, 4000),
                                            ("l2_resident_64_lanes", 2 << 20, 64, 1, 4000),
                                            ("far_0p54gb", 650 << 20, lanes, 1, 400),
                                            ("l2_resident_coherent", 2 << 20, lanes, 64, 4000),
                                            ("l1_resident_coherent", 16 << 10, lanes, 64, 4000)):
        if L.ctl_ceiling_node_chain(device, nbytes, act, share, 4, steps, 5, o) != 0:
            raise RuntimeError("ctl_ceiling_node_chain failed")
        chain[name] = {"lane_steps_per_s": round(o[0], 1), "ns_per_wave_step_per_simd": round(o[1], 2),
                       "active_lanes": act, "lanes_per_chain": share, "waves_per_simd": 4, "node_bytes": int(o[2])}
    out["node_chain"] = chain
    return out


def cpu_cores():
    """Host CPUs of this process: its affinity set, a cgroup CPU quota when there
    is one, and the job's stated CPU share (OMP_NUM_THREADS: a GPU box shares its
    256-thread host between 16 GPUs' jobs and sets it to 16).  The baseline runs
    on min(affinity, quota, share) threads and reports all of them."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    share = None
    try:
        share = int(os.environ["OMP_NUM_THREADS"])
    except (KeyError, ValueError):
        pass
    use = min(x for x in (aff, quota, share) if x)
    return {"threads": max(1, use), "affinity_cpus": aff, "cgroup_cpu_quota": quota, "job_cpu_share": share}


def cpu_baseline(desc, params, seconds, threads):
    """The oracle (CPU restatement of the reference path, oracle/) timed on the
    host cores on a bounded sample: every 4th pixel of consecutive passes."""
    import oracle
    O = oracle.load()
    fb = np.zeros((desc.camera.width * desc.camera.height, 7), np.float32)
    rays = 0
    passes = 0
    stats = np.zeros(4, np.uint64)
    t0 = time.perf_counter()
    while True:
        st = np.zeros(4, np.uint64)
        rays += O.oracle_render_pass(C.byref(desc), C.byref(params), 10_000 + passes, oracle.ptr(fb), 0, threads, 4,
                                     oracle.ptr(st))
        stats += st
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds or passes >= 64:
            break
    return {
        "value": round(rays / el / 1e6, 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle PathTrace<true> on the same triangles, every 4th pixel of {passes} pass(es), "
                  f"{rays} rays in {el:.1f} s",
        "per_thread_mrays_s": round(rays / el / 1e6 / threads, 4),
        "cpu_model": cpu_model(),
        "nproc": os.cpu_count(),
        "ref_nodes_per_ray": round(float(stats[1]) / max(1, float(stats[0])), 3),
        "ref_tris_per_ray": round(float(stats[2]) / max(1, float(stats[0])), 3),
    }


def primary_ray_leg(pt, dev, stream, sptr, torch, pass_index, prof, launches=10):
    """Primary-ray traversal through the batch C-ABI (ctl_camera_rays ->
    ctl_intersect): SURVEY §8(d)'s "C3 primary rays" roofline.  Algorithmic
    bytes per launch = 64*inner visits + 52*tri tests + 108*instance entries
    + 48 per ray (32-B ray in, 16-B hit out)."""
    pt.generate_samples(pass_index, sptr)
    n = pt.camera_rays(None, 0, sptr)
    rays = torch.empty((n, 8), dtype=torch.float32, device=dev)
    hits = torch.empty((n, 4), dtype=torch.int32, device=dev)
    pt.camera_rays(rays.data_ptr(), n, sptr)
    st = pt.intersect_stats(n, rays.data_ptr(), hits.data_ptr(), False, sptr)
    alg = 64 * st[1] + 52 * st[2] + 108 * st[3] + 48 * n
    for _ in range(2):
        pt.intersect_buffers(n, rays.data_ptr(), hits.data_ptr(), False, sptr)
    ev = []
    for _ in range(launches):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        pt.intersect_buffers(n, rays.data_ptr(), hits.data_ptr(), False, sptr)
        e1.record(stream)
        ev.append((e0, e1))
    torch.cuda.synchronize(dev)
    ms = sum(e0.elapsed_time(e1) for e0, e1 in ev) / launches
    kname = "intersect_kernel<closest,single,wide> (ctl_intersect over ctl_camera_rays)"
    rl = roofline(prof, "primary_intersect", ms, alg, kname, units=n)   # counters per ray, scaled to n rays
    rl["alg_model"].update({"inner_nodes": int(st[1]), "tri_tests": int(st[2]), "instances": int(st[3])})
    return {
        "kernel": kname,
        "rays_per_launch": int(n),
        "ms_per_launch": round(ms, 4),
        "mrays_s": round(n / ms / 1e3, 2),
        "roofline": rl,
    }


def single_pass_leg(pt, fb, stream, sptr, torch, pass_index, passes):
    """The same pass at the reference's DoPass granularity: one ctl_render_pass
    launch per pass (sampler tables generated before each), bracketed like the
    headline."""
    pt.generate_samples(pass_index, sptr)
    pt.render_pass(fb.data_ptr(), sptr)   # warm-up
    torch.cuda.synchronize()
    pt.reset_rays(sptr)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for k in range(passes):
        pt.generate_samples(pass_index + 1 + k, sptr)
        pt.render_pass(fb.data_ptr(), sptr)
    e1.record(stream)
    pt.sync(sptr)
    ms = e0.elapsed_time(e1)
    rays = pt.rays_traced()
    return {"passes": passes, "ms_per_pass": round(ms / passes, 3), "mrays_s": round(rays / ms / 1e3, 1),
            "note": "one ctl_render_pass launch per pass (reference DoPass granularity); the headline batches "
                    "--steps-per-launch steps per ctl_render_passes launch"}


def reference_dopass_leg(pt, desc, fb, stream, sptr, torch, pass_index, passes, ahead=False):
    """The reference's own pass loop as a drop-in drives it: Tracer::DoPass =
    UpdateKernel (ctl_scene_update on the unchanged scene: constants only, no
    copy, no sync) + the sampler tables + one render pass
    (Kernel/Tracer.h:209-248, TraceHelper.cu:182-217).  Device time of the loop
    between HIP events on the pass stream, and the host time of the update calls.
    ahead: the same calls with CTL_PT_RENDER_AHEAD (ctl_render_pass renders the
    loop's next passes in one launch and folds them call by call): 7 untimed
    calls reach the 8-pass windows, the timed calls are whole windows, so every
    ray counted belongs to a pass the loop folded."""
    import cudatracerlib_amd as ctl
    old = pt.params.flags
    if ahead:
        pt.params.flags = old | ctl.CTL_PT_RENDER_AHEAD
        passes = max(8, passes - passes % 8)
    try:
        warm = 7 if ahead else 1
        for k in range(warm):
            pt.update_scene(desc, 0, sptr)
            pt.generate_samples(pass_index + k, sptr)
            pt.render_pass(fb.data_ptr(), sptr)
        torch.cuda.synchronize()
        pt.reset_rays(sptr)
        upd = 0.0
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(passes):
            t0 = time.perf_counter()
            pt.update_scene(desc, 0, sptr)
            upd += time.perf_counter() - t0
            pt.generate_samples(pass_index + warm + k, sptr)
            pt.render_pass(fb.data_ptr(), sptr)
        e1.record(stream)
        pt.sync(sptr)
        ms = e0.elapsed_time(e1)
        rays = pt.rays_traced()
    finally:
        pt.params.flags = old
    out = {"passes": passes, "ms_per_pass": round(ms / passes, 3), "mrays_s": round(rays / ms / 1e3, 1),
           "update_host_ms_per_call": round(upd * 1e3 / passes, 4),
           "note": "per pass: ctl_scene_update(dirty=0) + ctl_sampler_generate + ctl_render_pass (reference "
                   "DoPass: UpdateKernel + DoRender)"}
    if ahead:
        out["note"] += ("; CTL_PT_RENDER_AHEAD: each 8th call renders 8 passes in one launch, the others fold "
                        "(bit-exact to one pass per call, tests/test_gpu_render_ahead.py)")
    return out


def closest_shadow_leg(pt, fb, stream, sptr, torch, pass_index, passes):
    """The same pass with the reference's own KernelDynamicScene::Occluded
    (a closest-hit shadow traversal tested against the light distance,
    KernelDynamicScene.cu:70-80) instead of any-hit shadow rays: the image is
    identical, the traversal work is not."""
    old = pt.params.shadow_any_hit
    pt.params.shadow_any_hit = 0
    try:
        pt.generate_samples(pass_index, sptr)
        pt.render_pass(fb.data_ptr(), sptr)   # warm-up
        torch.cuda.synchronize()
        pt.reset_rays(sptr)
        ev = []
        for k in range(passes):
            pt.generate_samples(pass_index + 1 + k, sptr)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            pt.render_pass(fb.data_ptr(), sptr)
            e1.record(stream)
            ev.append((e0, e1))
        pt.sync(sptr)
        ms = sum(e0.elapsed_time(e1) for e0, e1 in ev)
        rays = pt.rays_traced()
    finally:
        pt.params.shadow_any_hit = old
    return {"shadow_rays": "closest hit + distance test (reference Occluded)", "passes": passes,
            "ms_per_pass": round(ms / passes, 3), "mrays_s": round(rays / (ms * 1e-3) / 1e6, 2)}


def binary_leg(ctl, pt, desc, fb, stream, sptr, torch, pass_index, passes):
    """The reference-exact traversal (CTL_SCENE_BINARY_BVH: the uploaded binary
    BVH in the reference's own host visit order, so every hit equals the
    reference CPU traversal's, ties included) on the same context: the scene's
    trees switched by ctl_scene_update, one untimed launch, then `passes` passes
    in one ctl_render_passes launch between HIP events."""
    db = type(desc).from_buffer_copy(desc)
    db.flags |= ctl.CTL_SCENE_BINARY_BVH
    pt.update_scene(db, 0, sptr)
    pt.render_passes(fb.data_ptr(), pass_index, min(passes, 4), sptr)   # warm-up
    torch.cuda.synchronize()
    pt.reset_rays(sptr)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    pt.render_passes(fb.data_ptr(), pass_index + 4, passes, sptr)
    e1.record(stream)
    pt.sync(sptr)
    ms = e0.elapsed_time(e1)
    rays = pt.rays_traced()
    pt.update_scene(desc, 0, sptr)   # back to the 4-wide trees
    return {"traversal": "CTL_SCENE_BINARY_BVH: the reference's binary visit order (host branch of "
                         "BVHTraversal.h:122-232), hits bit-exact to its CPU traversal",
            "passes": passes, "ms_per_pass": round(ms / passes, 3), "mrays_s": round(rays / (ms * 1e-3) / 1e6, 2)}


def build_match(j, here):
    """Whether a committed record was measured on the libctl_trace.so this run
    loads: True (library hash), "sources" (a rebuild of the same sources,
    buildid.py: hipcc builds are not byte-reproducible) or False."""
    import hashlib
    lib = os.path.join(here, "cudatracerlib_amd", "_lib", "libctl_trace.so")
    if hashlib.sha256(open(lib, "rb").read()).hexdigest() == j.get("lib_sha256"):
        return True
    if j.get("src_sha256"):
        from buildid import source_fingerprint
        return "sources" if source_fingerprint(here) == j["src_sha256"] else False
    return False


def reference_order_record():
    """The newest committed distance of the shipped default from the reference's
    CPU path, one entry per PathTracer config (profiles/rNN_reference_order_<cfg>.json,
    written by tests/test_reference_order.py::test_full_size_reference_order_distance;
    a round-5 profiles/rNN_reference_order.json counts as C3): per-ray order
    classes, NEE visibility flips of the any-hit shadow query against the
    reference's closest-hit Occluded, and one full pass against the oracle's
    render of the reference's CPU path; `record_matches_binary` ties each to this
    run's library.  Plus the adversarial shadow-ray rooms
    (profiles/rNN_shadow_query_rooms.json, tests/test_shadow_query.py): where the
    any-hit query departs from the reference's Occluded."""
    import glob
    import re
    here = os.path.dirname(os.path.abspath(__file__))
    newest = {}
    for f in sorted(glob.glob(os.path.join(here, "profiles", "r[0-9][0-9]*_reference_order*.json"))):
        m = re.fullmatch(r"(r\d\d)_reference_order(?:_(c\d))?\.json", os.path.basename(f))
        if m:
            newest[m.group(2) or "c3"] = f     # sorted: a later round wins
    out = {}
    for cfg, path in sorted(newest.items()):
        j = json.load(open(path))
        t = j.get("total", {})
        ps = j.get("pass") or {}
        ref = ps.get("reference_cpu_path", ps)   # round 4 records: one comparison, any-hit on both sides
        e = {"rays": t.get("rays"), "differing_rays": t.get("differ"), "ties": t.get("ties"),
             "reference_culled": t.get("ref_culled"), "wide_culled": t.get("other_culled"),
             "ray_classes": sorted((j.get("classes") or {}).keys()),
             "pixels": ref.get("pixels"), "pixels_over_1e-4_rel": ref.get("pixels_over_1e-4_rel"),
             "pixels_differing": ref.get("pixels_differing"), "max_rel": ref.get("max_rel"),
             "vs": ("the reference CPU path (binary order, closest-hit Occluded)" if "reference_cpu_path" in ps
                    else "binary order with any-hit shadows"),
             "source": os.path.relpath(path, here),
             "record_matches_binary": build_match(j.get("build", {}), here) if j.get("build") else False}
        if j.get("nee_visibility"):
            e["nee_visibility_flips"] = j["nee_visibility"].get("visibility_flips")
            e["nee_rays"] = j["nee_visibility"].get("rays")
        out[cfg] = e
    rooms = sorted(glob.glob(os.path.join(here, "profiles", "r[0-9][0-9]_shadow_query_rooms.json")))
    if rooms:
        j = json.load(open(rooms[-1]))
        recs = [(k, kind, c) for k, v in j.items() if k != "build" for kind, c in v.items()]
        out["shadow_query_rooms"] = {
            "rays": sum(c["rays"] for _, _, c in recs),
            "flips": sum(c["flips"] for _, _, c in recs),
            "flips_no_cull": sum(c["flips_no_cull"] for _, _, c in recs),
            "flips_query_misses_occluder": sum(c["flips_query_misses_occluder"] for _, _, c in recs),
            "per_room": {f"{k}/{kind}": [c["flips"], c["rays"]] for k, kind, c in recs},
            "note": ("adversarial grazing shadow rays on grid walls at the origin, 1e4 and 5e4 away: every flip is "
                     "an occluder the any-hit query finds that the reference's own closest-hit cull skips "
                     "(flips == flips_no_cull); shipped shadow_any_hit = 1 departs from Occluded on these rays only"),
            "source": os.path.relpath(rooms[-1], here),
            "record_matches_binary": build_match(j["build"], here) if j.get("build") else False}
    return out or None


def wpt_leg(ctl, pt, dev, sptr, torch, W, H, pass_index, passes, flags=0):
    """WavefrontPathTracer::DoRender (ctl_wpt_render_pass) on the same context and
    scene: the batch traversal's second caller.  The first
    pass allocates the queues and is not counted.  flags: ctl_wpt_params.flags
    (CTL_WPT_SHADOW_ANY_HIT: shadow rays as the any-hit query)."""
    import ctypes as C
    fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)
    prm = ctl.WptParams(1, 50, 5, 0, flags)
    L = ctl.lib()
    ms, rays = [], []
    for k in range(passes + 1):
        pt.generate_samples(pass_index + k, sptr)
        prm.passes_done = k + 1
        pt.reset_rays(sptr)
        if L.ctl_wpt_render_pass(pt._ctx, C.byref(prm), C.c_void_p(fb.data_ptr()), C.c_void_p(sptr)) != 0:
            raise RuntimeError("ctl_wpt_render_pass: " + L.ctl_last_error(pt._ctx).decode())
        if k:
            ms.append(pt.last_pass_ms())
            rays.append(pt.rays_traced())
    per = sum(ms) / len(ms)
    return {"integrator": "WavefrontPathTracer (DoubleRayBuffer queues + batch traversal)",
            "shadow_rays": "any-hit query" if flags & 1 else "closest hit + distance compare (reference)",
            "passes": passes, "ms_per_pass": round(per, 3), "rays_per_pass": int(sum(rays) / len(rays)),
            "mrays_s": round(sum(rays) / (sum(ms) * 1e-3) / 1e6, 2)}


def c1_prim_leg(ctl, dev, torch, passes):
    """BASELINE configs[0]: PrimTracer (first_f) on the Cornell box at 256x256, 1 spp
    per pass, through ctl_prim_pass on its own context (Integrators/PrimTracer.cu:181-232).
    Per-pass device time from ctl_last_pass_ms; the first two passes are warmup."""
    hs = ctl.HostScene().generate(1, 1.0, 256, 256)
    d = hs.compile()
    pt = ctl.PrimTracer(dev.index or 0)
    try:
        pt.upload_scene(d)
        fb = torch.zeros((256 * 256, 7), dtype=torch.float32, device=dev)
        ms, rays = [], []
        for k in range(passes + 2):
            pt.reset_rays()
            pt.do_pass(fb.data_ptr(), k)
            pt.sync()
            if k >= 2:
                ms.append(pt.last_pass_ms())
                rays.append(pt.rays_traced())
    finally:
        pt.close()
    return {"integrator": "PrimTracer first_f (C1 Cornell box, 256x256, 1 spp)", "passes": passes,
            "ms_per_pass": round(sum(ms) / len(ms), 4), "rays_per_pass": int(sum(rays) / len(rays)),
            "mrays_s": round(sum(rays) / (sum(ms) * 1e-3) / 1e6, 2),
            "note": "plumbing config: 65 k rays per pass, launch-latency bound"}


def animation_leg(ctl, dev, torch, iters, n=1024):
    """ctl_scene_animate (AnimatedMesh::k_ComputeState with
    BVHRebuilder::Build(&p, true)'s recompute and SAH rotations) on the skinned grid
    of tools/tools_anim_bench.py (n x n quads, 2 n^2 triangles, 16 bones), on its
    own context: three untimed calls (the tree's shape carries over), then `iters`
    calls each bracketed by HIP events on the stream they run on.  A call includes
    the skinning, TriangleData, Woop data, the mesh tree's rebuild, the 4-wide copy,
    the instance boxes / epsilon and their read-back (one stream sync)."""
    import importlib.util
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("tools_anim_bench", os.path.join(here, "tools", "tools_anim_bench.py"))
    tab = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tab)
    V, N, BI, BW, T, UV = tab.grid(n, 16)
    s = ctl.HostScene()
    s.add_animated_mesh(V, N, BI, BW, T, [ctl.diffuse_material(0.5, 0.5, 0.5)], uvs=UV)
    s.add_node(0)
    s.set_camera([0, 8, -20], [0, 0, 0], [0, 1, 0], 50, 64, 64)
    d = s.compile()
    pt = ctl.PathTracer(dev.index or 0)
    try:
        pt.upload_scene(d)
        f0, f1 = tab.frames(16, 0.0), tab.frames(16, 1.0)
        for _ in range(3):
            pt.animate(0, f0, f1, 0.5)
        torch.cuda.synchronize()
        ms = []
        for k in range(iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pt.animate(0, f0, f1, (k + 0.5) / iters)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
    finally:
        pt.close()
    med = sorted(ms)[len(ms) // 2]
    return {"workload": f"skinned grid {n}x{n} quads: {V.shape[0]} vertices, {T.shape[0]} triangles, 16 bones, "
                        f"{int(d.n_bvh_nodes)} binary nodes rebuilt with rotations, the 4-wide copy refit",
            "calls": iters, "ms_per_animate_median": round(med, 4), "ms_min": round(min(ms), 4),
            "mtris_per_s": round(T.shape[0] / med / 1e3, 1),
            "note": "ctl_scene_animate per call (HIP events); the reference runs BVHRebuilder on the host after a "
                    "device-to-host copy (AnimatedMesh.cpp:170-180)"}


def c5_leg(ctl, dev, torch, stream, sptr, a, threads):
    """BASELINE configs[4] (C5, the textured / rough-material scene) on its own
    context: the full-shading path kernel (path_kernel_persistent FULL=1) at the
    headline's resolution, path length and launch shape.  One untimed launch,
    then --c5-passes passes in launches of --steps-per-launch, bracketed with
    HIP events on the launch stream."""
    t0 = time.perf_counter()
    hs = ctl.HostScene().generate(5, 1.0, a.width, a.height)
    hs.set_bvh_builder(a.builder, a.sbvh_alpha)
    d = hs.compile(threads=threads)
    apply_bvh(ctl, d, a.bvh)
    t_build = time.perf_counter() - t0
    pt = ctl.PathTracer(dev.index or 0, max_path_length=a.max_path_length, rr_start_depth=a.rr_start,
                        shadow_any_hit=bool(a.shadow_any_hit), tile_size=64, schedule="persistent")
    try:
        pt.upload_scene(d)
        fb = torch.zeros((a.width * a.height, 7), dtype=torch.float32, device=dev)
        G = max(1, a.steps_per_launch)
        W0 = min(G, 8)   # untimed warmup launch
        pt.render_passes(fb.data_ptr(), 0, W0, sptr)
        torch.cuda.synchronize(dev)
        pt.reset_rays(sptr)
        ev = []
        p = W0
        for g in launch_groups(a.c5_passes, G):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            pt.render_passes(fb.data_ptr(), p, g, sptr)
            e1.record(stream)
            ev.append((e0, e1))
            p += g
        torch.cuda.synchronize(dev)
        pt.sync(sptr)
        ms = sum(e0.elapsed_time(e1) for e0, e1 in ev)
        rays = pt.rays_traced()
    finally:
        pt.close()
    return {"workload": f"PathTracer C5 (BASELINE.json configs[4]): {d.n_tri_data} tris, {a.width}x{a.height}, "
                        f"{a.c5_passes} spp, textured + rough materials (path_kernel_persistent FULL=1)",
            "passes": a.c5_passes, "launches": len(ev), "ms_per_pass": round(ms / a.c5_passes, 3),
            "rays_per_pass": int(rays / a.c5_passes), "mrays_s": round(rays / (ms * 1e-3) / 1e6, 2),
            "scene_build_s": round(t_build, 1)}


def compile_scene(ctl, a, threads):
    hs = ctl.HostScene().generate(a.config, a.scale, a.width, a.height)
    if a.split_alpha is not None or a.bins or a.max_leaf:
        hs.set_bvh_params(a.split_alpha, a.split_depth, a.bins, a.max_leaf)
    hs.set_bvh_builder(a.builder, a.sbvh_alpha)
    return hs, hs.compile(threads=threads)


def build_scene_once(ctl, a, rank, world, dist, threads):
    """The scene of this run.  One rank per node compiles it (the SBVH build:
    ~36 s on 16 threads and a 3.5 GB host scene at C3 size) and writes the
    compiled desc to a cache file in /dev/shm (cudatracerlib_amd/scene_cache);
    the other ranks wait at a CPU (gloo) barrier and map that file, so the node
    builds once and holds one shared host copy.  Without a process group, or
    with --no-build-once, every rank compiles.  Returns (owner, desc, source):
    owner keeps the desc's arrays alive (a HostScene or a mapped cache)."""
    from cudatracerlib_amd import scene_cache
    if world == 1 or a.no_build_once:
        hs, desc = compile_scene(ctl, a, threads)
        return hs, desc, "compiled"
    cpu = dist.new_group(backend="gloo")
    key = f"c{a.config}_s{a.scale:g}_{a.width}x{a.height}_{a.builder}_{a.sbvh_alpha:g}_{a.split_alpha}_{a.bins}_" \
          f"{a.max_leaf}_{os.environ.get('MASTER_PORT', '0')}"
    path = os.path.join(a.scene_cache_dir, f"ctl_scene_{key}.bin")
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    import torch
    ok = 0
    if local_rank == 0:
        hs, desc = compile_scene(ctl, a, threads)
        try:
            scene_cache.save(desc, path)
            ok = 1
        except OSError as e:          # no room in /dev/shm: every rank compiles
            log(f"[rank {rank}] scene cache not written ({e}); the other ranks compile")
    # every rank learns whether a cache was written (a rank whose node has none finds no file)
    flag = torch.tensor([ok], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=cpu)
    if local_rank == 0:
        dist.barrier(group=cpu)   # the others have mapped it
        try:
            os.remove(path)       # the maps keep the pages until the ranks exit
        except OSError:
            pass
        return hs, desc, "compiled (cache written)" if ok else "compiled"
    if int(flag.item()) == 1 and os.path.exists(path):
        cached = scene_cache.load(path)
        dist.barrier(group=cpu)
        return cached, cached.desc, "mapped from the node's scene cache"
    dist.barrier(group=cpu)
    hs, desc = compile_scene(ctl, a, threads)
    return hs, desc, "compiled"


def apply_bvh(ctl, desc, bvh):
    """The device tree format --bvh selects (a scene flag of the desc)."""
    desc.flags |= {"wide": 0, "binary": ctl.CTL_SCENE_BINARY_BVH, "wideq": ctl._abi.CTL_SCENE_WIDE_QUANT}[bvh]


SCENE_SOURCES = ["compiled", "compiled (cache written)", "mapped from the node's scene cache"]


def host_peak_rss_gb():
    """Peak resident host memory of this process (getrusage ru_maxrss, KiB on
    Linux): a mapped scene cache counts the pages this rank touched."""
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0 ** 2


def rank_report(dist, world, elapsed_s, steps, reduce_ms, dev, build_s=0.0, source="compiled"):
    """Every rank's wall time per step of the timed region (its own bracket,
    the framebuffer reduce included) and the time of its reduce alone, plus the
    world size and backend the process group runs: the N-GPU line's `ranks`
    record, so a scaling run explains itself (slowest rank, reduce share).
    Also each rank's scene source (build-once: compiled, or mapped from the
    node's cache), its scene time and its peak host RSS.
    Collective: every rank calls it."""
    import torch
    src = SCENE_SOURCES.index(source) if source in SCENE_SOURCES else 0
    mine = torch.tensor([elapsed_s * 1e3 / max(1, steps), -1.0 if reduce_ms is None else float(reduce_ms),
                         float(build_s), host_peak_rss_gb(), float(src)], dtype=torch.float64, device=dev)
    if world > 1:
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
    else:
        allv = [mine]
    ms = [round(float(v[0]), 4) for v in allv]
    return {"world_size": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "ms_per_step": ms, "ms_per_step_min": min(ms), "ms_per_step_max": max(ms),
            "reduce_ms": [round(float(v[1]), 4) for v in allv] if world > 1 else None,
            "scene_s": [round(float(v[2]), 2) for v in allv],
            "scene_source": [SCENE_SOURCES[int(v[4])] for v in allv],
            "host_peak_rss_gb": [round(float(v[3]), 2) for v in allv],
            "note": "per rank: its timed-region wall time / steps (the reduce included) and the framebuffer "
                    "reduce alone (HIP events around shard.reduce_framebuffer); value uses the max over ranks; "
                    "scene_s / scene_source / host_peak_rss_gb: the build-once scene (bench.build_scene_once)"}


def launch_check(a, world, rank):
    """--launch-check: every rank joins the process group (gloo) and the ranks
    count themselves, reduce a 1920 x 64 PixelData framebuffer through
    shard.reduce_framebuffer and report their times like the bench's N-GPU
    line (`ranks`); rank 0 prints the line shape, with n_gpus = the ranks that
    reported.  No GPU, no scene."""
    import ctypes as C
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cudatracerlib_amd import shard
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.ones(1, dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    fb = torch.zeros((1920 * 64, 7), dtype=torch.float32)
    fb[rank::max(1, world), :] = 1.0   # disjoint pixels per rank, as the tile shards
    t0 = time.perf_counter()
    red_ms = None
    if world > 1:
        dist.barrier()
        r0 = time.perf_counter()
        img = shard.reduce_framebuffer(fb, dist, out=torch.empty_like(fb))
        red_ms = (time.perf_counter() - r0) * 1e3
        if rank == 0 and not bool((img == 1.0).all()):
            raise RuntimeError("launch-check: the reduced framebuffer is not the union of the shards")
    elapsed = time.perf_counter() - t0
    # the build-once scene path on a small scene: local rank 0 compiles and writes
    # the cache, the others map it; every rank's desc must be byte-identical
    scene = None
    t_build, source = 0.0, "compiled"
    if a.launch_check_scene:
        import hashlib
        import cudatracerlib_amd as ctl
        b = argparse.Namespace(**vars(a))
        b.config, b.scale, b.width, b.height = 2, 0.02, 64, 64
        tb = time.perf_counter()
        owner, desc, source = build_scene_once(ctl, b, rank, world, dist, 2)
        t_build = time.perf_counter() - tb
        from cudatracerlib_amd import scene_cache
        h = hashlib.sha256(bytes(desc.camera))
        for name, (et, count) in scene_cache._ARRAYS.items():
            p = scene_cache._addr(getattr(desc, name))
            if p:
                h.update(C.string_at(p, C.sizeof(et) * int(count(desc))))
        digest = torch.tensor(list(h.digest()[:8]), dtype=torch.int64)
        alld = [torch.zeros_like(digest) for _ in range(world)] if world > 1 else [digest]
        if world > 1:
            dist.all_gather(alld, digest)
        scene = {"triangles": int(desc.n_tri_data), "identical_on_every_rank": all(torch.equal(x, alld[0]) for x in alld)}
    ranks = rank_report(dist, world, elapsed, 1, red_ms, torch.device("cpu"), t_build, source)
    if rank == 0:
        print(json.dumps({"metric": "launch-check", "n_gpus": int(t.item()), "world_size": world,
                          "gpus_requested": a.gpus, "ranks": ranks, "scene": scene}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    plan = launch_plan(a, os.environ)
    if plan == "spawn":
        # No launcher around this process: start one rank per GPU as a child
        # (nothing here has touched the GPU) and report its status.
        cmd = launcher_cmd(argv, a.gpus, _free_port())
        log("bench: --gpus %d without a launcher; starting %s" % (a.gpus, " ".join(cmd)))
        return subprocess.call(cmd)
    if plan != "run":
        log("bench: " + plan)
        return 2
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.launch_check:
        launch_check(a, world, rank)
        return 0
    # image-tile shards: one per rank, or N emulated ranks in this one process
    shards = a.emulate_ranks if (world == 1 and a.emulate_ranks > 1) else world
    tile_rank = rank   # the tile shard this process renders
    if shards != world:
        if not 0 <= a.emulate_rank < shards:
            log(f"bench: --emulate-rank {a.emulate_rank} outside 0..{shards - 1}")
            return 2
        tile_rank = a.emulate_rank
    import torch
    import torch.distributed as dist
    if world > 1 and a.backend == "nccl" and torch.cuda.device_count() < world:
        log(f"bench: {world} RCCL ranks but {torch.cuda.device_count()} visible GPUs")
        return 2
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import cudatracerlib_amd as ctl
    from cudatracerlib_amd import shard

    # one GPU per rank; ranks beyond the visible GPUs wrap around (a gloo
    # rehearsal of the N-rank path on a one-GPU box)
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # bind the process group to this rank's GPU so RCCL never guesses the device
        if a.backend == "nccl":
            dist.init_process_group(a.backend, device_id=dev)
        else:
            dist.init_process_group(a.backend)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    threads = max(1, int(os.environ.get("OMP_NUM_THREADS", "8")))

    t0 = time.perf_counter()
    hs, desc, scene_source = build_scene_once(ctl, a, rank, world, dist, threads)
    apply_bvh(ctl, desc, a.bvh)
    t_build = time.perf_counter() - t0
    log(f"[rank {rank}] scene config {a.config}: {desc.n_tri_data} tris, {desc.n_bvh_nodes} BVH nodes, "
        f"{scene_source} in {t_build:.1f}s with {threads} threads")

    pt = ctl.PathTracer(local, max_path_length=a.max_path_length, rr_start_depth=a.rr_start,
                        shadow_any_hit=bool(a.shadow_any_hit), tile_size=64, num_ranks=shards, rank=tile_rank,
                        schedule=a.schedule)
    pt.upload_scene(desc)
    W, H = a.width, a.height
    fb = torch.zeros((W * H, 7), dtype=torch.float32, device=dev)

    # Instrumented pass (same kernel compiled with counters, untimed) for the
    # roofline's algorithmic bytes: 64 B per inner node visited, 52 B per
    # triangle tested (48 B Woop + 4 B index), 108 B per instance entry
    # (SURVEY.md §8d); per-launch = one pass over this rank's tiles.
    scratch = torch.zeros_like(fb)
    st = pt.pass_stats(scratch.data_ptr(), 1 << 40, sptr)
    alg_bytes_per_pass = 64 * st[1] + 52 * st[2] + 108 * st[3]
    del scratch

    pass_base = 0
    steps_done = 0

    # HIP events bracket every path-kernel launch (on the stream it runs on) so
    # the roofline uses that kernel's own average duration; the sampler-table
    # kernel of each pass stays outside the brackets but inside the step time.
    kev = []

    # The passes of G = --steps-per-launch consecutive steps (each step: this
    # rank's tiles of N passes when sharded, one full-image pass otherwise) go
    # through one ctl_render_passes launch: the same framebuffer as sequential
    # passes (bit-exact, tests/test_gpu_parity.py), with the next pass's paths
    # filling the CUs while the previous pass's longest paths finish (a
    # one-pass launch idles ~10 % of its time in that tail).
    G = max(1, a.steps_per_launch)

    def step(s, timed=False, nsteps=1):
        pidx = [p for k in range(nsteps) for p in shard.step_pass_indices(s + k, shards, pass_base)]
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
        if len(pidx) == 1:
            pt.generate_samples(pidx[0], sptr)
            if timed:
                e0.record(stream)
            pt.render_pass(fb.data_ptr(), sptr)
        else:
            if timed:
                e0.record(stream)
            pt.render_passes(fb.data_ptr(), pidx[0], len(pidx), sptr)
        if timed:
            e1.record(stream)
            kev.append((e0, e1))

    # launches of near-equal size (--steps 20 at 8 per launch: 7 + 7 + 6 steps)
    s = 0
    for g in launch_groups(a.warmup, G):
        step(s, nsteps=g)
        s += g
    steps_done = a.warmup
    torch.cuda.synchronize(dev)
    fb.zero_()
    pass_base = steps_done * shards   # fresh passes for the timed image
    image = torch.empty_like(fb) if world > 1 else fb   # the reduced image (rank 0)
    pt.reset_rays(sptr)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    s = 0
    for g in launch_groups(a.steps, G):
        step(s, timed=True, nsteps=g)
        s += g
    ev1.record(stream)
    red0 = red1 = None
    if world > 1:
        red0 = torch.cuda.Event(enable_timing=True)
        red1 = torch.cuda.Event(enable_timing=True)
        red0.record(stream)
        shard.reduce_framebuffer(fb, dist, out=image)   # RCCL over xGMI, into rank 0's image
        red1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1)
    kernel_ms = sum(e0.elapsed_time(e1) for e0, e1 in kev)
    pt.sync(sptr)   # raises if any traversal of the timed region overflowed its stack
    wsum = float(image[:, 6].sum().item()) if rank == 0 else 0.0   # the timed passes' image (before the legs)

    rays = pt.rays_traced()
    prof = pmc_profile()
    nxt = pass_base + a.steps * shards
    prim = primary_ray_leg(pt, dev, stream, sptr, torch, nxt, prof) if rank == 0 else None
    wpt = (wpt_leg(ctl, pt, dev, sptr, torch, W, H, nxt + 1, a.wpt_passes)
           if rank == 0 and a.wpt_passes > 0 else None)
    if wpt is not None:   # the same integrator with the any-hit shadow query (CTL_WPT_SHADOW_ANY_HIT)
        wpt["shadow_any_hit"] = wpt_leg(ctl, pt, dev, sptr, torch, W, H, nxt + 1, a.wpt_passes, flags=1)
    c1 = None
    if rank == 0 and a.prim_passes > 0:
        try:   # a side leg: its failure is reported in the line, not fatal to the headline
            c1 = c1_prim_leg(ctl, dev, torch, a.prim_passes)
        except Exception as e:
            c1 = {"error": f"{type(e).__name__}: {e}"}
    single = None
    if rank == 0 and shards == 1 and G > 1 and a.one_pass_leg > 0:
        single = single_pass_leg(pt, fb, stream, sptr, torch, nxt + 40, a.one_pass_leg)
    dopass = None
    if rank == 0 and shards == 1 and a.dopass_leg > 0:
        dopass = reference_dopass_leg(pt, desc, fb, stream, sptr, torch, nxt + 60, a.dopass_leg)
        dopass["render_ahead"] = reference_dopass_leg(pt, desc, fb, stream, sptr, torch, nxt + 100,
                                                      max(16, a.dopass_leg), ahead=True)
    closest = None
    if rank == 0 and a.closest_shadow_passes > 0 and shards == 1:
        scratch = torch.zeros_like(fb)
        closest = closest_shadow_leg(pt, scratch, stream, sptr, torch, nxt + 10, a.closest_shadow_passes)
        del scratch
    binary = None
    if rank == 0 and shards == 1 and a.binary_passes > 0 and a.bvh == "wide":
        try:   # a side leg: reported in the line, not fatal to the headline
            scratch = torch.zeros_like(fb)
            binary = binary_leg(ctl, pt, desc, scratch, stream, sptr, torch, nxt + 80, a.binary_passes)
            del scratch
        except Exception as e:
            binary = {"error": f"{type(e).__name__}: {e}"}
    c5 = None
    if rank == 0 and shards == 1 and a.c5_passes > 0 and a.config != 5:
        try:   # a side leg, like C1: reported in the line, not fatal to the headline
            c5 = c5_leg(ctl, dev, torch, stream, sptr, a, threads)
        except Exception as e:
            c5 = {"error": f"{type(e).__name__}: {e}"}
    anim = None
    if rank == 0 and a.anim_iters > 0:
        try:   # a side leg, like C1; last, so that it perturbs no other leg
            anim = animation_leg(ctl, dev, torch, a.anim_iters)
        except Exception as e:
            anim = {"error": f"{type(e).__name__}: {e}"}
    red = dev if a.backend == "nccl" else torch.device("cpu")
    ranks = rank_report(dist, world, elapsed, a.steps, red0.elapsed_time(red1) if red0 is not None else None, red,
                        t_build, scene_source)
    tt = torch.tensor([elapsed], dtype=torch.float64, device=red)
    rr = torch.tensor([rays, 1], dtype=torch.int64, device=red)   # rays, ranks that rendered
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dist.all_reduce(rr, op=dist.ReduceOp.SUM)
    elapsed = float(tt.item())
    total_rays = int(rr[0].item())
    ranks_rendered = int(rr[1].item())
    if ranks_rendered != world:
        raise RuntimeError(f"{ranks_rendered} of {world} ranks rendered")

    if rank == 0:
        passes = a.steps * shards
        launches = len(kev)   # path-kernel launches on this rank in the timed region
        per_launch_ms = kernel_ms / launches
        passes_per_launch = passes / launches   # this rank's passes (tiles of them when sharded) per launch
        fam = "path_kernel_full" if a.config == 5 else "path_kernel"
        # the profile's counters are per traced ray (rays_per_launch) and per pass, so
        # they scale to this run's launch shape, a rank's share of a sharded image
        # included (its launches trace 1/N of the image's rays of N passes); only the
        # workload (scene, resolution, schedule, tree) must match
        pj = prof[0] or {}
        same_workload = ("passes_per_launch" in pj and list(pj.get("config", []))[:4] == [a.config, a.scale, W, H]
                         and a.schedule == "persistent" and a.bvh == "wide")
        pk = (pj.get("kernels") or {}).get(fam, {})
        if pk.get("rays_per_launch"):
            rl = roofline(prof if same_workload else (None, None, False), fam, per_launch_ms,
                          alg_bytes_per_pass * passes_per_launch, KERNEL_NAME[a.schedule], units=rays / launches,
                          unit_key="rays_per_launch")
        else:
            rl = roofline(prof if same_workload and pj.get("shards", 1) == shards else (None, None, False), fam,
                          per_launch_ms, alg_bytes_per_pass * passes_per_launch, KERNEL_NAME[a.schedule],
                          units=passes_per_launch)
        rl.update({"launches_timed": launches, "gpu_step_ms": round(step_ms / a.steps, 3),
                   "passes_per_launch": round(passes_per_launch, 4),
                   "steps_per_launch": launch_groups(a.steps, G),
                   "visits_per_launch": {"inner_nodes": int(st[1]), "tri_tests": int(st[2]),
                                         "instances": int(st[3]), "rays": int(st[0])}})
        if a.ceiling and rank == 0:
            # the binding resources against their measured ceilings on this GPU
            lanes = int(round(64 * rl["valu_lane_util"])) if rl.get("valu_lane_util") else 26
            ce = measure_ceilings(local, lanes)
            node_steps_s = st[1] * passes_per_launch / (per_launch_ms * 1e-3)
            ce["path_kernel_node_steps_per_s"] = round(node_steps_s, 1)
            nc = ce["node_chain"]
            # against every probe: incoherent lanes (each its own random line: a floor the
            # kernel's coherence lifts it above), coherent lanes over L2 (the chain at the L2
            # hit latency, every step a miss in L1), coherent lanes over L1 (at the L1 latency)
            ce["frac_chain_by_probe"] = {k: round(node_steps_s / v["lane_steps_per_s"], 4) for k, v in nc.items()}
            ce["frac_chain"] = ce["frac_chain_by_probe"]["l2_resident_coherent"]
            # triangle tests are dependent fetches too (three 16-B loads against the node's seven)
            ce["frac_chain_with_tri_fetches"] = round(
                (st[1] + st[2] * 3.0 / 7.0) * passes_per_launch / (per_launch_ms * 1e-3)
                / nc["l2_resident_coherent"]["lane_steps_per_s"], 4)
            if rl.get("achieved"):
                ce["frac_hbm_of_measured_read"] = round(rl["achieved"] / ce["hbm_read_gbs"], 4)
            ce["note"] = ("frac_chain = the path kernel's 4-wide node steps per second (STATS pass x passes per "
                          "launch / its HIP-event launch time) over the dependent-chain probe at the kernel's lane "
                          "activity and occupancy with the wave's lanes on one chain of L2-resident nodes (one line "
                          "per load instruction; the kernel's L2 requests per vector-memory instruction are "
                          "l2_requests_per_vmem_inst); the kernel also shades, tests triangles and idles in "
                          "divergence, which the probe does not.  frac_chain_by_probe: against every probe")
            pkk = ((prof[0] or {}).get("kernels") or {}).get(fam, {})
            vm = (pkk.get("counters_per_launch") or {}).get("SQ_INSTS_VMEM_RD")
            if pkk.get("l2_read_bytes") and vm:
                ce["l2_requests_per_vmem_inst"] = round(pkk["l2_read_bytes"] / 128.0 / vm, 3)
            rl["ceilings"] = ce
            rl["hbm_ceiling_gbs"] = ce["hbm_read_gbs"]
            rl["frac_chain"] = ce["frac_chain"]
        if passes_per_launch > 1:
            rl["launch"] = ("ctl_render_passes: the launch's sampler tables, one path-kernel launch over all its "
                            "passes, slice fold (all inside the bracket)")
        out = {
            "metric": "Mrays/s (primary+secondary) at 1920x1080, San-Miguel-scale BVH",
            "value": round(total_rays / elapsed / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": ranks_rendered,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural scene, seed 0x5EED; SequenceSampler/XORWOW stream of the reference)",
            "config": {
                "workload": f"PathTracer C{a.config} (BASELINE.json configs[{a.config - 1}]): "
                            f"{desc.n_tri_data} tris, {W}x{H}, {passes} spp, Direct=1, MaxPathLength="
                            f"{a.max_path_length}, RRStartDepth={a.rr_start}, shadow rays any-hit="
                            f"{a.shadow_any_hit}",
                "triangles": int(desc.n_tri_data),
                "bvh_inner_nodes": int(desc.n_bvh_nodes),
                "bvh_refs": int(desc.n_tri_indices),
                "bvh": a.bvh, "builder": a.builder,
                "resolution": [W, H],
                "spp": passes,
                "tile": 64,
                "parallelism": (f"image-tile shard x{world} + {'RCCL' if a.backend == 'nccl' else a.backend} reduce"
                                if world > 1 else "single GPU"),
                "total_rays": total_rays,
                **({"emulated_ranks": shards, "emulated_rank": tile_rank} if shards != world else {}),
            },
            "roofline": rl,
            "ranks": ranks,
            "primary_rays": prim,
            "one_pass_launches": single,
            "reference_dopass": dopass,
            "closest_hit_shadows": closest,
            "binary_bvh": binary,
            "parity_vs_reference_order": reference_order_record(),
            "wavefront_tracer": wpt,
            "prim_tracer_c1": c1,
            "animation": anim,
            "path_tracer_c5": c5,
            "image_weight_sum": wsum,
            "scene_build_s": round(t_build, 2),
        }
        if world == 1 and not a.no_cpu_baseline:
            cc = cpu_cores()
            # the reference's CPU path runs on its own tree: SBVH with leaves <= 8
            # (SplitBVHBuilder Platform, BVHBuilderHelper.cpp:119), the same triangles
            ref_hs = ctl.HostScene().generate(a.config, a.scale, a.width, a.height)
            ref_hs.set_bvh_builder("sbvh", 1.0e-5).set_bvh_params(0.0, 8, 0, 8)
            ref_desc = ref_hs.compile(threads=threads)
            # and its own shadow test: a closest-hit traceRay + distance test (Occluded)
            ref_params = ctl.PTParams.from_buffer_copy(pt.params)
            ref_params.shadow_any_hit = 0
            out["cpu_baseline"] = cpu_baseline(ref_desc, ref_params, a.cpu_seconds, cc["threads"])
            out["cpu_baseline"].update({k: v for k, v in cc.items() if k != "threads"})
            out["cpu_baseline"]["bvh"] = ("SBVH, leaves <= 8 (the reference's SplitBVHBuilder configuration), binary "
                                          "visit order, closest-hit Occluded shadow rays: the reference's CPU path")
            anchor = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06_cpu_anchor.json")
            if os.path.exists(anchor):
                aj = json.load(open(anchor))
                w = aj["workloads"].get("soup_edge_0.01", {})
                out["cpu_baseline"]["per_thread_vs_reference"] = (w.get("threads_1") or {}).get("ratio_to_reference")
                out["cpu_baseline"]["anchor"] = {
                    "source": "profiles/r06_cpu_anchor.json (tools/cpu_anchor.py, this repo's container)",
                    "workload": "SURVEY 6: 1 M-triangle random soup, SBVH leaves <= 8, 2 M rays from one point",
                    "reference_mrays_s": aj["reference_mrays_s"],
                    "oracle_mrays_s_1_thread": {k: v["threads_1"]["mrays_s"] for k, v in aj["workloads"].items()},
                    "work_per_ray": {k: [v["threads_1"]["inner_visits_per_ray"], v["threads_1"]["tri_tests_per_ray"]]
                                     for k, v in aj["workloads"].items()},
                    "note": ("SURVEY did not record the soup's triangle size; the rate moves 14x with it (inner "
                             "visits and triangle tests per ray listed). per_thread_vs_reference is the soup where "
                             "every ray hits, as SURVEY records, and the work per ray is least (edge 0.01)")}
            out["cpu_baseline"]["note"] = (
                "threads = min(affinity set, cgroup quota, the job's CPU share OMP_NUM_THREADS); the oracle's "
                "rays are independent, so the rate scales about linearly with threads (per_thread_mrays_s)")
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    pt.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
