"""Multi-process (gloo, CPU) tests of the multi-GPU decomposition (shard.py):
row bands + one gather reassemble the frame bit for bit; frame assignment
covers every frame exactly once.  The per-band renderer here is the CPU oracle
standing in for the GPU (the GPU band path itself is covered by
test_gpu_parity.py::test_row_bands_assemble)."""
import importlib
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, h, w, k, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = importlib.import_module("2018rustraytracer_amd.shard")
    sc = importlib.import_module("2018rustraytracer_amd.scenes")
    r0, r1 = shard.row_band(h, world, rank)
    full = oracle.render(sc.scene_a_bench(), sc.eye_camera(), sc.shadow_camera(), w, h, k, 0)["rgba"]
    band = torch.zeros((shard.band_rows(h, world), w, 4), dtype=torch.float32)
    band[: r1 - r0] = torch.from_numpy(full[r0:r1])
    work, assembled = shard.gather_bands(band, rank, world, h, dist, async_op=True)
    if work is not None:
        work.wait()
    if rank == 0:
        q.put(assembled.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,h", [(2, 64), (2, 61), (3, 50), (4, 7)])
def test_band_gather_reassembles_frame(world, h, oracle, scenes):
    import multiprocessing as mp

    w, k = 48, 32
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, h, w, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = oracle.render(scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0)["rgba"]
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_row_bands_partition():
    shard = importlib.import_module("2018rustraytracer_amd.shard")
    for h in (1, 7, 61, 2160, 4320):
        for world in (1, 2, 3, 4, 8):
            bands = shard.row_bands(h, world)
            covered = [y for r0, r1 in bands for y in range(r0, r1)]
            assert covered == list(range(h))
            assert all(r1 - r0 <= shard.band_rows(h, world) for r0, r1 in bands)


def test_frames_for_rank_cover_each_frame_once():
    shard = importlib.import_module("2018rustraytracer_amd.shard")
    for n in (1, 10, 300):
        for world in (1, 2, 8):
            allf = sorted(f for r in range(world) for f in shard.frames_for_rank(n, r, world))
            assert allf == list(range(n))


def _run_bench(args, world, timeout=300):
    import subprocess
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    import json
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["rgba32f", "rgba8"])
def test_bench_tile_gather_gloo_rehearsal_world2(fmt):
    """bench.py --mode tile-gather end to end with two ranks sharing the box's GPU
    (gloo gathers the CPU-staged bands; the 8-GPU run uses RCCL): one JSON line,
    strong scaling, both ranks' pixels counted once."""
    res = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--mode", "tile-gather", "--format", fmt,
                      "--config", "2", "--steps", "3", "--warmup", "1", "--frames-per-step", "2", "--preroll-ms", "0", "--no-cpu-baseline",
                      "--no-alt"], 2)
    assert res["n_gpus"] == 2 and res["scaling"] == "strong" and res["value"] > 0
    assert res["tile_gather"]["format"] == fmt.upper() and "gloo" in res["tile_gather"]["gather"]
    assert res["config"]["rows_rank0"] == 540
    assert res["frames_per_step"] == 2 and res["tile_gather"]["frames"] == 6


@pytest.mark.gpu
def test_bench_frames_gloo_rehearsal_world2_carries_tile_gather():
    """The default (frames) mode with two ranks also reports the tile-gather figures."""
    res = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--config", "2", "--steps", "20", "--warmup", "5",
                      "--frames-per-step", "64", "--preroll-ms", "20", "--tile-gather-steps", "4", "--no-cpu-baseline",
                      "--no-alt"], 2)
    assert res["scaling"] == "weak" and res["n_gpus"] == 2
    # value = both ranks' frames of a step over the step time
    F = res["frames_per_step"]
    assert F >= 8 and res["value"] == pytest.approx(2 * F * 1920 * 1080 / (res["ms_per_step"] * 1e-3) / 1e6, rel=1e-2)
    assert set(res["tile_gather"]) == {"rgba32f", "rgba8"}
    assert all(v["value"] > 0 for v in res["tile_gather"].values())
    # the strong curve in the line itself: speed-up over one GPU's frame rate, root ingress
    for name, v in res["tile_gather"].items():
        assert v["scaling_vs_n1"] == pytest.approx(v["value"] / (res["value"] / 2), rel=1e-3)
        assert v["root_ingress_GBps"] == pytest.approx(v["root_ingress_bytes_per_frame"] / v["ms_per_step"] / 1e6,
                                                       rel=1e-3)


def test_tile_scaling_fields():
    """bench.tile_scaling: the tile-gather figures against one GPU's rate of the same
    run (alt_fused_shadow when measured, else the two-pass value), per format."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    tile = {"rgba32f": {"value": 1000.0, "ms_per_step": 2.0, "root_ingress_bytes_per_frame": 4_000_000},
            "rgba8": {"error": "x"}}
    bench.tile_scaling(tile, {"value": 3000.0, "alt_fused_shadow": {"value": 4000.0}}, 8)
    t = tile["rgba32f"]
    assert t["scaling_vs_n1"] == 2.0 and "alt_fused_shadow" in t["scaling_basis"]
    assert t["root_ingress_GBps"] == 2.0 and "scaling_vs_n1" not in tile["rgba8"]
    tile = {"rgba8": {"value": 600.0, "ms_per_step": 1.0, "root_ingress_bytes_per_frame": 0}}
    bench.tile_scaling(tile, {"value": 300.0, "alt_fused_shadow": None}, 2)
    assert tile["rgba8"]["scaling_vs_n1"] == 4.0 and tile["rgba8"]["root_ingress_GBps"] == 0.0


def test_bench_watchdog_prints_the_line_and_exits_nonzero():
    """bench.py's secondary-measurement watchdog: when it fires, rank 0 prints the
    line it holds (the secondary field marked), exactly once, and the process exits with
    a non-zero status (bench.WATCHDOG_EXIT): a stalled run never reads as a clean one."""
    import json
    import subprocess
    import sys
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench._Watchdog(0.2, {'value': 1.0, 'tile_gather': None}, 'tile_gather'); time.sleep(30)" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    sys.path.insert(0, ROOT)
    import bench
    assert r.returncode == bench.WATCHDOG_EXIT != 0, (r.returncode, r.stderr)
    assert "watchdog fired" in r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and "watchdog" in d["tile_gather"]["error"]


def test_stripe_partition_mirrors_library():
    """shard.stripe_rows_of / stripe_image_rows (the multi-GPU frame's cyclic stripes)
    agree with the library's rtm_stripe_rows (a host-only call) and tile every image
    row exactly once."""
    import importlib
    shard = importlib.import_module("2018rustraytracer_amd.shard")
    rtm = importlib.import_module("2018rustraytracer_amd")
    lib = rtm.load_library()
    for H in (1, 7, 8, 9, 255, 1080, 2160, 4320):
        for n in (1, 2, 3, 4, 7, 8):
            for S in (1, 3, 8, 64):
                rows = [shard.stripe_rows_of(H, n, S, r) for r in range(n)]
                assert sum(rows) == H
                assert rows == [lib.rtm_stripe_rows(H, S, n, r) for r in range(n)]
                seen = sorted(y for r in range(n) for y in shard.stripe_image_rows(H, n, S, r))
                assert seen == list(range(H))
                assert all(len(shard.stripe_image_rows(H, n, S, r)) == rows[r] for r in range(n))
    assert lib.rtm_stripe_rows(10, 0, 2, 0) == -1 and lib.rtm_stripe_rows(10, 8, 2, 2) == -1
