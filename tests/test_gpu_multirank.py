"""The multi-rank HIP path in one GPU test run: bench.py under
torch.distributed.run with two ranks sharing GPU 0 (PT_BENCH_SHARE_GPU).
RCCL refuses two ranks on one device, so the ranks reduce over gloo on the
host (--dist-backend gloo); every rank renders through its own context and
the library's tile split (pt_set_tiles).  --validate has rank 0 re-render
every frame in one context and compare the assembled image bit for bit.
The RCCL reduce itself is covered on one GPU by
test_gpu_parity.py::test_rccl_single_rank_reduce_and_errors; across GPUs
only the driver's 8-GPU run reaches it."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(*extra: str, timeout: int = 500) -> dict:
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "bench.py", "--gpus", "2",
           "--no-cpu-baseline", "--dist-backend", "gloo", *extra]
    env = dict(os.environ, PT_BENCH_SHARE_GPU="1", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config,scaling", [("c3", "weak"), ("c4", "strong")])
def test_two_ranks_tile_split_bit_exact(gpu, config, scaling):
    out = _bench("--config", config, "--width", "480", "--height", "272", "--spp", "4", "--steps", "2",
                 "--warmup", "1", "--validate")
    assert out["n_gpus"] == 2 and out["scaling"] == scaling
    frames = (1 + 2 + 1) * 4 * (2 if scaling == "weak" else 1)  # warm-up, timed steps, the per-launch timing step
    assert out["validation"] == {"frames": frames, "bit_exact": True}
    assert out["reduce_ms"] > 0 and out["value"] > 0
    # the default tile check agrees, and covers both ranks' tiles
    tc = out["tile_check"]
    assert tc["bit_exact"] is True and tc["frames"] == frames and tc["owner_ranks"] == [0, 1]


@pytest.mark.timeout(600)
def test_default_line_checks_its_tiles(gpu):
    """Without --validate the N > 1 line still proves itself (VERDICT r04
    item 1): rank 0 re-renders ~8 tiles over every accumulated frame and
    compares the assembled image bit for bit; per-rank render times give the
    tile split's balance; the c4_strong leg carries the same check."""
    out = _bench("--width", "480", "--height", "272", "--spp", "4", "--steps", "2", "--warmup", "1",
                 "--c4-steps", "1")
    tc = out["tile_check"]
    assert tc["bit_exact"] is True and tc["mismatched_texels"] == 0 and tc["ref_zero_outside"]
    assert tc["frames"] == (1 + 2 + 1) * 4 * 2 and tc["owner_ranks"] == [0, 1] and len(tc["tiles"]) >= 8
    pr = out["render_ms_per_rank"]
    assert 0 < pr["min"] <= pr["max"] and pr["max_over_min"] >= 1.0
    assert out["reduce_backend"] == "host" and "validation" not in out
    leg = out["c4_strong"]
    assert leg["tile_check"]["bit_exact"] is True and leg["tile_check"]["frames"] == 2 * 256
    assert leg["render_ms_per_rank"]["max"] == leg["render_ms_max_rank"]
    assert bench_exit_ok(out)


@pytest.mark.timeout(600)
def test_line_checks_non_finite_tiles(gpu):
    """the N > 1 line also re-renders every tile of the
    assembled image that holds a non-finite or negative-zero texel
    (bench.special_tiles) -- the texels a reduce's sum is most likely to
    alter.  C3 at 1080p holds NaN texels from its first 256 frames on (the
    reference's normalize of a zero vector), so a
    two-rank line over frames 1..512 must list them and match bit for bit."""
    out = _bench("--spp", "128", "--steps", "1", "--warmup", "0", "--c4-steps", "0")
    tc = out["tile_check"]
    assert tc["frames"] == (0 + 1 + 1) * 128 * 2
    assert len(tc["special_tiles"]) >= 1, tc
    assert tc["special_texels"] == 64 * len(tc["special_tiles"])
    assert set(tc["special_owner_ranks"]) <= {0, 1}
    assert tc["bit_exact"] is True and tc["mismatched_texels"] == 0
    assert out["valid"] is True and out["invalid_reasons"] == []


def bench_exit_ok(out: dict) -> bool:
    sys.path.insert(0, ROOT)
    import bench

    return bench.validation_failures(out) == []


@pytest.mark.timeout(600)
def test_one_gpu_validate_and_tile_check(gpu):
    """bench.py --validate on ONE rank (the solo-pipeline run
    had overwritten the image before the check): both checks bit-exact, and
    the table scene kernel's throughput on the line."""
    # (32 spp: enough samples per step for the binned pipeline, whose
    # solo-pipeline run used to overwrite the image)
    cmd = [sys.executable, "-u", "bench.py", "--no-cpu-baseline", "--width", "480", "--height", "272", "--spp", "32",
           "--steps", "2", "--warmup", "1", "--validate"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == 1
    assert out["validation"] == {"frames": (1 + 2) * 32, "bit_exact": True}
    assert out["tile_check"]["bit_exact"] is True and out["tile_check"]["frames"] == 96
    assert out["roofline"]["kernel"] == "pt_bin_trace_m_jit"
    assert out["table_kernel"]["value"] > 0 and out["config"]["chunks_per_dispatch"] == 1.0
    # the value edit: the table kernel renders at once,
    # the values-baked rebuild of a never-seen edit compiles and lands
    tk = out["table_kernel"]
    assert tk["table_kernel_meanwhile"] is True and tk["tier_active_after"] is True
    assert tk["tier_compile_s"] > 0.1 and tk["tier_up_s"] >= tk["tier_compile_s"] and 1 <= tk["edit_ulps"] < 4096
    assert out["valid"] is True and out["schedule"]["bin_table"]["slots"] == 4096


@pytest.mark.timeout(600)
def test_two_ranks_strong_config4_leg(gpu):
    """The default N > 1 line carries BASELINE config 4 split over the ranks
    (3840x2160, 256 spp) with its reduce timed on its own."""
    out = _bench("--width", "480", "--height", "272", "--spp", "2", "--steps", "1", "--warmup", "0",
                 "--c4-steps", "1")
    leg = out["c4_strong"]
    assert leg["scaling"] == "strong" and leg["n_gpus"] == 2
    assert leg["config"]["width"] == 3840 and leg["config"]["spp_per_step"] == 256
    assert leg["value"] > 0 and leg["reduce_ms"] > 0


@pytest.mark.timeout(600)
def test_bench_gpus_flag_launches_the_ranks(gpu):
    """`bench.py --gpus 2` with no launcher starts the two ranks itself
    (torch.distributed.run as a child process) and the line says so: n_gpus
    2, the tile split bit-exact against a one-context render (VERDICT r03:
    --gpus was parsed and ignored)."""
    cmd = [sys.executable, "-u", "bench.py", "--gpus", "2", "--no-cpu-baseline", "--dist-backend", "gloo",
           "--width", "480", "--height", "272", "--spp", "4", "--steps", "2", "--warmup", "1", "--validate"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PT_BENCH_SHARE_GPU="1", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["validation"]["bit_exact"] is True
    assert out["rccl_ranks"] is None  # (gloo host reduce: RCCL refuses two ranks on one device)
