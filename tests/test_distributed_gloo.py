"""Multi-rank path on CPU: world_size 2 over gloo.  Each rank renders its
cyclic 8x8 tiles (oracle as the stand-in renderer -- the same tile rule the
HIP kernel uses), TileSplitRender drives frames and the sum-reduce, and rank
0's assembled image must equal the single-rank render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from compute_path_tracer_amd import _native as N
from compute_path_tracer_amd import scenes
from compute_path_tracer_amd.distributed import TileSplitRender
from oracle import oracle as O

W, H, SPP, BOUNCES = 24, 17, 2, 3


class OracleRenderer:
    """CPU renderer with PathTracer's multi-GPU surface (test double)."""

    def __init__(self, rows, w, h):
        self.sc = O.OracleScene(rows)
        self.w, self.h = w, h
        self.img = np.zeros((h, w, 4), np.float32)
        self.rank, self.nranks = 0, 1
        self.reduced = None

    def set_tiles(self, rank, nranks):
        self.rank, self.nranks = rank, nranks
        self.img[:] = 0

    def comm_unique_id(self):
        return b"gloo"

    def comm_init(self, world, rank, uid):
        assert uid == b"gloo"

    def dispatch(self, c, spp):
        self.sc.render(self.w, self.h, O.Constants(c.time, c.frame, c.aspect, c.last_clear),
                       O.Settings(0, BOUNCES, 1.0, 1.0, 0), spp, image=self.img, rank=self.rank, nranks=self.nranks,
                       threads=1)

    def reduce(self, root):
        t = torch.from_numpy(self.img.copy())
        dist.reduce(t, dst=root, op=dist.ReduceOp.SUM)
        self.reduced = t.numpy()

    def read_reduced(self):
        return self.reduced

    def read_image(self):
        return self.img


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, mode, scaling="weak"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = scenes.c2_sphere_box_torus().rows()
    aspect = float(np.float32(W) / np.float32(H))
    tr = TileSplitRender(OracleRenderer(rows, W, H), rank, world, aspect, reduce=mode, scaling=scaling)
    tr.step(SPP)  # SPP * world frames of this rank's tiles
    tr.step(SPP)
    img = tr.image(0)
    if rank == 0:
        np.save(out, img, allow_pickle=False)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,scaling", [(2, "rccl", "weak"), (2, "host", "weak"), (3, "host", "weak"),
                                                (2, "rccl", "strong"), (3, "host", "strong")])
def test_tile_split_reduce_matches_single_rank(tmp_path, world, mode, scaling):
    """mode "rccl" drives the renderer's own reduce (RCCL in PathTracer, gloo
    in the test double); "host" is TileSplitRender's torch.distributed sum.
    Weak scaling renders SPP * world frames per step, strong SPP (BASELINE
    config 4's split of one image)."""
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, mode, scaling), nprocs=world, join=True)
    got = np.load(out, allow_pickle=False)
    rows = scenes.c2_sphere_box_torus().rows()
    aspect = float(np.float32(W) / np.float32(H))
    ref = O.OracleScene(rows).render(W, H, O.Constants(0.0, 1, aspect, 1), O.Settings(0, BOUNCES, 1.0, 1.0, 0),
                                     2 * SPP * (world if scaling == "weak" else 1))
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_tile_split_rejects_unknown_scaling():
    with pytest.raises(ValueError):
        TileSplitRender(OracleRenderer(scenes.c1_default().rows(), 8, 8), 0, 1, 1.0, scaling="linear")
