"""bench.py's self-check of an N-GPU line, host side:
which tiles rank 0 re-renders (every rank's share is among them), the
bit-for-bit tile comparison, and the exit status on a bad line -- an RCCL
communicator of the wrong size, a texel that differs -- for the headline and
the c4_strong leg.  The GPU side runs in tests/test_gpu_multirank.py."""
import numpy as np
import pytest

import bench


@pytest.mark.parametrize("width,height", [(1920, 1080), (3840, 2160), (480, 272), (72, 40)])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_tile_spec_covers_every_rank(width, height, world):
    n_tiles = -(-width // 8) * -(-height // 8)
    for seed in range(5):
        r, m = bench.check_tiles_spec(n_tiles, world, seed=seed)
        assert 0 <= r < m <= max(1, n_tiles // 8)
        tiles = list(range(r, n_tiles, m))
        assert 8 <= len(tiles) <= n_tiles
        if world > 1:
            assert m % world == 1
        # tile t belongs to rank t % world (distributed.py): min(8, world) ranks
        assert len({t % world for t in tiles}) == min(world, len(tiles))


def test_tile_ids_match_the_kernels_tiling():
    """pt_binned.h pixel_of: tile g's texels are x in [(g % tx) * 8, +8),
    y in [(g // tx) * 8, +8), ragged at the right and top edges."""
    ids = bench.tile_ids(20, 11)
    tx = 3
    for y in range(11):
        for x in range(20):
            assert ids[y, x] == (y // 8) * tx + x // 8
    assert ids.max() == 5


def _images(w=40, h=24, r=2, m=5, seed=0):
    rng = np.random.default_rng(seed)
    img = rng.standard_normal((h, w, 4)).astype(np.float32)
    img[3, 7] = np.nan  # NaN texels compare as bit patterns
    sel = bench.tile_ids(w, h) % m == r
    ref = np.where(sel[..., None], img, np.float32(0.0)).astype(np.float32)
    return img, ref, r, m


def test_compare_tiles_bit_exact_and_mismatch():
    img, ref, r, m = _images()
    ok = bench.compare_tiles(img, ref, r, m)
    assert ok["bit_exact"] and ok["mismatched_texels"] == 0 and ok["ref_zero_outside"]
    assert ok["texels"] == int(np.count_nonzero(bench.tile_ids(40, 24) % m == r))
    assert all(t % m == r for t in ok["tiles"])
    # one ulp in one texel of a checked tile
    bad = ref.copy()
    ys, xs = np.nonzero(bench.tile_ids(40, 24) % m == r)
    bad[ys[3], xs[3], 1] = np.nextafter(bad[ys[3], xs[3], 1], np.float32(np.inf))
    res = bench.compare_tiles(img, bad, r, m)
    assert not res["bit_exact"] and res["mismatched_texels"] == 1
    # -0 vs +0 differs as a bit pattern
    z = ref.copy()
    img2 = img.copy()
    img2[ys[0], xs[0], 0] = np.float32(0.0)
    z[ys[0], xs[0], 0] = np.float32(-0.0)
    assert not bench.compare_tiles(img2, z, r, m)["bit_exact"]
    # the reference render must be zero outside its tiles (pt_set_tiles)
    leak = ref.copy()
    ys2, xs2 = np.nonzero(bench.tile_ids(40, 24) % m != r)
    leak[ys2[0], xs2[0], 2] = 1.0
    res = bench.compare_tiles(img, leak, r, m)
    assert not res["ref_zero_outside"] and not res["bit_exact"]


def _line(**kw):
    out = {"n_gpus": 8, "reduce_backend": "rccl", "rccl_ranks": 8,
           "tile_check": {"bit_exact": True, "mismatched_texels": 0},
           "c4_strong": {"n_gpus": 8, "reduce_backend": "rccl", "rccl_ranks": 8,
                         "tile_check": {"bit_exact": True, "mismatched_texels": 0}}}
    out.update(kw)
    return out


def test_validation_failures():
    assert bench.validation_failures(_line()) == []
    assert bench.validation_failures({"n_gpus": 1, "reduce_backend": None, "rccl_ranks": None,
                                      "tile_check": {"bit_exact": True}}) == []
    # a gloo (host) reduce has no RCCL communicator to count
    assert bench.validation_failures(_line(reduce_backend="host", rccl_ranks=None, c4_strong=None)) == []
    f = bench.validation_failures(_line(rccl_ranks=1))
    assert len(f) == 1 and "RCCL communicator has 1 ranks" in f[0]
    f = bench.validation_failures(_line(tile_check={"bit_exact": False, "mismatched_texels": 64}))
    assert len(f) == 1 and "64 texels differ" in f[0]
    leg = dict(_line()["c4_strong"], rccl_ranks=4, tile_check={"bit_exact": False, "mismatched_texels": 3})
    f = bench.validation_failures(_line(c4_strong=leg))
    assert len(f) == 2 and all(x.startswith("c4_strong") for x in f)
    f = bench.validation_failures(_line(validation={"frames": 3, "bit_exact": False}))
    assert len(f) == 1 and "validation" in f[0]


def test_exit_status_paths(capsys):
    assert bench.exit_status(_line()) == 0
    assert bench.exit_status(None) == 0  # ranks other than 0
    assert capsys.readouterr().err == ""
    assert bench.exit_status(_line(rccl_ranks=7)) == 1
    assert "NOT valid" in capsys.readouterr().err
    assert bench.exit_status(_line(tile_check={"bit_exact": False, "mismatched_texels": 1})) == 1


def test_special_tiles_pick_non_finite_and_negative_zero_texels():
    """the tiles a sum-reduce could alter -- NaN / inf
    channels and negative zeros (-0 + +0 is +0) -- are the ones the N-GPU
    line re-renders on top of the ~8 spread tiles, at most 16, tile order."""
    w, h = 40, 24  # 5 x 3 tiles
    img = np.ones((h, w, 4), np.float32)
    assert bench.special_tiles(img) == []
    img[3, 7, 0] = np.nan    # tile 0
    img[20, 33, 2] = np.inf  # tile 14
    img[9, 17, 1] = -np.inf  # tile 7
    img[12, 2, 0] = np.float32(-0.0)  # tile 5
    img[12, 3, 1] = np.float32(0.0)   # +0: not special
    ids = bench.tile_ids(w, h)
    assert bench.special_tiles(img) == sorted({int(ids[3, 7]), int(ids[20, 33]), int(ids[9, 17]), int(ids[12, 2])})
    assert bench.special_tiles(img) == [0, 5, 7, 14]
    assert bench.special_tiles(img, limit=2) == [0, 5]
    # a NaN in every tile: the first 16
    many = np.ones((64, 64, 4), np.float32)
    many[::8, ::8, 3] = np.nan
    assert bench.special_tiles(many) == list(range(16))


def test_compare_one_tile():
    w, h = 40, 24
    rng = np.random.default_rng(1)
    img = rng.standard_normal((h, w, 4)).astype(np.float32)
    img[9, 17, 0] = np.nan
    t = int(bench.tile_ids(w, h)[9, 17])
    sel = bench.tile_ids(w, h) == t
    ref = np.where(sel[..., None], img, np.float32(0.0)).astype(np.float32)
    ok = bench.compare_one_tile(img, ref, t)
    assert ok == {"tile": t, "texels": 64, "mismatched_texels": 0, "ref_zero_outside": True}
    bad = ref.copy()
    bad.view(np.uint32)[9, 17, 0] ^= np.uint32(0x80000000)  # the same NaN with its sign bit flipped
    assert bench.compare_one_tile(img, bad, t)["mismatched_texels"] == 1
    leak = ref.copy()
    leak[0, 0, 0] = 1.0
    assert not bench.compare_one_tile(img, leak, t)["ref_zero_outside"]
