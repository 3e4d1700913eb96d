#!/usr/bin/env python3
"""How much a hashed bin mixes check[] sets: C3's 24 boxes,
rays with origins uniform in [-3, 3]^3 and uniform directions (a stand-in for
the real segment distribution), their bounds() masks in float64, then for
hashed bins of 11..16 bits and for one bin per set: the expected number of
boxes a 64-ray window drawn from one bin admits (the union of its rays'
sets), against the per-ray popcount.  CPU only.
    python scripts/bin_mix.py
"""
import ctypes
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from compute_path_tracer_amd import scenes, _native as N
from compute_path_tracer_amd.sdf_editor import CompData
prog = scenes.SCENES["c3"]().compile(CompData())
args = (prog.ops, prog.n_ops, prog.aabbs, prog.n_aabb, prog.data.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(prog.data), 1)
n = ctypes.c_size_t(); N.lib().pt_scene_kernel_source(*args, None, 0, ctypes.byref(n))
buf = ctypes.create_string_buffer(n.value); N.lib().pt_scene_kernel_source(*args, buf, n.value, ctypes.byref(n))
src = buf.value.decode()
boxes = []
for m in re.finditer(r"constexpr PtAabb A(\d+)\{\{(.*?)\}, \{(.*?)\}, (\d+), 0\};", src):
    lo = [float.fromhex(t.strip().rstrip('f')) for t in m.group(2).split(',')]
    hi = [float.fromhex(t.strip().rstrip('f')) for t in m.group(3).split(',')]
    boxes.append((lo, hi, int(m.group(4))))
boxes = boxes[:24]
lo = np.array([b[0] for b in boxes]); hi = np.array([b[1] for b in boxes]); back = np.array([b[2] for b in boxes])
print(len(boxes), lo.min(0), hi.max(0))
rng = np.random.default_rng(1)
M = 400000
o = rng.uniform([-3,-3,-3],[3,3,3], size=(M,3))
d = rng.normal(size=(M,3)); d /= np.linalg.norm(d, axis=1, keepdims=True)
with np.errstate(divide='ignore', invalid='ignore'):
    t1 = (lo[None] - o[:,None]) / d[:,None]; t2 = (hi[None] - o[:,None]) / d[:,None]
tn = np.minimum(t1,t2).max(2); tf = np.maximum(t1,t2).min(2)
hit = (tn < tf) & (tf > 0)
mask = (hit.astype(np.uint64) << back[None].astype(np.uint64)).sum(1).astype(np.uint64)
mx = (mask & 0xffffffff).astype(np.uint32); my = (mask >> 32).astype(np.uint32)
def bin_of(bits):
    h = (mx * np.uint32(0x9E3779B1)) ^ (my * np.uint32(0x85EBCA77))
    h = (h ^ (h >> np.uint32(15))) * np.uint32(0x2C1B3C6D)
    b = h >> np.uint32(32 - bits)
    small = (my == 0) & (mx < (1 << bits))
    return np.where(small, mx, b)
u, cnt = np.unique(mask, return_counts=True)
print("distinct masks", len(u), "mean popcount", np.mean([bin(int(x)).count('1') for x in mask[:20000]]))
pc = np.vectorize(lambda x: bin(int(x)).count('1'))
def mix(key):
    order = np.argsort(key, kind='stable')
    k = key[order]; m = mask[order]
    # windows of 64 consecutive rays within the sorted order (random order inside a bin)
    W = len(m)//64*64
    mw = m[:W].reshape(-1,64)
    orw = np.bitwise_or.reduce(mw, axis=1)
    return pc(orw).mean()
perm = rng.permutation(M); mask = mask[perm]; mx = mx[perm]; my = my[perm]
print("per-ray popcount", pc(mask[:50000]).mean())
for bits in (11, 12, 13, 14):
    print(bits, "window OR popcount", mix(bin_of(bits)))
print("exact", mix(mask))
print("--- straddle-free expectation, 64-ray windows drawn from one bin")
bitsmat = ((mask[:,None] >> np.arange(64, dtype=np.uint64)[None]) & np.uint64(1)).astype(np.float64)
used = bitsmat.sum(0) > 0
bitsmat = bitsmat[:, used]
def expected(key):
    ks, inv = np.unique(key, return_inverse=True)
    nb = len(ks)
    cnts = np.bincount(inv, minlength=nb).astype(np.float64)
    q = np.zeros((nb, bitsmat.shape[1]))
    np.add.at(q, inv, bitsmat)
    q /= cnts[:,None]
    e = (1 - (1 - q) ** 64).sum(1)
    return (e * cnts).sum() / cnts.sum(), nb
for bits in (11, 12, 13, 14, 16):
    print(bits, expected(bin_of(bits)))
print("exact", expected(mask))
