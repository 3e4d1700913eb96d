"""The C ABI from a compiled C caller (tests/abi_harness.c, VERDICT r04 item
6): built with gcc -std=c11 -Wall -Werror -pedantic against the in-tree
libpt.so.  Its _Static_asserts pin every struct's size and field offsets at
compile time (the Rust #[repr(C)] block of INTEGRATION.md 2 has the same
layout); the tests compare what it prints with the ctypes mirror and with
the Python compile of the same scene, and on the GPU it renders BASELINE
config 1 through pt_create .. pt_read_accum and checks the committed oracle
image bit for bit."""
import ctypes
import json
import os
import subprocess

import pytest

from compute_path_tracer_amd import _native as N
from compute_path_tracer_amd import build as B
from compute_path_tracer_amd import scenes
from compute_path_tracer_amd.sdf_editor import CompData

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "abi_harness.c")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not os.path.exists(B.LIB):
        pytest.fail(f"{B.LIB} is not built (run __graft_entry__.build())")
    libdir = os.path.dirname(B.LIB)
    exe = str(tmp_path_factory.mktemp("abi") / "abi_harness")
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-pedantic", "-O1", "-I", os.path.join(ROOT, "include"),
           SRC, "-o", exe, "-L", libdir, "-lpt", f"-Wl,-rpath,{libdir}"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return exe


def _run(exe, *args, timeout=120):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout)


def test_layout_matches_ctypes(harness):
    got = _run(harness, "layout")
    structs = {"pt_constants": N.Constants, "pt_settings": N.Settings, "pt_scene_node": N.SceneNode,
               "pt_op": N.Op, "pt_aabb": N.Aabb, "pt_float_key": N.FloatKey}
    seen = 0
    for cname, cls in structs.items():
        for fname, _ in cls._fields_:
            field = getattr(cls, fname)
            assert got[f"{cname}.{fname}"] == [field.offset, field.size], (cname, fname)
            seen += 1
    assert seen == len(got) - 1  # every field the harness prints, and no other
    assert got["sizes"] == [ctypes.sizeof(c) for c in structs.values()] == [16, 20, 132, 132, 56, 16]


def test_compile_matches_python(harness):
    """pt_compile_scene from C (two-call pattern, a short data[] capacity
    refused with PT_ERR_SIZE) gives the program the Python editor compiles
    for the same scene: 36 data[] slots with the 6969.69 sentinel
    (primitives.rs:53-56), one AABB, the same op list."""
    got = _run(harness, "compile")
    prog = scenes.c1_default().compile(CompData())
    assert (got["n_ops"], got["n_aabb"], got["n_check"]) == (prog.n_ops, prog.n_aabb, prog.n_check)
    assert got["n_data"] == len(prog.data) == 36
    assert got["data_bits"] == [int(v) for v in prog.data.view("uint32")]
    ops = [[o.opcode, o.shape, o.combine, o.check, o.scale, o.size[0], o.material[0]] for o in prog.ops[:prog.n_ops]]
    assert got["ops"] == ops
    boxes = [[a.back, a.so_kind, a.union_scale, a.shape_scale, a.aabb_exaggeration] for a in prog.aabbs[:prog.n_aabb]]
    assert got["aabbs"] == boxes


@pytest.mark.gpu
def test_c_caller_renders_config1(gpu, harness):
    """create -> set_program -> set_data -> dispatch -> read_accum from C:
    BASELINE config 1's scene, 32x32, 2 spp, 1 bounce, against the committed
    oracle image tests/golden/oracle_c1_32x32_s2_b1.npy, bit for bit."""
    got = _run(harness, "render", os.path.join(ROOT, "tests", "golden", "oracle_c1_32x32_s2_b1.npy"), timeout=300)
    assert got["mismatched"] == 0 and got["floats"] == 32 * 32 * 4 and got["mean_rgb"] > 0
