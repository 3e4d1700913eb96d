"""The C-ABI library: loads, exports every entry point include/pt_abi.h
declares, validates arguments, and builds scene kernels with hipRTC -- all
without a GPU (no compute calls here)."""
import ctypes
import os
import re

import pytest

from compute_path_tracer_amd import _native as N
from compute_path_tracer_amd import scenes
from compute_path_tracer_amd.sdf_editor import CompData

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    txt = open(os.path.join(ROOT, "include", "pt_abi.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported():
    L = N.lib()
    names = declared_functions()
    assert len(names) >= 20
    for name in names:
        assert hasattr(L, name), name
    assert set(names) == set(N.SYMBOLS)
    assert L.pt_abi_version() == 1


def test_struct_sizes_match_reference_blocks():
    assert ctypes.sizeof(N.Constants) == 16  # path_tracer.rs:149-155
    assert ctypes.sizeof(N.Settings) == 20   # path_tracer.rs:157-163


def test_null_and_state_errors_without_device():
    L = N.lib()
    assert L.pt_sync(None) == N.PT_ERR_INVALID
    assert L.pt_dispatch(None, None, None, 1) == N.PT_ERR_INVALID
    assert L.pt_last_error(None) == b"null context"
    ctx = ctypes.c_void_p()
    rc = L.pt_create(0, 8, 8, ctypes.byref(ctx))
    if rc == N.PT_OK:  # a GPU is present: exercise call-order checks
        c = N.Constants(0.0, 1, 1.0, 1)
        s = N.Settings(0, 1, 1.0, 1.0, 0)
        assert L.pt_dispatch(ctx, ctypes.byref(c), ctypes.byref(s), 1) == N.PT_ERR_STATE
        assert L.pt_set_data(ctx, None, 0) == N.PT_ERR_STATE
        L.pt_destroy(ctx)
    else:
        assert rc == N.PT_ERR_HIP and not ctx.value


@pytest.mark.parametrize("bake", ["0", "1"])
@pytest.mark.parametrize("name", ["c2", "c3"])
def test_scene_kernel_builds_with_hiprtc(name, bake, monkeypatch):
    # table and values-baked builds (the baked one also bakes the bounds()
    # boxes); the 124-entry "wide" scene (all four mask words) compiles in
    # the GPU parity tests, too slowly for this suite (~75 s)
    monkeypatch.setenv("PT_JIT_BAKE", bake)
    L = N.lib()
    prog = scenes.SCENES[name]().compile(CompData())
    log = ctypes.create_string_buffer(1 << 16)
    size = ctypes.c_size_t()
    rc = L.pt_jit_compile(prog.ops, prog.n_ops, prog.aabbs, prog.n_aabb,
                          prog.data.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(prog.data), log, len(log),
                          ctypes.byref(size))
    assert rc == N.PT_OK, log.value.decode()
    assert size.value > 10000


def test_jit_rejects_bad_slots():
    L = N.lib()
    prog = scenes.c1_default().compile(CompData())
    log = ctypes.create_string_buffer(4096)
    rc = L.pt_jit_compile(prog.ops, prog.n_ops, prog.aabbs, prog.n_aabb,
                          prog.data.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 5, log, len(log), None)
    assert rc == N.PT_ERR_INVALID and b"out of range" in log.value


def test_comm_argument_errors_without_device():
    """pt_comm_init / pt_reduce_accum / pt_read_reduced / pt_comm_get_unique_id
    reject null and out-of-range arguments before any HIP or RCCL call (the
    state errors with a live context are in test_gpu_parity.py)."""
    L = N.lib()
    uid = (ctypes.c_uint8 * N.PT_COMM_ID_BYTES)()
    assert L.pt_comm_get_unique_id(None) == N.PT_ERR_INVALID
    assert L.pt_comm_init(None, 2, 0, uid) == N.PT_ERR_INVALID
    assert L.pt_reduce_accum(None, 0) == N.PT_ERR_INVALID
    buf = (ctypes.c_float * 4)()
    assert L.pt_read_reduced(None, buf, 16) == N.PT_ERR_INVALID
    assert L.pt_accum_device_ptr(None, None, None) == N.PT_ERR_INVALID
