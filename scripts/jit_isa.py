"""Dump the scene-specialised kernel (hipRTC) for a scene: source, code
object, disassembly and per-kernel resource usage.  CPU-only (hipRTC
cross-compiles); usage: python scripts/jit_isa.py [scene] [outdir]."""
import ctypes
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
scene = sys.argv[1] if len(sys.argv) > 1 else "c3"
out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/jit_isa"
os.makedirs(out, exist_ok=True)
os.environ["PT_JIT_DUMP"] = os.path.join(out, f"{scene}.hip")
os.environ["PT_JIT_CODE_DUMP"] = os.path.join(out, f"{scene}.co")

from compute_path_tracer_amd import _native as N, scenes  # noqa: E402
from compute_path_tracer_amd.sdf_editor import CompData  # noqa: E402

prog = scenes.SCENES[scene]().compile(CompData())
log = ctypes.create_string_buffer(1 << 16)
rc = N.lib().pt_jit_compile(prog.ops, prog.n_ops, prog.aabbs, prog.n_aabb,
                            prog.data.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(prog.data), log, len(log),
                            None)
assert rc == 0, log.value.decode()
for l in log.value.decode().splitlines():
    if l.startswith("(rebuilt"):
        print(l)
llvm = "/opt/rocm/lib/llvm/bin"
dis = subprocess.run([f"{llvm}/llvm-objdump", "-d", "--mcpu=gfx950", os.environ["PT_JIT_CODE_DUMP"]],
                     capture_output=True, text=True).stdout
open(os.path.join(out, f"{scene}.s"), "w").write(dis)
notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", os.environ["PT_JIT_CODE_DUMP"]],
                       capture_output=True, text=True).stdout
for key in (".name:", ".vgpr_count:", ".sgpr_count:", ".agpr_count:", ".vgpr_spill_count:", ".sgpr_spill_count:",
            ".group_segment_fixed_size:", ".private_segment_fixed_size:"):
    for m in re.finditer(re.escape(key) + r"\s*(\S+)", notes):
        print(key, m.group(1))
print("instructions:", sum(1 for l in dis.splitlines() if re.match(r"^\s+[sv]_|^\s+ds_|^\s+buffer_|^\s+global_", l)))
