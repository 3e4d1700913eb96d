"""MI355X-native (gfx950) SDF sphere-trace + Monte-Carlo path-trace hot path.

Drop-in for the GLSL compute path of zachdedoo13/compute_path_tracer
(assets/shaders/path_tracer/test_compute.glsl dispatched by
src/path_tracer/path_tracer.rs).  The kernels live in ``csrc/`` and are reached
through the C ABI of ``include/pt_abi.h`` (``lib/libpt.so``); this package is the
host-side mirror of the reference's ``PathTracer`` and ``SDFEditor``.
"""
from .sdf_editor import CompData, Float, Material, SDFEditor, Shape, Shapes, Transform, Union, UnionType, V3  # noqa: F401

__all__ = ["CompData", "Float", "Material", "SDFEditor", "Shape", "Shapes", "Transform", "Union", "UnionType", "V3"]
