// pt_host.h -- host-side internals shared by pt_runtime.hip and pt_jit.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "pt_binned.h"
#include "pt_device.h"

// ahead-of-time kernels (pt_kernel.hip)
bool pt_use_simple_kernel(const PtLaunch &L);
void pt_launch_render(const PtLaunch &L, bool stats, hipStream_t stream);
enum class PtBinStage { Gen, Shade, Scan, Scatter, Trace, Fold };
void pt_launch_bin(PtBinStage stage, const PtPass &P, bool stats, unsigned grid, hipStream_t stream);
int pt_bin_trace_blocks_per_cu(bool stats);  // occupancy of the interpreter trace kernel
void pt_launch_display(const float *img, uint32_t w, uint32_t h, int fmt, void *out, hipStream_t stream);

// Expand (program, data[]) into the device tables (see pt_device.h).
int pt_derive(const std::vector<pt_op> &ops, const std::vector<pt_aabb> &aabbs, const float *data, uint32_t n,
              std::vector<PtNode> &nodes, std::vector<PtAabb> &boxes, std::vector<PtMat> &mats, std::string &err);

// Margin constant of the map() bound; NaN: no bound.
float pt_bound_k(const std::vector<PtNode> &nodes);

// Scene-specialised kernels (hipRTC).
struct PtJitModule {
    hipModule_t module = nullptr;
    hipFunction_t render = nullptr;
    hipFunction_t render_stats = nullptr;
    hipFunction_t trace = nullptr;        // binned pipeline trace pass (pt_binned.h)
    hipFunction_t trace_stats = nullptr;
    hipFunction_t trace_m = nullptr;        // march-only trace pass (normal taps in the shade pass)
    hipFunction_t trace_m_stats = nullptr;
    hipFunction_t shade_t = nullptr;        // shade pass with the normal taps (JitMapB)
    hipFunction_t shade_t_stats = nullptr;
    hipFunction_t gen = nullptr;  // camera rays + the scene's straight-line bounds()
    hipFunction_t gen_stats = nullptr;
    hipFunction_t trace_g = nullptr;  // first pass with its own camera rays (PtPass gen_trace)
    std::string key;  // generated source
};

// Source of the specialised kernel for these derived nodes.  bake=false:
// only the topology, per-node flags and material indices enter (values stay
// in the node table, value-only edits do not recompile); bake=true: node
// values become exact f32 literals too (no scalar loads; recompiles, cached,
// when a value changes).
std::string pt_jit_source(const std::vector<PtNode> &nodes, const std::vector<PtAabb> &boxes, bool fast_bounds,
                          bool bake);
// Compile with hipRTC for gfx950; returns the code object or an error log.
// on-disk cache first (*from_disk: the code object came from lib/jitcache)
bool pt_jit_compile_source(const std::string &src, std::vector<char> &code, std::string &log, bool *from_disk = nullptr);
// Load a code object on the current device.
bool pt_jit_load(const std::vector<char> &code, PtJitModule &m, std::string &err);
void pt_jit_unload(PtJitModule &m);
