// imenv_jit.h — run-time specialisation of the step kernel with hipRTC (host side).
//
// The ahead-of-time kernels (DynSpec) read every spec value from device memory. Specs are fixed for
// the lifetime of a handle, so imenv_jit.hip instead writes the spec out as a policy class whose
// accessors are all `static constexpr` (delays, capacities, prices, topology, observation map, the
// Poisson inversion table, and the per-call flags), and compiles step_body against it with hipRTC:
// every branch on the spec folds away, loops over nodes / children / features unroll to straight
// code, and no scalar registers are spent holding spec values. One code object per (spec, flags,
// arch) is cached for the process; modules are loaded per handle (device).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "imenv_device.h"

namespace imenv {

// Per-call properties the JIT kernel treats as compile-time constants.
struct JitFlags {
  bool act_f64 = false;
  bool obs_f64 = false;
  bool noisy_delay = false;
  bool noisy_demand = false;
  bool has_delay_u = false;
  int demand_layout = IMENV_LAYOUT_DRAW;
  bool metrics = false;       // evaluation-harness accumulators attached
  bool stream_store = false;  // IMENV_STORE_STREAM: non-temporal observation / reward stores
  bool wt_obs = false;        // write-through (sc1) observation / reward stores
  bool wt_state = false;      // write-through (sc1) state-row stores
  bool small_blocks = false;  // a launch of at most two waves per SIMD: 64-env blocks (imenv_jit.hip)
  bool info = true;           // info outputs requested (else the kernel carries no info-store code)
  bool full = false;          // n is a multiple of 2048 (so of every block size): no tail lanes
  bool aligned = false;       // 16-byte aligned observation buffer with whole-word rows per group
  uint32_t key() const {
    return (act_f64 ? 1u : 0u) | (obs_f64 ? 2u : 0u) | (noisy_delay ? 4u : 0u) | (noisy_demand ? 8u : 0u) |
           (has_delay_u ? 16u : 0u) | ((uint32_t)demand_layout << 5) | (metrics ? 1024u : 0u) |
           (stream_store ? 2048u : 0u) | (wt_obs ? 8192u : 0u) | (wt_state ? 16384u : 0u) |
           (small_blocks ? 32768u : 0u) | (info ? 0u : 65536u) | (full ? 131072u : 0u) |
           (aligned ? 262144u : 0u);
  }
};

struct JitKernel {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  int bs = 256;       // threads per block
  int ept = 1;        // envs per thread (step kernel)
  std::string tag;    // short description (kernel_info)
};

// Policy + kernel source for one specialisation (maxc: widest split, base: inv/backlog/order_u obs).
std::string jit_source(const SpecDev& d, int maxc, bool base, const JitFlags& f);

// Compile src with hipRTC for `arch` (e.g. "gfx950" or a device's gcnArchName); returns the code
// object through the process-wide cache. On failure returns null and sets msg (compiler log).
std::shared_ptr<const std::vector<char>> jit_compile(const std::string& src, const std::string& arch,
                                                     std::string& msg);

// Compile (cached) and load on the current device.
bool jit_load(const SpecDev& d, int maxc, bool base, const JitFlags& f, const std::string& arch, JitKernel& out,
              std::string& msg);

hipError_t jit_launch(const JitKernel& k, hipStream_t st, const SpecDev* sp, const StepArgs& A);

// Fused base-stock rollout kernel (rollout_body): compile-time properties of one launch.
struct RolloutFlags {
  bool table = false;         // host demand table (else in-kernel draws)
  bool noisy_delay = false;
  bool noisy_demand = false;  // drawn demand only
  bool objective = false;     // dfo_func objective (pmf given)
  int act = ROLL_BASE_STOCK;  // action source (rollout_body ACT): base-stock policy or an open-loop plan
  bool act_f64 = false;       // plan actions are float64 (else float32)
  uint32_t key() const {
    return (table ? 1u : 0u) | (noisy_delay ? 2u : 0u) | (noisy_demand ? 4u : 0u) | (objective ? 8u : 0u) |
           ((uint32_t)act << 4) | (act_f64 ? 64u : 0u);
  }
};

// Threads per block of the rollout kernel for this spec (0: does not fit LDS).
int rollout_block_size(const SpecDev& d, const RolloutFlags& f);
// Objective terms parked per thread in RolloutArgs::terms (trees with R > 1 retailers; 0: one replay
// per row).
int rollout_term_slots(const SpecDev& d, const RolloutFlags& f);
std::string jit_rollout_source(const SpecDev& d, int maxc, const RolloutFlags& f, int bs);
bool jit_rollout_load(const SpecDev& d, int maxc, const RolloutFlags& f, const std::string& arch, JitKernel& out,
                      std::string& msg);
hipError_t jit_rollout_launch(const JitKernel& k, hipStream_t st, const SpecDev* sp, const RolloutArgs& A);

}  // namespace imenv
