// Instantiates the ahead-of-time step kernels (runtime spec policy DynSpec) for one node capacity
// IMENV_NT, one translation unit per NT so the variants compile in parallel. Included by
// imenv_step_nt{1..8,16}.hip: NT <= 8 kernels are exact (N == NT), NT = 16 serves 9..16 nodes with
// runtime padding.
#include "imenv_device.h"

namespace imenv {
namespace {
template <int MC, bool BASE, typename ST>
void go(const LaunchCfg& c, const SpecDev* sp, const StepArgs& A) {
  hipLaunchKernelGGL((imenv_step_kernel<DynSpec<IMENV_NT, MC, BASE, ST>>), dim3(c.grid), dim3(256), 0, c.stream, sp,
                     A);
}
template <int MC, bool BASE>
void go_st(const LaunchCfg& c, const SpecDev* sp, const StepArgs& A) {
  if (c.es == 1) go<MC, BASE, uint8_t>(c, sp, A);
  else if (c.es == 2) go<MC, BASE, int16_t>(c, sp, A);
  else go<MC, BASE, int32_t>(c, sp, A);
}
template <int MC>
void go_mc(const LaunchCfg& c, const SpecDev* sp, const StepArgs& A) {
  if (c.base) go_st<MC, true>(c, sp, A);
  else go_st<MC, false>(c, sp, A);
}
}  // namespace

template <>
void launch_step_nt<IMENV_NT>(const LaunchCfg& c, const SpecDev* sp, const StepArgs& A) {
  if constexpr (IMENV_NT >= 6) {
    if (c.mc > 4) { go_mc<IMENV_MAX_CHILDREN>(c, sp, A); return; }
  }
  if constexpr (IMENV_NT >= 3) {
    if (c.mc > 0) { go_mc<4>(c, sp, A); return; }
  }
  go_mc<0>(c, sp, A);
}
}  // namespace imenv
