// The LP scripts' plan replay (SHLP_8.py:737-766) driven through the C ABI alone (include/imenv.h):
// one imenv_plan_rollout call replays every demand scenario's own plan. No Python, no torch.
// tests/test_c_abi_gpu.py runs it on the reference's plan-replay fixtures, bit for bit.
//
//   c_abi_plan <dir>
//
// <dir>/spec.bin     the ImEnvSpec struct (bytes, as include/imenv.h lays it out)
// <dir>/dims.txt     S T N R
// <dir>/demand.i32   customer demand, int32 [T][R][S]
// <dir>/plans.f64    float64 [T][S][N]: scenario s's action at period t (IMENV_PLAN_PER_EPISODE, one plan row)
// writes
// <dir>/rewards.f64  float64 [T][S]: profit[j, t] = r
// <dir>/stats.f64    float64 [IMENV_NUM_STATS][S]: lp_reward, 0, total_inventory, total_backlog,
//                    customer_backlog per scenario
// <dir>/mean_std.f64 float64 [IMENV_NUM_STATS][2]: np.mean / np.std over the scenarios
// <dir>/info.txt     the kernel description
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "imenv.h"

namespace {

#define HIP_OK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                         \
      std::exit(2);                                                                        \
    }                                                                                      \
  } while (0)

#define IMENV_OK_OR_DIE(x)                                                                 \
  do {                                                                                     \
    int rc_ = (x);                                                                         \
    if (rc_ != IMENV_OK) {                                                                 \
      std::fprintf(stderr, "%s -> %d: %s\n", #x, rc_, imenv_last_error());                 \
      std::exit(3);                                                                        \
    }                                                                                      \
  } while (0)

template <typename T>
std::vector<T> read_file(const std::string& path, size_t count) {
  std::vector<T> v(count);
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f || std::fread(v.data(), sizeof(T), count, f) != count) {
    std::fprintf(stderr, "cannot read %zu values from %s\n", count, path.c_str());
    std::exit(4);
  }
  std::fclose(f);
  return v;
}

template <typename T>
void write_file(const std::string& path, const std::vector<T>& v) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f || std::fwrite(v.data(), sizeof(T), v.size(), f) != v.size()) {
    std::fprintf(stderr, "cannot write %s\n", path.c_str());
    std::exit(4);
  }
  std::fclose(f);
}

template <typename T>
T* to_device(const std::vector<T>& v) {
  T* d = nullptr;
  HIP_OK(hipMalloc(&d, v.size() * sizeof(T)));
  HIP_OK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

template <typename T>
std::vector<T> to_host(const T* d, size_t count) {
  std::vector<T> v(count);
  HIP_OK(hipMemcpy(v.data(), d, count * sizeof(T), hipMemcpyDeviceToHost));
  return v;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s <dir>\n", argv[0]);
    return 1;
  }
  const std::string dir = argv[1];
  if (imenv_spec_size() != (int64_t)sizeof(ImEnvSpec)) {
    std::fprintf(stderr, "ImEnvSpec size mismatch\n");
    return 5;
  }
  long long S, T, N, R;
  {
    FILE* f = std::fopen((dir + "/dims.txt").c_str(), "r");
    if (!f || std::fscanf(f, "%lld %lld %lld %lld", &S, &T, &N, &R) != 4) {
      std::fprintf(stderr, "cannot read dims.txt\n");
      return 4;
    }
    std::fclose(f);
  }
  const std::vector<ImEnvSpec> spec = read_file<ImEnvSpec>(dir + "/spec.bin", 1);
  int32_t* d_demand = to_device(read_file<int32_t>(dir + "/demand.i32", (size_t)(T * R * S)));
  double* d_plans = to_device(read_file<double>(dir + "/plans.f64", (size_t)(T * S * N)));
  double *d_rew = nullptr, *d_ep = nullptr, *d_stats = nullptr;
  HIP_OK(hipMalloc(&d_rew, (size_t)(T * S) * sizeof(double)));
  HIP_OK(hipMalloc(&d_ep, (size_t)(IMENV_NUM_STATS * S) * sizeof(double)));
  HIP_OK(hipMalloc(&d_stats, (size_t)(IMENV_NUM_STATS * 2) * sizeof(double)));
  hipStream_t st;
  HIP_OK(hipStreamCreate(&st));

  ImEnv* env = nullptr;   // the handle lends the spec, device and kernel cache (1 env, never stepped)
  IMENV_OK_OR_DIE(imenv_create(&spec[0], 1, 0, 0, &env));
  ImEnvPlanRollout a = {};
  a.actions = d_plans;
  a.action_dtype = IMENV_F64;
  a.plan_layout = IMENV_PLAN_PER_EPISODE;
  a.num_plans = 1;
  a.num_scenarios = S;
  a.demand = d_demand;
  a.rewards = d_rew;
  a.episode_stats = d_ep;
  a.policy_stats = d_stats;
  IMENV_OK_OR_DIE(imenv_plan_rollout(env, &a, st));
  HIP_OK(hipStreamSynchronize(st));

  write_file(dir + "/rewards.f64", to_host(d_rew, (size_t)(T * S)));
  write_file(dir + "/stats.f64", to_host(d_ep, (size_t)(IMENV_NUM_STATS * S)));
  write_file(dir + "/mean_std.f64", to_host(d_stats, (size_t)(IMENV_NUM_STATS * 2)));
  char info[512];
  IMENV_OK_OR_DIE(imenv_kernel_info(env, info, sizeof info));
  FILE* f = std::fopen((dir + "/info.txt").c_str(), "w");
  std::fprintf(f, "%s\n", info);
  std::fclose(f);

  imenv_destroy(env);
  HIP_OK(hipStreamDestroy(st));
  HIP_OK(hipFree(d_demand));
  HIP_OK(hipFree(d_plans));
  HIP_OK(hipFree(d_rew));
  HIP_OK(hipFree(d_ep));
  HIP_OK(hipFree(d_stats));
  std::printf("ok %lld scenarios x %lld periods\n", S, T);
  return 0;
}
