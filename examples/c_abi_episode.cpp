// One episode of a batch of envs driven through the C ABI alone (include/imenv.h): no Python, no
// torch. What a C / C++ caller of libimenv.so writes. tests/test_c_abi_gpu.py runs it on the
// reference's golden cases and compares its outputs bit for bit.
//
//   c_abi_episode <dir>
//
// <dir>/spec.bin     the ImEnvSpec struct (bytes, as include/imenv.h lays it out)
// <dir>/dims.txt     n T N F R reward_cols noisy_delay_threshold (0: no noisy delay)
// <dir>/demand.i32   customer demand, int32 [T][R][n] (IMENV_LAYOUT_PER_ENV)
// <dir>/actions.f64  float64 [T][n][N]
// <dir>/delay_u.f64  float64 [T][N][n] host-fed noisy-delay uniforms (read when the threshold > 0)
// writes
// <dir>/obs0.f64     float64 [n][N][F] (reset)
// <dir>/obs.f64      float64 [T][n][N][F]
// <dir>/reward.f64   float64 [T][n][reward_cols]
// <dir>/done.txt     the done flag after every step, and the kernel description
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

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s <dir>\n", argv[0]);
    return 1;
  }
  const std::string dir = argv[1];
  if (imenv_spec_size() != (int64_t)sizeof(ImEnvSpec)) {
    std::fprintf(stderr, "ImEnvSpec size mismatch: header %zu, library %lld\n", sizeof(ImEnvSpec),
                 (long long)imenv_spec_size());
    return 5;
  }
  long long n, T, N, F, R, rc;
  double noisy = 0.0;
  {
    FILE* f = std::fopen((dir + "/dims.txt").c_str(), "r");
    if (!f || std::fscanf(f, "%lld %lld %lld %lld %lld %lld %lf", &n, &T, &N, &F, &R, &rc, &noisy) != 7) {
      std::fprintf(stderr, "cannot read dims.txt\n");
      return 4;
    }
    std::fclose(f);
  }
  const std::vector<ImEnvSpec> spec = read_file<ImEnvSpec>(dir + "/spec.bin", 1);
  const std::vector<int32_t> demand = read_file<int32_t>(dir + "/demand.i32", (size_t)(T * R * n));
  const std::vector<double> actions = read_file<double>(dir + "/actions.f64", (size_t)(T * n * N));

  int32_t *d_demand = nullptr;
  double *d_act = nullptr, *d_obs = nullptr, *d_obs0 = nullptr, *d_rew = nullptr, *d_u = nullptr;
  if (noisy > 0) {
    const std::vector<double> u = read_file<double>(dir + "/delay_u.f64", (size_t)(T * N * n));
    HIP_OK(hipMalloc(&d_u, u.size() * sizeof(double)));
    HIP_OK(hipMemcpy(d_u, u.data(), u.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  HIP_OK(hipMalloc(&d_demand, demand.size() * sizeof(int32_t)));
  HIP_OK(hipMalloc(&d_act, actions.size() * sizeof(double)));
  HIP_OK(hipMalloc(&d_obs0, (size_t)(n * N * F) * sizeof(double)));
  HIP_OK(hipMalloc(&d_obs, (size_t)(T * n * N * F) * sizeof(double)));
  HIP_OK(hipMalloc(&d_rew, (size_t)(T * n * rc) * sizeof(double)));
  HIP_OK(hipMemcpy(d_demand, demand.data(), demand.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_act, actions.data(), actions.size() * sizeof(double), hipMemcpyHostToDevice));
  hipStream_t st;
  HIP_OK(hipStreamCreate(&st));

  ImEnv* env = nullptr;
  IMENV_OK_OR_DIE(imenv_create(&spec[0], n, 0, 0, &env));
  IMENV_OK_OR_DIE(imenv_reset(env, d_demand, IMENV_LAYOUT_PER_ENV, noisy > 0 ? 1 : 0, noisy, d_u, -1, d_obs0,
                              IMENV_F64, st));
  std::string dones;
  for (long long t = 0; t < T; ++t) {
    int32_t done = -1;
    IMENV_OK_OR_DIE(imenv_step(env, d_act + t * n * N, IMENV_F64, d_obs + t * n * N * F, IMENV_F64,
                               d_rew + t * n * rc, nullptr, &done, st));
    dones += std::to_string(done) + " ";
  }
  int32_t extra = -1;   // one step past the horizon: the reference raises IndexError, the ABI returns an error
  const int past = imenv_step(env, d_act, IMENV_F64, d_obs, IMENV_F64, d_rew, nullptr, &extra, st);
  HIP_OK(hipStreamSynchronize(st));

  std::vector<double> obs0((size_t)(n * N * F)), obs((size_t)(T * n * N * F)), rew((size_t)(T * n * rc));
  HIP_OK(hipMemcpy(obs0.data(), d_obs0, obs0.size() * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(obs.data(), d_obs, obs.size() * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(rew.data(), d_rew, rew.size() * sizeof(double), hipMemcpyDeviceToHost));
  write_file(dir + "/obs0.f64", obs0);
  write_file(dir + "/obs.f64", obs);
  write_file(dir + "/reward.f64", rew);
  char info[512];
  IMENV_OK_OR_DIE(imenv_kernel_info(env, info, sizeof info));
  FILE* f = std::fopen((dir + "/done.txt").c_str(), "w");
  std::fprintf(f, "%s\npast_horizon_rc %d\n%s\n", dones.c_str(), past, info);
  std::fclose(f);

  imenv_destroy(env);
  HIP_OK(hipStreamDestroy(st));
  HIP_OK(hipFree(d_demand));
  HIP_OK(hipFree(d_act));
  HIP_OK(hipFree(d_obs0));
  HIP_OK(hipFree(d_obs));
  HIP_OK(hipFree(d_rew));
  if (d_u) HIP_OK(hipFree(d_u));
  std::printf("ok %lld envs x %lld periods\n", n, T);
  return 0;
}
