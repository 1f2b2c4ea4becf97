// Launch-cost probes for one small step launch (C2 at 131,072 envs: one wave generation). What does a
// launch pay before its first useful load, and how much of it depends on the kernel-argument path?
//   empty_noarg     a kernel with no argument at all (the dependent-launch boundary alone)
//   empty_bigarg    reads one field of a 384-byte by-value argument (the step kernel's StepArgs shape)
//   rec_bigarg      the C2 step's bytes as one 16-byte state record per env (actions float4, record
//                   dwordx4 load + store, a 12-float observation row through LDS, a float64 reward),
//                   every pointer taken from the 384-byte by-value argument
//   rec_ptrs        the same with the pointers as leading scalar arguments (preloadable into SGPRs)
//   rows_ptrs       the current row layout (net / order_u dwords, four 1-byte ring slots), scalar args
// Compiled twice by tools/probe_launch.py: plain, and with -mllvm -amdgpu-kernarg-preload-count=16 (the
// leading kernel arguments arrive in SGPRs at wave launch, no scalar load of the kernarg segment).
// Profiling tool only.
#include <hip/hip_runtime.h>

#include <cstdint>

struct BigArgs {          // StepArgs-sized: the pointers the probe uses first, then padding
  const float4* act;
  uint4* rec;
  float* obs;
  double* rew;
  int64_t n;
  int64_t pad[43];
};

namespace {
constexpr int kSC1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
}
__device__ __forceinline__ int64_t uniform(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef unsigned int u2 __attribute__((ext_vector_type(2)));

template <int BS>
__device__ __forceinline__ void rec_body(const float4* __restrict__ act, uint4* __restrict__ rec, float* __restrict__ obs,
                                         double* __restrict__ rew) {
  __shared__ __attribute__((aligned(16))) float s_obs[BS * 12];
  const int tid = threadIdx.x;
  const int64_t e0 = (int64_t)blockIdx.x * BS;
  const int64_t e = e0 + tid;
  const float4 a = act[e];
  const uint4 v = rec[e];
  const uint32_t s = v.x + v.y + (v.z & 0xFF) + (v.w >> 24) + (uint32_t)(int)a.x;
  const float f = (float)s;
#pragma unroll
  for (int q = 0; q < 12; ++q) s_obs[tid * 12 + q] = f + (float)q * a.y;
  const double rw = (double)s * a.z;
  const int64_t u0 = uniform(e0);
  u4 w = {v.x + s, v.y ^ s, v.z + s, v.w - s};
  __builtin_amdgcn_raw_buffer_store_b128(w, rsrc(rec + u0), 16 * tid, 0, kSC1);
  if constexpr (BS > 64) __syncthreads();
  else __builtin_amdgcn_wave_barrier();
  const float4* s4 = reinterpret_cast<const float4*>(s_obs);
  const auto ro = rsrc(obs + u0 * 12);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float4 x = s4[q * BS + tid];
    u4 ww;
    __builtin_memcpy(&ww, &x, 16);
    __builtin_amdgcn_raw_buffer_store_b128(ww, ro, (q * BS + tid) * 16, 0, kSC1);
  }
  u2 w2;
  __builtin_memcpy(&w2, &rw, 8);
  __builtin_amdgcn_raw_buffer_store_b64(w2, rsrc(rew + u0), tid * 8, 0, kSC1);
}

template <int BS>
__device__ __forceinline__ void rows_body(const float4* __restrict__ act, uint32_t* __restrict__ net,
                                          uint32_t* __restrict__ ou, uint8_t* __restrict__ r0, uint8_t* __restrict__ r1,
                                          uint8_t* __restrict__ r2, uint8_t* __restrict__ r3, float* __restrict__ obs,
                                          double* __restrict__ rew) {
  __shared__ __attribute__((aligned(16))) float s_obs[BS * 12];
  const int tid = threadIdx.x;
  const int64_t e0 = (int64_t)blockIdx.x * BS;
  const int64_t e = e0 + tid;
  const float4 a = act[e];
  const uint32_t vn = net[e], vo = ou[e];
  const uint8_t q0 = r0[e], q1 = r1[e], q2 = r2[e], q3 = r3[e];
  const uint32_t s = vn + vo + q0 + q1 + q2 + q3 + (uint32_t)(int)a.x;
  const float f = (float)s;
#pragma unroll
  for (int q = 0; q < 12; ++q) s_obs[tid * 12 + q] = f + (float)q * a.y;
  const double rw = (double)s * a.z;
  const int64_t u0 = uniform(e0);
  __builtin_amdgcn_raw_buffer_store_b32(vn + s, rsrc(net + u0), 4 * tid, 0, kSC1);
  __builtin_amdgcn_raw_buffer_store_b32(vo ^ s, rsrc(ou + u0), 4 * tid, 0, kSC1);
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(q0 + s), rsrc(r0 + u0), tid, 0, kSC1);
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(q1 + s), rsrc(r1 + u0), tid, 0, kSC1);
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(q2 + s), rsrc(r2 + u0), tid, 0, kSC1);
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(q3 + s), rsrc(r3 + u0), tid, 0, kSC1);
  if constexpr (BS > 64) __syncthreads();
  else __builtin_amdgcn_wave_barrier();
  const float4* s4 = reinterpret_cast<const float4*>(s_obs);
  const auto ro = rsrc(obs + u0 * 12);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float4 x = s4[q * BS + tid];
    u4 ww;
    __builtin_memcpy(&ww, &x, 16);
    __builtin_amdgcn_raw_buffer_store_b128(ww, ro, (q * BS + tid) * 16, 0, kSC1);
  }
  u2 w2;
  __builtin_memcpy(&w2, &rw, 8);
  __builtin_amdgcn_raw_buffer_store_b64(w2, rsrc(rew + u0), tid * 8, 0, kSC1);
}
}  // namespace

__global__ void __launch_bounds__(64) pl_empty_noarg() {}

__global__ void __launch_bounds__(64) pl_empty_bigarg(const BigArgs A) {
  if (A.n < 0) A.rew[threadIdx.x] = 0.0;   // never taken: keeps the argument live
}

template <int BS>
__global__ void __launch_bounds__(BS) pl_rec_bigarg(const BigArgs A) {
  rec_body<BS>(A.act, A.rec, A.obs, A.rew);
}

template <int BS>
__global__ void __launch_bounds__(BS) pl_rec_ptrs(const float4* __restrict__ act, uint4* __restrict__ rec,
                                                  float* __restrict__ obs, double* __restrict__ rew) {
  rec_body<BS>(act, rec, obs, rew);
}

__global__ void __launch_bounds__(64) pl_rows_ptrs(const float4* __restrict__ act, uint32_t* __restrict__ net,
                                                   uint32_t* __restrict__ ou, uint8_t* __restrict__ r0,
                                                   uint8_t* __restrict__ r1, uint8_t* __restrict__ r2,
                                                   uint8_t* __restrict__ r3, float* __restrict__ obs,
                                                   double* __restrict__ rew) {
  rows_body<64>(act, net, ou, r0, r1, r2, r3, obs, rew);
}

struct PLArgs {
  const float4* act;
  uint4* rec;
  uint32_t* net;
  uint32_t* ou;
  uint8_t* ring[4];
  float* obs;
  double* rew;
  int64_t n;
};

extern "C" int probe_launch_run(int which, const PLArgs* P, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t n = P->n;
  BigArgs B{};
  B.act = P->act; B.rec = P->rec; B.obs = P->obs; B.rew = P->rew; B.n = n;
  switch (which) {
    case 0: pl_empty_noarg<<<(unsigned)(n / 64), 64, 0, st>>>(); break;
    case 1: pl_empty_bigarg<<<(unsigned)(n / 64), 64, 0, st>>>(B); break;
    case 2: pl_rec_bigarg<64><<<(unsigned)(n / 64), 64, 0, st>>>(B); break;
    case 3: pl_rec_ptrs<64><<<(unsigned)(n / 64), 64, 0, st>>>(P->act, P->rec, P->obs, P->rew); break;
    case 4: pl_rows_ptrs<<<(unsigned)(n / 64), 64, 0, st>>>(P->act, P->net, P->ou, P->ring[0], P->ring[1], P->ring[2],
                                                           P->ring[3], P->obs, P->rew); break;
    case 5: pl_rec_ptrs<128><<<(unsigned)(n / 128), 128, 0, st>>>(P->act, P->rec, P->obs, P->rew); break;
    case 6: pl_rec_ptrs<256><<<(unsigned)(n / 256), 256, 0, st>>>(P->act, P->rec, P->obs, P->rew); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
