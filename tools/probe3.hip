// Memory-footprint probes for the uint8 C2 layout of the step kernel (tools/probe3.py): per env
// 32 B read (actions 16, inv/backlog/order_u rows 3 x 4, ring 4 x 1) and 72 B written (state rows
// 12, ring 4, obs 48, reward 8) = 104 B. No env arithmetic: each probe's time is the floor for its
// access shape. Variants: envs per thread and whether consecutive envs share a thread (wide
// per-lane accesses: 4 envs -> uint4 state rows, uint32 ring words). Profiling tool only.
#include <hip/hip_runtime.h>

#include <cstdint>

struct P3Args {
  const float4* act;
  uint32_t* inv;
  uint32_t* bl;
  uint32_t* ou;
  uint8_t* ring;
  float* obs;
  double* rew;
  int64_t n;
  int32_t ring_row[4];
};

// one env per thread (the current kernel's shape), BS threads, obs staged through LDS
template <int BS>
__global__ void __launch_bounds__(BS) probe_u8(const P3Args A) {
  __shared__ __attribute__((aligned(16))) float s_obs[BS * 12];
  const int tid = threadIdx.x;
  const int64_t e = (int64_t)blockIdx.x * BS + tid;
  const float4 a = A.act[e];
  uint32_t vi = A.inv[e], vb = A.bl[e], vo = A.ou[e];
  uint8_t r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = A.ring[(int64_t)A.ring_row[i] * A.n + e];
  const uint32_t s = vi + vb + vo + r[0] + r[1] + r[2] + r[3] + (uint32_t)a.x;
  A.inv[e] = vi + s;
  A.bl[e] = vb ^ s;
  A.ou[e] = vo - s;
#pragma unroll
  for (int i = 0; i < 4; ++i) A.ring[(int64_t)A.ring_row[i] * A.n + e] = (uint8_t)(r[i] + s);
  const float f = (float)s;
#pragma unroll
  for (int q = 0; q < 12; ++q) s_obs[tid * 12 + q] = f + (float)q * a.y;
  __syncthreads();
  float4* g4 = reinterpret_cast<float4*>(A.obs + ((int64_t)blockIdx.x * BS) * 12);
  const float4* s4 = reinterpret_cast<const float4*>(s_obs);
#pragma unroll
  for (int q = 0; q < 3; ++q) g4[q * BS + tid] = s4[q * BS + tid];
  A.rew[e] = (double)s * a.z;
}

// four consecutive envs per thread: wide loads / stores for every stream
template <int BS>
__global__ void __launch_bounds__(BS) probe_u8x4(const P3Args A) {
  __shared__ __attribute__((aligned(16))) float s_obs[BS * 48];
  const int tid = threadIdx.x;
  const int64_t q4 = (int64_t)blockIdx.x * BS + tid;     // group of 4 envs
  const int64_t e0 = q4 * 4;
  float4 a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = A.act[e0 + k];
  const uint4 vi = reinterpret_cast<const uint4*>(A.inv)[q4];
  const uint4 vb = reinterpret_cast<const uint4*>(A.bl)[q4];
  const uint4 vo = reinterpret_cast<const uint4*>(A.ou)[q4];
  uint32_t r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = reinterpret_cast<const uint32_t*>(A.ring + (int64_t)A.ring_row[i] * A.n)[q4];
  const uint32_t s = vi.x + vb.y + vo.z + r[0] + r[1] + r[2] + r[3] + (uint32_t)a[0].x + (uint32_t)a[3].w;
  reinterpret_cast<uint4*>(A.inv)[q4] = make_uint4(vi.x + s, vi.y + s, vi.z + s, vi.w + s);
  reinterpret_cast<uint4*>(A.bl)[q4] = make_uint4(vb.x ^ s, vb.y ^ s, vb.z ^ s, vb.w ^ s);
  reinterpret_cast<uint4*>(A.ou)[q4] = make_uint4(vo.x - s, vo.y - s, vo.z - s, vo.w - s);
#pragma unroll
  for (int i = 0; i < 4; ++i) reinterpret_cast<uint32_t*>(A.ring + (int64_t)A.ring_row[i] * A.n)[q4] = r[i] + s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float f = (float)s + (float)k;
#pragma unroll
    for (int q = 0; q < 12; ++q) s_obs[(tid * 4 + k) * 12 + q] = f + (float)q * a[k].y;
  }
  __syncthreads();
  float4* g4 = reinterpret_cast<float4*>(A.obs + ((int64_t)blockIdx.x * BS * 4) * 12);
  const float4* s4 = reinterpret_cast<const float4*>(s_obs);
#pragma unroll
  for (int q = 0; q < 12; ++q) g4[q * BS + tid] = s4[q * BS + tid];
  double2* r2 = reinterpret_cast<double2*>(A.rew + e0);
  r2[0] = make_double2((double)s * a[0].z, (double)s * a[1].z);
  r2[1] = make_double2((double)s * a[2].z, (double)s * a[3].z);
}

// two envs per thread, interleaved by block (e = (blockIdx * 2 + k) * BS + tid), loads first
template <int BS>
__global__ void __launch_bounds__(BS) probe_u8_ept2(const P3Args A) {
  __shared__ __attribute__((aligned(16))) float s_obs[BS * 12];
  const int tid = threadIdx.x;
  float4 a[2];
  uint32_t vi[2], vb[2], vo[2];
  uint8_t r[2][4];
  int64_t e[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    e[k] = ((int64_t)blockIdx.x * 2 + k) * BS + tid;
    a[k] = A.act[e[k]];
    vi[k] = A.inv[e[k]]; vb[k] = A.bl[e[k]]; vo[k] = A.ou[e[k]];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[k][i] = A.ring[(int64_t)A.ring_row[i] * A.n + e[k]];
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t s = vi[k] + vb[k] + vo[k] + r[k][0] + r[k][1] + r[k][2] + r[k][3] + (uint32_t)a[k].x;
    A.inv[e[k]] = vi[k] + s; A.bl[e[k]] = vb[k] ^ s; A.ou[e[k]] = vo[k] - s;
#pragma unroll
    for (int i = 0; i < 4; ++i) A.ring[(int64_t)A.ring_row[i] * A.n + e[k]] = (uint8_t)(r[k][i] + s);
    const float f = (float)s;
#pragma unroll
    for (int q = 0; q < 12; ++q) s_obs[tid * 12 + q] = f + (float)q * a[k].y;
    __syncthreads();
    float4* g4 = reinterpret_cast<float4*>(A.obs + (((int64_t)blockIdx.x * 2 + k) * BS) * 12);
    const float4* s4 = reinterpret_cast<const float4*>(s_obs);
#pragma unroll
    for (int q = 0; q < 3; ++q) g4[q * BS + tid] = s4[q * BS + tid];
    __syncthreads();
    A.rew[e[k]] = (double)s * a[k].z;
  }
}

// persistent blocks over 256-env tiles (tile += gridDim), the next tile's loads issued before the
// current tile's arithmetic and stores (software pipelining: more bytes in flight per wave)
struct P3Tile {
  float4 a;
  uint32_t vi, vb, vo;
  uint8_t r[4];
};
__device__ __forceinline__ void p3_load(const P3Args& A, int64_t e, P3Tile& x) {
  x.a = A.act[e];
  x.vi = A.inv[e]; x.vb = A.bl[e]; x.vo = A.ou[e];
#pragma unroll
  for (int i = 0; i < 4; ++i) x.r[i] = A.ring[(int64_t)A.ring_row[i] * A.n + e];
}
template <int BS>
__global__ void __launch_bounds__(BS) probe_u8_persist(const P3Args A) {
  __shared__ __attribute__((aligned(16))) float s_obs[BS * 12];
  const int tid = threadIdx.x;
  const int64_t ntiles = A.n / BS;
  int64_t tile = blockIdx.x;
  P3Tile cur, nxt;
  if (tile < ntiles) p3_load(A, tile * BS + tid, cur);
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t e = tile * BS + tid;
    const int64_t tn = tile + gridDim.x;
    if (tn < ntiles) p3_load(A, tn * BS + tid, nxt);
    const uint32_t s = cur.vi + cur.vb + cur.vo + cur.r[0] + cur.r[1] + cur.r[2] + cur.r[3] + (uint32_t)cur.a.x;
    A.inv[e] = cur.vi + s;
    A.bl[e] = cur.vb ^ s;
    A.ou[e] = cur.vo - s;
#pragma unroll
    for (int i = 0; i < 4; ++i) A.ring[(int64_t)A.ring_row[i] * A.n + e] = (uint8_t)(cur.r[i] + s);
    const float f = (float)s;
#pragma unroll
    for (int q = 0; q < 12; ++q) s_obs[tid * 12 + q] = f + (float)q * cur.a.y;
    __syncthreads();
    float4* g4 = reinterpret_cast<float4*>(A.obs + (tile * BS) * 12);
    const float4* s4 = reinterpret_cast<const float4*>(s_obs);
#pragma unroll
    for (int q = 0; q < 3; ++q) g4[q * BS + tid] = s4[q * BS + tid];
    A.rew[e] = (double)s * cur.a.z;
    __syncthreads();
    cur = nxt;
  }
}

extern "C" int probe3_run(int which, const P3Args* A, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t n = A->n;
  switch (which) {
    case 0: hipLaunchKernelGGL((probe_u8<256>), dim3(n / 256), dim3(256), 0, st, *A); break;
    case 1: hipLaunchKernelGGL((probe_u8<512>), dim3(n / 512), dim3(512), 0, st, *A); break;
    case 2: hipLaunchKernelGGL((probe_u8_ept2<256>), dim3(n / 512), dim3(256), 0, st, *A); break;
    case 3: hipLaunchKernelGGL((probe_u8x4<64>), dim3(n / 256), dim3(64), 0, st, *A); break;
    case 4: hipLaunchKernelGGL((probe_u8x4<128>), dim3(n / 512), dim3(128), 0, st, *A); break;
    case 5: hipLaunchKernelGGL((probe_u8x4<256>), dim3(n / 1024), dim3(256), 0, st, *A); break;
    case 6: hipLaunchKernelGGL((probe_u8_persist<256>), dim3(2048), dim3(256), 0, st, *A); break;
    case 7: hipLaunchKernelGGL((probe_u8_persist<256>), dim3(1024), dim3(256), 0, st, *A); break;
    case 8: hipLaunchKernelGGL((probe_u8_persist<256>), dim3(512), dim3(256), 0, st, *A); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
