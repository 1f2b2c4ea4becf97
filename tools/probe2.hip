// Memory-footprint probes for the current step-kernel layout (C2, int16 state, node-major ring):
// per env 48 B read (actions 16, inv/backlog/order_u rows 3 x 8, ring 4 x 2) and 88 B written
// (state rows 24, ring 8, obs 48, reward 8). No env arithmetic: each probe's time is the floor for
// that access shape, so the gap to the real kernel is compute / latency exposure. Profiling tool
// only (tools/probe2.py).
#include <hip/hip_runtime.h>

#include <cstdint>

struct P2Args {
  const float4* act;
  uint2* inv;
  uint2* bl;
  uint2* ou;
  uint16_t* ring;
  float* obs;
  double* rew;
  int64_t n;
  int32_t ring_row[4];
};

template <bool NT_STORE>
__device__ __forceinline__ void st_f4(float4* p, float4 v) {
  if (NT_STORE) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
  } else {
    *p = v;
  }
}

// EPT envs per thread: env (blockIdx.x * EPT + k) * BS + tid. All loads of all EPT envs first.
template <int BS, int EPT, bool NT_STORE, bool STAGE>
__global__ void __launch_bounds__(BS) probe_mirror(const P2Args A) {
  __shared__ __attribute__((aligned(16))) float s_obs[STAGE ? BS * 12 : 4];
  const int tid = threadIdx.x;
  float4 a[EPT];
  uint2 vi[EPT], vb[EPT], vo[EPT];
  uint16_t r[EPT][4];
  int64_t e[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    e[k] = ((int64_t)blockIdx.x * EPT + k) * BS + tid;
    a[k] = A.act[e[k]];
    vi[k] = A.inv[e[k]];
    vb[k] = A.bl[e[k]];
    vo[k] = A.ou[e[k]];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[k][i] = A.ring[(int64_t)A.ring_row[i] * A.n + e[k]];
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const uint32_t s = vi[k].x + vb[k].y + vo[k].x + r[k][0] + r[k][1] + r[k][2] + r[k][3] + (uint32_t)a[k].x;
    vi[k].x += s; vb[k].y ^= s; vo[k].x -= s;
    A.inv[e[k]] = vi[k];
    A.bl[e[k]] = vb[k];
    A.ou[e[k]] = vo[k];
#pragma unroll
    for (int i = 0; i < 4; ++i) A.ring[(int64_t)A.ring_row[i] * A.n + e[k]] = (uint16_t)(r[k][i] + s);
    const float f = (float)s;
    float o[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) o[q] = f + (float)q * a[k].y;
    if (STAGE) {
#pragma unroll
      for (int q = 0; q < 12; ++q) s_obs[tid * 12 + q] = o[q];
      __syncthreads();
      float4* g4 = reinterpret_cast<float4*>(A.obs + (((int64_t)blockIdx.x * EPT + k) * BS) * 12);
      const float4* s4 = reinterpret_cast<const float4*>(s_obs);
#pragma unroll
      for (int q = 0; q < 3; ++q) st_f4<NT_STORE>(g4 + q * BS + tid, s4[q * BS + tid]);
      __syncthreads();
    } else {
      float4* g4 = reinterpret_cast<float4*>(A.obs + e[k] * 12);
#pragma unroll
      for (int q = 0; q < 3; ++q) st_f4<NT_STORE>(g4 + q, make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]));
    }
    if (NT_STORE) __builtin_nontemporal_store((double)s * a[k].z, A.rew + e[k]);
    else A.rew[e[k]] = (double)s * a[k].z;
  }
}

extern "C" int probe2_run(int which, const P2Args* A, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t n = A->n;
  switch (which) {
    case 0: hipLaunchKernelGGL((probe_mirror<256, 1, false, true>), dim3(n / 256), dim3(256), 0, st, *A); break;
    case 1: hipLaunchKernelGGL((probe_mirror<256, 1, true, true>), dim3(n / 256), dim3(256), 0, st, *A); break;
    case 2: hipLaunchKernelGGL((probe_mirror<256, 2, false, true>), dim3(n / 512), dim3(256), 0, st, *A); break;
    case 3: hipLaunchKernelGGL((probe_mirror<256, 4, false, true>), dim3(n / 1024), dim3(256), 0, st, *A); break;
    case 4: hipLaunchKernelGGL((probe_mirror<256, 1, false, false>), dim3(n / 256), dim3(256), 0, st, *A); break;
    case 5: hipLaunchKernelGGL((probe_mirror<512, 1, false, true>), dim3(n / 512), dim3(512), 0, st, *A); break;
    case 6: hipLaunchKernelGGL((probe_mirror<128, 1, false, true>), dim3(n / 128), dim3(128), 0, st, *A); break;
    case 7: hipLaunchKernelGGL((probe_mirror<256, 2, true, true>), dim3(n / 512), dim3(256), 0, st, *A); break;
    case 8: hipLaunchKernelGGL((probe_mirror<1024, 1, false, true>), dim3(n / 1024), dim3(1024), 0, st, *A); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
