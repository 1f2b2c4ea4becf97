// Memory-pattern probes for the step kernel's byte budget (C2: 80 B read + 120 B written per env).
// No env arithmetic: each probe moves exactly the step kernel's bytes with a given access shape,
// so its time is the floor for that layout. Profiling tool only (tools/probe.py).
#include <hip/hip_runtime.h>
#include <cstdint>

// (a) current layout: fields SoA [field][node][env] int32, per-node dword accesses
__global__ void __launch_bounds__(256) probe_soa(const float4* __restrict__ act, int32_t* __restrict__ st,
                                                 int32_t* __restrict__ ring, float* __restrict__ obs,
                                                 double* __restrict__ rew, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const float4 a = act[e];
  int v[12], r[4];
#pragma unroll
  for (int k = 0; k < 12; ++k) v[k] = st[k * n + e];
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = ring[k * n + e];
  int s = 0;
#pragma unroll
  for (int k = 0; k < 12; ++k) { v[k] += (int)a.x + r[k & 3]; s += v[k]; st[k * n + e] = v[k]; }
#pragma unroll
  for (int k = 0; k < 4; ++k) ring[(4 + k) * n + e] = r[k] + s;
  float4* o = reinterpret_cast<float4*>(obs + e * 12);
  o[0] = make_float4(v[0], v[1], v[2], v[3]);
  o[1] = make_float4(v[4], v[5], v[6], v[7]);
  o[2] = make_float4(v[8], v[9], v[10], v[11]);
  rew[e] = (double)s * a.y;
}

// (b) packed: fields [field][env][4] int32 (one int4 per field per env), arrival ring time-major
// [slot][env][4] (one int4 load), departures scattered dword stores into later slots
__global__ void __launch_bounds__(256) probe_packed(const float4* __restrict__ act, int4* __restrict__ st,
                                                    int32_t* __restrict__ ring, float4* __restrict__ obs,
                                                    double* __restrict__ rew, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const float4 a = act[e];
  int4 f0 = st[e], f1 = st[n + e], f2 = st[2 * n + e];
  const int4 ar = reinterpret_cast<const int4*>(ring)[e];
  f0.x += ar.x; f1.y += ar.y; f2.z += ar.z; f0.w += (int)a.x + ar.w;
  const int s = f0.x + f1.y + f2.z + f0.w;
  st[e] = f0; st[n + e] = f1; st[2 * n + e] = f2;
#pragma unroll
  for (int k = 0; k < 4; ++k) ring[((int64_t)(1 + k) * n + e) * 4 + k] = s + k;
  obs[3 * e + 0] = make_float4(f0.x, f0.y, f0.z, f0.w);
  obs[3 * e + 1] = make_float4(f1.x, f1.y, f1.z, f1.w);
  obs[3 * e + 2] = make_float4(f2.x, f2.y, f2.z, f2.w);
  rew[e] = (double)s * a.y;
}

// (c) plain float4 copy of the same bytes: 80 B read, 120 B written per env
__global__ void __launch_bounds__(256) probe_copy(const float4* __restrict__ src, float4* __restrict__ dst,
                                                  int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  float4 v[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) v[k] = src[k * n + e];
  float4 w = make_float4(v[0].x + v[1].y, v[2].z, v[3].w, v[4].x);
#pragma unroll
  for (int k = 0; k < 5; ++k) dst[k * n + e] = v[k];
  dst[5 * n + e] = w;
  dst[6 * n + e] = v[1];
  reinterpret_cast<float2*>(dst + 7 * n)[e] = make_float2(w.x, w.y);
}

extern "C" int probe_run(int which, void* a, void* b, void* c, void* d, void* e, int64_t n, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (which == 0)
    hipLaunchKernelGGL(probe_soa, dim3(grid), dim3(256), 0, st, (const float4*)a, (int32_t*)b, (int32_t*)c,
                       (float*)d, (double*)e, n);
  else if (which == 1)
    hipLaunchKernelGGL(probe_packed, dim3(grid), dim3(256), 0, st, (const float4*)a, (int4*)b, (int32_t*)c,
                       (float4*)d, (double*)e, n);
  else
    hipLaunchKernelGGL(probe_copy, dim3(grid), dim3(256), 0, st, (const float4*)a, (float4*)b, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
