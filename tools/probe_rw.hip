// Read / write / mixed HBM bandwidth probe (tools only; not part of the library).
// Measures, for a given total byte count per launch, float4-per-lane streaming kernels:
//   read   : every lane loads float4s and folds them into one value per thread (stored once)
//   write  : every lane stores float4s
//   copy   : load + store (50 / 50)
//   mixRW  : reads R% of the bytes, writes the rest (the step kernel's mix is ~30 / 70)
// Each kernel runs back to back K times between two HIP events; prints GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -o probe_rw tools/probe_rw.hip && ./probe_rw [MB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void __launch_bounds__(256) k_read(const float4* __restrict__ a, size_t n, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[threadIdx.x] = s;   // never true for zeroed input: keeps the loads alive
}

__global__ void __launch_bounds__(256) k_write(float4* __restrict__ b, size_t n, float c) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    b[i] = make_float4(c, c, c, c);
}

// one pass, one element per thread (like the step kernel: no grid-stride loop)
__global__ void __launch_bounds__(256) k_write1(float4* __restrict__ b, size_t n, float c) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) b[i] = make_float4(c, c, c, c);
}

__global__ void __launch_bounds__(256) k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

// per thread: RD float4 loads from a, WR float4 stores to b (one "env" per thread, no grid-stride)
template <int RD, int WR>
__global__ void __launch_bounds__(256) k_mix(const float4* __restrict__ a, float4* __restrict__ b, size_t nthr) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= nthr) return;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < RD; ++k) {   // layout [k][thread]: each load instruction is 1 KiB per wave
    const float4 v = a[k * nthr + t];
    s += v.x + v.y + v.z + v.w;
  }
#pragma unroll
  for (int k = 0; k < WR; ++k) b[k * nthr + t] = make_float4(s, s, s, (float)k);
  if (WR == 0 && s == 12345.f) b[t] = make_float4(s, s, s, s);   // keeps read-only loads alive
}

int main(int argc, char** argv) {
  const size_t MB = argc > 1 ? std::atoll(argv[1]) : 100;
  const size_t bytes = MB << 20;
  const size_t n = bytes / 16;
  float4 *a, *b;
  float* o;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&o, 4096));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int K = 50;
  const int grid_gs = 256 * 8 * 4;   // grid-stride kernels: 4 waves of 256-thread blocks per SIMD pair
  auto timeit = [&](const char* name, double traffic, auto launch) {
    for (int w = 0; w < 5; ++w) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int k = 0; k < K; ++k) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / K;
    std::printf("%-16s %8.2f us  %7.1f GB/s  (%.1f MB per launch)\n", name, us, traffic / (us * 1e-6) / 1e9,
                traffic / 1e6);
  };
  timeit("read", (double)bytes, [&] { k_read<<<grid_gs, 256>>>(a, n, o); });
  timeit("write", (double)bytes, [&] { k_write<<<grid_gs, 256>>>(b, n, 1.f); });
  timeit("write1", (double)bytes, [&] { k_write1<<<(unsigned)((n + 255) / 256), 256>>>(b, n, 1.f); });
  timeit("copy(half each)", (double)bytes, [&] { k_copy<<<grid_gs, 256>>>(a, b, n / 2); });
  // mixes of 8 float4 per thread = 128 B per thread
  const size_t nt = bytes / 128;
  timeit("mix r1 w7", (double)nt * 128, [&] { k_mix<1, 7><<<(unsigned)((nt + 255) / 256), 256>>>(a, b, nt); });
  timeit("mix r2 w6", (double)nt * 128, [&] { k_mix<2, 6><<<(unsigned)((nt + 255) / 256), 256>>>(a, b, nt); });
  timeit("mix r3 w5", (double)nt * 128, [&] { k_mix<3, 5><<<(unsigned)((nt + 255) / 256), 256>>>(a, b, nt); });
  timeit("mix r4 w4", (double)nt * 128, [&] { k_mix<4, 4><<<(unsigned)((nt + 255) / 256), 256>>>(a, b, nt); });
  timeit("mix r6 w2", (double)nt * 128, [&] { k_mix<6, 2><<<(unsigned)((nt + 255) / 256), 256>>>(a, b, nt); });
  timeit("mix r8 w0", (double)nt * 128, [&] { k_mix<8, 0><<<(unsigned)((nt + 255) / 256), 256>>>(a, b, nt); });
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(o));
  return 0;
}
