// PMC calibration kernels: known-byte streams at the access widths the step kernel uses,
// so rocprofv3 FETCH_SIZE / WRITE_SIZE can be converted to bytes (MI355X_MICROARCH.md §HBM:
// "calibrate on a known byte count in your own access pattern"). Profiling tool only.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void read_dword(const int32_t* __restrict__ src, int32_t* __restrict__ sink, int64_t n) {
  int32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc ^= src[i];
  if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ void read_dwordx4(const int4* __restrict__ src, int32_t* __restrict__ sink, int64_t n4) {
  int32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ void write_dword(int32_t* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (int32_t)i;
}

__global__ void write_dwordx4(int4* __restrict__ dst, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = make_int4((int)i, 1, 2, 3);
}

extern "C" int pmc_calib_run(void* buf, int64_t bytes, void* sink) {
  const int64_t n = bytes / 4;
  hipLaunchKernelGGL(read_dword, dim3(4096), dim3(256), 0, 0, (const int32_t*)buf, (int32_t*)sink, n);
  hipLaunchKernelGGL(read_dwordx4, dim3(4096), dim3(256), 0, 0, (const int4*)buf, (int32_t*)sink, n / 4);
  hipLaunchKernelGGL(write_dword, dim3(4096), dim3(256), 0, 0, (int32_t*)buf, n);
  hipLaunchKernelGGL(write_dwordx4, dim3(4096), dim3(256), 0, 0, (int4*)buf, n / 4);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
