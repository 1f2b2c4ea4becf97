// Vector-ALU issue-rate probe (tools only; not part of the library). The rollout kernel is bound by
// vector-instruction issue and a large share of its instructions are float64; the microarch guide
// prices float32 ops only. Each kernel here runs one instruction kind in 8 independent register
// chains (inline asm, so nothing is folded or reordered), 8 waves per SIMD, and reports the
// measured cost as SIMD cycles per wave-instruction at the nominal clock (run it under rocprofv3
// --pmc SQ_INSTS_VALU_* to see which class counter each instruction kind increments):
//   cyc = (launch time x clock x SIMDs) / (waves x instructions per wave)
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/probe_valu tools/probe_valu.hip && tools/bin/probe_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

constexpr int ITERS = 512;   // loop trips; 8 chains x 8 unrolled = 64 instructions per trip
constexpr int BS = 256;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ void __launch_bounds__(BS) k_valu(double* __restrict__ out, double seed) {
  double d[8];
  float f[8];
  int i32[8];
  uint64_t u64[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    d[j] = seed + j + threadIdx.x;
    f[j] = (float)d[j];
    i32[j] = (int)threadIdx.x + j;
    u64[j] = (uint64_t)threadIdx.x * 7 + j;
  }
  const double b = seed * 0.5;
  const float bf = (float)b;
  const int bi = (int)seed;
  const uint32_t m32 = __builtin_amdgcn_readfirstlane(0x55555555u * (uint32_t)bi);
  const uint64_t mask = ((uint64_t)m32 << 32) | m32;               // an SGPR-pair lane mask
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#define STEP(j)                                                                                               \
  if constexpr (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[j]) : "v"(bf));                       \
  if constexpr (OP == 1) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[j]) : "v"(b));                        \
  if constexpr (OP == 2) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[j]) : "v"(b));                        \
  if constexpr (OP == 3) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[j]) : "v"(b));                    \
  if constexpr (OP == 4) asm volatile("v_max_f64 %0, %0, %1" : "+v"(d[j]) : "v"(b));                        \
  if constexpr (OP == 5) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[j]) : "v"(i32[j]));                  \
  if constexpr (OP == 6) asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(i32[j]) : "v"(d[j]));                  \
  if constexpr (OP == 7) asm volatile("v_rndne_f64 %0, %0" : "+v"(d[j]));                                   \
  if constexpr (OP == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(i32[j]) : "v"(bi));                     \
  if constexpr (OP == 9) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(u64[j]) : "v"(i32[j]), "v"(bi) : "vcc"); \
  if constexpr (OP == 10) asm volatile("v_mov_b64 %0, %1" : "=v"(u64[j]) : "v"(d[j]));                     \
  if constexpr (OP == 11) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(i32[j]) : "v"(bi), "s"(mask));  \
  if constexpr (OP == 12) asm volatile("v_lshl_add_u64 %0, %0, 3, %1" : "+v"(u64[j]) : "v"(u64[(j + 1) & 7])); \
  if constexpr (OP == 13) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(i32[j]) : "v"(bi));                    \
  if constexpr (OP == 14) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(i32[j]) : "v"(bi));                \
  if constexpr (OP == 15) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(i32[j]) : "v"(bi), "v"(i32[(j + 1) & 7])); \
  if constexpr (OP == 16) asm volatile("v_add_f32_e64 %0, %0, %1" : "+v"(f[j]) : "v"(bf));                 \
  if constexpr (OP == 17) asm volatile("v_mov_b32 %0, %1" : "=v"(i32[j]) : "v"(i32[(j + 3) & 7]));
      REP8(STEP)
#undef STEP
    }
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += d[j] + (double)f[j] + (double)i32[j] + (double)u64[j];
  if (s == 1.2345e300) out[threadIdx.x] = s;   // never true: keeps the chains alive
}

template <int OP>
float time_op(double* out, int blocks, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(BS), 0, 0, out, 3.0);   // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(BS), 0, 0, out, 3.0);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main() {
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  const double clk = 2.4e9;                    // nominal peak engine clock (MI355X)
  const int waves_per_simd = 8;
  const int blocks = cus * 4 * waves_per_simd / (BS / 64);
  double* out;
  CK(hipMalloc(&out, BS * sizeof(double)));
  const char* names[] = {"v_add_f32", "v_add_f64", "v_mul_f64", "v_fma_f64", "v_max_f64", "v_cvt_f64_i32",
                         "v_cvt_i32_f64", "v_rndne_f64", "v_add_u32", "v_mad_u64_u32", "v_mov_b64",
                         "v_cndmask_b32", "v_lshl_add_u64", "v_xor_b32", "v_add_u32_e64", "v_med3_i32", "v_add_f32_e64",
                         "v_mov_b32"};
  constexpr int NOPS = 18;
  float ms[NOPS];
  ms[0] = time_op<0>(out, blocks, 20);
  ms[1] = time_op<1>(out, blocks, 20);
  ms[2] = time_op<2>(out, blocks, 20);
  ms[3] = time_op<3>(out, blocks, 20);
  ms[4] = time_op<4>(out, blocks, 20);
  ms[5] = time_op<5>(out, blocks, 20);
  ms[6] = time_op<6>(out, blocks, 20);
  ms[7] = time_op<7>(out, blocks, 20);
  ms[8] = time_op<8>(out, blocks, 20);
  ms[9] = time_op<9>(out, blocks, 20);
  ms[10] = time_op<10>(out, blocks, 20);
  ms[11] = time_op<11>(out, blocks, 20);
  ms[12] = time_op<12>(out, blocks, 20);
  ms[13] = time_op<13>(out, blocks, 20);
  ms[14] = time_op<14>(out, blocks, 20);
  ms[15] = time_op<15>(out, blocks, 20);
  ms[16] = time_op<16>(out, blocks, 20);
  ms[17] = time_op<17>(out, blocks, 20);
  const double waves = (double)blocks * (BS / 64);
  const double instr = (double)ITERS * 64;   // per wave
  std::printf("{\"cus\": %d, \"waves_per_simd\": %d, \"instr_per_wave\": %.0f, \"clock_hz\": %.3g, \"ops\": {", cus,
              waves_per_simd, instr, clk);
  for (int k = 0; k < NOPS; ++k) {
    const double cyc = (ms[k] * 1e-3) * clk * (cus * 4.0) / (waves * instr);
    std::printf("%s\"%s\": {\"ms\": %.4f, \"simd_cycles_per_wave_instr\": %.3f}", k ? ", " : "", names[k], ms[k], cyc);
  }
  std::printf("}}\n");
  CK(hipFree(out));
  return 0;
}
