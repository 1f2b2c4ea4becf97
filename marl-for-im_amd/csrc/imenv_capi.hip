// imenv_capi.hip — host side of the C ABI in include/imenv.h: spec validation and derivation,
// buffer ownership, the reset / state-unpack kernels and step-kernel dispatch.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "imenv_device.h"
#include "imenv_jit.h"

using imenv::LaunchCfg;
using imenv::SpecDev;
using imenv::StepArgs;

namespace {

// ------------------------------------------------------------------ reset kernel
// Period-0 observation (IM_env.py:221-229): inv = init_inv, everything else 0 — the same
// [N][F] row for every env (host-built template), written with 16-B stores. It also clears the
// split-guard flags and advances the device-resident episode counter (the Philox counter word):
// set to `episode` if >= 0, else incremented, so a captured reset+steps graph draws fresh demand
// on every replay.
__global__ void __launch_bounds__(256) imenv_reset_kernel(const SpecDev* __restrict__ sp, void* obs, int obs_f64,
                                                          int64_t n, uint32_t* episode_word, int64_t episode,
                                                          uint32_t* err, uint32_t* err_any) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *episode_word = episode >= 0 ? (uint32_t)episode : *episode_word + 1u;
    *err_any = 0u;
  }
  const int row = sp->s.num_nodes * sp->s.num_features;
  const int64_t total = n * row;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t q = q0; q < n; q += stride) err[q] = 0u;
  // the template index q mod (row words) advances by stride mod (row words) per iteration: one 64-bit
  // division per thread instead of one per 16-byte store
  if (!obs_f64 && (row & 3) == 0) {
    const int r4 = row >> 2;
    float4* o4 = static_cast<float4*>(obs);
    const float4* tpl = reinterpret_cast<const float4*>(sp->reset_f32);
    int k = (int)(q0 % r4);
    const int ks = (int)(stride % r4);
    for (int64_t q = q0; q < total / 4; q += stride) {
      o4[q] = tpl[k];
      k += ks;
      if (k >= r4) k -= r4;
    }
  } else if (obs_f64 && (row & 1) == 0) {
    const int r2 = row >> 1;
    double2* o2 = static_cast<double2*>(obs);
    const double2* tpl = reinterpret_cast<const double2*>(sp->reset_f64);
    int k = (int)(q0 % r2);
    const int ks = (int)(stride % r2);
    for (int64_t q = q0; q < total / 2; q += stride) {
      o2[q] = tpl[k];
      k += ks;
      if (k >= r2) k -= r2;
    }
  } else {
    for (int64_t q = q0; q < total; q += stride) {
      if (obs_f64) static_cast<double*>(obs)[q] = sp->reset_f64[q % row];
      else static_cast<float*>(obs)[q] = sp->reset_f32[q % row];
    }
  }
}

// packed [n][np] state rows -> int32 [N][n] SoA (imenv_get_state): inventory and backlog are the
// positive and negative parts of the signed net row, order_u its own row; one pass over both rows
template <typename SN, typename ST>
__global__ void __launch_bounds__(256) imenv_state_kernel(const SN* __restrict__ net, const ST* __restrict__ ou,
                                                          int32_t* __restrict__ inv_out, int32_t* __restrict__ bl_out,
                                                          int32_t* __restrict__ ou_out, int64_t n, int np, int N) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  for (int i = 0; i < N; ++i) {
    const int32_t v = (int32_t)net[e * np + i];
    if (inv_out) inv_out[i * n + e] = max(v, 0);
    if (bl_out) bl_out[i * n + e] = max(-v, 0);
    if (ou_out) ou_out[i * n + e] = (int32_t)ou[e * np + i];
  }
}

// policy_stats of a base-stock rollout: one block per (policy, metric) merges the rollout kernel's
// per-block (sum, M2 about the block mean, count) triples with Chan et al.'s pairwise update
//   M2 = sum_b M2_b + sum_b n_b (mean_b - mean)^2,  mean = sum_b sum_b / S
// -> np.mean and np.std (population). Strided per-thread sums, wavefront shuffles and a fixed
// wave order through LDS: deterministic, the same bits for the same inputs.
__global__ void __launch_bounds__(256) imenv_rollout_stats_kernel(const double* __restrict__ partial,
                                                                  double* __restrict__ out, int64_t P, int64_t S,
                                                                  int64_t bpp) {
  __shared__ double s_w[4];
  const int64_t pol = blockIdx.x;
  const int m = blockIdx.y;
  const int tid = threadIdx.x;
  auto block_sum = [&](double v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((tid & 63) == 0) s_w[tid >> 6] = v;
    __syncthreads();
    const double r = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
    __syncthreads();
    return r;
  };
  const double* pb = partial + ((int64_t)m * P + pol) * bpp * 3;
  // unrolled so that 8 loads per thread are in flight (the sums stay in k order: same bits)
  double a = 0.0;
#pragma unroll 8
  for (int64_t k = tid; k < bpp; k += 256) a += pb[3 * k];
  const double mean = block_sum(a) / (double)S;
  double q = 0.0;
#pragma unroll 8
  for (int64_t k = tid; k < bpp; k += 256) {
    const double nb = pb[3 * k + 2];
    const double d = pb[3 * k] / nb - mean;
    q += pb[3 * k + 1] + nb * (d * d);
  }
  const double var = block_sum(q) / (double)S;
  if (tid == 0) {
    out[(pol * IMENV_NUM_STATS + m) * 2 + 0] = mean;
    out[(pol * IMENV_NUM_STATS + m) * 2 + 1] = sqrt(var);
  }
}

// np.mean / np.std (population) of every column of a row-major [rows][cols] float64 matrix, in the
// two-pass form np.std uses (the mean, then the mean of squared deviations). Each pass: a grid of
// row-chunk blocks x 64-column tiles writes one partial sum per (chunk, column); a finalize kernel adds
// the partials of each column in chunk order. Within a block, lane l of a wave reads column
// c0 + l % cw of row l / cw (cw = the tile's columns, 64 / cw rows per wave step), so a wave moves
// whole consecutive rows (512 B for 8 columns); lanes of one column and the 4 waves are combined
// through LDS in a fixed order. Deterministic: the same bits for the same input and grid.
template <bool SQ>
__global__ void __launch_bounds__(256) imenv_colsum_partial_kernel(const double* __restrict__ x, int64_t rows,
                                                                   int32_t cols, int64_t chunk,
                                                                   const double* __restrict__ mean_sd,
                                                                   double* __restrict__ part) {
  __shared__ double s_acc[256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c0 = blockIdx.y * 64;
  const int cw = (cols - c0) < 64 ? (cols - c0) : 64;
  const int rpw = 64 / cw;                        // rows per wave step
  const bool active = lane < rpw * cw;
  const int c = c0 + lane % cw;
  const int64_t r0 = (int64_t)blockIdx.x * chunk;
  const int64_t r1 = (r0 + chunk) < rows ? (r0 + chunk) : rows;
  const double mu = (SQ && active) ? mean_sd[2 * c] : 0.0;
  double acc = 0.0;
  if (active) {
    for (int64_t r = r0 + (int64_t)w * rpw + lane / cw; r < r1; r += 4 * rpw) {
      const double v = x[r * cols + c];
      if (SQ) {
        const double d = v - mu;
        acc += d * d;
      } else {
        acc += v;
      }
    }
  }
  s_acc[tid] = acc;
  __syncthreads();
  if (tid < cw) {
    double sum = 0.0;
    for (int q = 0; q < 4; ++q)
      for (int k = 0; k < rpw; ++k) sum += s_acc[q * 64 + k * cw + tid];
    part[(int64_t)blockIdx.x * cols + c0 + tid] = sum;
  }
}

// one block per column: strided per-thread sums of the chunk partials, then the waves' sums in a fixed
// order (the partials' loads are independent, so 256 threads keep them in flight)
template <bool SQ>
__global__ void __launch_bounds__(256) imenv_colsum_finalize_kernel(const double* __restrict__ part, int64_t nb,
                                                                    int64_t rows, int32_t cols,
                                                                    double* __restrict__ out) {
  __shared__ double s_w[4];
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  double v = 0.0;
  for (int64_t b = tid; b < nb; b += 256) v += part[b * cols + c];
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((tid & 63) == 0) s_w[tid >> 6] = v;
  __syncthreads();
  if (tid == 0) {
    const double sum = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
    if (SQ) out[2 * c + 1] = sqrt(sum / (double)rows);
    else out[2 * c] = sum / (double)rows;
  }
}

// Centralised-critic observations (models/CC_Model.py:196-214 central_critic_observer + :165-193
// FillInActions), flattened the way RLlib flattens the Dict space {own_obs, opponent_obs,
// opponent_action} for the value model (gym sorts Dict keys): per env e and agent m, a row of
// N*F + N - 1 values
//   [ clip(action[o], lo, hi) for o != m ][ obs[o][:] for o != m ][ obs[m][:] ]
// (o in agent order). One thread per output element: the writes are one contiguous stream, the
// reads gather from the env's own [N][F] obs row and [N] action row (cache-resident).
// np.clip (models/CC_Model.py:165-193; oracle/cc_obs.py:20): NaN passes through (fmin/fmax alone would turn it into lo)
__device__ __forceinline__ double np_clip(double x, double lo, double hi) {
  return x != x ? x : fmin(fmax(x, lo), hi);
}

template <typename OT, typename AT>
__global__ void __launch_bounds__(256) imenv_cc_obs_kernel(const OT* __restrict__ obs, const AT* __restrict__ act,
                                                           int64_t n, int N, int F, double lo, double hi,
                                                           OT* __restrict__ out) {
  const int Fcc = N * F + N - 1;
  const int64_t per_env = (int64_t)N * Fcc;
  const int64_t total = n * per_env;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += stride) {
    const int64_t e = q / per_env;
    const int r = (int)(q - e * per_env);
    const int m = r / Fcc;
    const int j = r - m * Fcc;
    OT v;
    if (j < N - 1) {                          // opponent_action
      const int o = j < m ? j : j + 1;
      v = act ? (OT)np_clip((double)act[e * N + o], lo, hi) : (OT)0;
    } else if (j < (N - 1) * (F + 1)) {       // opponent_obs
      const int k = j - (N - 1);
      const int oi = k / F;
      const int o = oi < m ? oi : oi + 1;
      v = obs[(e * N + o) * F + (k - oi * F)];
    } else {                                  // own_obs
      v = obs[(e * N + m) * F + (j - (N - 1) * (F + 1))];
    }
    out[q] = v;
  }
}

// The same rows, one thread per (env, agent) row: a block of E = 256 / N envs stages its obs [E][N][F]
// and clipped actions in LDS with coalesced loads, each thread assembles its row of N*F + N - 1 values
// in an LDS slab (odd row stride: no bank conflicts), and the block writes the slab, which is one
// contiguous run of the output, with 16-byte stores. Used when the slab fits 48 KiB.
template <typename OT, typename AT, int BS, bool NT = false>
__global__ void __launch_bounds__(BS) imenv_cc_obs_slab_kernel(const OT* __restrict__ obs, const AT* __restrict__ act,
                                                               int64_t n, int N, int F, double lo, double hi,
                                                               OT* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  const int W = N * F + N - 1;
  const int WP = W | 1;                               // odd stride
  const int E = BS / N;
  const int tid = threadIdx.x;
  const int64_t e0 = (int64_t)blockIdx.x * E;
  const int ne = (n - e0) < E ? (int)(n - e0) : E;
  double* s_act = reinterpret_cast<double*>(s_raw);                       // [E][N]
  OT* s_obs = reinterpret_cast<OT*>(s_act + E * N);                       // [E][N][F]
  OT* s_out = s_obs + E * N * F;                                          // [E * N][WP]
  for (int q = tid; q < ne * N * F; q += BS) s_obs[q] = obs[e0 * N * F + q];
  for (int q = tid; q < ne * N; q += BS)
    s_act[q] = act ? np_clip((double)act[e0 * N + q], lo, hi) : 0.0;
  __syncthreads();
  if (tid < ne * N) {
    const int el = tid / N, m = tid - el * N;
    OT* row = s_out + tid * WP;
    const OT* eo = s_obs + el * N * F;
    int k = 0;
    for (int o = 0; o < N; ++o)
      if (o != m) row[k++] = (OT)s_act[el * N + o];     // opponent_action
    for (int o = 0; o < N; ++o)
      if (o != m)
        for (int f = 0; f < F; ++f) row[k++] = eo[o * F + f];   // opponent_obs
    for (int f = 0; f < F; ++f) row[k++] = eo[m * F + f];      // own_obs
  }
  __syncthreads();
  const int total = ne * N * W;
  OT* g = out + e0 * N * W;
  constexpr int V = 16 / (int)sizeof(OT);            // values per 16-byte store
  const bool dense16 = WP == W && (reinterpret_cast<uintptr_t>(s_out) & 15) == 0;
  if (total % V == 0 && (reinterpret_cast<uintptr_t>(g) & 15) == 0) {
    for (int q = tid; q < total / V; q += BS) {
      OT v[V];
      if (dense16) {                                // 16-byte LDS read of the same values
        if constexpr (V == 4) {
          const float4 x = reinterpret_cast<const float4*>(s_out)[q];
          v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        } else {
          const double2 x = reinterpret_cast<const double2*>(s_out)[q];
          v[0] = x.x; v[1] = x.y;
        }
      } else {
#pragma unroll
        for (int u = 0; u < V; ++u) {
          const int i = q * V + u;
          v[u] = WP == W ? s_out[i] : s_out[(i / W) * WP + i % W];
        }
      }
      if constexpr (V == 4) imenv::store16<NT>(reinterpret_cast<float4*>(g) + q, make_float4(v[0], v[1], v[2], v[3]));
      else imenv::store16<NT>(reinterpret_cast<double2*>(g) + q, make_double2(v[0], v[1]));
    }
  } else {
    for (int i = tid; i < total; i += BS) g[i] = WP == W ? s_out[i] : s_out[(i / W) * WP + i % W];
  }
}

template <int BS, bool NT>
void launch_cc_slab(dim3 g, size_t lds, hipStream_t st, const void* obs, int obs_dtype, const void* actions,
                    int action_dtype, int64_t n, int N, int F, double lo, double hi, void* out) {
  const dim3 b(BS);
  if (obs_dtype == IMENV_F32 && action_dtype == IMENV_F32)
    hipLaunchKernelGGL((imenv_cc_obs_slab_kernel<float, float, BS, NT>), g, b, lds, st,
                       static_cast<const float*>(obs), static_cast<const float*>(actions), n, N, F, lo, hi,
                       static_cast<float*>(out));
  else if (obs_dtype == IMENV_F32)
    hipLaunchKernelGGL((imenv_cc_obs_slab_kernel<float, double, BS, NT>), g, b, lds, st,
                       static_cast<const float*>(obs), static_cast<const double*>(actions), n, N, F, lo, hi,
                       static_cast<float*>(out));
  else if (action_dtype == IMENV_F32)
    hipLaunchKernelGGL((imenv_cc_obs_slab_kernel<double, float, BS, NT>), g, b, lds, st,
                       static_cast<const double*>(obs), static_cast<const float*>(actions), n, N, F, lo, hi,
                       static_cast<double*>(out));
  else
    hipLaunchKernelGGL((imenv_cc_obs_slab_kernel<double, double, BS, NT>), g, b, lds, st,
                       static_cast<const double*>(obs), static_cast<const double*>(actions), n, N, F, lo, hi,
                       static_cast<double*>(out));
}

// GAE over a [T][n] rollout (RLlib 1.5 compute_advantages with use_gae, as called by
// models/CC_Policy.py:238-250; gamma / lambda from utils.py:19-23). One thread per env walks t from
// T-1 down to 0; each step reads one coalesced row of rewards and values per wave. Arithmetic is
// that of the reference path for a completed episode (last_r = 0.0 makes vpred_t float64):
//   delta_t = (r_t + gamma * v_{t+1}) - v_t                     float64 (float32 terms with a float32
//                                                               bootstrap value, see below)
//   adv_t   = c * adv_{t+1} + delta_t, c = gamma * lambda      float64 (scipy lfilter's
//             direct-form-II recursion of discount_cumsum; adv_{T-1} = 0.0 + delta_{T-1})
//   advantages = float32(adv_t), value_targets = float32(adv_t + v_t)
template <typename RT, typename VT, bool NT = false>
__global__ void __launch_bounds__(256) imenv_gae_kernel(const RT* __restrict__ rew, const VT* __restrict__ val,
                                                        const VT* __restrict__ last, int64_t n, int T, double gamma,
                                                        double c, float* __restrict__ adv_out,
                                                        float* __restrict__ vt_out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  // a float32 bootstrap value keeps vpred_t float32 in the reference (np.concatenate of float32
  // arrays), so gamma * v_{t+1} is a float32 product (NumPy casts the Python float to float32) and
  // the sum / difference take the wider of the operands' types; last_r = 0.0 makes it all float64
  const bool f32_path = sizeof(VT) == 4 && last != nullptr;
  const float gamma32 = (float)gamma;
  double vnext = last ? (double)last[e] : 0.0;
  double adv = 0.0;
  for (int t = T - 1; t >= 0; --t) {
    const double v = (double)val[(int64_t)t * n + e];
    const RT rr = rew[(int64_t)t * n + e];
    const double r = (double)rr;
    double delta;
    if (f32_path) {
      const float gv = gamma32 * (float)vnext;
      if (sizeof(RT) == 4) delta = (double)(((float)rr + gv) - (float)v);
      else delta = (r + (double)gv) - v;
    } else {
      delta = (r + gamma * vnext) - v;
    }
    adv = (t == T - 1) ? 0.0 + delta : c * adv + delta;
    if constexpr (NT) {
      __builtin_nontemporal_store((float)adv, adv_out + (int64_t)t * n + e);
      if (vt_out) __builtin_nontemporal_store((float)(adv + v), vt_out + (int64_t)t * n + e);
    } else {
      adv_out[(int64_t)t * n + e] = (float)adv;
      if (vt_out) vt_out[(int64_t)t * n + e] = (float)(adv + v);
    }
    vnext = v;
  }
}

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                                    \
  do {                                                                                               \
    hipError_t _e = (x);                                                                             \
    if (_e != hipSuccess) return fail(IMENV_E_HIP, std::string(#x ": ") + hipGetErrorString(_e));    \
  } while (0)

// Integer tuning switch from the environment, read on every call (a getenv is cheap next to a kernel
// launch, and a test that changes the variable between calls sees its new value). Unset or
// unparsable: dflt.
int env_switch(const char* name, int dflt) {
  int v = dflt;
  if (const char* e = std::getenv(name)) {
    char* end = nullptr;
    const long x = std::strtol(e, &end, 10);
    if (end && end != e) v = (int)x;
  }
  return v;
}

uint64_t prob_thr32(double p) {
  if (!(p > 0.0)) return 0;   // also NaN: the reference's `uniform() < nan` is never true
  double v = std::ceil(p * 4294967296.0);
  if (v < 0) v = 0;
  if (v > 4294967296.0) v = 4294967296.0;
  return (uint64_t)v;
}

// Host twin of obs_map: the same IEEE double expression, so table entries are bit-identical
// to what the device would compute (both built with -ffp-contract=off).
double host_obs_map(int mode, double v, double a, double bma, double den, double clip) {
  if (mode == IMENV_OBS_RAW) return v;
  if (mode == IMENV_OBS_SCALED) return a + (v * bma) / den;
  if (mode == IMENV_OBS_CLAMP_SCALED) return a + (std::fmin(v, clip) * bma) / den;
  return 0.0;
}

// Largest demand a node can see in one period: retailers are capped at inv_max
// (IM_env.py:306), other nodes receive at most the sum of their children's order_max.
int64_t demand_bound(const ImEnvSpec& s, int i) {
  if (s.retailer_slot[i] >= 0) return s.inv_max[i];
  int64_t b = 0;
  for (int c = 0; c < s.num_nodes; ++c)
    if (s.demand_parent[c] == i) b += s.order_max[c];
  return b;
}

// Observation lookup tables: for every scaled group and node, the exact value for each integer
// raw value the state can take (bounded by the capacities); values outside fall back to the
// in-kernel expression. Also the period-0 row shared by every env.
void build_obs_tables(SpecDev& d, std::vector<float>& l32, std::vector<double>& l64) {
  const ImEnvSpec& s = d.s;
  const int N = s.num_nodes;
  const double a = s.a, bma = s.b - s.a;
  l32.clear();
  l64.clear();
  for (int g = 0; g < IMENV_NUM_GROUPS; ++g) {
    for (int i = 0; i < IMENV_MAX_NODES; ++i) { d.lut_off[g][i] = 0; d.lut_max[g][i] = -1; }
    const int mode = s.group_mode[g];
    if (mode != IMENV_OBS_SCALED && mode != IMENV_OBS_CLAMP_SCALED) continue;
    for (int i = 0; i < N; ++i) {
      int64_t vmax = 0;
      switch (g) {
        case IMENV_G_INV: case IMENV_G_ORDER_U: vmax = s.inv_max[i]; break;
        case IMENV_G_BACKLOG: vmax = s.backlog_cap[i] >= 0 ? s.backlog_cap[i] : s.inv_max[i]; break;
        case IMENV_G_DEMAND_HIST: vmax = demand_bound(s, i); break;
        case IMENV_G_ORDER_HIST: vmax = s.order_max[i]; break;
        case IMENV_G_TRANSIT:
          vmax = mode == IMENV_OBS_CLAMP_SCALED ? (int64_t)std::fmin(s.group_clip[g][i], 4096.0)
                                                : (s.parent[i] >= 0 ? s.inv_max[s.parent[i]] : s.order_max[i]);
          break;
        case IMENV_G_NODE_ID: vmax = N; break;
        default: vmax = -1;
      }
      if (vmax > 4096) vmax = 4096;
      if (vmax < 0) continue;
      d.lut_off[g][i] = (int32_t)l64.size();
      d.lut_max[g][i] = (int32_t)vmax;
      for (int64_t v = 0; v <= vmax; ++v) {
        const double o = host_obs_map(mode, (double)v, a, bma, s.group_den[g][i], s.group_clip[g][i]);
        l64.push_back(o);
        l32.push_back((float)o);
      }
    }
  }
  const int F = s.num_features;
  for (int i = 0; i < N; ++i) {
    for (int f = 0; f < F; ++f) {
      const int g = s.feat_group[f];
      double v = 0.0;
      if (g == IMENV_G_INV) v = s.init_inv[i];
      else if (g == IMENV_G_NODE_ID) v = i;
      const double o = host_obs_map(s.group_mode[g], v, a, bma, s.group_den[g][i], s.group_clip[g][i]);
      d.reset_f64[i * F + f] = o;
      d.reset_f32[i * F + f] = (float)o;
    }
  }
}

// 1/x when x is a (signed) power of two, so that y / x == y * (1/x) exactly; else 0.
double exact_reciprocal(double x) {
  if (!(x != 0.0) || !std::isfinite(x)) return 0.0;
  int ex = 0;
  const double m = std::frexp(std::fabs(x), &ex);
  if (m != 0.5) return 0.0;
  return 1.0 / x;
}

// Upper bound of every value held in the packed state (inventory, backlog, unfulfilled orders,
// shipments in transit, demand / order history); all of them are >= 0. Backlog grows by at most one
// period's demand per period when uncapped; a shipment is at most backlog + demand, plus the split's
// overshoot of (children - 1) units (its inner loop does not re-check the remaining amount).
int64_t state_bound(const ImEnvSpec& s) {
  const int N = s.num_nodes;
  int64_t B = 0;
  auto upd = [&](int64_t v) { if (v > B) B = v; };
  for (int i = 0; i < N; ++i) {
    const int64_t dm = demand_bound(s, i);
    const int64_t blb = s.backlog_cap[i] >= 0 ? s.backlog_cap[i] : (int64_t)s.num_periods * dm;
    upd(s.inv_max[i]); upd(s.init_inv[i]); upd(blb); upd(dm); upd(s.order_max[i]);
    const int64_t shipb = blb + dm + IMENV_MAX_CHILDREN;
    upd(shipb);
  }
  return B;
}

// Largest magnitude of a split child's backlog_to (the reference's signed per-child backlog, IM_div_env.py
// :396-502): each period adds at most the child's order (<= order_max: A adds the unshipped part of it,
// C and D add order - ship_to with ship_to >= 0, B adds nothing), so backlog_to <= T x order_max. It goes
// below zero only in case C, where a backlog-first shipment s <= backlog_to is subtracted twice (drained,
// then order - ship_to with ship_to = s): the result is >= -backlog_to. Loops A and D decrement only
// positive counts. So |backlog_to| <= T x order_max of the child. (validate_and_derive inlines this.)

// Largest magnitude of the signed net-inventory row (inv - backlog): inventory up to its capacity or
// initial level, backlog up to its cap or T periods of demand.
int64_t net_bound(const ImEnvSpec& s) {
  int64_t B = 0;
  for (int i = 0; i < s.num_nodes; ++i) {
    const int64_t dm = demand_bound(s, i);
    const int64_t blb = s.backlog_cap[i] >= 0 ? s.backlog_cap[i] : (int64_t)s.num_periods * dm;
    B = std::max<int64_t>(B, std::max<int64_t>(blb, std::max<int64_t>(s.inv_max[i], s.init_inv[i])));
  }
  return B;
}

int validate_and_derive(const ImEnvSpec& s, SpecDev& d, int& maxc) {
  if (s.abi_version != IMENV_ABI_VERSION) return fail(IMENV_E_INVALID, "abi_version mismatch");
  const int N = s.num_nodes;
  if (N < 1 || N > IMENV_MAX_NODES) return fail(IMENV_E_INVALID, "num_nodes out of range");
  if (s.num_periods < 1 || s.num_periods > IMENV_MAX_PERIODS) return fail(IMENV_E_INVALID, "num_periods out of range");
  std::memset(&d, 0, sizeof(d));
  d.s = s;
  int roots = 0;
  d.factory = -1;
  d.dmax = 1;
  for (int i = 0; i < N; ++i) {
    if (s.parent[i] < 0) { ++roots; d.factory = i; }
    else if (s.parent[i] >= N || s.parent[i] == i) return fail(IMENV_E_INVALID, "bad parent index");
    if (s.delay[i] < 1)
      return fail(IMENV_E_UNSUPPORTED, "delay must be >= 1 in this build (delay 0 is a degenerate lead time)");
    if (s.delay[i] > IMENV_MAX_DELAY) return fail(IMENV_E_INVALID, "delay too large");
    if (s.delay[i] > d.dmax) d.dmax = s.delay[i];
    d.ring_off[i] = d.ring_total;
    d.ring_total += s.delay[i];
    if (s.inv_max[i] < 0 || s.order_max[i] < 0 || s.init_inv[i] < 0) return fail(IMENV_E_INVALID, "negative capacity");
    if (s.num_children[i] < 0 || s.num_children[i] > IMENV_MAX_CHILDREN)
      return fail(IMENV_E_UNSUPPORTED, "too many children");
  }
  if (roots != 1) return fail(IMENV_E_INVALID, "topology needs exactly one factory (parent = -1)");
  maxc = 0;
  d.num_split = 0;
  for (int i = 0; i < N; ++i) { d.split_child[i] = 0; d.single_parent[i] = -1; }
  for (int p = 0; p < N; ++p) {
    const int m = s.num_children[p];
    for (int k = 0; k < m; ++k) {
      const int c = s.children[p][k];
      if (c < 0 || c >= N || s.parent[c] != p) return fail(IMENV_E_INVALID, "children/parent mismatch");
    }
    if (m == 1) d.single_parent[s.children[p][0]] = p;
    if (m > 1) {
      d.split_node[d.num_split++] = p;
      if (m > maxc) maxc = m;
      for (int k = 0; k < m; ++k) d.split_child[s.children[p][k]] = 1;
    }
  }
  // compact backlog_to rows (imenv_device.h BtoRow): one slot per split child, in node order; int16 when
  // bto_bound fits it (IMENV_BTO_BYTES=4 forces int32: testing)
  d.num_bto = 0;
  for (int i = 0; i < IMENV_MAX_NODES; ++i) d.bto_slot[i] = -1;
  int64_t bto_om = 0;
  for (int i = 0; i < N; ++i)
    if (d.split_child[i]) {
      d.bto_slot[i] = d.num_bto++;
      bto_om = std::max<int64_t>(bto_om, s.order_max[i]);
    }
  d.bto_es = (int64_t)s.num_periods * bto_om <= 32767 ? 2 : 4;
  if (const char* v = std::getenv("IMENV_BTO_BYTES"))
    if (std::atoi(v) == 4) d.bto_es = 4;
  int nret = 0;
  for (int i = 0; i < N; ++i) {
    if (s.retailer_slot[i] >= 0) {
      ++nret;
      if (s.retailer_slot[i] >= s.num_retailers) return fail(IMENV_E_INVALID, "retailer_slot out of range");
    }
    if (s.demand_parent[i] >= N) return fail(IMENV_E_INVALID, "bad demand_parent");
  }
  if (nret != s.num_retailers || nret < 1) return fail(IMENV_E_INVALID, "retailer count mismatch");
  if (s.num_features < 1 || s.num_features > IMENV_MAX_FEATURES) return fail(IMENV_E_INVALID, "num_features out of range");
  if (s.prev_length < 1 || s.prev_length > IMENV_MAX_HIST) return fail(IMENV_E_INVALID, "prev_length out of range");
  for (int f = 0; f < s.num_features; ++f) {
    if (s.feat_group[f] < 0 || s.feat_group[f] >= IMENV_NUM_GROUPS) return fail(IMENV_E_INVALID, "bad feature group");
    if (s.feat_index[f] < 0) return fail(IMENV_E_INVALID, "bad feature index");
    if ((s.feat_group[f] == IMENV_G_DEMAND_HIST || s.feat_group[f] == IMENV_G_ORDER_HIST) &&
        s.feat_index[f] >= s.prev_length)
      return fail(IMENV_E_INVALID, "history feature index >= prev_length");
    if (s.feat_group[f] == IMENV_G_TRANSIT && s.feat_index[f] >= d.dmax)
      return fail(IMENV_E_INVALID, "transit feature index >= max delay");
  }
  for (int g = 0; g < IMENV_NUM_GROUPS; ++g)
    if (s.group_mode[g] < IMENV_OBS_ZERO || s.group_mode[g] > IMENV_OBS_CLAMP_SCALED)
      return fail(IMENV_E_INVALID, "bad group mode");
  if (s.decode_mode != IMENV_DECODE_CLIP_ROUND && s.decode_mode != IMENV_DECODE_ROUND_CLIP)
    return fail(IMENV_E_INVALID, "bad decode_mode");
  if (s.reward_mode < IMENV_REWARD_SUM || s.reward_mode > IMENV_REWARD_INDEPENDENT)
    return fail(IMENV_E_INVALID, "bad reward_mode");
  if (s.standardise_actions && !(s.b - s.a != 0.0)) return fail(IMENV_E_INVALID, "a == b");
  // the reference's numbers are finite (MAIM_env.py:166-168 asserts the price order, which no NaN
  // passes); a non-finite price / cost / scale would only turn rewards or observations into NaN
  if (!std::isfinite(s.a) || !std::isfinite(s.b)) return fail(IMENV_E_INVALID, "a and b must be finite");
  for (int i = 0; i < N; ++i) {
    if (!std::isfinite(s.sell_price[i]) || !std::isfinite(s.buy_price[i]) || !std::isfinite(s.stock_cost[i]) ||
        !std::isfinite(s.backlog_cost[i]) || !std::isfinite(s.inv_target[i]))
      return fail(IMENV_E_INVALID, "prices, costs and inventory targets must be finite");
    for (int q = 0; q < 4; ++q)
      // the closed-form round robin (rr_closed) counts rounds up to limit + 1 in int32; the reference's
      // guards are a few multiples of a node's demand bound, far below 2^30
      if (s.split_limit[i][q] < 0 || s.split_limit[i][q] > (1 << 30))
        return fail(IMENV_E_INVALID, "split guard limits must be in [0, 2^30]");
  }
  for (int g = 0; g < IMENV_NUM_GROUPS; ++g) {
    if (s.group_mode[g] != IMENV_OBS_SCALED && s.group_mode[g] != IMENV_OBS_CLAMP_SCALED) continue;
    for (int i = 0; i < N; ++i) {
      if (std::isnan(s.group_den[g][i])) return fail(IMENV_E_INVALID, "observation denominator is NaN");
      if (s.group_mode[g] == IMENV_OBS_CLAMP_SCALED && !(s.group_clip[g][i] >= 0.0 && std::isfinite(s.group_clip[g][i])))
        return fail(IMENV_E_INVALID, "observation clamp must be finite and >= 0");
    }
  }
  d.table_len = 0;
  if (s.demand_dist == IMENV_DEMAND_POISSON) {
    // thr[k] = ceil(CDF(k) * 2^32) by the pmf recurrence (oracle/philox.py:poisson_thresholds)
    const double mu = s.poisson_mu;
    if (!(mu > 0.0) || !std::isfinite(mu)) return fail(IMENV_E_INVALID, "Poisson mean must be positive and finite");
    double p = std::exp(-mu), cdf = 0.0;
    int k = 0;
    for (;;) {
      cdf += p;
      const double tv = std::ceil(cdf * 4294967296.0);
      if (tv >= 4294967296.0) break;
      if (!(tv >= 0.0)) return fail(IMENV_E_INVALID, "Poisson table: non-finite probability");
      if (k >= IMENV_TABLE_MAX) return fail(IMENV_E_UNSUPPORTED, "Poisson mean too large for the inversion table");
      d.table[k] = (uint32_t)tv;
      ++k;
      p = p * mu / (double)k;
    }
    d.table_len = k;
    // indexed-search guide (rollout_body's poisson_guided): count of thresholds <= g << (32 - bits)
    int c = 0;
    for (int g = 0; g < (1 << IMENV_GUIDE_BITS); ++g) {
      const uint64_t lo = (uint64_t)g << (32 - IMENV_GUIDE_BITS);
      while (c < k && (uint64_t)d.table[c] <= lo) ++c;
      d.guide[g] = (uint16_t)c;
    }
  } else if (s.demand_dist == IMENV_DEMAND_UNIFORM) {
    if (s.uniform_low >= s.uniform_high)
      return fail(IMENV_E_INVALID, "Lower bound cannot be larger than upper bound");
  } else if (s.demand_dist != IMENV_DEMAND_CUSTOM) {
    return fail(IMENV_E_INVALID, "Unrecognised, Distribution Not Implemented");
  }
  // narrowest element type the bounds allow; IMENV_STATE_BYTES=2|4 forces a wider one (testing)
  const int64_t bound = state_bound(s);
  d.vbound = (int32_t)std::min<int64_t>(std::max<int64_t>(bound, N), INT32_MAX);
  d.es = bound <= 255 ? 1 : (bound <= 32767 ? 2 : 4);
  if (d.es == 1 && net_bound(s) > 127) d.es = 2;   // the net row is signed (int8 beside uint8 rows)
  if (d.es == 1 && (int64_t)s.num_periods * bound > 32767) d.es = 2;   // int16 noisy-delay carry (CarryOf)
  if (const char* v = std::getenv("IMENV_STATE_BYTES")) {
    const int want = std::atoi(v);
    if ((want == 2 || want == 4) && want > d.es) d.es = want;
  }
  d.inv_bma = exact_reciprocal(s.b - s.a);
  d.inv_n = exact_reciprocal((double)N);
  d.np = d.es == 1 ? ((N + 3) & ~3) : (d.es == 2 ? ((N + 1) & ~1) : N);
  return IMENV_OK;
}

template <typename T>
int alloc(T** p, size_t count) {
  if (count == 0) { *p = nullptr; return IMENV_OK; }
  HIPCHK(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  return IMENV_OK;
}

// IMENV_STORE_DEFAULT: the state rows are written through as well when a launch's observation and
// reward bytes are at most 24 MiB (L2 is 8 XCDs x 4 MiB): then nearly every line a launch writes
// would still be dirty at its end and the dependent-launch boundary would write it back (+ bytes /
// 6 TB/s, MI355X_MICROARCH.md); larger launches evict their lines during the launch anyway, and there
// a state row written through (a 64-byte ring row per wave: partial lines) costs more than it saves.
// Measured (profiles/r03/store_sweep): state rows written through are 4-20% faster for C2 at 131,072 /
// 262,144 envs (7.3 / 14.7 MB of outputs) and C4 at 131,072 (13.6 MB), 2-9% slower for C2 at 2^19 /
// 2^20 (29 / 59 MB) and C3 at 262,144 (27 MB).
// IMENV_WT_STATE_MAX_BYTES overrides the 24 MiB limit (read once; tuning sweeps).
// at most two waves per SIMD (256 CUs x 4 SIMDs x 64 lanes x 2): the JIT step kernel then uses 64-env
// blocks (JitFlags::small_blocks, imenv_jit.hip jit_step_block_size)
constexpr int64_t kSmallLaunchEnvs = 2 * 64 * 4 * 256;

// State records (imenv_device.h: one 16- or 32-byte record per env holding the net and order_u rows and
// every ring slot) for launches of at most this many envs: one wave generation, where the launch is a
// latency chain and one 16-byte load and store per lane beats two row accesses plus one byte access per
// node (tools/probe_small.py: 3.79 vs 3.97 us for C2's access shape at 131,072 envs). Larger launches
// keep the rows: there the record's unused ring slots are extra bytes (104 vs 96 B per env-step for C2)
// for no gain. IMENV_REC=0 / 1 turns records off / on at any size; IMENV_REC_MAX_ENVS moves the limit.
int rec_bytes_for(const SpecDev& d, int64_t n) {
  const int N = d.s.num_nodes;
  const int need = 2 * d.np + d.ring_total;
  if (d.es != 1 || N > 8 || need > 32) return 0;
  int64_t lim = kSmallLaunchEnvs;
  if (const char* v = std::getenv("IMENV_REC_MAX_ENVS")) lim = std::atoll(v);
  if (const char* v = std::getenv("IMENV_REC")) lim = std::atoi(v) != 0 ? INT64_MAX : -1;
  if (n > lim) return 0;
  return need <= 16 ? 16 : 32;
}

// Drawn-demand table for launches of at most this many envs, where the step kernel is a latency chain
// and its demand draw (a Philox block on the episode word, then the inversion) sits on it: C2 at
// 131,072 envs 3.91 -> 3.40 us per launch without the draw (profiles/r05/ablate). A Philox block gives
// four periods, so the step at t % 4 == 0 draws all four and parks the next three in the table
// (imenv_device.h step_finish); the other three steps read one element per retailer. (Drawing the whole
// episode in the reset instead costs a VALU-bound kernel of 11-17 us per episode, more than the steps
// save; profiles/r05/dtab.) Measured in the graph-replayed window: C2 at 131,072 envs 3.97 -> 3.87 us
// per launch on average; C4 (two retailers: eight inversions at t % 4 == 0) 5.49 -> 5.99, so by default
// the table is for a single retailer only. The element is the narrowest integer holding every value a
// draw makes: [0, table_len] for Poisson, [low, high) for uniform, doubled when demand is noisy.
// IMENV_DTAB=0 / 1 turns it off / on at any size and retailer count; IMENV_DTAB_MAX_ENVS moves the limit.
int dtab_es_for(const SpecDev& d, int64_t n) {
  const ImEnvSpec& s = d.s;
  if (s.demand_dist != IMENV_DEMAND_POISSON && s.demand_dist != IMENV_DEMAND_UNIFORM) return 0;
  int64_t lim = s.num_retailers == 1 ? kSmallLaunchEnvs : -1;
  if (const char* v = std::getenv("IMENV_DTAB_MAX_ENVS")) lim = std::atoll(v);
  if (const char* v = std::getenv("IMENV_DTAB")) lim = std::atoi(v) != 0 ? INT64_MAX : -1;
  if (n > lim) return 0;
  int64_t lo = 0, hi = d.table_len;
  if (s.demand_dist == IMENV_DEMAND_UNIFORM) { lo = s.uniform_low; hi = s.uniform_high; }
  if (s.noisy_demand) { lo = std::min<int64_t>(std::min<int64_t>(lo, 2 * lo), 0); hi = std::max<int64_t>(hi, 2 * hi); }
  if (lo >= 0 && hi <= 255) return 1;
  if (lo >= -32768 && hi <= 32767) return 2;
  return 4;
}

bool jit_slim() {
  static const bool v = [] {
    const char* e = std::getenv("IMENV_JIT_SLIM");
    return !(e && std::atoi(e) == 0);
  }();
  return v;
}

int64_t wt_state_limit() {
  static const int64_t lim = [] {
    const char* v = std::getenv("IMENV_WT_STATE_MAX_BYTES");
    return v ? (int64_t)std::atoll(v) : (int64_t(24) << 20);
  }();
  return lim;
}
bool wt_state_pays(const ImEnvSpec& s, int64_t n, bool obs_f64) {
  const int64_t per_env = (int64_t)s.num_nodes * s.num_features * (obs_f64 ? 8 : 4) +
                          (s.reward_mode == IMENV_REWARD_INDEPENDENT ? 8 * s.num_nodes : 8);
  return n * per_env <= wt_state_limit();
}

bool is_base_obs(const ImEnvSpec& s) {
  return s.num_features == 3 && s.feat_group[0] == IMENV_G_INV && s.feat_group[1] == IMENV_G_BACKLOG &&
         s.feat_group[2] == IMENV_G_ORDER_U;
}

}  // namespace

// ==================================================================== handle
struct ImEnv {
  SpecDev host;        // host copy of the device spec
  SpecDev* d_spec = nullptr;
  int device = 0;
  int64_t n = 0;
  int64_t env_offset = 0;
  int maxc = 0;
  size_t es = 4;       // state element size (1, 2 or 4)
  void *d_net = nullptr, *d_ou = nullptr, *d_ring = nullptr, *d_hist_d = nullptr, *d_hist_o = nullptr;
  int32_t *d_carry = nullptr, *d_demand = nullptr;
  void* d_bto = nullptr;   // compact backlog_to rows [n][row_len(num_bto)] of bto_es bytes
  void* d_dtab = nullptr;  // the episode's drawn demand [T][R][n] of dtab_es bytes (dtab_es_for)
  double* d_delay_u = nullptr;
  float* d_lut32 = nullptr;
  double* d_lut64 = nullptr;
  std::vector<float> lut32;
  std::vector<double> lut64;
  uint32_t *d_err = nullptr, *d_err_any = nullptr;
  uint32_t* d_episode = nullptr;
  int t = 0;
  bool reset_done = false;
  bool noisy_delay = false;
  double noisy_thr = 0.0;
  bool have_delay_u = false;
  int demand_layout = IMENV_LAYOUT_DRAW;
  size_t demand_cap = 0;
  // kernel selection (imenv_set_jit): hipRTC-specialised kernels per JitFlags, else ahead-of-time
  int jit = 1;
  int store_policy = IMENV_STORE_DEFAULT;   // imenv_set_store_policy
  bool jit_strict = false;   // IMENV_JIT_STRICT=1: a JIT failure is an error instead of an AOT fallback
  std::string arch;
  std::unordered_map<uint32_t, imenv::JitKernel> jit_k;
  std::string jit_err;
  std::string last_kernel;   // the last AOT kernel's tag (a JIT launch names its kernel through last_jit)
  const imenv::JitKernel* last_jit = nullptr;   // entries of jit_k stay put (node-based map)
  uint32_t cached_key = 0xFFFFFFFFu;            // the previous call's JitFlags key and kernel: no lookup
  const imenv::JitKernel* cached_jit = nullptr; // when consecutive steps use the same flags
  // base-stock rollout: kernels per RolloutFlags, scratch for per-episode metrics and block sums
  std::unordered_map<uint32_t, imenv::JitKernel> roll_k;
  double* d_roll_part = nullptr;
  size_t roll_part_cap = 0;
  double* d_roll_terms = nullptr;   // parked objective terms of the single-pass tree rollout
  size_t roll_terms_cap = 0;
  std::string last_rollout;
  double* d_metrics = nullptr;   // caller-owned [n][4 + N] (imenv_set_episode_metrics)
  uint64_t* d_stamps = nullptr;  // diagnostics: per-wave phase stamps of IMENV_STAMPS kernel builds
  int64_t n_stamps = 0;
};

extern "C" {

int imenv_abi_version(void) { return IMENV_ABI_VERSION; }

int64_t imenv_spec_size(void) { return (int64_t)sizeof(ImEnvSpec); }

const char* imenv_last_error(void) { return g_err.c_str(); }

void imenv_destroy(ImEnv* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  void* ptrs[] = {h->d_spec, h->d_net, h->d_ou, h->d_ring, h->d_carry, h->d_bto, h->d_hist_d,
                  h->d_hist_o, h->d_demand, h->d_delay_u, h->d_err, h->d_err_any, h->d_lut32, h->d_lut64,
                  h->d_episode, h->d_roll_part, h->d_roll_terms, h->d_stamps, h->d_dtab};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (auto& kv : h->jit_k)
    if (kv.second.mod) (void)hipModuleUnload(kv.second.mod);
  for (auto& kv : h->roll_k)
    if (kv.second.mod) (void)hipModuleUnload(kv.second.mod);
  delete h;
}

int imenv_create(const ImEnvSpec* spec, int64_t n_envs, int64_t env_offset, int device, ImEnv** out) {
  if (!spec || !out) return fail(IMENV_E_INVALID, "null argument");
  *out = nullptr;
  if (n_envs < 1 || n_envs > (int64_t(1) << 31)) return fail(IMENV_E_INVALID, "n_envs out of range");
  if (env_offset < 0 || env_offset + n_envs > (int64_t(1) << 32)) return fail(IMENV_E_INVALID, "env ids must fit 32 bits");
  ImEnv* h = new ImEnv();
  int rc = validate_and_derive(*spec, h->host, h->maxc);
  if (rc != IMENV_OK) { delete h; return rc; }
  h->device = device;
  h->n = n_envs;
  h->env_offset = env_offset;
  h->noisy_delay = spec->noisy_delay != 0;
  h->noisy_thr = spec->noisy_delay_threshold;
  h->es = (size_t)h->host.es;
  const ImEnvSpec& s = *spec;
  const size_t n = n_envs, np = h->host.np, rowb = n * np * h->es;
  // history rows only when an observation reads an entry older than this step (feature index >= 1)
  bool uses_hist = false;
  for (int f = 0; f < s.num_features; ++f)
    if ((s.feat_group[f] == IMENV_G_DEMAND_HIST || s.feat_group[f] == IMENV_G_ORDER_HIST) && s.feat_index[f] >= 1)
      uses_hist = true;
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) { delete h; return fail(IMENV_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he)); }
  char **net = reinterpret_cast<char**>(&h->d_net), **ou = reinterpret_cast<char**>(&h->d_ou),
       **ring = reinterpret_cast<char**>(&h->d_ring), **bto = reinterpret_cast<char**>(&h->d_bto);
  const int nbt = h->host.num_bto;
  h->host.rec_bytes = rec_bytes_for(h->host, n_envs);
  h->host.dtab_es = dtab_es_for(h->host, n_envs);
  const bool rec = h->host.rec_bytes > 0;
  const size_t bto_row = (size_t)h->host.bto_es * (h->host.bto_es == 2 ? ((nbt + 1) & ~1) : nbt);
  if ((rc = alloc(&h->d_spec, 1)) || (rc = alloc(net, rec ? n * h->host.rec_bytes : rowb)) ||
      (rc = alloc(ou, rec ? 0 : rowb)) || (rc = alloc(ring, rec ? 0 : n * h->es * h->host.ring_total)) ||
      (rc = alloc(&h->d_carry, n * np)) ||
      (rc = alloc(bto, h->maxc > 0 ? n * bto_row : 0)) || (rc = alloc(&h->d_err, n)) ||
      (rc = alloc(&h->d_err_any, 1)) || (rc = alloc(&h->d_episode, 1)) ||
      (rc = alloc(reinterpret_cast<char**>(&h->d_dtab), n * s.num_periods * s.num_retailers * (size_t)h->host.dtab_es))) {
    imenv_destroy(h);
    return rc;
  }
  if (uses_hist) {
    char **hd = reinterpret_cast<char**>(&h->d_hist_d), **ho = reinterpret_cast<char**>(&h->d_hist_o);
    if ((rc = alloc(hd, rowb * s.prev_length)) || (rc = alloc(ho, rowb * s.prev_length))) {
      imenv_destroy(h);
      return rc;
    }
  }
  build_obs_tables(h->host, h->lut32, h->lut64);
  if ((rc = alloc(&h->d_lut32, h->lut32.size() + 1)) || (rc = alloc(&h->d_lut64, h->lut64.size() + 1))) {
    imenv_destroy(h);
    return rc;
  }
  he = hipMemcpy(h->d_spec, &h->host, sizeof(SpecDev), hipMemcpyHostToDevice);
  if (he == hipSuccess && !h->lut32.empty())
    he = hipMemcpy(h->d_lut32, h->lut32.data(), h->lut32.size() * sizeof(float), hipMemcpyHostToDevice);
  if (he == hipSuccess && !h->lut64.empty())
    he = hipMemcpy(h->d_lut64, h->lut64.data(), h->lut64.size() * sizeof(double), hipMemcpyHostToDevice);
  if (he == hipSuccess) he = hipMemset(h->d_err, 0, n * sizeof(uint32_t));
  if (he == hipSuccess) he = hipMemset(h->d_err_any, 0, sizeof(uint32_t));
  if (he == hipSuccess) he = hipMemset(h->d_episode, 0xFF, sizeof(uint32_t));   // first auto reset -> 0
  if (he != hipSuccess) { imenv_destroy(h); return fail(IMENV_E_HIP, std::string("init copy: ") + hipGetErrorString(he)); }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) h->arch = prop.gcnArchName;
  if (h->arch.empty()) h->jit = 0;
  if (const char* v = std::getenv("IMENV_JIT")) h->jit = (std::atoi(v) != 0 && !h->arch.empty()) ? 1 : 0;
  if (const char* v = std::getenv("IMENV_JIT_STRICT")) h->jit_strict = std::atoi(v) != 0;
  if (const char* v = std::getenv("IMENV_STAMPS")) {   // diagnostics (imenv_debug_stamps)
    if (std::atoi(v) != 0) {
      h->n_stamps = ((int64_t)n + 63) / 64 * 8 + 64 * 8;   // 8 per wave (+ a block's tail waves)
      if ((rc = alloc(&h->d_stamps, (size_t)h->n_stamps)) != IMENV_OK) { imenv_destroy(h); return rc; }
      (void)hipMemset(h->d_stamps, 0, (size_t)h->n_stamps * sizeof(uint64_t));
    }
  }
  *out = h;
  return IMENV_OK;
}

int imenv_reset(ImEnv* h, const int32_t* demand, int demand_layout, int noisy_delay, double noisy_delay_threshold,
                const double* delay_uniforms, int64_t episode, void* obs, int obs_dtype, void* stream) {
  if (!h || !obs) return fail(IMENV_E_INVALID, "null argument");
  if (obs_dtype != IMENV_F32 && obs_dtype != IMENV_F64) return fail(IMENV_E_INVALID, "bad obs dtype");
  const ImEnvSpec& s = h->host.s;
  hipStream_t st = static_cast<hipStream_t>(stream);
  HIPCHK(hipSetDevice(h->device));
  const size_t T = s.num_periods, R = s.num_retailers, n = h->n, N = s.num_nodes;
  if (demand_layout == IMENV_LAYOUT_DRAW) {
    if (demand) return fail(IMENV_E_INVALID, "IMENV_LAYOUT_DRAW takes no demand table");
    if (s.demand_dist != IMENV_DEMAND_POISSON && s.demand_dist != IMENV_DEMAND_UNIFORM)
      return fail(IMENV_E_INVALID, "custom demand needs a table (IMENV_LAYOUT_BROADCAST)");
  } else if (demand_layout == IMENV_LAYOUT_PER_ENV || demand_layout == IMENV_LAYOUT_BROADCAST) {
    if (!demand) return fail(IMENV_E_INVALID, "missing customer-demand table");
    const size_t cnt = (demand_layout == IMENV_LAYOUT_PER_ENV) ? T * R * n : T * R;
    if (h->demand_cap < cnt) {
      if (h->d_demand) { HIPCHK(hipStreamSynchronize(st)); HIPCHK(hipFree(h->d_demand)); h->d_demand = nullptr; }
      int rc = alloc(&h->d_demand, cnt);
      if (rc) return rc;
      h->demand_cap = cnt;
    }
    HIPCHK(hipMemcpyAsync(h->d_demand, demand, cnt * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
  } else {
    return fail(IMENV_E_INVALID, "bad demand_layout");
  }
  h->demand_layout = demand_layout;
  if (noisy_delay) {             // IM_env.py:180-182: latched until the env is rebuilt
    h->noisy_delay = true;
    h->noisy_thr = noisy_delay_threshold;
  }
  h->have_delay_u = false;
  if (delay_uniforms) {
    if (!h->d_delay_u) {
      int rc = alloc(&h->d_delay_u, T * N * n);
      if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(h->d_delay_u, delay_uniforms, T * N * n * sizeof(double), hipMemcpyDeviceToDevice, st));
    h->have_delay_u = true;
  }
  h->t = 0;
  h->reset_done = true;
  int64_t blocks = ((int64_t)n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(imenv_reset_kernel, dim3((unsigned)blocks), dim3(256), 0, st, h->d_spec, obs,
                     obs_dtype == IMENV_F64 ? 1 : 0, (int64_t)n, h->d_episode, episode, h->d_err, h->d_err_any);
  HIPCHK(hipGetLastError());
  return IMENV_OK;
}

int imenv_step(ImEnv* h, const void* actions, int action_dtype, void* obs, int obs_dtype, double* reward,
               const ImEnvInfo* info, int32_t* done_out, void* stream) {
  if (!h || !actions || !obs || !reward) return fail(IMENV_E_INVALID, "null argument");
  if (!h->reset_done) return fail(IMENV_E_NOT_RESET, "step() before reset()");
  const ImEnvSpec& s = h->host.s;
  if (h->t >= s.num_periods) return fail(IMENV_E_DONE, "step() past num_periods (episode is done; call reset)");
  if (action_dtype != IMENV_F32 && action_dtype != IMENV_F64) return fail(IMENV_E_INVALID, "bad action dtype");
  if (obs_dtype != IMENV_F32 && obs_dtype != IMENV_F64) return fail(IMENV_E_INVALID, "bad obs dtype");
  hipStream_t st = static_cast<hipStream_t>(stream);
  HIPCHK(hipSetDevice(h->device));
  StepArgs A;
  std::memset(&A, 0, sizeof(A));
  A.actions = actions;
  A.obs = obs;
  A.reward = reward;
  A.net = h->d_net; A.ou = h->d_ou;
  A.ring = h->d_ring; A.carry = h->d_carry; A.bto = h->d_bto;
  A.hist_d = h->d_hist_d; A.hist_o = h->d_hist_o;
  A.demand = h->d_demand;
  A.delay_u = h->have_delay_u ? h->d_delay_u : nullptr;
  A.err = h->d_err; A.err_any = h->d_err_any;
  if (info) {
    A.i_order = info->order; A.i_demand = info->demand; A.i_acq = info->acquisition; A.i_ship = info->ship;
    A.i_profit = info->profit; A.i_ship_to = info->ship_to; A.i_bto = info->backlog_to;
    if (!A.i_order && (A.i_demand || A.i_acq || A.i_ship || A.i_profit || A.i_ship_to || A.i_bto))
      return fail(IMENV_E_INVALID, "info.order is required when any other info field is requested");
  }
  A.lut32 = h->d_lut32;
  A.lut64 = h->d_lut64;
  A.episode = h->d_episode;
  A.dtab = (h->demand_layout == IMENV_LAYOUT_DRAW && h->host.dtab_es > 0) ? h->d_dtab : nullptr;
  A.metrics = h->d_metrics;
  A.stamps = h->d_stamps;
  A.n = h->n;
  A.env_offset = (uint32_t)h->env_offset;
  A.t = h->t;
  A.action_f64 = action_dtype == IMENV_F64;
  A.obs_f64 = obs_dtype == IMENV_F64;
  A.demand_layout = h->demand_layout;
  A.noisy_demand = (s.noisy_demand && h->demand_layout != IMENV_LAYOUT_PER_ENV) ? 1 : 0;
  A.noisy_delay = h->noisy_delay ? 1 : 0;
  A.noisy_delay_thr = h->noisy_thr;
  A.noisy_delay_thr32 = prob_thr32(h->noisy_thr);
  A.noisy_demand_thr32 = prob_thr32(s.noisy_demand_threshold);
  for (int i = 0; i < s.num_nodes; ++i)   // rows: element offset of the slot's row; records: the slot's byte
    A.ring_at[i] = h->host.rec_bytes ? (int64_t)(2 * h->host.np + h->host.ring_off[i] + h->t % s.delay[i])
                                     : (int64_t)(h->host.ring_off[i] + h->t % s.delay[i]) * h->n;
  LaunchCfg c;
  c.mc = h->maxc;
  c.base = is_base_obs(s);
  c.es = h->host.es;
  c.grid = (unsigned)((h->n + 255) / 256);
  c.stream = st;
  const int N = s.num_nodes;
  if (h->jit) {
    imenv::JitFlags f;
    f.act_f64 = A.action_f64 != 0;
    f.obs_f64 = A.obs_f64 != 0;
    f.noisy_delay = A.noisy_delay != 0;
    f.noisy_demand = A.noisy_demand != 0;
    f.has_delay_u = A.delay_u != nullptr;
    f.demand_layout = A.demand_layout;
    f.metrics = A.metrics != nullptr;
    f.stream_store = h->store_policy == IMENV_STORE_STREAM;
    f.wt_obs = h->store_policy == IMENV_STORE_DEFAULT || h->store_policy == IMENV_STORE_WRITETHROUGH;
    f.wt_state = h->store_policy == IMENV_STORE_WRITETHROUGH ||
                 (h->store_policy == IMENV_STORE_DEFAULT && wt_state_pays(s, h->n, A.obs_f64 != 0));
    f.small_blocks = h->n <= kSmallLaunchEnvs;
    // code only for what this call uses (IMENV_JIT_SLIM=0 keeps the general kernel): a kernel without the
    // info stores, and without tail-lane guards when every block is whole, is ~25% less code, which a
    // launch fetches into cold instruction caches
    const bool slim = jit_slim();
    f.info = !slim || A.i_order != nullptr;
    f.full = slim && h->n % 2048 == 0;
    // a 16-byte aligned observation buffer and whole blocks: every group's contiguous run (64 or BS envs
    // x the row) then starts on a 16-byte boundary and is a whole number of 16-byte words
    f.aligned = f.full && (reinterpret_cast<uintptr_t>(obs) & 15) == 0;
    const uint32_t key = f.key();
    if (key == h->cached_key && h->cached_jit && h->cached_jit->fn) {   // the per-step fast path
      HIPCHK(imenv::jit_launch(*h->cached_jit, st, h->d_spec, A));
      h->last_jit = h->cached_jit;
      h->t += 1;
      if (done_out) *done_out = h->t >= s.num_periods ? 1 : 0;
      return IMENV_OK;
    }
    auto it = h->jit_k.find(key);
    if (it == h->jit_k.end()) {
      // compiling + loading a module is not stream work: never do it while the stream is being
      // captured into a graph (that launch takes the ahead-of-time kernel instead)
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(st, &cs);
      if (cs == hipStreamCaptureStatusNone) {
        imenv::JitKernel k;
        std::string msg;
        if (imenv::jit_load(h->host, h->maxc, c.base, f, h->arch, k, msg)) {
          it = h->jit_k.emplace(f.key(), k).first;
        } else {
          h->jit_err = msg;
          if (h->jit_strict) return fail(IMENV_E_UNSUPPORTED, "JIT step kernel: " + msg);
          // recorded in imenv_kernel_info; the ahead-of-time kernels take over for THIS flag set only
          // (an empty entry: no retry per step), other flag sets of the handle keep their JIT kernels
          it = h->jit_k.emplace(f.key(), imenv::JitKernel{}).first;
        }
      }
    }
    if (it != h->jit_k.end() && it->second.fn) {
      HIPCHK(imenv::jit_launch(it->second, st, h->d_spec, A));
      h->last_jit = &it->second;
      h->cached_key = key;
      h->cached_jit = &it->second;
      h->t += 1;
      if (done_out) *done_out = h->t >= s.num_periods ? 1 : 0;
      return IMENV_OK;
    }
  }
  {
    char tag[96];
    std::snprintf(tag, sizeof tag, "aot:imenv_step_kernel[NT=%d,MC=%d,base=%d,es=%d]", N <= 8 ? N : 16, c.mc,
                  c.base ? 1 : 0, c.es);
    h->last_kernel = tag;
    h->last_jit = nullptr;
  }
  switch (N) {   // exact kernels for N <= 8, padded NT = 16 above
    case 1: imenv::launch_step_nt<1>(c, h->d_spec, A); break;
    case 2: imenv::launch_step_nt<2>(c, h->d_spec, A); break;
    case 3: imenv::launch_step_nt<3>(c, h->d_spec, A); break;
    case 4: imenv::launch_step_nt<4>(c, h->d_spec, A); break;
    case 5: imenv::launch_step_nt<5>(c, h->d_spec, A); break;
    case 6: imenv::launch_step_nt<6>(c, h->d_spec, A); break;
    case 7: imenv::launch_step_nt<7>(c, h->d_spec, A); break;
    case 8: imenv::launch_step_nt<8>(c, h->d_spec, A); break;
    default: imenv::launch_step_nt<16>(c, h->d_spec, A); break;
  }
  HIPCHK(hipGetLastError());
  h->t += 1;
  if (done_out) *done_out = h->t >= s.num_periods ? 1 : 0;
  return IMENV_OK;
}

static int launch_rollout(ImEnv* h, const imenv::RolloutFlags& f, imenv::RolloutArgs A, double* policy_stats,
                          hipStream_t st);

int imenv_base_stock_rollout(ImEnv* h, const ImEnvRollout* r, void* stream) {
  if (!h || !r || !r->policy) return fail(IMENV_E_INVALID, "null argument");
  const ImEnvSpec& s = h->host.s;
  if (s.reward_mode == IMENV_REWARD_INDEPENDENT)
    return fail(IMENV_E_UNSUPPORTED, "base-stock rollout needs a scalar reward (independent multi-agent rewards)");
  if (r->num_policies < 1 || r->num_scenarios < 1) return fail(IMENV_E_INVALID, "num_policies / num_scenarios < 1");
  if (r->scenario_offset < 0 || r->scenario_offset + r->num_scenarios > (int64_t(1) << 32))
    return fail(IMENV_E_INVALID, "scenario ids must fit 32 bits");
  if (r->episode < 0 || r->episode > 0xFFFFFFFFll) return fail(IMENV_E_INVALID, "episode must fit 32 bits");
  if (!r->demand && s.demand_dist != IMENV_DEMAND_POISSON && s.demand_dist != IMENV_DEMAND_UNIFORM)
    return fail(IMENV_E_INVALID, "custom demand needs a table");
  if (r->demand_pmf && (r->pmf_len < 1 || (int64_t)s.num_retailers * s.num_periods > 128))
    return fail(r->pmf_len < 1 ? IMENV_E_INVALID : IMENV_E_UNSUPPORTED,
                "objective: pmf_len >= 1 and num_retailers * num_periods <= 128 (np.sum without recursion)");
  if (h->arch.empty()) return fail(IMENV_E_UNSUPPORTED, "base-stock rollout needs hipRTC (device arch unknown)");
  hipStream_t st = static_cast<hipStream_t>(stream);
  HIPCHK(hipSetDevice(h->device));
  imenv::RolloutFlags f;
  f.table = r->demand != nullptr;
  f.noisy_delay = r->noisy_delay != 0;
  f.noisy_demand = !f.table && s.noisy_demand != 0;
  f.objective = r->demand_pmf != nullptr;
  imenv::RolloutArgs A;
  std::memset(&A, 0, sizeof(A));
  A.policy = r->policy;
  A.demand = r->demand;
  A.pmf = r->demand_pmf;
  A.pmf_len = r->demand_pmf ? r->pmf_len : 0;
  A.ep = r->episode_stats;
  A.S = r->num_scenarios;
  A.P = r->num_policies;
  A.scen_offset = (uint32_t)r->scenario_offset;
  A.episode = (uint32_t)r->episode;
  A.noisy_delay_thr32 = prob_thr32(r->noisy_delay_threshold);
  return launch_rollout(h, f, A, r->policy_stats, st);
}

int imenv_plan_rollout(ImEnv* h, const ImEnvPlanRollout* r, void* stream) {
  if (!h || !r || !r->actions) return fail(IMENV_E_INVALID, "null argument");
  const ImEnvSpec& s = h->host.s;
  if (s.reward_mode == IMENV_REWARD_INDEPENDENT)
    return fail(IMENV_E_UNSUPPORTED, "plan rollout needs a scalar reward (independent multi-agent rewards)");
  if (r->num_plans < 1 || r->num_scenarios < 1) return fail(IMENV_E_INVALID, "num_plans / num_scenarios < 1");
  // the inventory / backlog sums are sums of the raw state, which equal the LP scripts' sum(s[:, 0]) /
  // sum(s[:, 1]) only for raw observations (every LP script sets standardise_state False)
  if (s.group_mode[IMENV_G_INV] != IMENV_OBS_RAW || s.group_mode[IMENV_G_BACKLOG] != IMENV_OBS_RAW)
    return fail(IMENV_E_UNSUPPORTED, "plan rollout sums raw state: needs standardise_state False (raw observations)");
  if (r->action_dtype != IMENV_F32 && r->action_dtype != IMENV_F64)
    return fail(IMENV_E_INVALID, "action_dtype must be IMENV_F32 or IMENV_F64");
  if (r->plan_layout != IMENV_PLAN_SHARED && r->plan_layout != IMENV_PLAN_PER_EPISODE)
    return fail(IMENV_E_INVALID, "plan_layout must be IMENV_PLAN_SHARED or IMENV_PLAN_PER_EPISODE");
  if (r->scenario_offset < 0 || r->scenario_offset + r->num_scenarios > (int64_t(1) << 32))
    return fail(IMENV_E_INVALID, "scenario ids must fit 32 bits");
  if (r->episode < 0 || r->episode > 0xFFFFFFFFll) return fail(IMENV_E_INVALID, "episode must fit 32 bits");
  if (!r->demand && s.demand_dist != IMENV_DEMAND_POISSON && s.demand_dist != IMENV_DEMAND_UNIFORM)
    return fail(IMENV_E_INVALID, "custom demand needs a table");
  if (h->arch.empty()) return fail(IMENV_E_UNSUPPORTED, "plan rollout needs hipRTC (device arch unknown)");
  {
    // per-episode rows are loaded as whole 16 / 8-byte words (load_words), shared rows element-wise
    const size_t row = (r->action_dtype == IMENV_F64 ? 8 : 4) * (size_t)s.num_nodes;
    const size_t align = r->plan_layout == IMENV_PLAN_SHARED ? (r->action_dtype == IMENV_F64 ? 8 : 4)
                         : row % 16 == 0 ? 16 : row % 8 == 0 ? 8 : 4;
    if (reinterpret_cast<uintptr_t>(r->actions) % align)
      return fail(IMENV_E_INVALID, "plan actions must be aligned to " + std::to_string(align) + " bytes");
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  HIPCHK(hipSetDevice(h->device));
  imenv::RolloutFlags f;
  f.table = r->demand != nullptr;
  f.noisy_delay = r->noisy_delay != 0;
  f.noisy_demand = !f.table && s.noisy_demand != 0;
  f.act = r->plan_layout == IMENV_PLAN_SHARED ? imenv::ROLL_PLAN_SHARED : imenv::ROLL_PLAN_EPISODE;
  f.act_f64 = r->action_dtype == IMENV_F64;
  imenv::RolloutArgs A;
  std::memset(&A, 0, sizeof(A));
  A.plan = r->actions;
  A.rewards = r->rewards;
  A.demand = r->demand;
  A.ep = r->episode_stats;
  A.S = r->num_scenarios;
  A.P = r->num_plans;
  A.scen_offset = (uint32_t)r->scenario_offset;
  A.episode = (uint32_t)r->episode;
  A.noisy_delay_thr32 = prob_thr32(r->noisy_delay_threshold);
  return launch_rollout(h, f, A, r->policy_stats, st);
}

// The fused rollout launch shared by the base-stock and plan rollouts: kernel lookup (compiled once per
// flag set), per-block partials and parked-term scratch, the rollout kernel, then the stats merge.
static int launch_rollout(ImEnv* h, const imenv::RolloutFlags& f, imenv::RolloutArgs A, double* policy_stats,
                          hipStream_t st) {
  const ImEnvSpec& s = h->host.s;
  auto it = h->roll_k.find(f.key());
  if (it == h->roll_k.end()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone)
      return fail(IMENV_E_UNSUPPORTED, "first rollout of a flag combination cannot be captured (it compiles)");
    imenv::JitKernel k;
    std::string msg;
    if (!imenv::jit_rollout_load(h->host, h->maxc, f, h->arch, k, msg))
      return fail(IMENV_E_UNSUPPORTED, "rollout kernel: " + msg);
    it = h->roll_k.emplace(f.key(), k).first;
  }
  const imenv::JitKernel& k = it->second;
  const int64_t P = A.P, S = A.S;
  const int64_t bpp = (S + k.bs - 1) / k.bs;
  if (P * bpp > 0x7FFFFFFFll) return fail(IMENV_E_INVALID, "num_policies * ceil(num_scenarios / block) too large");
  const size_t pneed = (size_t)IMENV_NUM_STATS * P * bpp * 3;
  if (h->roll_part_cap < pneed) {
    if (h->d_roll_part) { HIPCHK(hipStreamSynchronize(st)); HIPCHK(hipFree(h->d_roll_part)); h->d_roll_part = nullptr; }
    int rc = alloc(&h->d_roll_part, pneed);
    if (rc) return rc;
    h->roll_part_cap = pneed;
  }
  const size_t tneed = (size_t)imenv::rollout_term_slots(h->host, f) * P * bpp * k.bs;
  if (h->roll_terms_cap < tneed) {
    if (h->d_roll_terms) { HIPCHK(hipStreamSynchronize(st)); HIPCHK(hipFree(h->d_roll_terms)); h->d_roll_terms = nullptr; }
    int rc = alloc(&h->d_roll_terms, tneed);
    if (rc) return rc;
    h->roll_terms_cap = tneed;
  }
  A.terms = h->d_roll_terms;
  A.partial = h->d_roll_part;
  A.bpp = bpp;
  A.noisy_delay = f.noisy_delay ? 1 : 0;
  A.noisy_demand = f.noisy_demand ? 1 : 0;
  A.noisy_demand_thr32 = prob_thr32(s.noisy_demand_threshold);
  HIPCHK(imenv::jit_rollout_launch(k, st, h->d_spec, A));
  h->last_rollout = k.tag;
  if (policy_stats) {
    hipLaunchKernelGGL(imenv_rollout_stats_kernel, dim3((unsigned)P, IMENV_NUM_STATS), dim3(256), 0, st,
                       h->d_roll_part, policy_stats, P, S, bpp);
    HIPCHK(hipGetLastError());
  }
  return IMENV_OK;
}

int imenv_set_episode_metrics(ImEnv* h, double* acc) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  h->d_metrics = acc;
  return IMENV_OK;
}

int imenv_column_stats(const double* x, int64_t rows, int32_t cols, double* out, void* stream) {
  if (!x || !out) return fail(IMENV_E_INVALID, "null argument");
  if (rows < 1 || cols < 1 || cols > 65535) return fail(IMENV_E_INVALID, "rows >= 1 and 1 <= cols <= 65535");
  hipStream_t st = static_cast<hipStream_t>(stream);
  // row chunks: up to 1024 blocks per column tile, at most 2^20 partials, at least 256 rows per chunk
  int64_t nb = std::min<int64_t>(1024, std::max<int64_t>(1, (int64_t(1) << 20) / cols));
  nb = std::min<int64_t>(nb, (rows + 255) / 256);
  const int64_t chunk = (rows + nb - 1) / nb;
  nb = (rows + chunk - 1) / chunk;
  double* part = nullptr;   // stream-ordered scratch (capturable), returned to the pool after the last use
  HIPCHK(hipMallocAsync(reinterpret_cast<void**>(&part), (size_t)nb * cols * sizeof(double), st));
  const dim3 g((unsigned)nb, (unsigned)((cols + 63) / 64)), b(256);
  const dim3 gf((unsigned)cols), bf(256);
  hipLaunchKernelGGL(imenv_colsum_partial_kernel<false>, g, b, 0, st, x, rows, cols, chunk, out, part);
  hipLaunchKernelGGL(imenv_colsum_finalize_kernel<false>, gf, bf, 0, st, part, nb, rows, cols, out);
  hipLaunchKernelGGL(imenv_colsum_partial_kernel<true>, g, b, 0, st, x, rows, cols, chunk, out, part);
  hipLaunchKernelGGL(imenv_colsum_finalize_kernel<true>, gf, bf, 0, st, part, nb, rows, cols, out);
  const hipError_t e = hipGetLastError();
  (void)hipFreeAsync(part, st);
  if (e != hipSuccess) return fail(IMENV_E_HIP, std::string("column stats: ") + hipGetErrorString(e));
  return IMENV_OK;
}

int imenv_cc_observation(int64_t n, int32_t num_agents, int32_t num_features, const void* obs, int obs_dtype,
                         const void* actions, int action_dtype, double clip_lo, double clip_hi, void* out,
                         void* stream) {
  if (!obs || !out) return fail(IMENV_E_INVALID, "null argument");
  if (n < 1 || num_agents < 2 || num_features < 1) return fail(IMENV_E_INVALID, "n >= 1, num_agents >= 2, F >= 1");
  if ((obs_dtype != IMENV_F32 && obs_dtype != IMENV_F64) || (action_dtype != IMENV_F32 && action_dtype != IMENV_F64))
    return fail(IMENV_E_INVALID, "bad dtype");
  hipStream_t st = static_cast<hipStream_t>(stream);
  {
    // staged (env, agent)-row kernel when the block's slab fits 48 KiB
    const int BSC = env_switch("IMENV_CC_BS", 256) == 512 ? 512 : 256;   // 512-thread blocks (tuning)
    const int N = num_agents, F = num_features, W = N * F + N - 1, E = BSC / N;
    const size_t osz = obs_dtype == IMENV_F64 ? 8 : 4;
    const size_t lds = (size_t)E * N * 8 + (size_t)E * N * F * osz + (size_t)E * N * (W | 1) * osz;
    if (N <= 256 && lds <= 48 * 1024) {
      const dim3 g((unsigned)((n + E - 1) / E)), b(BSC);
      // non-temporal row stores (default; IMENV_CC_NT=0 turns them off): the rows are read back only by
      // a later training pass, and streamed past the caches the kernel runs at 76% of HBM peak instead
      // of 54% (tools/bench_kernels.py, 2^20 envs, profiles/r02/kernels_cc_nt.log)
      const bool nt = env_switch("IMENV_CC_NT", 1) != 0;
      if (BSC == 512 && nt)
        launch_cc_slab<512, true>(g, lds, st, obs, obs_dtype, actions, action_dtype, n, N, F, clip_lo, clip_hi, out);
      else if (BSC == 512)
        launch_cc_slab<512, false>(g, lds, st, obs, obs_dtype, actions, action_dtype, n, N, F, clip_lo, clip_hi, out);
      else if (nt)
        launch_cc_slab<256, true>(g, lds, st, obs, obs_dtype, actions, action_dtype, n, N, F, clip_lo, clip_hi, out);
      else
        launch_cc_slab<256, false>(g, lds, st, obs, obs_dtype, actions, action_dtype, n, N, F, clip_lo, clip_hi, out);
      HIPCHK(hipGetLastError());
      return IMENV_OK;
    }
  }
  const int64_t total = n * num_agents * (int64_t)(num_agents * num_features + num_agents - 1);
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  const dim3 g((unsigned)blocks), b(256);
  if (obs_dtype == IMENV_F32 && action_dtype == IMENV_F32)
    hipLaunchKernelGGL((imenv_cc_obs_kernel<float, float>), g, b, 0, st, static_cast<const float*>(obs),
                       static_cast<const float*>(actions), n, num_agents, num_features, clip_lo, clip_hi,
                       static_cast<float*>(out));
  else if (obs_dtype == IMENV_F32)
    hipLaunchKernelGGL((imenv_cc_obs_kernel<float, double>), g, b, 0, st, static_cast<const float*>(obs),
                       static_cast<const double*>(actions), n, num_agents, num_features, clip_lo, clip_hi,
                       static_cast<float*>(out));
  else if (action_dtype == IMENV_F32)
    hipLaunchKernelGGL((imenv_cc_obs_kernel<double, float>), g, b, 0, st, static_cast<const double*>(obs),
                       static_cast<const float*>(actions), n, num_agents, num_features, clip_lo, clip_hi,
                       static_cast<double*>(out));
  else
    hipLaunchKernelGGL((imenv_cc_obs_kernel<double, double>), g, b, 0, st, static_cast<const double*>(obs),
                       static_cast<const double*>(actions), n, num_agents, num_features, clip_lo, clip_hi,
                       static_cast<double*>(out));
  HIPCHK(hipGetLastError());
  return IMENV_OK;
}

int imenv_gae(int64_t n, int32_t T, const void* rewards, int reward_dtype, const void* values, int value_dtype,
              const void* last_value, double gamma, double lambda, float* advantages, float* value_targets,
              void* stream) {
  if (!rewards || !values || !advantages) return fail(IMENV_E_INVALID, "null argument");
  if (n < 1 || T < 1) return fail(IMENV_E_INVALID, "n >= 1 and T >= 1");
  if ((reward_dtype != IMENV_F32 && reward_dtype != IMENV_F64) || (value_dtype != IMENV_F32 && value_dtype != IMENV_F64))
    return fail(IMENV_E_INVALID, "bad dtype");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  const double c = gamma * lambda;
  // non-temporal advantage / value-target stores (default; IMENV_GAE_NT=0 turns them off): they are
  // read by the loss pass after the whole batch, and streamed the kernel takes 109 us instead of
  // 113-116 us for 2^20 envs x 30 periods (profiles/r02/kernels_gae_nt.log)
  const bool nt = env_switch("IMENV_GAE_NT", 1) != 0;
  auto launch = [&](auto nt_tag) {
    constexpr bool NTS = decltype(nt_tag)::value;
    if (reward_dtype == IMENV_F32 && value_dtype == IMENV_F32)
      hipLaunchKernelGGL((imenv_gae_kernel<float, float, NTS>), g, b, 0, st, static_cast<const float*>(rewards),
                         static_cast<const float*>(values), static_cast<const float*>(last_value), n, T, gamma, c,
                         advantages, value_targets);
    else if (reward_dtype == IMENV_F64 && value_dtype == IMENV_F32)
      hipLaunchKernelGGL((imenv_gae_kernel<double, float, NTS>), g, b, 0, st, static_cast<const double*>(rewards),
                         static_cast<const float*>(values), static_cast<const float*>(last_value), n, T, gamma, c,
                         advantages, value_targets);
    else if (reward_dtype == IMENV_F32)
      hipLaunchKernelGGL((imenv_gae_kernel<float, double, NTS>), g, b, 0, st, static_cast<const float*>(rewards),
                         static_cast<const double*>(values), static_cast<const double*>(last_value), n, T, gamma, c,
                         advantages, value_targets);
    else
      hipLaunchKernelGGL((imenv_gae_kernel<double, double, NTS>), g, b, 0, st, static_cast<const double*>(rewards),
                         static_cast<const double*>(values), static_cast<const double*>(last_value), n, T, gamma, c,
                         advantages, value_targets);
  };
  if (nt) launch(std::true_type{});
  else launch(std::false_type{});
  HIPCHK(hipGetLastError());
  return IMENV_OK;
}

int imenv_get_state(ImEnv* h, int32_t* inv, int32_t* backlog, int32_t* order_u, int32_t* period, void* stream) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  const ImEnvSpec& s = h->host.s;
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t bytes = (size_t)s.num_nodes * h->n * sizeof(int32_t);
  if (h->t == 0) {
    // period-0 state is implicit in the step kernel; materialise it for the caller
    if (inv) {
      std::vector<int32_t> tmp((size_t)s.num_nodes * h->n);
      for (int i = 0; i < s.num_nodes; ++i)
        for (int64_t e = 0; e < h->n; ++e) tmp[(size_t)i * h->n + e] = s.init_inv[i];
      HIPCHK(hipMemcpyAsync(inv, tmp.data(), bytes, hipMemcpyHostToDevice, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    if (backlog) HIPCHK(hipMemsetAsync(backlog, 0, bytes, st));
    if (order_u) HIPCHK(hipMemsetAsync(order_u, 0, bytes, st));
  } else {
    const unsigned grid = (unsigned)((h->n + 255) / 256);
    // inventory and backlog are the two sides of the signed net row (imenv_device.h, NetOf)
    if (h->host.rec_bytes)   // state records: net row at byte 0, order_u row at byte np, record stride
      hipLaunchKernelGGL((imenv_state_kernel<int8_t, uint8_t>), dim3(grid), dim3(256), 0, st,
                         static_cast<const int8_t*>(h->d_net), static_cast<const uint8_t*>(h->d_net) + h->host.np,
                         inv, backlog, order_u, h->n, h->host.rec_bytes, s.num_nodes);
    else if (h->host.es == 1)
      hipLaunchKernelGGL((imenv_state_kernel<int8_t, uint8_t>), dim3(grid), dim3(256), 0, st,
                         static_cast<const int8_t*>(h->d_net), static_cast<const uint8_t*>(h->d_ou), inv, backlog,
                         order_u, h->n, h->host.np, s.num_nodes);
    else if (h->host.es == 2)
      hipLaunchKernelGGL((imenv_state_kernel<int16_t, int16_t>), dim3(grid), dim3(256), 0, st,
                         static_cast<const int16_t*>(h->d_net), static_cast<const int16_t*>(h->d_ou), inv, backlog,
                         order_u, h->n, h->host.np, s.num_nodes);
    else
      hipLaunchKernelGGL((imenv_state_kernel<int32_t, int32_t>), dim3(grid), dim3(256), 0, st,
                         static_cast<const int32_t*>(h->d_net), static_cast<const int32_t*>(h->d_ou), inv, backlog,
                         order_u, h->n, h->host.np, s.num_nodes);
    HIPCHK(hipGetLastError());
  }
  if (period) *period = h->t;
  return IMENV_OK;
}

int imenv_get_errors(ImEnv* h, uint32_t* flags, uint32_t* any_out, void* stream) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (flags) HIPCHK(hipMemcpyAsync(flags, h->d_err, h->n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
  if (any_out) {
    uint32_t v = 0;
    HIPCHK(hipMemcpyAsync(&v, h->d_err_any, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *any_out = v;
  }
  return IMENV_OK;
}

int imenv_dims(const ImEnv* h, int32_t* num_nodes, int32_t* num_features, int32_t* num_retailers,
               int32_t* num_periods) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  const ImEnvSpec& s = h->host.s;
  if (num_nodes) *num_nodes = s.num_nodes;
  if (num_features) *num_features = s.num_features;
  if (num_retailers) *num_retailers = s.num_retailers;
  if (num_periods) *num_periods = s.num_periods;
  return IMENV_OK;
}

int imenv_poisson_table(const ImEnv* h, uint32_t* out, int32_t cap, int32_t* len_out) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  if (len_out) *len_out = h->host.table_len;
  if (out) {
    const int m = cap < h->host.table_len ? cap : h->host.table_len;
    for (int k = 0; k < m; ++k) out[k] = h->host.table[k];
  }
  return IMENV_OK;
}

int imenv_state_layout(const ImEnv* h, int32_t* elem_bytes, int32_t* row_len, int32_t* ring_depth) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  if (elem_bytes) *elem_bytes = (int32_t)h->es;
  if (row_len) *row_len = h->host.np;
  if (ring_depth) *ring_depth = h->host.ring_total;
  return IMENV_OK;
}

int imenv_draw_layout(const ImEnv* h, int32_t* elem_bytes) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  if (elem_bytes) *elem_bytes = h->host.dtab_es;
  return IMENV_OK;
}

int imenv_split_layout(const ImEnv* h, int32_t* num_split_children, int32_t* elem_bytes) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  if (num_split_children) *num_split_children = h->maxc > 0 ? h->host.num_bto : 0;
  if (elem_bytes) *elem_bytes = h->host.bto_es;
  return IMENV_OK;
}

int imenv_set_delay_uniforms(ImEnv* h, int32_t period, const double* u, void* stream) {
  if (!h || !u) return fail(IMENV_E_INVALID, "null argument");
  if (!h->reset_done) return fail(IMENV_E_NOT_RESET, "set_delay_uniforms() before reset()");
  const ImEnvSpec& s = h->host.s;
  if (period < h->t || period >= s.num_periods)
    return fail(IMENV_E_INVALID, "period must lie in [current period, num_periods)");
  hipStream_t st = static_cast<hipStream_t>(stream);
  HIPCHK(hipSetDevice(h->device));
  const size_t T = s.num_periods, N = s.num_nodes, n = h->n;
  if (!h->d_delay_u) {
    int rc = alloc(&h->d_delay_u, T * N * n);
    if (rc) return rc;
  }
  if (!h->have_delay_u) {   // rows not written by the caller read as 1.0 (no extra delay unless thr >= 1)
    std::vector<double> ones(T * N * n, 1.0);
    HIPCHK(hipMemcpyAsync(h->d_delay_u, ones.data(), ones.size() * sizeof(double), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    h->have_delay_u = true;
  }
  HIPCHK(hipMemcpyAsync(h->d_delay_u + (size_t)period * N * n, u, N * n * sizeof(double), hipMemcpyDeviceToDevice,
                        st));
  return IMENV_OK;
}

int imenv_set_store_policy(ImEnv* h, int policy) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  if (policy < IMENV_STORE_DEFAULT || policy > IMENV_STORE_WRITETHROUGH)
    return fail(IMENV_E_INVALID, "policy must be one of IMENV_STORE_DEFAULT / STREAM / PLAIN / WRITETHROUGH");
  h->store_policy = policy;
  return IMENV_OK;
}

int imenv_set_jit(ImEnv* h, int mode) {
  if (!h) return fail(IMENV_E_INVALID, "null handle");
  if (mode != 0 && mode != 1) return fail(IMENV_E_INVALID, "mode must be 0 (ahead-of-time) or 1 (hipRTC)");
  if (mode == 1 && h->arch.empty()) return fail(IMENV_E_UNSUPPORTED, "device architecture unknown");
  h->jit = mode;
  if (mode == 1) {   // retry flag sets whose compile failed
    h->jit_err.clear();
    for (auto it = h->jit_k.begin(); it != h->jit_k.end();) it = it->second.fn ? std::next(it) : h->jit_k.erase(it);
  }
  return IMENV_OK;
}

int imenv_kernel_info(const ImEnv* h, char* buf, int64_t len) {
  if (!h || !buf || len < 1) return fail(IMENV_E_INVALID, "null argument");
  std::string s = h->last_jit ? h->last_jit->tag
                 : h->last_kernel.empty() ? std::string(h->jit ? "jit (no step yet)" : "aot (no step yet)")
                                          : h->last_kernel;
  if (!h->jit_err.empty()) s += " | jit failed: " + h->jit_err;
  if (!h->last_rollout.empty()) s += " | rollout " + h->last_rollout;
  std::snprintf(buf, (size_t)len, "%s", s.c_str());
  return IMENV_OK;
}

int imenv_debug_stamps(ImEnv* h, uint64_t* out, int64_t cap, int64_t* count) {
  if (!h || !count) return fail(IMENV_E_INVALID, "null argument");
  *count = h->n_stamps;
  if (!h->d_stamps || !out || cap <= 0) return IMENV_OK;
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, h->d_stamps, (size_t)std::min(cap, h->n_stamps) * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return IMENV_OK;
}

int imenv_jit_check(const ImEnvSpec* spec, const char* arch, uint32_t flags, char* log, int64_t log_len) {
  if (!spec || !arch) return fail(IMENV_E_INVALID, "null argument");
  SpecDev d;
  std::memset(&d, 0, sizeof(d));
  int maxc = 0;
  int rc = validate_and_derive(*spec, d, maxc);
  if (rc != IMENV_OK) return rc;
  std::vector<float> l32;
  std::vector<double> l64;
  build_obs_tables(d, l32, l64);
  imenv::JitFlags f;
  f.act_f64 = flags & 1u;
  f.obs_f64 = flags & 2u;
  f.noisy_delay = flags & 4u;
  f.noisy_demand = flags & 8u;
  f.has_delay_u = flags & 16u;
  f.metrics = flags & 1024u;
  f.stream_store = flags & 2048u;
  f.wt_obs = flags & 8192u;
  f.wt_state = flags & 16384u;
  f.small_blocks = flags & 32768u;
  f.info = !(flags & 65536u);
  f.full = flags & 131072u;
  f.aligned = flags & 262144u;
  f.demand_layout = (int)((flags >> 5) & 31u);
  d.rec_bytes = rec_bytes_for(d, f.small_blocks ? 1 : INT64_MAX);   // as a handle of that size would
  d.dtab_es = dtab_es_for(d, f.small_blocks ? 1 : INT64_MAX);
  std::string msg;
  std::string src;
  if (flags & (1u << 12)) {   // the rollout kernel; bits 13..19 = RolloutFlags::key()
    imenv::RolloutFlags rf;
    const uint32_t rk = flags >> 13;
    rf.table = rk & 1u;
    rf.noisy_delay = rk & 2u;
    rf.noisy_demand = rk & 4u;
    rf.objective = rk & 8u;
    rf.act = (int)((rk >> 4) & 3u);
    rf.act_f64 = rk & 64u;
    if (rf.act > imenv::ROLL_PLAN_EPISODE || (rf.act != imenv::ROLL_BASE_STOCK && rf.objective))
      return fail(IMENV_E_INVALID, "rollout flags: unknown action source, or a plan with an objective");
    const int bs = imenv::rollout_block_size(d, rf);
    if (bs == 0) return fail(IMENV_E_UNSUPPORTED, "rollout does not fit LDS");
    src = imenv::jit_rollout_source(d, maxc, rf, bs);
  } else {
    src = imenv::jit_source(d, maxc, is_base_obs(*spec), f);
  }
  auto code = imenv::jit_compile(src, arch, msg);
  if (log && log_len > 0) std::snprintf(log, (size_t)log_len, "%s", code ? "ok" : msg.c_str());
  if (!code) return fail(IMENV_E_UNSUPPORTED, "hipRTC: " + msg);
  return IMENV_OK;
}

}  // extern "C"
