// imenv_kernels.hip — MI355X (gfx950) step/reset kernels and the C ABI of include/imenv.h.
//
// One fused kernel advances every env by one period: order decode (rev_scale +
// round/clip), demand assembly, lead-time arrivals from a per-node ring buffer,
// shipment, the divergent per-edge split, backlog / order_u / inventory balance,
// per-node profit and reward, and the next observation. It restates
// environments/IM_env.py:287-456, MAIM_env.py:330-519, IM_div_env.py:361-645 and
// MAIM_div_env.py:441-739 (every quirk listed in SURVEY.md §8a), batched over envs.
//
// Layout: one thread per env; every node of that env in registers
// (the node loop is unrolled for NT >= N nodes); state is int32 SoA [field][node][env]
// so a wave's 64 lanes read/write 256 contiguous bytes per field; actions [env][N]
// and obs [env][N][F] are the policy's row layout (vector loads/stores per lane).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (no FMA contraction,
// IEEE division: float64 rewards/obs are bit-exact with NumPy).
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/imenv.h"

#define IMENV_TABLE_MAX 1024

namespace {

// ------------------------------------------------------------------ device spec
struct SpecDev {
  ImEnvSpec s;
  int32_t ring_off[IMENV_MAX_NODES];   // first ring row of node i (rows = sum of delays)
  int32_t bto_slot[IMENV_MAX_NODES];   // backlog_to row of child c (-1: parent does not split)
  int32_t num_split;                   // nodes with >1 child, ascending
  int32_t split_node[IMENV_MAX_NODES];
  int32_t single_parent[IMENV_MAX_NODES];  // parent if it has exactly one child, else -1
  int32_t factory;
  int32_t table_len;
  uint32_t table[IMENV_TABLE_MAX];
};

struct StepArgs {
  const void* actions;
  void* obs;
  double* reward;
  int32_t* inv;
  int32_t* bl;
  int32_t* ou;
  int32_t* ring;
  int32_t* carry;
  int32_t* bto;
  int32_t* hist_d;
  int32_t* hist_o;
  const int32_t* demand;      // PER_ENV: [T][R][n]; BROADCAST: [T][R]
  const double* delay_u;      // [T][N][n] or null
  uint32_t* err;              // [n]
  uint32_t* err_any;          // [1]
  int32_t* i_order;
  int32_t* i_demand;
  int32_t* i_acq;
  int32_t* i_ship;
  double* i_profit;
  int32_t* i_ship_to;
  int32_t* i_bto;
  int64_t n;
  uint32_t env_offset;
  uint32_t episode;
  int32_t t;
  int32_t action_f64;
  int32_t obs_f64;
  int32_t demand_layout;      // IMENV_LAYOUT_*
  int32_t noisy_demand;       // applies to drawn / broadcast demand
  int32_t noisy_delay;
  double noisy_delay_thr;
  uint64_t noisy_delay_thr32;
  uint64_t noisy_demand_thr32;
};

constexpr uint32_t PH_M0 = 0xD2511F53u, PH_M1 = 0xCD9E8D57u;
constexpr uint32_t PH_W0 = 0x9E3779B9u, PH_W1 = 0xBB67AE85u;
constexpr uint32_t STREAM_DEMAND = 0, STREAM_ND_DOUBLE = 1, STREAM_ND_ZERO = 2, STREAM_NOISY_DELAY = 3;

// Philox4x32-10 (Salmon et al. SC'11); oracle/philox.py is the CPU twin.
__device__ __forceinline__ uint32_t philox_word(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                uint32_t k0, uint32_t k1, int w) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += PH_W0; k1 += PH_W1; }
    const uint32_t hi0 = __umulhi(PH_M0, c0), lo0 = PH_M0 * c0;
    const uint32_t hi1 = __umulhi(PH_M1, c2), lo1 = PH_M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return w == 0 ? c0 : (w == 1 ? c1 : (w == 2 ? c2 : c3));
}

__device__ __forceinline__ int ceil_div_pos(int a, int b) { return (a + b - 1) / b; }

// Round-robin unit shipping, closed form. Restates the reference's
//   while <cond> and amt > 0: for k in children: if x[k] > 0: s[k]+=1; x[k]-=1; amt-=1
// (IM_div_env.py:413-428, 440-450, 472-484; the inner loop does not re-check amt).
// SUMCHECK: loop also requires sum(x) > 0 (backlog-first / outstanding-order loops).
// Without it (capped loop, IM_div_env.py:488-498) an env with nothing eligible spins
// until the guard trips. Phases: while the set P = {k: x[k] > 0} is fixed, every
// round moves |P| units, so a phase lasts min(min_P x, ceil(S/|P|), ceil(amt/|P|))
// rounds. Returns false if the guard (rounds > lim) trips; rounds stop at lim+1.
template <int MC, bool SUMCHECK>
__device__ __forceinline__ bool rr_closed(int m, int (&x)[MC], int (&s)[MC], int& amt, int lim) {
  int rounds = 0;
#pragma unroll 1
  for (int ph = 0; ph <= MC + 1; ++ph) {
    int S = 0, cnt = 0, mn = INT_MAX;
#pragma unroll
    for (int k = 0; k < MC; ++k) {
      if (k < m) {
        S += x[k];
        if (x[k] > 0) { ++cnt; mn = min(mn, x[k]); }
      }
    }
    if (amt <= 0) break;
    if (SUMCHECK && S <= 0) break;
    if (cnt == 0) { rounds = lim + 1; break; }   // no progress possible: guard trips
    int r = min(mn, ceil_div_pos(amt, cnt));
    if (SUMCHECK) r = min(r, ceil_div_pos(S, cnt));
    const int rem = lim + 1 - rounds;
    if (r > rem) r = rem;
#pragma unroll
    for (int k = 0; k < MC; ++k)
      if (k < m && x[k] > 0) { x[k] -= r; s[k] += r; }
    amt -= r * cnt;
    rounds += r;
    if (rounds > lim) break;
  }
  return rounds <= lim;
}

template <int NT>
__device__ __forceinline__ int sel(const int (&v)[NT], int idx) {
  int r = 0;
#pragma unroll
  for (int j = 0; j < NT; ++j) r = (idx == j) ? v[j] : r;
  return r;
}

__device__ __forceinline__ double obs_map(int mode, double v, double a, double bma, double den, double clip) {
  // rescale(val, 0, max, a, b) = a + ((val - 0) * (b - a)) / (max - 0)   (IM_env.py:435-444)
  if (mode == IMENV_OBS_RAW) return v;
  if (mode == IMENV_OBS_SCALED) return a + (v * bma) / den;
  if (mode == IMENV_OBS_CLAMP_SCALED) return a + (fmin(v, clip) * bma) / den;
  return 0.0;
}

__device__ __forceinline__ void store_obs(void* obs, int f64, int64_t idx, double v) {
  if (f64) static_cast<double*>(obs)[idx] = v;
  else static_cast<float*>(obs)[idx] = static_cast<float>(v);
}

// ------------------------------------------------------------------ step kernel
// NT: compile-time node capacity (>= N). MC: max children of a splitting node (0 = no split).
// BASE: observation is exactly [inv, backlog, order_u] (F = 3), vector-stored.
template <int NT, int MC, bool BASE>
__global__ void __launch_bounds__(256) imenv_step_kernel(const SpecDev* __restrict__ sp, StepArgs A) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const ImEnvSpec& S = sp->s;
  __shared__ uint32_t s_tab[IMENV_TABLE_MAX];
  const bool poisson = A.demand_layout == IMENV_LAYOUT_DRAW && S.demand_dist == IMENV_DEMAND_POISSON;
  if (poisson) {
    for (int k = threadIdx.x; k < sp->table_len; k += blockDim.x) s_tab[k] = sp->table[k];
    __syncthreads();
  }
  if (e >= A.n) return;
  const int N = S.num_nodes;
  const int T = S.num_periods;
  const int t = A.t;
  const int64_t n = A.n;
  const double a = S.a;
  const double bma = S.b - S.a;
  const uint32_t gid = A.env_offset + (uint32_t)e;
  const uint32_t k0 = (uint32_t)S.seed, k1 = (uint32_t)(S.seed >> 32);

  int inv[NT], bl[NT], ou[NT], order[NT], dem[NT], acq[NT], ship[NT], sto[NT], push[NT];
  double prof[NT];

  // ---- state (period-0 state is implicit: no loads at t == 0)
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i < N) {
      if (t == 0) { inv[i] = S.init_inv[i]; bl[i] = 0; ou[i] = 0; }
      else { inv[i] = A.inv[i * n + e]; bl[i] = A.bl[i * n + e]; ou[i] = A.ou[i * n + e]; }
    }
  }

  // ---- order decode (IM_env.py:298-302; MAIM_env.py:340-347)
  double x[NT];
  if (A.action_f64) {
    const double* ap = static_cast<const double*>(A.actions) + e * N;
    if (N == NT && (NT % 2) == 0) {
#pragma unroll
      for (int i = 0; i < NT; i += 2) {
        const double2 v = *reinterpret_cast<const double2*>(ap + i);
        x[i] = v.x; x[i + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NT; ++i) x[i] = (i < N) ? ap[i] : 0.0;
    }
  } else {
    const float* ap = static_cast<const float*>(A.actions) + e * N;
    if (N == NT && (NT % 4) == 0) {
#pragma unroll
      for (int i = 0; i < NT; i += 4) {
        const float4 v = *reinterpret_cast<const float4*>(ap + i);
        x[i] = v.x; x[i + 1] = v.y; x[i + 2] = v.z; x[i + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NT; ++i) x[i] = (i < N) ? (double)ap[i] : 0.0;
    }
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i < N) {
      const double om = (double)S.order_max[i];
      double v = S.standardise_actions ? (((x[i] - a) * (om - 0.0)) / bma) + 0.0 : x[i];
      double o;
      if (S.decode_mode == IMENV_DECODE_CLIP_ROUND) o = rint(fmin(fmax(v, 0.0), om));
      else o = fmin(fmax(rint(v), 0.0), om);
      order[i] = (int)o;
    }
  }

  // ---- demand (IM_env.py:306-308, IM_div_env.py:380-387)
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i < N) {
      const int r = S.retailer_slot[i];
      if (r >= 0) {
        const int R = S.num_retailers;
        int cd;
        if (A.demand_layout == IMENV_LAYOUT_PER_ENV) {
          cd = A.demand[((int64_t)t * R + r) * n + e];
        } else if (A.demand_layout == IMENV_LAYOUT_BROADCAST) {
          cd = A.demand[t * R + r];
        } else {
          const uint32_t w = philox_word(gid, A.episode, (uint32_t)t, (STREAM_DEMAND << 16) | (uint32_t)(r >> 2),
                                         k0, k1, r & 3);
          if (poisson) {
            int lo = 0, hi = sp->table_len;
            while (lo < hi) {
              const int mid = (lo + hi) >> 1;
              if (w >= s_tab[mid]) lo = mid + 1; else hi = mid;
            }
            cd = lo;
          } else {
            const uint64_t rng = (uint64_t)(S.uniform_high - S.uniform_low);
            cd = S.uniform_low + (int)(((uint64_t)w * rng) >> 32);
          }
        }
        if (A.noisy_demand) {
          const uint32_t wd = philox_word(gid, A.episode, (uint32_t)t, (STREAM_ND_DOUBLE << 16) | (uint32_t)(r >> 2),
                                          k0, k1, r & 3);
          const uint32_t wz = philox_word(gid, A.episode, (uint32_t)t, (STREAM_ND_ZERO << 16) | (uint32_t)(r >> 2),
                                          k0, k1, r & 3);
          if ((uint64_t)wd < A.noisy_demand_thr32) cd = 2 * cd;
          if ((uint64_t)wz < A.noisy_demand_thr32) cd = 0;
        }
        dem[i] = min(cd, S.inv_max[i]);
      } else {
        int s = 0;
#pragma unroll
        for (int c = 0; c < NT; ++c)
          if (c < N && S.demand_parent[c] == i) s += order[c];
        dem[i] = s;
      }
    }
  }

  // ---- arrivals: ring slot (t mod d) holds what was shipped d periods ago (IM_env.py:376-414)
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i < N) {
      const int d = S.delay[i];
      const int slot = t % d;
      int arr = 0;
      if (t >= d) arr = A.ring[(int64_t)(sp->ring_off[i] + slot) * n + e];
      int q = arr;
      if (A.noisy_delay) {
        if (t > 0) q += A.carry[i * n + e];
        int co = 0;
        if (t >= d) {
          bool extra;
          if (A.delay_u) extra = A.delay_u[((int64_t)t * N + i) * n + e] <= A.noisy_delay_thr;
          else extra = (uint64_t)philox_word(gid, A.episode, (uint32_t)t,
                                             (STREAM_NOISY_DELAY << 16) | (uint32_t)(i >> 2), k0, k1, i & 3) <
                       A.noisy_delay_thr32;
          if (extra && t < T - 1) { co = q; q = 0; }
        }
        A.carry[i * n + e] = co;
      }
      acq[i] = q;
      ship[i] = min(bl[i] + dem[i], inv[i] + acq[i]);   // IM_env.py:315
    }
  }

  // ---- shipments into each node: whole ship of a single-child parent, else the split
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    sto[c] = 0;
    if (c < N) {
      const int p = sp->single_parent[c];
      if (p >= 0) sto[c] = sel<NT>(ship, p);
    }
  }
  if constexpr (MC > 0) {
#pragma unroll 1
    for (int si = 0; si < sp->num_split; ++si) {
      const int p = sp->split_node[si];
      const int m = S.num_children[p];
      const int shp = sel<NT>(ship, p), dmp = sel<NT>(dem, p), blp = sel<NT>(bl, p);
      int bto[MC], oc[MC], s[MC];
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        s[k] = 0; bto[k] = 0; oc[k] = 0;
        if (k < m) {
          const int c = S.children[p][k];
          oc[k] = sel<NT>(order, c);
          if (t > 0) bto[k] = A.bto[(int64_t)sp->bto_slot[c] * n + e];
        }
      }
      int amt = shp;
      bool ok = true;
      if (shp >= dmp) {
        if (blp > 0) {        // backlog first, then outstanding orders (IM_div_env.py:409-454)
          ok = rr_closed<MC, true>(m, bto, s, amt, S.split_limit[p][0]);
          if (ok && amt > 0 && dmp > 0) {
            int out[MC];
#pragma unroll
            for (int k = 0; k < MC; ++k) out[k] = oc[k];
            ok = rr_closed<MC, true>(m, out, s, amt, S.split_limit[p][1]);
#pragma unroll
            for (int k = 0; k < MC; ++k) bto[k] += out[k];
          }
        } else {              // IM_div_env.py:457-460
#pragma unroll
          for (int k = 0; k < MC; ++k) s[k] += oc[k];
        }
      } else {
        if (blp > 0) {        // IM_div_env.py:468-484
          ok = rr_closed<MC, true>(m, bto, s, amt, S.split_limit[p][2]);
        } else {              // IM_div_env.py:486-498: cap at order + backlog_to
          int cap[MC];
#pragma unroll
          for (int k = 0; k < MC; ++k) cap[k] = oc[k] + bto[k];
          ok = rr_closed<MC, false>(m, cap, s, amt, S.split_limit[p][3]);
        }
#pragma unroll
        for (int k = 0; k < MC; ++k) bto[k] += oc[k] - s[k];   // IM_div_env.py:501-502
      }
      if (!ok) {
        A.err[e] |= 1u;
        atomicOr(A.err_any, 1u);
      }
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        if (k < m) {
          const int c = S.children[p][k];
#pragma unroll
          for (int j = 0; j < NT; ++j) sto[j] = (c == j) ? s[k] : sto[j];
          A.bto[(int64_t)sp->bto_slot[c] * n + e] = bto[k];
          if (A.i_bto) A.i_bto[e * N + c] = bto[k];
        }
      }
    }
  }

  // ---- balance equations, ring push, profit (IM_env.py:318-340, 362-374)
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i < N) {
      int b2 = bl[i] + dem[i] - ship[i];
      if (S.backlog_cap[i] >= 0) b2 = min(b2, S.backlog_cap[i]);
      const int im = S.inv_max[i];
      const int ou2 = min(max(ou[i] + order[i] - acq[i], 0), im);
      const int inv2 = min(max(inv[i] + acq[i] - ship[i], 0), im);
      push[i] = (i == sp->factory) ? order[i] : sto[i];
      A.ring[(int64_t)(sp->ring_off[i] + t % S.delay[i]) * n + e] = push[i];
      prof[i] = ((S.sell_price[i] * (double)ship[i] - S.buy_price[i] * (double)order[i]) -
                 S.stock_cost[i] * fabs((double)inv2 - S.inv_target[i])) -
                S.backlog_cost[i] * (double)b2;
      bl[i] = b2; ou[i] = ou2; inv[i] = inv2;
      A.inv[i * n + e] = inv2;
      A.bl[i * n + e] = b2;
      A.ou[i * n + e] = ou2;
    }
  }
  const int L = S.prev_length;
  if (A.hist_d) {
#pragma unroll
    for (int i = 0; i < NT; ++i) if (i < N) A.hist_d[((int64_t)(t % L) * N + i) * n + e] = dem[i];
  }
  if (A.hist_o) {
#pragma unroll
    for (int i = 0; i < NT; ++i) if (i < N) A.hist_o[((int64_t)(t % L) * N + i) * n + e] = order[i];
  }

  // ---- reward (IM_env.py:372 np.sum order; MAIM_env.py:418-434)
  if (S.reward_mode == IMENV_REWARD_INDEPENDENT) {
#pragma unroll
    for (int i = 0; i < NT; ++i) if (i < N) A.reward[e * N + i] = prof[i];
  } else if (S.reward_mode == IMENV_REWARD_SHARED_MEAN || N < 8) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NT; ++i) if (i < N) s += prof[i];
    A.reward[e] = (S.reward_mode == IMENV_REWARD_SHARED_MEAN) ? s / (double)N : s;
  } else {
    double r8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r8[j] = (j < NT) ? prof[j < NT ? j : 0] : 0.0;
    const int full = N - (N % 8);
#pragma unroll
    for (int i0 = 8; i0 < NT; i0 += 8) {
      if (i0 < full) {
#pragma unroll
        for (int j = 0; j < 8; ++j) if (i0 + j < NT) r8[j] += prof[(i0 + j) < NT ? i0 + j : 0];
      }
    }
    double s = ((r8[0] + r8[1]) + (r8[2] + r8[3])) + ((r8[4] + r8[5]) + (r8[6] + r8[7]));
#pragma unroll
    for (int i = 8; i < NT; ++i) if (i >= full && i < N) s += prof[i];
    A.reward[e] = s;
  }

  // ---- info (IM_env.py:345-350)
  if (A.i_order) {
#pragma unroll
    for (int i = 0; i < NT; ++i) if (i < N) {
      A.i_order[e * N + i] = order[i];
      if (A.i_demand) A.i_demand[e * N + i] = dem[i];
      if (A.i_acq) A.i_acq[e * N + i] = acq[i];
      if (A.i_ship) A.i_ship[e * N + i] = ship[i];
      if (A.i_profit) A.i_profit[e * N + i] = prof[i];
      if (A.i_ship_to) A.i_ship_to[e * N + i] = sto[i];
    }
  }

  // ---- observation for period t+1 (IM_env.py:231-285, MAIM_env.py:242-328, ...)
  if constexpr (BASE) {
    const int gm0 = S.group_mode[0], gm1 = S.group_mode[1], gm2 = S.group_mode[2];
    double ov[3 * NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      if (i < N) {
        ov[3 * i + 0] = obs_map(gm0, (double)inv[i], a, bma, S.group_den[0][i], 0.0);
        ov[3 * i + 1] = obs_map(gm1, (double)bl[i], a, bma, S.group_den[1][i], 0.0);
        ov[3 * i + 2] = obs_map(gm2, (double)ou[i], a, bma, S.group_den[2][i], 0.0);
      } else {
        ov[3 * i + 0] = ov[3 * i + 1] = ov[3 * i + 2] = 0.0;
      }
    }
    if (N == NT && !A.obs_f64 && ((3 * NT) % 4) == 0) {
      float4* op = reinterpret_cast<float4*>(static_cast<float*>(A.obs) + e * (3 * NT));
#pragma unroll
      for (int q = 0; q < (3 * NT) / 4; ++q)
        op[q] = make_float4((float)ov[4 * q], (float)ov[4 * q + 1], (float)ov[4 * q + 2], (float)ov[4 * q + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 3 * NT; ++q)
        if (q < 3 * N) store_obs(A.obs, A.obs_f64, e * (3 * N) + q, ov[q]);
    }
  } else {
    const int F = S.num_features;
    const int tp = t + 1;   // observation period
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      if (i < N) {
        const int d = S.delay[i];
#pragma unroll 1
        for (int f = 0; f < F; ++f) {
          const int g = S.feat_group[f];
          const int j = S.feat_index[f];
          double v = 0.0;
          if (g == IMENV_G_INV) v = inv[i];
          else if (g == IMENV_G_BACKLOG) v = bl[i];
          else if (g == IMENV_G_ORDER_U) v = ou[i];
          else if (g == IMENV_G_DEMAND_HIST || g == IMENV_G_ORDER_HIST) {
            const int pr = tp - 1 - j;     // period of the entry; 0 when j >= tp
            if (pr >= 0) {
              if (j == 0) v = (g == IMENV_G_DEMAND_HIST) ? dem[i] : order[i];
              else {
                const int32_t* h = (g == IMENV_G_DEMAND_HIST) ? A.hist_d : A.hist_o;
                v = h[((int64_t)(pr % L) * N + i) * n + e];
              }
            }
          } else if (g == IMENV_G_TRANSIT) {
            // slot k: amount arriving at period tp + k, shipped at tp + k - d (IM_env.py:416-432)
            if (j < d && tp + j - d >= 0) {
              if (j == d - 1) v = push[i];
              else v = A.ring[(int64_t)(sp->ring_off[i] + (tp + j) % d) * n + e];
            }
          } else if (g == IMENV_G_NODE_ID) {
            v = i;
          }
          const double o = obs_map(S.group_mode[g], v, a, bma, S.group_den[g][i], S.group_clip[g][i]);
          store_obs(A.obs, A.obs_f64, (e * N + i) * F + f, o);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ reset kernel
// Period-0 observation (IM_env.py:221-229): inv = init_inv, everything else 0.
__global__ void __launch_bounds__(256) imenv_reset_kernel(const SpecDev* __restrict__ sp, void* obs, int obs_f64,
                                                          int64_t n) {
  const ImEnvSpec& S = sp->s;
  const int N = S.num_nodes, F = S.num_features;
  const int64_t row = (int64_t)N * F;
  const int64_t total = n * row;
  const double a = S.a, bma = S.b - S.a;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(q % row);
    const int i = r / F, f = r % F;
    const int g = S.feat_group[f];
    double v = 0.0;
    if (g == IMENV_G_INV) v = S.init_inv[i];
    else if (g == IMENV_G_NODE_ID) v = i;
    store_obs(obs, obs_f64, q, obs_map(S.group_mode[g], v, a, bma, S.group_den[g][i], S.group_clip[g][i]));
  }
}

}  // namespace

// ==================================================================== host side
struct ImEnv {
  SpecDev host;        // host copy of the device spec
  SpecDev* d_spec = nullptr;
  int device = 0;
  int64_t n = 0;
  int64_t env_offset = 0;
  int maxc = 0;
  int ring_rows = 0;
  int32_t *d_inv = nullptr, *d_bl = nullptr, *d_ou = nullptr, *d_ring = nullptr, *d_carry = nullptr,
          *d_bto = nullptr, *d_hist_d = nullptr, *d_hist_o = nullptr, *d_demand = nullptr;
  double* d_delay_u = nullptr;
  uint32_t *d_err = nullptr, *d_err_any = nullptr;
  int t = 0;
  int64_t episode = -1;
  bool reset_done = false;
  bool noisy_delay = false;
  double noisy_thr = 0.0;
  bool have_delay_u = false;
  int demand_layout = IMENV_LAYOUT_DRAW;
  size_t demand_cap = 0;
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t _e = (x);                                                                   \
    if (_e != hipSuccess) return fail(IMENV_E_HIP, std::string(#x ": ") + hipGetErrorString(_e)); \
  } while (0)

uint64_t prob_thr32(double p) {
  double v = std::ceil(p * 4294967296.0);
  if (v < 0) v = 0;
  if (v > 4294967296.0) v = 4294967296.0;
  return (uint64_t)v;
}

int validate_and_derive(const ImEnvSpec& s, SpecDev& d, int& maxc, int& ring_rows) {
  if (s.abi_version != IMENV_ABI_VERSION) return fail(IMENV_E_INVALID, "abi_version mismatch");
  const int N = s.num_nodes;
  if (N < 1 || N > IMENV_MAX_NODES) return fail(IMENV_E_INVALID, "num_nodes out of range");
  if (s.num_periods < 1 || s.num_periods > IMENV_MAX_PERIODS) return fail(IMENV_E_INVALID, "num_periods out of range");
  std::memset(&d, 0, sizeof(d));
  d.s = s;
  int roots = 0;
  d.factory = -1;
  ring_rows = 0;
  for (int i = 0; i < N; ++i) {
    if (s.parent[i] < 0) { ++roots; d.factory = i; }
    else if (s.parent[i] >= N || s.parent[i] == i) return fail(IMENV_E_INVALID, "bad parent index");
    if (s.delay[i] < 1)
      return fail(IMENV_E_UNSUPPORTED, "delay must be >= 1 in this build (delay 0 is a degenerate lead time)");
    if (s.delay[i] > IMENV_MAX_DELAY) return fail(IMENV_E_INVALID, "delay too large");
    if (s.inv_max[i] < 0 || s.order_max[i] < 0) return fail(IMENV_E_INVALID, "negative capacity");
    if (s.num_children[i] < 0 || s.num_children[i] > IMENV_MAX_CHILDREN) return fail(IMENV_E_UNSUPPORTED, "too many children");
    d.ring_off[i] = ring_rows;
    ring_rows += s.delay[i];
  }
  if (roots != 1) return fail(IMENV_E_INVALID, "topology needs exactly one factory (parent = -1)");
  maxc = 0;
  d.num_split = 0;
  int bto_rows = 0;
  for (int i = 0; i < N; ++i) { d.bto_slot[i] = -1; d.single_parent[i] = -1; }
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
      for (int k = 0; k < m; ++k) d.bto_slot[s.children[p][k]] = bto_rows++;
    }
  }
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
    if ((s.feat_group[f] == IMENV_G_DEMAND_HIST || s.feat_group[f] == IMENV_G_ORDER_HIST) && s.feat_index[f] >= s.prev_length)
      return fail(IMENV_E_INVALID, "history feature index >= prev_length");
  }
  for (int g = 0; g < IMENV_NUM_GROUPS; ++g)
    if (s.group_mode[g] < IMENV_OBS_ZERO || s.group_mode[g] > IMENV_OBS_CLAMP_SCALED) return fail(IMENV_E_INVALID, "bad group mode");
  if (s.decode_mode != IMENV_DECODE_CLIP_ROUND && s.decode_mode != IMENV_DECODE_ROUND_CLIP) return fail(IMENV_E_INVALID, "bad decode_mode");
  if (s.reward_mode < IMENV_REWARD_SUM || s.reward_mode > IMENV_REWARD_INDEPENDENT) return fail(IMENV_E_INVALID, "bad reward_mode");
  if (s.standardise_actions && !(s.b - s.a != 0.0)) return fail(IMENV_E_INVALID, "a == b");
  d.table_len = 0;
  if (s.demand_dist == IMENV_DEMAND_POISSON) {
    // thr[k] = ceil(CDF(k) * 2^32) by the pmf recurrence (oracle/philox.py:poisson_thresholds)
    const double mu = s.poisson_mu;
    if (!(mu > 0.0)) return fail(IMENV_E_INVALID, "Poisson mean must be positive");
    double p = std::exp(-mu), cdf = 0.0;
    int k = 0;
    for (;;) {
      cdf += p;
      const double tv = std::ceil(cdf * 4294967296.0);
      if (tv >= 4294967296.0) break;
      if (k >= IMENV_TABLE_MAX) return fail(IMENV_E_UNSUPPORTED, "Poisson mean too large for the inversion table");
      d.table[k] = (uint32_t)tv;
      ++k;
      p = p * mu / (double)k;
    }
    d.table_len = k;
  } else if (s.demand_dist == IMENV_DEMAND_UNIFORM) {
    if (s.uniform_low >= s.uniform_high) return fail(IMENV_E_INVALID, "Lower bound cannot be larger than upper bound");
  } else if (s.demand_dist != IMENV_DEMAND_CUSTOM) {
    return fail(IMENV_E_INVALID, "Unrecognised, Distribution Not Implemented");
  }
  return IMENV_OK;
}

template <int NT, int MC, bool BASE>
void launch_step(const ImEnv* h, const StepArgs& A, hipStream_t st) {
  const int threads = 256;
  const int64_t blocks = (h->n + threads - 1) / threads;
  hipLaunchKernelGGL((imenv_step_kernel<NT, MC, BASE>), dim3((unsigned)blocks), dim3(threads), 0, st, h->d_spec, A);
}

template <int NT, int MC>
void dispatch_base(const ImEnv* h, const StepArgs& A, hipStream_t st, bool base) {
  if (base) launch_step<NT, MC, true>(h, A, st);
  else launch_step<NT, MC, false>(h, A, st);
}

template <int NT>
void dispatch_mc(const ImEnv* h, const StepArgs& A, hipStream_t st, bool base) {
  if (h->maxc == 0) dispatch_base<NT, 0>(h, A, st, base);
  else if (h->maxc <= 4) dispatch_base<NT, 4>(h, A, st, base);
  else dispatch_base<NT, IMENV_MAX_CHILDREN>(h, A, st, base);
}

bool is_base_obs(const ImEnvSpec& s) {
  return s.num_features == 3 && s.feat_group[0] == IMENV_G_INV && s.feat_group[1] == IMENV_G_BACKLOG &&
         s.feat_group[2] == IMENV_G_ORDER_U;
}

template <typename T>
int alloc(T** p, size_t count) {
  if (count == 0) { *p = nullptr; return IMENV_OK; }
  HIPCHK(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  return IMENV_OK;
}

}  // namespace

extern "C" {

int imenv_abi_version(void) { return IMENV_ABI_VERSION; }

int64_t imenv_spec_size(void) { return (int64_t)sizeof(ImEnvSpec); }

const char* imenv_last_error(void) { return g_err.c_str(); }

int imenv_create(const ImEnvSpec* spec, int64_t n_envs, int64_t env_offset, int device, ImEnv** out) {
  if (!spec || !out) return fail(IMENV_E_INVALID, "null argument");
  *out = nullptr;
  if (n_envs < 1 || n_envs > (int64_t(1) << 31)) return fail(IMENV_E_INVALID, "n_envs out of range");
  if (env_offset < 0 || env_offset + n_envs > (int64_t(1) << 32)) return fail(IMENV_E_INVALID, "env ids must fit 32 bits");
  ImEnv* h = new ImEnv();
  int rc = validate_and_derive(*spec, h->host, h->maxc, h->ring_rows);
  if (rc != IMENV_OK) { delete h; return rc; }
  h->device = device;
  h->n = n_envs;
  h->env_offset = env_offset;
  h->noisy_delay = spec->noisy_delay != 0;
  h->noisy_thr = spec->noisy_delay_threshold;
  const ImEnvSpec& s = *spec;
  const size_t N = s.num_nodes, n = n_envs;
  int bto_rows = 0;
  for (int i = 0; i < s.num_nodes; ++i) if (h->host.bto_slot[i] >= 0) ++bto_rows;
  bool uses_hist = false;
  for (int f = 0; f < s.num_features; ++f)
    if (s.feat_group[f] == IMENV_G_DEMAND_HIST || s.feat_group[f] == IMENV_G_ORDER_HIST) uses_hist = true;
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) { delete h; return fail(IMENV_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he)); }
  if ((rc = alloc(&h->d_spec, 1)) || (rc = alloc(&h->d_inv, N * n)) || (rc = alloc(&h->d_bl, N * n)) ||
      (rc = alloc(&h->d_ou, N * n)) || (rc = alloc(&h->d_ring, (size_t)h->ring_rows * n)) ||
      (rc = alloc(&h->d_carry, N * n)) || (rc = alloc(&h->d_bto, (size_t)bto_rows * n)) ||
      (rc = alloc(&h->d_err, n)) || (rc = alloc(&h->d_err_any, 1))) {
    imenv_destroy(h);
    return rc;
  }
  if (uses_hist) {
    if ((rc = alloc(&h->d_hist_d, (size_t)s.prev_length * N * n)) || (rc = alloc(&h->d_hist_o, (size_t)s.prev_length * N * n))) {
      imenv_destroy(h);
      return rc;
    }
  }
  he = hipMemcpy(h->d_spec, &h->host, sizeof(SpecDev), hipMemcpyHostToDevice);
  if (he == hipSuccess) he = hipMemset(h->d_err, 0, n * sizeof(uint32_t));
  if (he == hipSuccess) he = hipMemset(h->d_err_any, 0, sizeof(uint32_t));
  if (he != hipSuccess) { imenv_destroy(h); return fail(IMENV_E_HIP, std::string("init copy: ") + hipGetErrorString(he)); }
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
  h->episode = (episode >= 0) ? episode : h->episode + 1;
  h->t = 0;
  h->reset_done = true;
  HIPCHK(hipMemsetAsync(h->d_err, 0, n * sizeof(uint32_t), st));
  HIPCHK(hipMemsetAsync(h->d_err_any, 0, sizeof(uint32_t), st));
  const int64_t total = (int64_t)n * N * s.num_features;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(imenv_reset_kernel, dim3((unsigned)blocks), dim3(256), 0, st, h->d_spec, obs,
                     obs_dtype == IMENV_F64 ? 1 : 0, (int64_t)n);
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
  HIPCHK(hipSetDevice(h->device));
  StepArgs A;
  std::memset(&A, 0, sizeof(A));
  A.actions = actions;
  A.obs = obs;
  A.reward = reward;
  A.inv = h->d_inv; A.bl = h->d_bl; A.ou = h->d_ou;
  A.ring = h->d_ring; A.carry = h->d_carry; A.bto = h->d_bto;
  A.hist_d = h->d_hist_d; A.hist_o = h->d_hist_o;
  A.demand = h->d_demand;
  A.delay_u = h->have_delay_u ? h->d_delay_u : nullptr;
  A.err = h->d_err; A.err_any = h->d_err_any;
  if (info) {
    A.i_order = info->order; A.i_demand = info->demand; A.i_acq = info->acquisition; A.i_ship = info->ship;
    A.i_profit = info->profit; A.i_ship_to = info->ship_to; A.i_bto = info->backlog_to;
    if (!A.i_order && (A.i_demand || A.i_acq || A.i_ship || A.i_profit || A.i_ship_to))
      return fail(IMENV_E_INVALID, "info.order is required when any other info field is requested");
    if (A.i_bto) HIPCHK(hipMemsetAsync(A.i_bto, 0, (size_t)h->n * s.num_nodes * sizeof(int32_t), static_cast<hipStream_t>(stream)));
  }
  A.n = h->n;
  A.env_offset = (uint32_t)h->env_offset;
  A.episode = (uint32_t)h->episode;
  A.t = h->t;
  A.action_f64 = action_dtype == IMENV_F64;
  A.obs_f64 = obs_dtype == IMENV_F64;
  A.demand_layout = h->demand_layout;
  A.noisy_demand = (s.noisy_demand && h->demand_layout != IMENV_LAYOUT_PER_ENV) ? 1 : 0;
  A.noisy_delay = h->noisy_delay ? 1 : 0;
  A.noisy_delay_thr = h->noisy_thr;
  A.noisy_delay_thr32 = prob_thr32(h->noisy_thr);
  A.noisy_demand_thr32 = prob_thr32(s.noisy_demand_threshold);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool base = is_base_obs(s);
  const int N = s.num_nodes;
  if (N <= 4) dispatch_mc<4>(h, A, st, base);
  else if (N <= 8) dispatch_mc<8>(h, A, st, base);
  else dispatch_mc<16>(h, A, st, base);
  HIPCHK(hipGetLastError());
  h->t += 1;
  if (done_out) *done_out = h->t >= s.num_periods ? 1 : 0;
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
    std::vector<int32_t> tmp((size_t)s.num_nodes * h->n);
    if (inv) {
      for (int i = 0; i < s.num_nodes; ++i)
        for (int64_t e = 0; e < h->n; ++e) tmp[(size_t)i * h->n + e] = s.init_inv[i];
      HIPCHK(hipMemcpy(inv, tmp.data(), bytes, hipMemcpyHostToDevice));
    }
    if (backlog) HIPCHK(hipMemsetAsync(backlog, 0, bytes, st));
    if (order_u) HIPCHK(hipMemsetAsync(order_u, 0, bytes, st));
  } else {
    if (inv) HIPCHK(hipMemcpyAsync(inv, h->d_inv, bytes, hipMemcpyDeviceToDevice, st));
    if (backlog) HIPCHK(hipMemcpyAsync(backlog, h->d_bl, bytes, hipMemcpyDeviceToDevice, st));
    if (order_u) HIPCHK(hipMemcpyAsync(order_u, h->d_ou, bytes, hipMemcpyDeviceToDevice, st));
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

int imenv_dims(const ImEnv* h, int32_t* num_nodes, int32_t* num_features, int32_t* num_retailers, int32_t* num_periods) {
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

void imenv_destroy(ImEnv* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  void* ptrs[] = {h->d_spec, h->d_inv, h->d_bl, h->d_ou, h->d_ring, h->d_carry, h->d_bto,
                  h->d_hist_d, h->d_hist_o, h->d_demand, h->d_delay_u, h->d_err, h->d_err_any};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete h;
}

}  // extern "C"
