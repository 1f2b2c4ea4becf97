// imenv_device.h — device-side data structures and the fused step kernel body (gfx950).
//
// One kernel advances every env by one period: order decode (rev_scale + round/clip),
// demand assembly (host-fed or in-kernel Philox), lead-time arrivals, shipment, the
// divergent per-edge split, backlog / order_u / inventory balance, per-node profit and
// reward, and the next observation. It restates environments/IM_env.py:287-456,
// MAIM_env.py:330-519, IM_div_env.py:361-645 and MAIM_div_env.py:441-739 (every quirk
// listed in SURVEY.md §8a), batched over envs, one thread per env.
//
// The body is a template over a spec policy P:
//   DynSpec<NT, MC, BASE, ST>  reads the spec from device memory (ahead-of-time kernels, any spec)
//   JitSpec (generated)        every spec value is a constexpr: hipRTC compiles one kernel per
//                              spec with all constants folded into immediates (imenv_jit.cpp)
//
// HBM layout. ST = uint8 / int16 when the spec's bounds prove every value fits
// (0..255 / 32767), else int32. NP = row length in ST elements (N rounded up so rows are 4-byte
// aligned: to a multiple of 4 for uint8, of 2 for int16).
//   net, order_u            [n][NP] ST      one packed row per env: 4 B per lane for N=4 uint8; the
//                                           net row holds inv - backlog (signed: NetOf<ST>)
//   ring (in transit)       [sum d_i][n] ST node-major, d_i slots per node: node i's slot
//                                           (t mod d_i) holds what arrives at t (shipped at t - d_i)
//                                           and is then overwritten by what ships at t, so the
//                                           arrival load and departure store hit one address and a
//                                           wave moves whole 128-byte lines (a time-major ring
//                                           scatters 2-byte stores that dirty partial sectors)
//   record (small launches) [n][16|32 B]    uint8 state of up to 8 nodes as ONE record per env instead of
//                                           the three arrays above: net row, order_u row, then every ring
//                                           slot (node i's slot s at byte 2 NP + ring_off[i] + s), zero
//                                           padded; one 16/32-byte load and store per lane (SpecDev::rec_bytes)
//   hist_d / hist_o         [L][n][NP] ST   demand / order history rows (prev_* observations)
//   backlog_to              [n][E] int16|int32  split state of the E split children only (trees);
//                                           int16 when T x the children's order_max fits (bto_bound)
//   carry                   [n][NP] CarryOf<ST> noisy-delay carry
//   actions [n][N] f32|f64, obs [n][N][F] f32|f64, reward [n] or [n][N] f64 (policy layout)
// Build: --offload-arch=gfx950 -O3 -ffp-contract=off (no FMA contraction, IEEE division:
// float64 rewards/obs are bit-exact with NumPy).
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#else
typedef signed char int8_t;
typedef unsigned char uint8_t;
typedef short int16_t;
typedef unsigned short uint16_t;
typedef int int32_t;
typedef unsigned int uint32_t;
typedef long long int64_t;
typedef unsigned long long uint64_t;
#define INT_MAX 2147483647
#endif

#include "imenv.h"

#define IMENV_TABLE_MAX 1024
#ifndef IMENV_NT_STORE
#define IMENV_NT_STORE 0     // 1: observation / reward stores of the step kernel are non-temporal
#endif
#ifndef IMENV_WAVE_SLAB
#define IMENV_WAVE_SLAB 0    // 1: each wave writes out its own staged observation rows (step_body)
#endif
#ifndef IMENV_WT_STORE
#define IMENV_WT_STORE 0     // 1: observation / reward stores of the step kernel are write-through (sc1)
#endif
#ifndef IMENV_WT_STATE
#define IMENV_WT_STATE 0     // 1: the step kernel's state-row stores are write-through (sc1)
#endif
#ifndef IMENV_STAMPS
#define IMENV_STAMPS 0       // 1 (diagnostic builds only): per-wave phase timestamps into StepArgs::stamps
#endif
// Ablations (diagnostic builds only, WRONG results: timing where the compute goes): bit 0 skips the
// divergent split, bit 1 the demand draw (Philox + Poisson), bit 2 computes observations as (float)v,
// bit 3 skips profit / reward arithmetic, bit 4 skips the order decode (order = the action's sign bit:
// the action load stays), bit 5 replaces the scalar load of the device episode word by 0. Every
// ablation keeps every load and store, so IMENV_ABLATE=63 is the access-shape floor of the kernel.
#ifndef IMENV_ABLATE
#define IMENV_ABLATE 0
#endif
#ifndef IMENV_PRIO
#define IMENV_PRIO 0         // > 0: waves in odd hardware slots of a SIMD raise their issue priority (stagger)
#endif
#ifndef IMENV_BUF_LOAD
#define IMENV_BUF_LOAD 0     // 1: exact-row step loads as buffer loads off the block's first env (SGPR bases)
#endif
#ifndef IMENV_XCD_REMAP
#define IMENV_XCD_REMAP 0    // 1: XCD-aware env chunks for small-block launches (measured slower: step_body)
#endif
#ifndef IMENV_SLAB_BATCH
#define IMENV_SLAB_BATCH 1   // 1: a whole group's observation slab is written out in batches of LDS reads
#endif
#define IMENV_GUIDE_BITS 10

namespace imenv {

// 16-byte store, non-temporal under NT (streamed past the caches)
template <bool NT, typename V>
__device__ __forceinline__ void store16(V* p, const V& v) {
  if constexpr (NT) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    u4 w;
    __builtin_memcpy(&w, &v, 16);
    __builtin_nontemporal_store(w, reinterpret_cast<u4*>(p));
  } else {
    *p = v;
  }
}

// Write-through stores (cache policy sc1): the line is written to memory at once and dropped from
// the XCD's L2 (MI355X_MICROARCH.md, "stores of each flavour"), so a launch leaves no dirty lines for
// the end-of-kernel write-back (the dependent-boundary cost "+ B / 6 TB/s") and its HBM writes overlap
// the rest of the launch. Raw buffer stores carry the policy bits; the resource's base is wave-uniform
// (a block's slab), the per-lane part is the 32-bit byte offset.
constexpr int CPOL_SC1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
}
template <typename V>
__device__ __forceinline__ void wt_store16(__amdgpu_buffer_rsrc_t r, int off, const V& v) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  u4 w;
  __builtin_memcpy(&w, &v, 16);
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, CPOL_SC1);
}
__device__ __forceinline__ void wt_store8(__amdgpu_buffer_rsrc_t r, int off, double v) {
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  u2 w;
  __builtin_memcpy(&w, &v, 8);
  __builtin_amdgcn_raw_buffer_store_b64(w, r, off, 0, CPOL_SC1);
}
// a value every lane of the wave holds (e.g. the block's first env), as a scalar: a buffer resource
// built from it stays in SGPRs (from a value the compiler cannot prove uniform it would emit a
// readfirstlane waterfall loop around every buffer store)
__device__ __forceinline__ int64_t uniform_i64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  return reinterpret_cast<T*>(uniform_i64(reinterpret_cast<int64_t>(p)));
}

struct SpecDev {
  ImEnvSpec s;
  int32_t num_split;                        // nodes with > 1 child, ascending
  int32_t split_node[IMENV_MAX_NODES];
  int32_t split_child[IMENV_MAX_NODES];     // 1 if node's parent splits its shipment
  int32_t single_parent[IMENV_MAX_NODES];   // parent if it has exactly one child, else -1
  int32_t num_bto;                          // split children: nodes whose parent splits its shipment
  int32_t bto_es;                           // backlog_to element bytes: 2 (int16) or 4 (int32)
  int32_t bto_slot[IMENV_MAX_NODES];        // node -> its slot in the compact backlog_to row, or -1
  int32_t rec_bytes;                        // 0: state rows + ring; 16 / 32: one state record per env
  int32_t dtab_es;                          // 0: every step draws its period's demand; 1 (uint8) / 2 / 4: the
                                            // step at t % 4 == 0 parks periods t+1..t+3 in a [T][R][n] table
  int32_t factory;
  int32_t dmax;                             // max delay
  int32_t ring_off[IMENV_MAX_NODES];        // first ring row of node i (sum of earlier delays)
  int32_t ring_total;                       // ring rows = sum of delays
  int32_t np;                               // packed row length (elements)
  int32_t es;                               // state element bytes: 1 (uint8), 2 (int16) or 4 (int32)
  int32_t vbound;                           // proven bound of every raw value an observation reads (>= N)
  int32_t table_len;
  uint32_t table[IMENV_TABLE_MAX];          // Poisson inversion thresholds
  uint16_t guide[1 << IMENV_GUIDE_BITS];    // indexed-search guide: #{thresholds <= g << (32 - bits)}
  // observation lookup: value of group g, node i for raw v in [0, lut_max] at lut[lut_off + v]
  int32_t lut_off[IMENV_NUM_GROUPS][IMENV_MAX_NODES];
  int32_t lut_max[IMENV_NUM_GROUPS][IMENV_MAX_NODES];   // -1: not tabulated
  // period-0 observation row (the same for every env)
  alignas(16) float reset_f32[IMENV_MAX_NODES * IMENV_MAX_FEATURES];
  alignas(16) double reset_f64[IMENV_MAX_NODES * IMENV_MAX_FEATURES];
  double inv_bma;                           // 1/(b - a) when b - a is a power of two, else 0
  double inv_n;                             // 1/N when N is a power of two, else 0
};

struct StepArgs {
  const void* actions;
  void* obs;
  double* reward;
  void* net;                  // net inventory rows: inv - backlog (NetOf<ST>; see Row below)
  void* ou;
  void* ring;
  void* carry;                // noisy-delay carry rows (CarryOf<ST>)
  void* bto;                  // compact backlog_to rows (BtoRow)
  void* hist_d;
  void* hist_o;
  const int32_t* demand;      // PER_ENV: [T][R][n]; BROADCAST: [T][R]
  void* dtab;                 // drawn demand, [T][R][n] of SpecDev::dtab_es bytes (LAYOUT_DRAW), or null: read at
                              // t % 4 != 0, written (periods t+1..t+3) at t % 4 == 0
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
  const float* lut32;
  const double* lut64;
  const uint32_t* episode;    // device word written by the reset kernel (graph-replay safe)
  double* metrics;            // [n][4 + N] evaluation-harness accumulators (imenv_set_episode_metrics) or null
  uint64_t* stamps;           // diagnostics (IMENV_STAMPS builds): [waves][8] s_memrealtime phase stamps, or null
  int64_t n;
  uint32_t env_offset;
  int32_t t;
  int32_t action_f64;
  int32_t obs_f64;
  int32_t demand_layout;      // IMENV_LAYOUT_*
  int32_t noisy_demand;       // applies to drawn / broadcast demand
  int32_t noisy_delay;
  double noisy_delay_thr;
  uint64_t noisy_delay_thr32;
  uint64_t noisy_demand_thr32;
  int64_t ring_at[IMENV_MAX_NODES];   // element offset of node i's ring row this step: (ring_off[i] + t mod delay[i]) * n;
                                      // with state records: that slot's byte in the record, 2 NP + ring_off[i] + t mod delay[i]
};

// Fused base-stock rollout (imenv_base_stock_rollout): whole episodes of P policies x S demand
// scenarios in one launch, state in registers, the in-transit queue in LDS.
struct RolloutArgs {
  const double* policy;       // [P][N] order-up-to levels (base-stock rollouts)
  const void* plan;           // plan rollouts: [P][T][N] (PLAN_SHARED) or [T][P][S][N] (PLAN_PER_EPISODE) actions
  double* rewards;            // [T][P][S] per-step rewards (plan rollouts), or null
  const int32_t* demand;      // [T][R][S] customer demand per scenario, or null: drawn in-kernel
  const double* pmf;          // [pmf_len] dfo_func weight of a customer-demand value (objective only)
  double* ep;                 // [IMENV_NUM_STATS][P][S] per-episode metrics, or null
  double* partial;            // [IMENV_NUM_STATS][P][bpp][3] per-block (sum, M2, count)
  double* terms;              // [P * bpp][TBUF][BS] parked objective terms (trees, rollout_body TBUF > 0)
  int64_t S;                  // scenarios per policy
  int64_t P;                  // policies
  int64_t bpp;                // blocks per policy = ceil(S / BS)
  uint32_t scen_offset;       // global id of scenario 0 (Philox key, sharding)
  uint32_t episode;           // Philox counter word
  int32_t pmf_len;
  int32_t noisy_delay;
  int32_t noisy_demand;
  int32_t pad_;
  uint64_t noisy_delay_thr32;
  uint64_t noisy_demand_thr32;
};

constexpr uint32_t PH_M0 = 0xD2511F53u, PH_M1 = 0xCD9E8D57u;
constexpr uint32_t PH_W0 = 0x9E3779B9u, PH_W1 = 0xBB67AE85u;
constexpr uint32_t STREAM_DEMAND = 0, STREAM_ND_DOUBLE = 1, STREAM_ND_ZERO = 2, STREAM_NOISY_DELAY = 3;

// Philox4x32-10 (Salmon et al. SC'11); oracle/philox.py is the CPU twin. Each round's two 32x32
// products are taken as 64-bit products (one v_mad_u64_u32 each instead of a mul_lo + mul_hi pair).
__device__ __forceinline__ uint4 philox4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                         uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += PH_W0; k1 += PH_W1; }
    const uint64_t p0 = (uint64_t)PH_M0 * c0;
    const uint64_t p1 = (uint64_t)PH_M1 * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return make_uint4(c0, c1, c2, c3);
}

// The episode word through the constant address space: a scalar load even where the kernel also
// stores through other pointers (the drawn-demand hand-over), which would otherwise make it a vector
// load that queues behind the step's state loads. The word is written only by the reset kernel, an
// earlier launch, so it is constant for the life of this one.
__device__ __forceinline__ uint32_t load_episode_word(const uint32_t* p) {
  return *(const __attribute__((address_space(4))) uint32_t*)(unsigned long long)p;
}

// (Round 5 tried a branch-free select on the index bits, which let the compiler issue the step's loads
// before the draw: 1.5x slower per launch in normal runs at 2^20 and 131,072 envs, yet as fast as this
// one under a rocprofv3 kernel trace, profiles/r05/ab/ab_word_select.log; not kept.)
__device__ __forceinline__ uint32_t word_of(const uint4& b, int w) {
  return w == 0 ? b.x : (w == 1 ? b.y : (w == 2 ? b.z : b.w));
}

// The env's random stream: the 32-bit word for (stream, lane, period t) of env `gid`
// in episode `ep` is word t mod 4 of Philox(counter = (gid, ep, t / 4, stream << 16 | lane), key =
// seed). lane = retailer row (demand, noisy demand) or node (noisy delay). One block serves four
// consecutive periods, so a kernel that runs whole episodes (rollout_body) draws once per 4 periods.
__device__ __forceinline__ uint4 rng_block(uint32_t gid, uint32_t ep, int t, uint32_t stream, int lane, uint32_t k0,
                                           uint32_t k1) {
  return philox4(gid, ep, (uint32_t)t >> 2, (stream << 16) | (uint32_t)lane, k0, k1);
}
__device__ __forceinline__ uint32_t rng_word(uint32_t gid, uint32_t ep, int t, uint32_t stream, int lane, uint32_t k0,
                                             uint32_t k1) {
  return word_of(rng_block(gid, ep, t, stream, lane, k0, k1), t & 3);
}
// Noisy delay draws one word per node per period: word i mod 4 of Philox(counter = (gid, ep, t,
// STREAM_NOISY_DELAY << 16 | i / 4)), so one block serves four nodes of the same period and a
// one-period kernel (the step kernel) pays one block per four nodes instead of one per node.
__device__ __forceinline__ uint4 rng_node_block(uint32_t gid, uint32_t ep, int t, uint32_t stream, int group,
                                                uint32_t k0, uint32_t k1) {
  return philox4(gid, ep, (uint32_t)t, (stream << 16) | (uint32_t)group, k0, k1);
}

// ceil(a / b) for a > 0, 1 <= b <= 8 (b = number of eligible children): the common b = 1, 2 without
// an integer division
__device__ __forceinline__ int ceil_div_pos(int a, int b) {
  if (b == 1) return a;
  if (b == 2) return (a + 1) >> 1;
  return (a + b - 1) / b;
}

// Round-robin unit shipping, closed form. Restates the reference's
//   while <cond> and amt > 0: for k in children: if x[k] > 0: s[k]+=1; x[k]-=1; amt-=1
// (IM_div_env.py:413-428, 440-450, 472-484; the inner loop does not re-check amt).
// sumcheck: the loop also requires sum(x) > 0 (backlog-first / outstanding-order loops). Without it
// (capped loop, IM_div_env.py:488-498) an env with nothing eligible spins until the guard trips.
// Phases: while the set P = {k: x[k] > 0} is fixed, every round moves |P| units, so a phase lasts
// min(min_P x, ceil(S/|P|), ceil(amt/|P|)) rounds. Returns false if the guard (rounds > lim) trips;
// rounds stop at lim+1. amt <= 0 returns true at once. sumcheck is a per-lane value so that every
// branch of the split runs this one loop (no divergent copies of it in a wave).
template <int MC>
__device__ __forceinline__ bool rr_closed(int m, int (&x)[MC], int (&s)[MC], int& amt, int lim, bool sumcheck) {
  if constexpr (MC == 2) {
    // Two children (m == 2: a split needs two), straight-line, two phases and the guard:
    //  1. both eligible: each round moves 2 units, r1 = min(x0, x1, ceil(amt / 2)) rounds (with the
    //     sum check, ceil(S / 2) >= min(x0, x1) never binds). amt may end at -1 (the reference's
    //     inner loop does not re-check amt).
    //  2. at most one eligible child c left: one unit per round, r2 = min(x_c, amt[, S]) (the other
    //     child's count is <= 0, so with the sum check S = x_c + x_other stops it first). After it,
    //     amt <= 0, S <= 0, or nothing is eligible: the loop ends, or without the sum check (the
    //     capped loop, IM_div_env.py:488-498) spins until its guard trips.
    // Rounds are capped at lim + 1 (the guard, IM_div_env.py:424-498) as the loop would be.
    // Equal to the literal loop on every (x0, x1, amt, lim, sumcheck) with x in [-4, 13], amt in
    // [-2, 31] and 8 guard limits (tools/check_rr_closed.py).
    const bool go1 = amt > 0 && (!sumcheck || x[0] + x[1] > 0);
    int r1 = min(min(min(x[0], x[1]), (amt + 1) >> 1), lim + 1);
    if (!(go1 && x[0] > 0 && x[1] > 0)) r1 = 0;
    x[0] -= r1; x[1] -= r1; s[0] += r1; s[1] += r1;
    amt -= 2 * r1;
    const bool e0 = x[0] > 0, e1 = x[1] > 0;
    const bool go2 = go1 && amt > 0 && r1 <= lim;
    int r2 = min(e0 ? x[0] : (e1 ? x[1] : 0), amt);
    if (sumcheck) r2 = min(r2, x[0] + x[1]);
    r2 = min(r2, lim + 1 - r1);
    r2 = go2 ? max(r2, 0) : 0;
    const int r2a = e0 ? r2 : 0, r2b = r2 - r2a;   // r2 == 0 when neither child is eligible: no branches
    x[0] -= r2a; s[0] += r2a;
    x[1] -= r2b; s[1] += r2b;
    amt -= r2;
    const bool trip = go2 && !sumcheck && amt > 0;
    return r1 + r2 <= lim && !trip;
  }
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
    if (sumcheck && S <= 0) break;
    if (cnt == 0) { rounds = lim + 1; break; }   // no progress possible: guard trips
    int r = min(mn, ceil_div_pos(amt, cnt));
    if (sumcheck) r = min(r, ceil_div_pos(S, cnt));
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

// ---------------------------------------------------------------- raw loads
// Loads move bytes into raw 32-bit words and nothing else: all unpacking happens after every load
// of the step has been issued, so hipcc places a single vmcnt wait at the first use instead of one
// wait per load (a wave's loads then overlap instead of paying HBM latency one after another).
template <int BYTES>
__device__ __forceinline__ void load_words(const void* __restrict__ p, uint32_t (&w)[BYTES / 4]) {
  constexpr int W = BYTES / 4;
  if constexpr (BYTES % 16 == 0) {
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
      const uint4 x = reinterpret_cast<const uint4*>(p)[q];
      w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
    }
  } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
    for (int q = 0; q < W / 2; ++q) {
      const uint2 x = reinterpret_cast<const uint2*>(p)[q];
      w[2 * q] = x.x; w[2 * q + 1] = x.y;
    }
  } else {
#pragma unroll
    for (int q = 0; q < W; ++q) w[q] = reinterpret_cast<const uint32_t*>(p)[q];
  }
}

// load_words from a buffer resource at byte offset off (lanes past the resource's range read 0)
template <int BYTES>
__device__ __forceinline__ void buf_load_words(__amdgpu_buffer_rsrc_t r, int off, uint32_t (&w)[BYTES / 4]) {
  constexpr int W = BYTES / 4;
  if constexpr (BYTES % 16 == 0) {
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * q, 0, 0);
      w[4 * q] = x[0]; w[4 * q + 1] = x[1]; w[4 * q + 2] = x[2]; w[4 * q + 3] = x[3];
    }
  } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
    for (int q = 0; q < W / 2; ++q) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, off + 8 * q, 0, 0);
      w[2 * q] = x[0]; w[2 * q + 1] = x[1];
    }
  } else {
#pragma unroll
    for (int q = 0; q < W; ++q) w[q] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * q, 0, 0);
  }
}
// a read-only resource over cnt elements of BYTES bytes from base (base and cnt wave-uniform)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ld_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <typename T>
__device__ __forceinline__ T buf_load_elem(__amdgpu_buffer_rsrc_t r, int off) {
  if constexpr (sizeof(T) == 1) return (T)__builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
  else if constexpr (sizeof(T) == 2) return (T)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
  else if constexpr (sizeof(T) == 4) {
    const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    T v;
    __builtin_memcpy(&v, &x, 4);
    return v;
  } else {
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    T v;
    __builtin_memcpy(&v, &x, 8);
    return v;
  }
}

// store_words as write-through buffer stores at byte offset off of resource r
template <int BYTES>
__device__ __forceinline__ void wt_store_words(__amdgpu_buffer_rsrc_t r, int off, const uint32_t (&w)[BYTES / 4]) {
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  constexpr int W = BYTES / 4;
  if constexpr (BYTES % 16 == 0) {
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
      const u4 x = {w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(x, r, off + 16 * q, 0, CPOL_SC1);
    }
  } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
    for (int q = 0; q < W / 2; ++q) {
      const u2 x = {w[2 * q], w[2 * q + 1]};
      __builtin_amdgcn_raw_buffer_store_b64(x, r, off + 8 * q, 0, CPOL_SC1);
    }
  } else {
#pragma unroll
    for (int q = 0; q < W; ++q) __builtin_amdgcn_raw_buffer_store_b32(w[q], r, off + 4 * q, 0, CPOL_SC1);
  }
}

template <int BYTES>
__device__ __forceinline__ void store_words(void* __restrict__ p, const uint32_t (&w)[BYTES / 4]) {
  constexpr int W = BYTES / 4;
  if constexpr (BYTES % 16 == 0) {
#pragma unroll
    for (int q = 0; q < W / 4; ++q)
      reinterpret_cast<uint4*>(p)[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
    for (int q = 0; q < W / 2; ++q) reinterpret_cast<uint2*>(p)[q] = make_uint2(w[2 * q], w[2 * q + 1]);
  } else {
#pragma unroll
    for (int q = 0; q < W; ++q) reinterpret_cast<uint32_t*>(p)[q] = w[q];
  }
}

// A packed row is N elements of ST padded to a 4-byte multiple (row_len), at base + e*row_len. EXACT
// rows (N == NT) move as whole 4/8/16-byte words (one vector instruction per lane); padded rows
// element-wise. Both forms use the same stride for a given N and element type, so kernels of either
// form can continue each other's episode. Both deliver raw words; unpack() turns them into ints.
template <int ES>
__host__ __device__ constexpr int row_len(int N) {
  return ES == 1 ? ((N + 3) & ~3) : (ES == 2 ? ((N + 1) & ~1) : N);
}

template <typename ST, int NT, bool EXACT>
struct Row {
  static constexpr int ES = (int)sizeof(ST);
  static constexpr int NPT = row_len<ES>(NT);
  static constexpr int BYTES = NPT * (int)sizeof(ST);
  static constexpr int WORDS = BYTES / 4;

  // (the np argument is unused: the stride is row_len<ES>(N), the same for every row of one type)
  __device__ static __forceinline__ void load(const ST* __restrict__ base, int64_t e, int /*np*/, int N,
                                              uint32_t (&w)[WORDS]) {
    const int np = row_len<ES>(N);
    if (EXACT || np == NPT) {
      load_words<BYTES>(base + e * NPT, w);
    } else {
#pragma unroll
      for (int q = 0; q < WORDS; ++q) w[q] = 0;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (i < N) {
          if constexpr (ES == 1) w[i >> 2] |= ((uint32_t)(uint8_t)base[e * np + i]) << ((i & 3) * 8);
          else if constexpr (ES == 2) w[i >> 1] |= ((uint32_t)(uint16_t)base[e * np + i]) << ((i & 1) * 16);
          else w[i] = (uint32_t)base[e * np + i];
        }
      }
    }
  }

  __device__ static __forceinline__ void unpack(const uint32_t (&w)[WORDS], int (&v)[NT]) {
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      if constexpr (ES == 1) v[i] = (int)(ST)(uint8_t)((w[i >> 2] >> ((i & 3) * 8)) & 0xFFu);   // sign per ST
      else if constexpr (ES == 2) v[i] = (int)(int16_t)((w[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu);
      else v[i] = (int)w[i];
    }
  }

  __device__ static __forceinline__ void load_unpacked(const ST* __restrict__ base, int64_t e, int np, int N,
                                                       int (&v)[NT]) {
    uint32_t w[WORDS];
    load(base, e, np, N, w);
    unpack(w, v);
  }

  __device__ static __forceinline__ void store(ST* __restrict__ base, int64_t e, int /*np*/, int N,
                                               const int (&v)[NT]) {
    const int np = row_len<ES>(N);
    if (EXACT || np == NPT) {
      uint32_t w[WORDS];
#pragma unroll
      for (int q = 0; q < WORDS; ++q) w[q] = 0;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int x = (i < N) ? v[i] : 0;
        if constexpr (ES == 1) w[i >> 2] |= ((uint32_t)(uint8_t)x) << ((i & 3) * 8);
        else if constexpr (ES == 2) w[i >> 1] |= ((uint32_t)(uint16_t)(int16_t)x) << ((i & 1) * 16);
        else w[i] = (uint32_t)x;
      }
      store_words<BYTES>(base + e * NPT, w);
    } else {
#pragma unroll
      for (int i = 0; i < NT; ++i) if (i < N) base[e * np + i] = (ST)v[i];
    }
  }

  // the raw words of an exact row (the inverse of unpack)
  __device__ static __forceinline__ void pack(const int (&v)[NT], uint32_t (&w)[WORDS]) {
#pragma unroll
    for (int q = 0; q < WORDS; ++q) w[q] = 0;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      if constexpr (ES == 1) w[i >> 2] |= ((uint32_t)(uint8_t)v[i]) << ((i & 3) * 8);
      else if constexpr (ES == 2) w[i >> 1] |= ((uint32_t)(uint16_t)(int16_t)v[i]) << ((i & 1) * 16);
      else w[i] = (uint32_t)v[i];
    }
  }

  // write-through form for exact rows: e0 is the wave-uniform first env, lane = e - e0
  __device__ static __forceinline__ void store_wt(ST* __restrict__ base, int64_t e0, int lane, const int (&v)[NT]) {
    uint32_t w[WORDS];
    pack(v, w);
    wt_store_words<BYTES>(wt_rsrc(base + e0 * NPT), lane * BYTES, w);
  }
};

// Inventory and backlog share one signed row: net = inv - backlog. After every step one of the two is
// zero (ship = min(backlog + demand, inv + acquisition): either the backlog is cleared or the
// inventory is used up, IM_env.py:315-340), and period 0 has no backlog, so
// inv = max(net, 0), backlog = max(-net, 0). One row read and written per step instead of two.
// The row's element is the signed twin of the state type (validate_and_derive widens the state type
// when a bound does not fit it).
template <typename ST> struct NetOf { using type = ST; };
template <> struct NetOf<uint8_t> { using type = int8_t; };
// The noisy-delay carry (arrivals deferred to the next period; a deferral can defer earlier ones again,
// so up to T shipments) is int16 beside uint8 state (validate_and_derive widens the state to int16
// when T x the state bound exceeds int16), int32 beside int16 / int32 state.
template <typename ST> struct CarryOf { using type = int32_t; };
template <> struct CarryOf<uint8_t> { using type = int16_t; };

// The split state: backlog_to of the E = nb() split children only (a single child's and the factory's
// are always 0), one row [n][E] of int16 (when the spec proves |backlog_to| <= T x the children's
// order_max fits: the only decrement below zero is the reference's double subtraction of a backlog-first
// shipment, IM_div_env.py:468-484 + 501, which is bounded by the positive part) or int32. Slot k of the
// row belongs to the node with bto_slot(node) == k. P::NBT is the compile-time capacity: the exact E for
// a JIT policy, NT for the ahead-of-time kernels (runtime E and element width).
template <class P>
struct BtoRow {
  static constexpr int CAP = P::NBT > 0 ? P::NBT : 1;
  using R16 = Row<int16_t, CAP, P::JIT>;
  using R32 = Row<int32_t, CAP, P::JIT>;
  static constexpr int WORDS = R32::WORDS;   // >= R16::WORDS
  __device__ static __forceinline__ void load(const P& p, const void* base, int64_t e, uint32_t (&w)[WORDS]) {
    const int nb = p.nb();
    if (p.bto_es() == 2) {
      uint32_t w16[R16::WORDS];
      R16::load(static_cast<const int16_t*>(base), e, nb, nb, w16);
#pragma unroll
      for (int q = 0; q < WORDS; ++q) w[q] = q < R16::WORDS ? w16[q < R16::WORDS ? q : 0] : 0u;
    } else {
      R32::load(static_cast<const int32_t*>(base), e, nb, nb, w);
    }
  }
  // node-indexed backlog_to (0 for nodes that are not split children)
  __device__ static __forceinline__ void unpack(const P& p, const uint32_t (&w)[WORDS], int (&btoc)[P::NT]) {
    int v[CAP];
    if (p.bto_es() == 2) {
      uint32_t w16[R16::WORDS];
#pragma unroll
      for (int q = 0; q < R16::WORDS; ++q) w16[q] = w[q];
      R16::unpack(w16, v);
    } else {
      R32::unpack(w, v);
    }
#pragma unroll
    for (int j = 0; j < P::NT; ++j) {
      const int k = j < p.N() ? p.bto_slot(j) : -1;
      btoc[j] = k >= 0 ? sel<CAP>(v, k) : 0;
    }
  }
  __device__ static __forceinline__ void pack(const P& p, const int (&btoc)[P::NT], int (&v)[CAP]) {
#pragma unroll
    for (int k = 0; k < CAP; ++k) v[k] = 0;
#pragma unroll
    for (int j = 0; j < P::NT; ++j) {
      const int k = j < p.N() ? p.bto_slot(j) : -1;
#pragma unroll
      for (int q = 0; q < CAP; ++q) v[q] = (k == q) ? btoc[j] : v[q];
    }
  }
  __device__ static __forceinline__ void store(const P& p, void* base, int64_t e, const int (&btoc)[P::NT]) {
    int v[CAP];
    pack(p, btoc, v);
    const int nb = p.nb();
    if (p.bto_es() == 2) R16::store(static_cast<int16_t*>(base), e, nb, nb, v);
    else R32::store(static_cast<int32_t*>(base), e, nb, nb, v);
  }
  // write-through form (exact rows: JIT policies)
  __device__ static __forceinline__ void store_wt(const P& p, void* base, int64_t e0, int lane, const int (&btoc)[P::NT]) {
    int v[CAP];
    pack(p, btoc, v);
    if (p.bto_es() == 2) R16::store_wt(static_cast<int16_t*>(base), e0, lane, v);
    else R32::store_wt(static_cast<int32_t*>(base), e0, lane, v);
  }
};

// ---------------------------------------------------------------- runtime spec policy
// Every accessor reads the spec from device memory (scalar loads). Per-call flags come from A.
template <int NT_, int MC_, bool BASE_, typename ST_>
struct DynSpec {
  static constexpr int NT = NT_;
  static constexpr int MC = MC_;
  static constexpr bool BASE = BASE_;
  static constexpr bool EXACT = NT_ <= 8;    // AOT kernels for N <= 8 are compiled for N == NT
  static constexpr bool JIT = false;
  static constexpr int TAB_LDS = IMENV_TABLE_MAX;   // Poisson table staged in LDS
  static constexpr int BS = 256;                     // threads per block
  static constexpr int EPT = 1;                      // envs per thread
  static constexpr int OBS_ROW = 0;                  // general observation rows are stored directly
  static constexpr bool OBS_STAGE64 = false;         // float64 observations are stored directly
  static constexpr int TD_PRE = 0;                   // in-transit obs slots are loaded after the step
  static constexpr bool XCD_REMAP = false;           // (step_body)
  static constexpr bool FULL = false;                // a tail block is possible (n not a multiple of the block)
  static constexpr bool INFO = true;                 // info outputs are checked per call (A.i_order)
  static constexpr bool ALIGNED = false;             // observation alignment is checked per group
  using ST = ST_;
  const SpecDev* __restrict__ sp;
  const StepArgs& A;
  __device__ DynSpec(const SpecDev* __restrict__ s, const StepArgs& a) : sp(s), A(a) {}
  __device__ int N() const { return EXACT ? NT : sp->s.num_nodes; }
  __device__ int T() const { return sp->s.num_periods; }
  __device__ int np() const { return EXACT ? Row<ST, NT, EXACT>::NPT : sp->np; }
  __device__ int D() const { return sp->dmax; }
  __device__ int factory() const { return sp->factory; }
  __device__ int num_retailers() const { return sp->s.num_retailers; }
  __device__ int prev_length() const { return sp->s.prev_length; }
  __device__ int num_features() const { return sp->s.num_features; }
  __device__ int num_split() const { return sp->num_split; }
  __device__ int delay(int i) const { return sp->s.delay[i]; }
  __device__ int ring_off(int i) const { return sp->ring_off[i]; }
  __device__ int init_inv(int i) const { return sp->s.init_inv[i]; }
  __device__ int inv_max(int i) const { return sp->s.inv_max[i]; }
  __device__ int order_max(int i) const { return sp->s.order_max[i]; }
  __device__ int backlog_cap(int i) const { return sp->s.backlog_cap[i]; }
  __device__ int retailer_slot(int i) const { return sp->s.retailer_slot[i]; }
  __device__ int demand_parent(int c) const { return sp->s.demand_parent[c]; }
  __device__ int single_parent(int c) const { return sp->single_parent[c]; }
  __device__ int split_child(int c) const { return sp->split_child[c]; }
  __device__ int split_node(int si) const { return sp->split_node[si]; }
  static constexpr int NBT = NT_;                    // backlog_to row capacity (runtime count nb())
  // state records (uint8 state, N <= 8): capacity 32 bytes, runtime size rec_words()
  static constexpr int RECW = (sizeof(ST_) == 1 && NT_ <= 8) ? 8 : 0;
  __device__ int rec_words() const { return RECW > 0 ? sp->rec_bytes / 4 : 0; }
  __device__ int dtab_es() const { return sp->dtab_es; }
  __device__ int nb() const { return sp->num_bto; }
  __device__ int bto_es() const { return sp->bto_es; }
  __device__ int bto_slot(int i) const { return sp->bto_slot[i]; }
  __device__ int num_children(int p) const { return sp->s.num_children[p]; }
  __device__ int child(int p, int k) const { return sp->s.children[p][k]; }
  __device__ int split_limit(int p, int q) const { return sp->s.split_limit[p][q]; }
  __device__ double sell(int i) const { return sp->s.sell_price[i]; }
  __device__ double buy(int i) const { return sp->s.buy_price[i]; }
  __device__ double stock_cost(int i) const { return sp->s.stock_cost[i]; }
  __device__ double backlog_cost(int i) const { return sp->s.backlog_cost[i]; }
  __device__ double inv_target(int i) const { return sp->s.inv_target[i]; }
  __device__ bool std_actions() const { return sp->s.standardise_actions != 0; }
  __device__ bool clip_round() const { return sp->s.decode_mode == IMENV_DECODE_CLIP_ROUND; }
  __device__ double a() const { return sp->s.a; }
  __device__ double bma() const { return sp->s.b - sp->s.a; }
  __device__ double inv_bma() const { return sp->inv_bma; }
  __device__ int reward_mode() const { return sp->s.reward_mode; }
  __device__ double inv_n() const { return sp->inv_n; }
  __device__ int group_mode(int g) const { return sp->s.group_mode[g]; }
  __device__ double group_den(int g, int i) const { return sp->s.group_den[g][i]; }
  __device__ double group_clip(int g, int i) const { return sp->s.group_clip[g][i]; }
  __device__ int lut_max(int g, int i) const { return sp->lut_max[g][i]; }
  __device__ int lut_off(int g, int i) const { return sp->lut_off[g][i]; }
  __device__ int feat_group(int f) const { return sp->s.feat_group[f]; }
  __device__ int feat_index(int f) const { return sp->s.feat_index[f]; }
  __device__ int demand_dist() const { return sp->s.demand_dist; }
  __device__ int uniform_low() const { return sp->s.uniform_low; }
  __device__ int uniform_high() const { return sp->s.uniform_high; }
  __device__ uint64_t seed() const { return sp->s.seed; }
  // per-call flags
  __device__ bool act_f64() const { return A.action_f64 != 0; }
  __device__ bool obs_f64() const { return A.obs_f64 != 0; }
  __device__ int demand_layout() const { return A.demand_layout; }
  __device__ bool noisy_delay() const { return A.noisy_delay != 0; }
  __device__ bool noisy_demand() const { return A.noisy_demand != 0; }
  __device__ bool has_delay_u() const { return A.delay_u != nullptr; }
  __device__ bool uses_hist() const { return A.hist_d != nullptr; }
  __device__ bool has_metrics() const { return A.metrics != nullptr; }
  // observation value of group g, node i for raw value v (table lookup, see obs_value32)
  __device__ float obs32(int g, int i, int v, const float* __restrict__ lut) const;
  __device__ double obs64(int g, int i, int v, const double* __restrict__ lut) const;
  // Poisson inversion: binary search over the LDS copy of the table
  __device__ int poisson_draw(uint32_t w, const uint32_t* s_tab) const {
    int lo = 0, hi = sp->table_len;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (w >= s_tab[mid]) lo = mid + 1; else hi = mid;
    }
    return lo;
  }
  __device__ void stage_tables(uint32_t* s_tab, bool poisson) const {
    if (poisson) {
      for (int k = threadIdx.x; k < sp->table_len; k += BS) s_tab[k] = sp->table[k];
      __syncthreads();
    }
  }
};

// Exact observation value for integer raw value v: table lookup (host-built with the same IEEE
// double expression, so bit-identical) inside the tabulated range, else computed.
template <class P>
__device__ __forceinline__ double obs_value64(const P& p, const double* __restrict__ lut, int g, int i, int v) {
  const int mx = p.lut_max(g, i);
  if (v >= 0 && v <= mx) return lut[p.lut_off(g, i) + v];
  return obs_map(p.group_mode(g), (double)v, p.a(), p.bma(), p.group_den(g, i), p.group_clip(g, i));
}
template <class P>
__device__ __forceinline__ float obs_value32(const P& p, const float* __restrict__ lut, int g, int i, int v) {
  const int mx = p.lut_max(g, i);
  if (v >= 0 && v <= mx) return lut[p.lut_off(g, i) + v];
  return (float)obs_map(p.group_mode(g), (double)v, p.a(), p.bma(), p.group_den(g, i), p.group_clip(g, i));
}

template <int NT_, int MC_, bool BASE_, typename ST_>
__device__ __forceinline__ float DynSpec<NT_, MC_, BASE_, ST_>::obs32(int g, int i, int v,
                                                                      const float* __restrict__ lut) const {
  return obs_value32(*this, lut, g, i, v);
}
template <int NT_, int MC_, bool BASE_, typename ST_>
__device__ __forceinline__ double DynSpec<NT_, MC_, BASE_, ST_>::obs64(int g, int i, int v,
                                                                       const double* __restrict__ lut) const {
  return obs_value64(*this, lut, g, i, v);
}

// ---------------------------------------------------------------- one period of one env
// The arithmetic of step() on register state (IM_env.py:287-374 and siblings), given the decoded
// orders: demand, arrivals (noisy-delay deferral decided by the caller), shipment, divergent split,
// balance equations, profit and reward. inv / bl / ou / btoc are updated in place. Shared by the
// step kernel (state in HBM rows) and the fused rollout kernel (state in registers, in-transit
// queue in LDS), so both compute one function.
// order decode (IM_env.py:298-302; MAIM_env.py:340-347). Division by b - a is replaced by an exact
// multiply when b - a is a power of two (inv_bma != 0).
template <class P>
__device__ __forceinline__ void decode_orders(const P& p, const double (&x)[P::NT], int (&order)[P::NT]) {
  constexpr int NT = P::NT;
  const int N = p.N();
  const double a = p.a();
  const double bma = p.bma();
  // A power-of-two 1 / (b - a) folds into order_max exactly: scaling by 2^k commutes with rounding, so
  // (d * om) * 2^k == d * (om * 2^k) bit for bit while no product leaves the normal range, which holds
  // when a is 0 or at least 2^-900 in magnitude (then x - a is 0 or >= 2^-953) and 2^k >= 2^-60.
  // rescale's trailing "+ 0" (rev_scale, IM_env.py:446-456) only turns -0.0 into +0.0, which the clip
  // and the integer conversion below ignore, so it is dropped. Every step is checked against the
  // reference's golden vectors and the oracle (tests/test_gpu_parity.py, tests/test_fuzz_gpu.py).
  const double ib = p.inv_bma();
  const bool fold = ib >= 0x1p-60 && (a == 0.0 || fabs(a) >= 0x1p-900);
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    order[i] = 0;
    if (i < N) {
      const double om = (double)p.order_max(i);
      double v = x[i];
      if (p.std_actions()) {
        const double d = x[i] - a;
        v = fold ? d * (om * ib) : (ib != 0.0 ? (d * om) * ib : (d * om) / bma);
      }
      const double o = p.clip_round() ? rint(fmin(fmax(v, 0.0), om)) : fmin(fmax(rint(v), 0.0), om);
      // (the ablation keeps the action load: order 0 or 1 from the action's sign, no decode arithmetic)
      order[i] = (IMENV_ABLATE & 16) ? (x[i] > 0.0 ? 1 : 0) : (int)o;
    }
  }
}

template <class P>
__device__ __forceinline__ void step_core(const P& p, const int t, const int (&order)[P::NT], const int (&cust)[P::NT],
                                          const bool (&defer)[P::NT], const int (&arr)[P::NT],
                                          const int (&cin)[P::NT], int (&inv)[P::NT], int (&bl)[P::NT],
                                          int (&ou)[P::NT], int (&btoc)[P::NT], int (&dem)[P::NT],
                                          int (&acq)[P::NT], int (&ship)[P::NT], int (&sto)[P::NT],
                                          int (&cout)[P::NT], int (&push)[P::NT], double (&prof)[P::NT],
                                          double& rew, bool& split_ok) {
  constexpr int NT = P::NT;
  constexpr int MC = P::MC;
  const int N = p.N();
  const int T = p.T();
  // demand (IM_env.py:306-308, IM_div_env.py:380-387)
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    dem[i] = 0;
    if (i < N) {
      const int r = p.retailer_slot(i);
      if (r >= 0) {
        dem[i] = min(cust[i], p.inv_max(i));
      } else {
        int s = 0;
#pragma unroll
        for (int c = 0; c < NT; ++c)
          if (c < N && p.demand_parent(c) == i) s += order[c];
        dem[i] = s;
      }
    }
  }
  // arrivals (IM_env.py:376-414); noisy delay defers the whole arrival (plus any carried amount)
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    acq[i] = ship[i] = cout[i] = 0;
    if (i < N) {
      int q = arr[i] + cin[i];
      if (defer[i] && t < T - 1) { cout[i] = q; q = 0; }
      acq[i] = q;
      ship[i] = min(bl[i] + dem[i], inv[i] + acq[i]);   // IM_env.py:315
    }
  }
  // shipments into each node: a single-child parent's whole shipment, else the split
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    sto[c] = 0;
    if (c < N) {
      const int par = p.single_parent(c);
      if (par >= 0) sto[c] = sel<NT>(ship, par);
    }
  }
  split_ok = true;
  if constexpr (MC > 0 && !(IMENV_ABLATE & 1)) {
#pragma unroll
    for (int si = 0; si < NT; ++si) {
      if (si >= p.num_split()) break;
      const int q = p.split_node(si);
      const int m = p.num_children(q);
      const int shp = sel<NT>(ship, q), dmp = sel<NT>(dem, q), blp = sel<NT>(bl, q);
      int bto[MC], oc[MC], s[MC];
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        s[k] = 0; bto[k] = 0; oc[k] = 0;
        if (k < m) {
          const int c = p.child(q, k);
          oc[k] = sel<NT>(order, c);
          bto[k] = sel<NT>(btoc, c);
        }
      }
      // the four branches of IM_div_env.py:409-502 as one straight-line sequence (per-lane choices,
      // one round-robin loop that every lane runs):
      //   A ship >= demand, backlog > 0: backlog-first loop over backlog_to, then outstanding orders
      //   B ship >= demand, no backlog:  ship_to += order                      (IM_div_env.py:457-460)
      //   C ship <  demand, backlog > 0: backlog-first loop, backlog_to += order - ship_to (:468-484, 501)
      //   D ship <  demand, no backlog:  loop capped at order + backlog_to, then the same (:486-502)
      const bool caseA = shp >= dmp && blp > 0;
      const bool caseB = shp >= dmp && blp <= 0;
      const bool caseD = shp < dmp && blp <= 0;
      int x1[MC];
#pragma unroll
      for (int k = 0; k < MC; ++k) x1[k] = caseD ? oc[k] + bto[k] : bto[k];
      int amt = caseB ? 0 : shp;
      const int lim1 = caseA ? p.split_limit(q, 0) : (caseD ? p.split_limit(q, 3) : p.split_limit(q, 2));
      // a lane with nothing to ship (amt <= 0) leaves the loop at once with x1, s and amt unchanged
      // (rounds 0 <= limit): when that holds for the whole wave, the loop is skipped (wave-uniform)
      bool ok = true;
      if (__builtin_amdgcn_ballot_w64(amt > 0) != 0) ok = rr_closed<MC>(m, x1, s, amt, lim1, !caseD);
      if (!caseD) {
#pragma unroll
        for (int k = 0; k < MC; ++k) bto[k] = x1[k];   // A and C drain backlog_to in place
      }
      // (after a guard trip in the first loop the reference has raised, "Infinite Loop 1": no state
      // follows it. The env's error flag is set; the outstanding-order loop still runs, as in the
      // oracle's non-raising restatement, so a tripped episode's later values are the oracle's too.
      // The rollout kernels, which report no per-episode errors, relied on that; plan case 400179.)
      const bool second = caseA && amt > 0 && dmp > 0;
      int out[MC];
#pragma unroll
      for (int k = 0; k < MC; ++k) out[k] = oc[k];
      int amt2 = second ? amt : 0;
      if (__builtin_amdgcn_ballot_w64(second) != 0) ok = rr_closed<MC>(m, out, s, amt2, p.split_limit(q, 1), true) && ok;
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        if (second) bto[k] += out[k];
        if (caseB) s[k] += oc[k];
        if (!caseA && !caseB) bto[k] += oc[k] - s[k];   // IM_div_env.py:501-502
      }
      split_ok = split_ok && ok;
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        if (k < m) {
          const int c = p.child(q, k);
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            sto[j] = (c == j) ? s[k] : sto[j];
            btoc[j] = (c == j) ? bto[k] : btoc[j];
          }
        }
      }
    }
  }
  // balance equations and profit (IM_env.py:318-340, 362-367)
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    prof[i] = 0.0;
    push[i] = 0;
    if (i < N) {
      int b2 = bl[i] + dem[i] - ship[i];
      if (p.backlog_cap(i) >= 0) b2 = min(b2, p.backlog_cap(i));
      const int im = p.inv_max(i);
      const int ou2 = min(max(ou[i] + order[i] - acq[i], 0), im);
      const int inv2 = min(max(inv[i] + acq[i] - ship[i], 0), im);
      // With integral prices of at most 2^12 (JIT constants), 8-bit state (0 <= ship <= inv + acq <
      // 2^8 + 2^15 with the int16 noisy-delay carry) and order_max < 2^16, sell * ship - buy * order
      // is an integer below 2^29 in magnitude that float64 holds exactly, as it holds both products:
      // the integer difference converted once is the reference's float64 difference bit for bit (one
      // conversion instead of two conversions, two products and a sum).
      const double sv = p.sell(i), bv = p.buy(i);
      const bool int_rev = P::JIT && sizeof(typename P::ST) == 1 && p.order_max(i) < 65536 && sv == rint(sv) &&
                           bv == rint(bv) && fabs(sv) <= 0x1p12 && fabs(bv) <= 0x1p12;
      const double rev = int_rev ? (double)((int)sv * ship[i] - (int)bv * order[i])
                                 : sv * (double)ship[i] - bv * (double)order[i];
      if constexpr (IMENV_ABLATE & 8) prof[i] = (double)(ship[i] - order[i]); else
      prof[i] = (rev - p.stock_cost(i) * fabs((double)inv2 - p.inv_target(i))) - p.backlog_cost(i) * (double)b2;
      bl[i] = b2; ou[i] = ou2; inv[i] = inv2;
      push[i] = (i == p.factory()) ? order[i] : sto[i];
    }
  }
  // reward (IM_env.py:372 np.sum order; MAIM_env.py:418-434)
  rew = 0.0;
  if (p.reward_mode() != IMENV_REWARD_INDEPENDENT) {
    if (p.reward_mode() == IMENV_REWARD_SHARED_MEAN || N < 8) {
#pragma unroll
      for (int i = 0; i < NT; ++i) if (i < N) rew += prof[i];
      if (p.reward_mode() == IMENV_REWARD_SHARED_MEAN) rew = (p.inv_n() != 0.0) ? rew * p.inv_n() : rew / (double)N;
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
      rew = ((r8[0] + r8[1]) + (r8[2] + r8[3])) + ((r8[4] + r8[5]) + (r8[6] + r8[7]));
#pragma unroll
      for (int i = 8; i < NT; ++i) if (i >= full && i < N) rew += prof[i];
    }
  }

}

// ---------------------------------------------------------------- step body
// Observation values per env of the block's LDS slab: the base observation [N][3] (N <= 8), or, for a
// JIT policy with a general feature list, the whole [N][F] row when the block slab fits 48 KiB
// (OBS_ROW; imenv_jit.hip picks the block size). Values are float32, or float64 for a JIT policy
// specialised for float64 observations (OBS_STAGE64); the AOT kernels stage float32 only.
template <class P>
constexpr int stage_row() {
  return (P::BASE && P::NT <= 8) ? 3 * P::NT : (!P::BASE ? P::OBS_ROW : 0);
}
// Values between consecutive envs of the slab. Each lane writes its own row. float32 rows of a multiple
// of 4 values are written and read as float4 (ds_write_b128 / ds_read_b128: 16 B per lane, no index
// arithmetic in the write-out); a multiple of 8 puts a wave's 16-byte writes on a bank period of 8
// dwords, so such rows get 4 pad values (stride = row + 4, which keeps the 16-byte alignment and
// spreads 8 consecutive lanes over all 32 banks). Other rows, and float64 rows of an even length
// (one pad value), are written value by value and gathered back into packed order.
template <class P>
constexpr int stage_stride() {
  constexpr int r = stage_row<P>();
  if (r <= 0) return r;
  if (P::OBS_STAGE64) return r % 2 == 0 ? r + 1 : r;
  return r % 8 == 0 ? r + 4 : r;
}
// One lane's float32 row into its LDS slot (16-byte stores when the row and the stride allow them).
template <int ROW, int SSTR>
__device__ __forceinline__ void lds_row_store(float* __restrict__ s, const float (&v)[ROW]) {
  if constexpr (ROW % 4 == 0 && SSTR % 4 == 0) {
#pragma unroll
    for (int q = 0; q < ROW / 4; ++q)
      reinterpret_cast<float4*>(s)[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < ROW; ++k) s[k] = v[k];
  }
}
// Whether this call's observations go through the slab (the slab's value type matches the call's).
// Write-out of a whole group's slab: QT 16-byte words, word q = lane + k * GS. The reads of up to 8
// words are issued before the first of their stores, so a lane waits for LDS once per batch (a loop
// with a runtime trip count waits once per word: ~6 serialised LDS round trips for a 24-float row).
template <int QT, int GS, class RQ, class WQ>
__device__ __forceinline__ void slab_copy(const int gl, const RQ& rq, const WQ& wq) {
  constexpr int K = (QT + GS - 1) / GS;
  constexpr int B = 8;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += B) {
    decltype(rq(0)) v[B];
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int q = gl + (k0 + j) * GS;
      if (k0 + j < K && (QT % GS == 0 || q < QT)) v[j] = rq(q);
    }
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int q = gl + (k0 + j) * GS;
      if (k0 + j < K && (QT % GS == 0 || q < QT)) wq(q, v[j]);
    }
  }
}

template <class P>
__device__ __forceinline__ bool staged_obs(const P& p) {
  return P::OBS_STAGE64 ? p.obs_f64() : !p.obs_f64();
}

// Structure: (A) issue every load that does not depend on this step's arithmetic (raw words),
// (B) compute in registers, (C) store; float32 BASE observations are staged through LDS so the
// block writes its contiguous obs slab with full 1 KiB-per-wave float4 stores.
// Per-env raw words of one step, loaded before any of them is used (step_load) so that the loads
// of all the envs a thread owns overlap; step_finish unpacks and computes.
// State records: byte b of a record held as W raw words (b wave-uniform: a kernel argument or a
// function of the period), read or replaced through the 64-bit word pair that holds it: one 64-bit
// shift and mask per byte, the pair chosen by a uniform compare. Ring bytes start at 2 NP, so pairs
// below Q0 = 2 NP / 8 never hold one (a 16-byte record of 4 nodes: pair 1 only, no compare at all).
template <int W, int Q0 = 0>
__device__ __forceinline__ uint32_t rec_byte(const uint32_t (&w)[W], int b) {
  const int k = b >> 3, sh = (b & 7) * 8;
  uint64_t c = 0;
#pragma unroll
  for (int q = Q0; q < W / 2; ++q)
    if (k == q || q == W / 2 - 1 && q == Q0) c = ((uint64_t)w[2 * q + 1] << 32) | w[2 * q];
  return (uint32_t)(c >> sh) & 0xFFu;
}
template <int W, int Q0 = 0>
__device__ __forceinline__ void rec_put(uint32_t (&w)[W], int b, uint32_t v) {
  const int k = b >> 3, sh = (b & 7) * 8;
  const uint64_t m = 0xFFull << sh, x = (uint64_t)(v & 0xFFu) << sh;
#pragma unroll
  for (int q = Q0; q < W / 2; ++q) {
    if (k == q || q == W / 2 - 1 && q == Q0) {
      const uint64_t c = ((((uint64_t)w[2 * q + 1] << 32) | w[2 * q]) & ~m) | x;
      w[2 * q] = (uint32_t)c;
      w[2 * q + 1] = (uint32_t)(c >> 32);
    }
  }
}

template <class P>
struct StepLoad {
  using R = Row<typename P::ST, P::NT, P::EXACT>;
  using RC = Row<typename CarryOf<typename P::ST>::type, P::NT, P::EXACT>;
  uint32_t aw[2 * P::NT];
  uint32_t w_net[R::WORDS], w_ou[R::WORDS], w_cin[RC::WORDS], w_bto[BtoRow<P>::WORDS];
  uint32_t w_rec[P::RECW > 0 ? P::RECW : 1];   // the env's state record (P::RECW > 0 and rec_words() > 0)
  typename P::ST r_arr[P::NT];
  int cdem[P::NT];
  double du[P::NT];
  double macc[4 + P::NT];
  typename P::ST r_td[P::NT][P::TD_PRE > 0 ? P::TD_PRE : 1];   // in-transit slots of the next obs
};

template <class P>
__device__ __forceinline__ void step_load(const P& p, const StepArgs& A, const int64_t e, StepLoad<P>& L) {
  constexpr int NT = P::NT;
  constexpr int MC = P::MC;
  constexpr bool EXACT = P::EXACT;
  using ST = typename P::ST;
  using R = Row<ST, NT, EXACT>;
  using RB = BtoRow<P>;
  using SN = typename NetOf<ST>::type;
  using RN = Row<SN, NT, EXACT>;
  const int64_t n = A.n;
  const bool valid = P::FULL || e < n;   // FULL: every block is whole (no tail lanes)
  const int N = p.N();
  const int np = p.np();
  const int t = A.t;
  const SN* __restrict__ p_net = static_cast<const SN*>(A.net);
  const ST* __restrict__ p_ou = static_cast<const ST*>(A.ou);
  const ST* __restrict__ p_ring = static_cast<const ST*>(A.ring);
  using CT = typename CarryOf<ST>::type;
  using RC = Row<CT, NT, EXACT>;
  const CT* __restrict__ p_carry = static_cast<const CT*>(A.carry);
  const void* __restrict__ p_bto = A.bto;
  // ================= (A) loads: raw words only, every independent load issued before any use
  uint32_t (&aw)[2 * NT] = L.aw;
  uint32_t (&w_net)[R::WORDS] = L.w_net;
  uint32_t (&w_ou)[R::WORDS] = L.w_ou;
  uint32_t (&w_cin)[RC::WORDS] = L.w_cin;
  uint32_t (&w_bto)[RB::WORDS] = L.w_bto;
  ST (&r_arr)[NT] = L.r_arr;
  int (&cdem)[NT] = L.cdem;
  double (&du)[NT] = L.du;
  double (&macc)[4 + NT] = L.macc;
#pragma unroll
  for (int k = 0; k < 4 + NT; ++k) macc[k] = 0.0;
#pragma unroll
  for (int q = 0; q < 2 * NT; ++q) aw[q] = 0;
#pragma unroll
  for (int q = 0; q < R::WORDS; ++q) w_net[q] = w_ou[q] = 0;
#pragma unroll
  for (int q = 0; q < RC::WORDS; ++q) w_cin[q] = 0;
#pragma unroll
  for (int q = 0; q < RB::WORDS; ++q) w_bto[q] = 0;
#pragma unroll
  for (int i = 0; i < NT; ++i) { cdem[i] = 0; du[i] = 1.0; r_arr[i] = 0; }
  const bool rec = P::RECW > 0 && p.rec_words() > 0;
#pragma unroll
  for (int q = 0; q < (P::RECW > 0 ? P::RECW : 1); ++q) L.w_rec[q] = 0;
  if constexpr (IMENV_BUF_LOAD && EXACT && P::RECW == 0) {
    // buffer loads off the slab's first env: the bases are scalars, the lane's byte offset is shared by
    // every row of one element size, and lanes past n read 0 (the resource ends at the last env), so
    // no 64-bit address arithmetic and no tail clamp
    const int lane = threadIdx.x;
    const int64_t e0 = uniform_i64(e - lane);
    const int64_t left = n - e0;
    const uint32_t cnt = (uint32_t)(left < (int64_t)P::BS ? left : (int64_t)P::BS);
    if (p.act_f64()) {
      buf_load_words<8 * NT>(ld_rsrc(static_cast<const double*>(A.actions) + e0 * NT, cnt * 8 * NT), lane * 8 * NT, aw);
    } else {
      uint32_t (&a32)[NT] = *reinterpret_cast<uint32_t(*)[NT]>(aw);
      buf_load_words<4 * NT>(ld_rsrc(static_cast<const float*>(A.actions) + e0 * NT, cnt * 4 * NT), lane * 4 * NT, a32);
    }
    buf_load_words<RN::BYTES>(ld_rsrc(p_net + e0 * RN::NPT, cnt * RN::BYTES), lane * RN::BYTES, w_net);
    buf_load_words<R::BYTES>(ld_rsrc(p_ou + e0 * R::NPT, cnt * R::BYTES), lane * R::BYTES, w_ou);
    constexpr int ES = (int)sizeof(ST);
#pragma unroll
    for (int i = 0; i < NT; ++i)
      r_arr[i] = buf_load_elem<ST>(ld_rsrc(p_ring + A.ring_at[i] + e0, cnt * ES), lane * ES);
    if (p.noisy_delay()) buf_load_words<RC::BYTES>(ld_rsrc(p_carry + e0 * RC::NPT, cnt * RC::BYTES), lane * RC::BYTES, w_cin);
    if (MC > 0) RB::load(p, p_bto, valid ? e : n - 1, w_bto);
    if (p.demand_layout() == IMENV_LAYOUT_PER_ENV) {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int r = p.retailer_slot(i);
        if (r >= 0)
          cdem[i] = buf_load_elem<int>(ld_rsrc(A.demand + ((int64_t)t * p.num_retailers() + r) * n + e0, cnt * 4), lane * 4);
      }
    }
    if (p.has_delay_u()) {
#pragma unroll
      for (int i = 0; i < NT; ++i)
        du[i] = buf_load_elem<double>(ld_rsrc(A.delay_u + ((int64_t)t * N + i) * n + e0, cnt * 8), lane * 8);
    }
    if constexpr (P::TD_PRE > 0) {   // (as below)
#pragma unroll
      for (int i = 0; i < NT; ++i) {
#pragma unroll
        for (int j = 0; j < P::TD_PRE; ++j) {
          L.r_td[i][j] = 0;
          const int d = p.delay(i);
          if (j < d - 1) {   // loaded at every period (a valid ring row), used from t = d - 1 - j on
            const ST v = buf_load_elem<ST>(ld_rsrc(p_ring + (int64_t)(p.ring_off(i) + (t + 1 + j) % d) * n + e0, cnt * ES),
                                           lane * ES);
            L.r_td[i][j] = (t + 1 + j - d >= 0) ? v : (ST)0;
          }
        }
      }
    }
    if (p.has_metrics() && t > 0) {
      const int64_t el = valid ? e : n - 1;
#pragma unroll
      for (int k = 0; k < 4 + NT; ++k) if (k < 4 + N) macc[k] = A.metrics[el * (4 + N) + k];
    }
  } else {
    // every lane loads (a tail lane re-reads the last env; only stores are guarded): no branch, so the
    // loads and the draws below share one basic block and the draws run under the loads' latency
    const int64_t el = valid ? e : n - 1;
    if (EXACT) {
      if (p.act_f64()) {
        load_words<8 * NT>(static_cast<const double*>(A.actions) + el * NT, aw);
      } else {
        uint32_t (&a32)[NT] = *reinterpret_cast<uint32_t(*)[NT]>(aw);
        load_words<4 * NT>(static_cast<const float*>(A.actions) + el * NT, a32);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (i < N) {
          if (p.act_f64()) {
            const uint2 v = reinterpret_cast<const uint2*>(static_cast<const double*>(A.actions) + el * N)[i];
            aw[2 * i] = v.x; aw[2 * i + 1] = v.y;
          } else {
            aw[i] = reinterpret_cast<const uint32_t*>(static_cast<const float*>(A.actions) + el * N)[i];
          }
        }
      }
    }
    // state and arrivals are loaded even at t == 0 (then ignored): unconditional, branch-free loads
    if constexpr (P::RECW > 0) {
      if (rec) {   // one record: net, order_u and every ring slot (unpacked in step_finish)
        const uint32_t* __restrict__ rb = static_cast<const uint32_t*>(A.net);
        if (P::RECW == 4 || p.rec_words() == 4) {
          uint32_t (&w4)[4] = *reinterpret_cast<uint32_t(*)[4]>(L.w_rec);
          load_words<16>(rb + el * 4, w4);
        } else if constexpr (P::RECW == 8) {
          load_words<32>(rb + el * 8, L.w_rec);
        }
      }
    }
    if (!rec) {
      RN::load(p_net, el, np, N, w_net);
      R::load(p_ou, el, np, N, w_ou);
#pragma unroll
      for (int i = 0; i < NT; ++i)
        if (i < N) r_arr[i] = p_ring[A.ring_at[i] + el];
    }
    if (p.noisy_delay()) RC::load(p_carry, el, np, N, w_cin);
    if (MC > 0) RB::load(p, p_bto, el, w_bto);
    if (p.demand_layout() == IMENV_LAYOUT_PER_ENV) {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int r = (i < N) ? p.retailer_slot(i) : -1;
        if (r >= 0) cdem[i] = A.demand[((int64_t)t * p.num_retailers() + r) * n + el];
      }
    } else if (p.demand_layout() == IMENV_LAYOUT_DRAW && p.dtab_es() > 0 && (t & 3) != 0) {
      // this period's drawn demand, drawn three periods ago or less by the step at the Philox block's
      // first period (step_finish): one byte / short / word per retailer instead of a block and an inversion
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int r = (i < N) ? p.retailer_slot(i) : -1;
        if (r >= 0) {
          const int64_t q = ((int64_t)t * p.num_retailers() + r) * n + el;
          if (p.dtab_es() == 1) cdem[i] = static_cast<const uint8_t*>(A.dtab)[q];
          else if (p.dtab_es() == 2) cdem[i] = static_cast<const int16_t*>(A.dtab)[q];
          else cdem[i] = static_cast<const int32_t*>(A.dtab)[q];
        }
      }
    }
    if (p.has_delay_u()) {
#pragma unroll
      for (int i = 0; i < NT; ++i) if (i < N) du[i] = A.delay_u[((int64_t)t * N + i) * n + el];
    }
    if (P::TD_PRE > 0 && !rec) {
      // time-dependent observation of period t+1: slot j < d_i - 1 of node i is ring slot
      // (t + 1 + j) mod d_i, never the slot this step overwrites (t mod d_i), so it loads here with
      // the state instead of after the step (IM_env.py:416-432); a state record holds them already
#pragma unroll
      for (int i = 0; i < NT; ++i) {
#pragma unroll
        for (int j = 0; j < P::TD_PRE; ++j) {
          L.r_td[i][j] = 0;
          if (i < N) {
            const int d = p.delay(i);
            // loaded at every period (a valid ring row), used from t = d - 1 - j on: no branch around the
            // load, so the kernel's argument loads and all of its state loads form one block
            if (j < d - 1) {
              const ST v = p_ring[(int64_t)(p.ring_off(i) + (t + 1 + j) % d) * n + el];
              L.r_td[i][j] = (t + 1 + j - d >= 0) ? v : (ST)0;
            }
          }
        }
      }
    }
    if (p.has_metrics() && t > 0) {   // period 0 starts the episode's sums from zero
#pragma unroll
      for (int k = 0; k < 4 + NT; ++k) if (k < 4 + N) macc[k] = A.metrics[el * (4 + N) + k];
    }
  }
}

// One env's step after its loads: the random draws, unpack, step_core, the stores and the next
// observation. With a staged float32 base observation the row goes to the block's LDS slab s_obs
// (written out by step_body after a barrier); every other observation is stored directly.
template <class P>
__device__ __forceinline__ void step_finish(const P& p, const StepArgs& A, const int64_t e, const StepLoad<P>& L,
                                            uint32_t* s_tab, float* s_obs) {
  constexpr int NT = P::NT;
  constexpr int MC = P::MC;
  constexpr bool EXACT = P::EXACT;
  constexpr bool STAGE = P::BASE && NT <= 8;
  constexpr int OROW = P::BASE ? 0 : P::OBS_ROW;   // general rows staged in LDS (JIT)
  using ST = typename P::ST;
  using R = Row<ST, NT, EXACT>;
  using RB = BtoRow<P>;
  using SN = typename NetOf<ST>::type;
  using RN = Row<SN, NT, EXACT>;
  const int tid = threadIdx.x;
  const int64_t n = A.n;
  const bool valid = P::FULL || e < n;
  const int N = p.N();
  const int np = p.np();
  const int t = A.t;
  // drawn demand: one Philox block gives four periods (word t & 3). With a demand table (dtab, small
  // launches) the step at a block's first period draws all four and parks the next three periods' demand
  // in the table, which the next three steps read (`cached`): three of four steps have no draw on their
  // latency chain. Without it every step draws its own word.
  const bool pre = p.demand_layout() == IMENV_LAYOUT_DRAW && p.dtab_es() > 0;
  const bool cached = pre && (t & 3) != 0;
  const bool draw_here = p.demand_layout() == IMENV_LAYOUT_DRAW && !cached;
  const bool poisson = draw_here && p.demand_dist() == IMENV_DEMAND_POISSON;
  const bool need_ep = draw_here || (p.noisy_demand() && !cached) || (p.noisy_delay() && !p.has_delay_u());
  // (diagnostic IMENV_ABLATE & 32: no scalar load of the episode word)
  const uint32_t ep = ((IMENV_ABLATE & 32) || !need_ep) ? 0u : load_episode_word(A.episode);
  const uint32_t gid = A.env_offset + (uint32_t)e;
  const uint64_t seed = p.seed();
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);

  SN* __restrict__ p_net = static_cast<SN*>(A.net);
  ST* __restrict__ p_ou = static_cast<ST*>(A.ou);
  ST* __restrict__ p_ring = static_cast<ST*>(A.ring);
  using CT = typename CarryOf<ST>::type;
  using RC = Row<CT, NT, EXACT>;
  CT* __restrict__ p_carry = static_cast<CT*>(A.carry);
  void* __restrict__ p_bto = A.bto;
  const int64_t ring_rows = n * np;   // elements per packed-row array (history)
  const uint32_t (&aw)[2 * NT] = L.aw;
  const uint32_t (&w_net)[R::WORDS] = L.w_net;
  const uint32_t (&w_ou)[R::WORDS] = L.w_ou;
  const uint32_t (&w_cin)[RC::WORDS] = L.w_cin;
  const uint32_t (&w_bto)[RB::WORDS] = L.w_bto;
  const ST (&r_arr)[NT] = L.r_arr;
  const int (&cdem)[NT] = L.cdem;
  const double (&du)[NT] = L.du;
  const double (&macc)[4 + NT] = L.macc;
  const auto& r_td = L.r_td;

  // (A2) random draws depend on no loaded value: placed before the first use of a load, they
  // execute under the loads' latency instead of after the wait
  int cdraw[NT];
  bool nd_double[NT], nd_zero[NT], nd_delay[NT];
  constexpr int NG = (NT + 3) / 4;
  uint4 dblk[NG];   // noisy delay: one block per four nodes (rng_node_block)
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    dblk[g] = make_uint4(0u, 0u, 0u, 0u);
    if (p.noisy_delay() && !p.has_delay_u() && 4 * g < N)
      dblk[g] = rng_node_block(gid, ep, t, STREAM_NOISY_DELAY, g, k0, k1);
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    cdraw[i] = 0;
    nd_double[i] = nd_zero[i] = nd_delay[i] = false;
    if (i < N) {
      const int r = p.retailer_slot(i);
      if (r >= 0) {
        if (draw_here && pre) {   // t % 4 == 0: this period's demand, the next three periods' into the table
          const uint4 b = rng_block(gid, ep, t, STREAM_DEMAND, r, k0, k1);
          uint4 b2 = make_uint4(0u, 0u, 0u, 0u), bz = b2;
          if (p.noisy_demand()) {
            b2 = rng_block(gid, ep, t, STREAM_ND_DOUBLE, r, k0, k1);
            bz = rng_block(gid, ep, t, STREAM_ND_ZERO, r, k0, k1);
          }
          int c4[4];
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const uint32_t x = word_of(b, w);
            if (poisson) {
              c4[w] = (IMENV_ABLATE & 2) ? 5 : p.poisson_draw(x, s_tab);
            } else {
              const uint64_t rng = (uint64_t)(p.uniform_high() - p.uniform_low());
              c4[w] = p.uniform_low() + (int)(((uint64_t)x * rng) >> 32);
            }
            if (p.noisy_demand()) {   // IM_div_env.py:246-255: double, then zero
              if ((uint64_t)word_of(b2, w) < A.noisy_demand_thr32) c4[w] = 2 * c4[w];
              if ((uint64_t)word_of(bz, w) < A.noisy_demand_thr32) c4[w] = 0;
            }
          }
          cdraw[i] = c4[0];
          if (P::FULL || e < n) {
#pragma unroll
            for (int w = 1; w < 4; ++w) {
              if (t + w < p.T()) {
                const int64_t q = ((int64_t)(t + w) * p.num_retailers() + r) * n + e;
                if (p.dtab_es() == 1) static_cast<uint8_t*>(A.dtab)[q] = (uint8_t)c4[w];
                else if (p.dtab_es() == 2) static_cast<int16_t*>(A.dtab)[q] = (int16_t)c4[w];
                else static_cast<int32_t*>(A.dtab)[q] = c4[w];
              }
            }
          }
        } else if (draw_here) {
          const uint32_t w = rng_word(gid, ep, t, STREAM_DEMAND, r, k0, k1);
          if (poisson) {
            cdraw[i] = (IMENV_ABLATE & 2) ? 5 : p.poisson_draw(w, s_tab);
          } else {
            const uint64_t rng = (uint64_t)(p.uniform_high() - p.uniform_low());
            cdraw[i] = p.uniform_low() + (int)(((uint64_t)w * rng) >> 32);
          }
        }
        if (p.noisy_demand() && !pre) {   // (with a table, the draw above applied it, or the table holds it)
          const uint32_t wd = rng_word(gid, ep, t, STREAM_ND_DOUBLE, r, k0, k1);
          const uint32_t wz = rng_word(gid, ep, t, STREAM_ND_ZERO, r, k0, k1);
          nd_double[i] = (uint64_t)wd < A.noisy_demand_thr32;
          nd_zero[i] = (uint64_t)wz < A.noisy_demand_thr32;
        }
      }
      if (p.noisy_delay() && !p.has_delay_u() && t >= p.delay(i))
        nd_delay[i] = (uint64_t)word_of(dblk[i >> 2], i & 3) < A.noisy_delay_thr32;
    }
  }

  // unpack (first use of the loaded words)
  double x[NT];
  int inv[NT], bl[NT], ou[NT], arr[NT], cin[NT], btoc[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (p.act_f64()) x[i] = __hiloint2double((int)aw[2 * i + 1], (int)aw[2 * i]);
    else x[i] = (double)__uint_as_float(aw[i]);
  }
  // a state record (small launches) holds the net and order_u rows as its first words and every ring
  // slot after them: the arrival of node i is the byte the host names in ring_at[i]
  constexpr int RECW = P::RECW > 0 ? P::RECW : 1;
  const bool rec = P::RECW > 0 && p.rec_words() > 0;
  [[maybe_unused]] const uint32_t (&w_rec)[RECW] = L.w_rec;
  uint32_t wn[R::WORDS], wo[R::WORDS];
  ST ra[NT];
  [[maybe_unused]] ST rtd[NT][P::TD_PRE > 0 ? P::TD_PRE : 1];
#pragma unroll
  for (int q = 0; q < R::WORDS; ++q) {
    wn[q] = w_net[q];
    wo[q] = w_ou[q];
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    ra[i] = r_arr[i];
#pragma unroll
    for (int j = 0; j < (P::TD_PRE > 0 ? P::TD_PRE : 1); ++j) rtd[i][j] = r_td[i][j];
  }
  if constexpr (P::RECW > 0) {
    if (rec) {
      constexpr int RW = R::WORDS;   // = NP / 4 (uint8 rows, N == NT)
#pragma unroll
      for (int q = 0; q < RW; ++q) {
        wn[q] = w_rec[q];
        wo[q] = w_rec[RW + q];
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        ra[i] = (ST)rec_byte<RECW, RW>(w_rec, (int)A.ring_at[i]);
#pragma unroll
        for (int j = 0; j < P::TD_PRE; ++j) {
          rtd[i][j] = 0;
          const int d = p.delay(i);
          if (j < d - 1 && t + 1 + j - d >= 0)
            rtd[i][j] = (ST)rec_byte<RECW, RW>(w_rec, 8 * RW + p.ring_off(i) + (t + 1 + j) % d);
        }
      }
    }
  }
  RN::unpack(wn, inv);
#pragma unroll
  for (int i = 0; i < NT; ++i) {   // net -> (inv, backlog): one of them is 0
    bl[i] = max(-inv[i], 0);
    inv[i] = max(inv[i], 0);
  }
  R::unpack(wo, ou);
#pragma unroll
  for (int i = 0; i < NT; ++i) arr[i] = (int)ra[i];
  RC::unpack(w_cin, cin);
  if constexpr (MC > 0) RB::unpack(p, w_bto, btoc);
  else {
#pragma unroll
    for (int i = 0; i < NT; ++i) btoc[i] = 0;
  }
  if (t == 0) {              // period-0 state is implicit (IM_env.py:221-224); one uniform branch
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      inv[i] = (i < N) ? p.init_inv(i) : 0;
      bl[i] = ou[i] = cin[i] = btoc[i] = 0;
    }
  }
#pragma unroll
  for (int i = 0; i < NT; ++i)
    if (i >= N || t < p.delay(i < N ? i : 0)) arr[i] = 0;   // nothing shipped d periods ago yet

  // per-period inputs that do not come from the state rows: customer demand (layout + noise) and
  // the noisy-delay deferral decision
  int cust[NT];
  bool defer[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    cust[i] = 0;
    defer[i] = false;
    if (i < N) {
      const int r = p.retailer_slot(i);
      if (r >= 0) {
        int cd;
        if (p.demand_layout() == IMENV_LAYOUT_PER_ENV || cached) cd = cdem[i];
        else if (p.demand_layout() == IMENV_LAYOUT_BROADCAST) cd = A.demand[t * p.num_retailers() + r];
        else cd = cdraw[i];
        if (p.noisy_demand() && !pre) {   // IM_div_env.py:246-255: double, then zero
          if (nd_double[i]) cd = 2 * cd;
          if (nd_zero[i]) cd = 0;
        }
        cust[i] = cd;
      }
      if (p.noisy_delay() && t >= p.delay(i)) defer[i] = p.has_delay_u() ? (du[i] <= A.noisy_delay_thr) : nd_delay[i];
    }
  }

  // ================= (B) compute
  int order[NT], dem[NT], acq[NT], ship[NT], sto[NT], cout[NT], push[NT];
  double prof[NT];
  double rew;
  bool split_ok;
  decode_orders(p, x, order);
  step_core(p, t, order, cust, defer, arr, cin, inv, bl, ou, btoc, dem, acq, ship, sto, cout, push, prof, rew,
            split_ok);

  // ================= (C) stores
  if (valid) {
    int net[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) net[i] = inv[i] - bl[i];   // inv[i] * bl[i] == 0 after step_core
    bool state_done = false;
    if constexpr (P::RECW > 0) {
      if (rec) {   // the whole record back: new rows, this step's departures in their ring slots
        constexpr int RW = R::WORDS;
        uint32_t wr[RECW], pn[RW], po[RW];
#pragma unroll
        for (int q = 0; q < RECW; ++q) wr[q] = w_rec[q];
        RN::pack(net, pn);
        R::pack(ou, po);
#pragma unroll
        for (int q = 0; q < RW; ++q) {
          wr[q] = pn[q];
          wr[RW + q] = po[q];
        }
#pragma unroll
        for (int i = 0; i < NT; ++i)
          if (i < N) rec_put<RECW, RW>(wr, (int)A.ring_at[i], (uint32_t)push[i]);
        uint32_t* __restrict__ rb = static_cast<uint32_t*>(A.net);
        if (P::RECW == 4 || p.rec_words() == 4) {
          const uint32_t (&w4)[4] = *reinterpret_cast<const uint32_t(*)[4]>(wr);
          if constexpr (IMENV_WT_STATE) wt_store_words<16>(wt_rsrc(rb + uniform_i64(e - tid) * 4), tid * 16, w4);
          else store_words<16>(rb + e * 4, w4);
        } else if constexpr (P::RECW == 8) {
          if constexpr (IMENV_WT_STATE) wt_store_words<32>(wt_rsrc(rb + uniform_i64(e - tid) * 8), tid * 32, wr);
          else store_words<32>(rb + e * 8, wr);
        }
        state_done = true;
      }
    }
    if (state_done) {
      if (p.noisy_delay()) RC::store(p_carry, e, np, N, cout);
      if constexpr (MC > 0) RB::store(p, p_bto, e, btoc);
    } else if constexpr (IMENV_WT_STATE && EXACT) {
      const int64_t e0 = uniform_i64(e - tid);
      RN::store_wt(p_net, e0, tid, net);
      R::store_wt(p_ou, e0, tid, ou);
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const auto rr = wt_rsrc(p_ring + A.ring_at[i] + e0);
        if constexpr (sizeof(ST) == 1) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)push[i], rr, tid, 0, CPOL_SC1);
        else if constexpr (sizeof(ST) == 2) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)push[i], rr, 2 * tid, 0, CPOL_SC1);
        else __builtin_amdgcn_raw_buffer_store_b32((uint32_t)push[i], rr, 4 * tid, 0, CPOL_SC1);
      }
      if (p.noisy_delay()) RC::store_wt(p_carry, e0, tid, cout);
      if constexpr (MC > 0) {
        if constexpr (P::JIT) RB::store_wt(p, p_bto, e0, tid, btoc);
        else RB::store(p, p_bto, e, btoc);
      }
    } else {
      RN::store(p_net, e, np, N, net);
      R::store(p_ou, e, np, N, ou);
#pragma unroll
      for (int i = 0; i < NT; ++i)
        if (i < N) p_ring[A.ring_at[i] + e] = (ST)push[i];
      if (p.noisy_delay()) RC::store(p_carry, e, np, N, cout);
      if constexpr (MC > 0) RB::store(p, p_bto, e, btoc);
    }
    if (!split_ok) {          // no-return atomics
      atomicOr(A.err + e, 1u);
      atomicOr(A.err_any, 1u);
    }
    if (p.uses_hist()) {
      const int L = p.prev_length();
      R::store(static_cast<ST*>(A.hist_d) + (int64_t)(t % L) * ring_rows, e, np, N, dem);
      R::store(static_cast<ST*>(A.hist_o) + (int64_t)(t % L) * ring_rows, e, np, N, order);
    }
    if (p.reward_mode() == IMENV_REWARD_INDEPENDENT) {
#pragma unroll
      for (int i = 0; i < NT; ++i) if (i < N) A.reward[e * N + i] = prof[i];
    } else if constexpr (IMENV_NT_STORE) {
      __builtin_nontemporal_store(rew, A.reward + e);
    } else if constexpr (IMENV_WT_STORE) {
      const int64_t e0 = uniform_i64(e - tid);     // the block's first env of this slab
      wt_store8(wt_rsrc(A.reward + e0), tid * 8, rew);
    } else {
      A.reward[e] = rew;
    }
    if (p.has_metrics()) {
      // the reference's evaluation harness, per env (inv_management.py:586-597, MA_inv_management.py:559-572,
      // MA_inv_management_div.py:540-553): episode_reward += reward (each agent's, in agent order, for
      // the multi-agent envs); per step, the sum over agents of rev_scale(obs[m][0 | 1], 0, inv_max[m], a, b)
      // from the float64 observation; customer backlog from agent 0's; stage_rewards[m] += profit[m]
      const double a = p.a(), bma = p.bma();
      double r0 = macc[0];
      if (p.reward_mode() == IMENV_REWARD_SUM) {
        r0 += rew;
      } else {
#pragma unroll
        for (int i = 0; i < NT; ++i)
          if (i < N) r0 += (p.reward_mode() == IMENV_REWARD_SHARED_MEAN) ? rew : prof[i];
      }
      double si = 0.0, sb = 0.0, c0 = 0.0;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (i < N) {
          const double im = (double)p.inv_max(i) - 0.0;
          const double ri = ((p.obs64(IMENV_G_INV, i, inv[i], A.lut64) - a) * im) / bma + 0.0;
          const double rb = ((p.obs64(IMENV_G_BACKLOG, i, bl[i], A.lut64) - a) * im) / bma + 0.0;
          si += ri;
          sb += rb;
          if (i == 0) c0 = rb;
        }
      }
      double* row = A.metrics + e * (4 + N);
      row[0] = r0;
      row[1] = macc[1] + si;
      row[2] = macc[2] + sb;
      row[3] = macc[3] + c0;
#pragma unroll
      for (int i = 0; i < NT; ++i) if (i < N) row[4 + i] = macc[4 + i] + prof[i];
    }
    if (P::INFO && A.i_order) {   // info (IM_env.py:345-350); a JIT kernel without info has no such code
#pragma unroll
      for (int i = 0; i < NT; ++i) if (i < N) {
        A.i_order[e * N + i] = order[i];
        if (A.i_demand) A.i_demand[e * N + i] = dem[i];
        if (A.i_acq) A.i_acq[e * N + i] = acq[i];
        if (A.i_ship) A.i_ship[e * N + i] = ship[i];
        if (A.i_profit) A.i_profit[e * N + i] = prof[i];
        if (A.i_ship_to) A.i_ship_to[e * N + i] = sto[i];
        if (A.i_bto) A.i_bto[e * N + i] = p.split_child(i) ? btoc[i] : 0;
      }
    }
  }

  // observation for period t+1 (IM_env.py:231-285, MAIM_env.py:242-328, IM_div_env.py:304-359,
  // MAIM_div_env.py:343-439)
  if constexpr (P::BASE) {
    if (STAGE && staged_obs(p)) {
      constexpr int row = stage_stride<P>();
      [[maybe_unused]] float rv32[3 * NT];   // the env's float32 row, stored to LDS in one go
      if (valid) {
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          if (i < N) {
            if constexpr (P::OBS_STAGE64) {
              double* sd = reinterpret_cast<double*>(s_obs);
              sd[tid * row + 3 * i + 0] = p.obs64(IMENV_G_INV, i, inv[i], A.lut64);
              sd[tid * row + 3 * i + 1] = p.obs64(IMENV_G_BACKLOG, i, bl[i], A.lut64);
              sd[tid * row + 3 * i + 2] = p.obs64(IMENV_G_ORDER_U, i, ou[i], A.lut64);
            } else {
              rv32[3 * i + 0] = p.obs32(IMENV_G_INV, i, inv[i], A.lut32);
              rv32[3 * i + 1] = p.obs32(IMENV_G_BACKLOG, i, bl[i], A.lut32);
              rv32[3 * i + 2] = p.obs32(IMENV_G_ORDER_U, i, ou[i], A.lut32);
            }
          }
        }
        if constexpr (!P::OBS_STAGE64) lds_row_store<3 * NT, row>(s_obs + tid * row, rv32);
      }
    } else if (valid) {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (i < N) {
          const int64_t base = (e * N + i) * 3;
          if (p.obs_f64()) {
            double* o = static_cast<double*>(A.obs);
            o[base + 0] = p.obs64(IMENV_G_INV, i, inv[i], A.lut64);
            o[base + 1] = p.obs64(IMENV_G_BACKLOG, i, bl[i], A.lut64);
            o[base + 2] = p.obs64(IMENV_G_ORDER_U, i, ou[i], A.lut64);
          } else {
            float* o = static_cast<float*>(A.obs);
            o[base + 0] = p.obs32(IMENV_G_INV, i, inv[i], A.lut32);
            o[base + 1] = p.obs32(IMENV_G_BACKLOG, i, bl[i], A.lut32);
            o[base + 2] = p.obs32(IMENV_G_ORDER_U, i, ou[i], A.lut32);
          }
        }
      }
    }
  } else if (valid) {
    const int F = p.num_features();
    const int L = p.prev_length();
    const int tp = t + 1;   // observation period
    [[maybe_unused]] float rv32[OROW > 0 ? OROW : 1];   // staged float32 row (JIT: constant indices)
    auto feature = [&](const int f) {
      const int g = p.feat_group(f);
      const int j = p.feat_index(f);
      int v[NT];
#pragma unroll
      for (int i = 0; i < NT; ++i) v[i] = 0;
      if (g == IMENV_G_INV) {
#pragma unroll
        for (int i = 0; i < NT; ++i) v[i] = inv[i];
      } else if (g == IMENV_G_BACKLOG) {
#pragma unroll
        for (int i = 0; i < NT; ++i) v[i] = bl[i];
      } else if (g == IMENV_G_ORDER_U) {
#pragma unroll
        for (int i = 0; i < NT; ++i) v[i] = ou[i];
      } else if (g == IMENV_G_DEMAND_HIST || g == IMENV_G_ORDER_HIST) {
        const int pr = tp - 1 - j;     // period of the entry; 0 when j >= tp
        if (pr >= 0) {
          if (j == 0) {
#pragma unroll
            for (int i = 0; i < NT; ++i) v[i] = (g == IMENV_G_DEMAND_HIST) ? dem[i] : order[i];
          } else {
            const ST* h = static_cast<const ST*>(g == IMENV_G_DEMAND_HIST ? A.hist_d : A.hist_o);
            R::load_unpacked(h + (int64_t)(pr % L) * ring_rows, e, np, N, v);
          }
        }
      } else if (g == IMENV_G_TRANSIT) {
        // slot j: amount arriving at period tp + j, shipped at tp + j - d_i (IM_env.py:416-432);
        // it sits in node i's ring slot (tp + j) mod d_i, except j = d_i - 1: this step's shipment
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          const int d = (i < N) ? p.delay(i) : 1;
          v[i] = 0;
          if (i < N && j < d && tp + j - d >= 0) {
            if (j == d - 1) {
              v[i] = push[i];
            } else if constexpr (P::TD_PRE > 0) {
#pragma unroll
              for (int q = 0; q < P::TD_PRE; ++q) if (q == j) v[i] = (int)rtd[i][q];
            } else if (rec) {
              if constexpr (P::RECW > 0)
                v[i] = (int)rec_byte<RECW, Row<ST, NT, EXACT>::WORDS>(w_rec, 2 * p.np() + p.ring_off(i) + (tp + j) % d);
            } else {
              v[i] = (int)p_ring[(int64_t)(p.ring_off(i) + (tp + j) % d) * n + e];
            }
          }
        }
      } else if (g == IMENV_G_NODE_ID) {
#pragma unroll
        for (int i = 0; i < NT; ++i) v[i] = i;
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (i < N) {
          const int64_t idx = (e * N + i) * F + f;
          if (p.obs_f64()) {
            if constexpr (OROW > 0 && P::OBS_STAGE64)
              reinterpret_cast<double*>(s_obs)[tid * stage_stride<P>() + i * F + f] = p.obs64(g, i, v[i], A.lut64);
            else
              static_cast<double*>(A.obs)[idx] = p.obs64(g, i, v[i], A.lut64);
          } else if constexpr (OROW > 0 && !P::OBS_STAGE64) {
            rv32[i * F + f] = p.obs32(g, i, v[i], A.lut32);
          } else {
            static_cast<float*>(A.obs)[idx] = p.obs32(g, i, v[i], A.lut32);
          }
        }
      }
    };
    if constexpr (P::JIT) {   // feature list is a compile-time constant: unroll it
#pragma unroll
      for (int f = 0; f < F; ++f) feature(f);
    } else {
#pragma unroll 1
      for (int f = 0; f < F; ++f) feature(f);
    }
    if constexpr (OROW > 0 && !P::OBS_STAGE64) {
      if (!p.obs_f64()) lds_row_store<OROW, stage_stride<P>()>(s_obs + tid * stage_stride<P>(), rv32);
    }
  }
}

// The step kernel body: each thread owns P::EPT envs, one per BS-env slab of the block's EPT*BS
// envs (env = (blockIdx * EPT + k) * BS + tid). Every load of every owned env is issued first, then
// each env is finished in turn; a staged float32 base observation is written out slab by slab as
// contiguous float4 runs after one barrier.
template <class P>
__device__ __forceinline__ void step_body(const P& p, const StepArgs& A, uint32_t* s_tab, float* s_obs) {
  constexpr int BS = P::BS;
  constexpr int EPT = P::EPT;
  constexpr int SROW = stage_row<P>();   // LDS floats per env (0: observations stored directly)
  const int tid = threadIdx.x;
  const int64_t n = A.n;
  // XCD-aware env chunks (IMENV_XCD_REMAP=1, small-block launches): blocks go round-robin to the 8
  // XCDs (block b to XCD b mod 8), each with its own L2. A 64-env block's 1-byte ring rows are half a
  // 128-byte line, so two neighbouring chunks on different XCDs both fetch the line. Chunk
  // c = (b mod 8) * G/8 + b / 8 puts chunks c and c + 1 on one XCD (a bijection when 8 divides the
  // grid G). It removes those fetches (C4: 6.54 -> 5.90 MB read per launch) but the launch gets slower
  // (5.64 -> 6.04 us, C2 at 131,072 4.20 -> 4.52 us; profiles/r03/xcd_remap/): off by default.
  int64_t bid = blockIdx.x;
  if constexpr (P::XCD_REMAP && IMENV_XCD_REMAP) {
    const int64_t G = gridDim.x;
    if ((G & 7) == 0) bid = (bid & 7) * (G >> 3) + (bid >> 3);
  }
  const int64_t eb = bid * EPT * BS;
  const bool poisson = p.demand_layout() == IMENV_LAYOUT_DRAW && p.demand_dist() == IMENV_DEMAND_POISSON;
  // diagnostic phase stamps (IMENV_STAMPS builds, 10 ns ticks of s_memrealtime): 0 entry, 1 loads issued,
  // 2 loads landed (an added vmcnt(0) wait), 3 computed, 4 after the slab barrier, 5 stores issued,
  // 6 stores acknowledged
  [[maybe_unused]] uint64_t stamp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (IMENV_STAMPS) stamp[0] = __builtin_amdgcn_s_memrealtime();
  if constexpr (IMENV_PRIO > 0) {
    // Two waves per SIMD run the same phases in lockstep (load, compute, store). With one of them at a
    // higher issue priority it finishes its arithmetic first and its stores overlap the other's
    // arithmetic (MI355X_MICROARCH.md, "Two waves per SIMD", item 4). HW_ID bits 3:0 = wave slot.
    const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (3 << 11));
    if (hw & 1u) __builtin_amdgcn_s_setprio(IMENV_PRIO);
  }
  StepLoad<P> L[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) step_load(p, A, eb + k * BS + tid, L[k]);
#ifndef IMENV_LOAD_FENCE
#define IMENV_LOAD_FENCE 1
#endif
  // Issue the loads here when the drawn-demand hand-over is on: the compiler otherwise places them after
  // the t % 4 == 0 branch that draws four periods, behind the episode word's load and the draw (C2 at
  // 131,072 envs: 3.89 -> 3.77 us per launch). Elsewhere the fence costs (C4 5.51 -> 5.83 us, C2 at 2^20
  // 18.5 -> 19.1: profiles/r05/ab/ab_load_fence.log), so only hipRTC kernels with the table get it
  // (IMENV_LOAD_FENCE=0: A/B through IMENV_JIT_OPTS)
  if constexpr (IMENV_LOAD_FENCE && P::JIT) {
    if (p.demand_layout() == IMENV_LAYOUT_DRAW && p.dtab_es() > 0) asm volatile("" ::: "memory");
  }
  p.stage_tables(s_tab, poisson);
  constexpr int SSTR = stage_stride<P>();
  constexpr int SLAB = BS * SSTR * (P::OBS_STAGE64 ? 2 : 1);   // floats per BS-env slab
  if constexpr (IMENV_STAMPS) {
    stamp[1] = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp[2] = __builtin_amdgcn_s_memrealtime();
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) step_finish(p, A, eb + k * BS + tid, L[k], s_tab, s_obs + k * SLAB);
  if constexpr (IMENV_STAMPS) stamp[3] = __builtin_amdgcn_s_memrealtime();
  // Write-out group: the block (one barrier), or with IMENV_WAVE_SLAB each wave on its own (the 64 rows
  // it staged itself: LDS ops of one wave complete in order, so a wavefront fence replaces the block
  // barrier and no wave waits for its block's slowest wave)
  constexpr int GS = IMENV_WAVE_SLAB ? 64 : BS;
  [[maybe_unused]] const int gl = tid % GS, gi = tid / GS;
  if constexpr (SROW > 0) {
    if (staged_obs(p)) {
      if constexpr (IMENV_WAVE_SLAB) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else {
        __syncthreads();
      }
    }
  }
  if constexpr (IMENV_STAMPS) stamp[4] = __builtin_amdgcn_s_memrealtime();
  if constexpr (SROW > 0 && P::OBS_STAGE64) {
    // float64 rows: the same write-out in 16-byte double2 runs
    if (staged_obs(p)) {
      constexpr int row = SROW;
      auto at = [](const double* so, int q) { return so[(q / row) * SSTR + q % row]; };
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int64_t e0 = eb + k * BS + gi * GS;
        if (P::FULL || e0 < n) {
          const int cnt = (P::FULL || (n - e0) >= GS) ? GS : (int)(n - e0);
          const int total = cnt * row;
          double* gobs = static_cast<double*>(A.obs) + e0 * row;
          const double* so = reinterpret_cast<const double*>(s_obs + k * SLAB) + gi * GS * SSTR;
          // 16-byte stores need a 16-byte aligned destination (a caller's obs_out view may be offset)
          // (ALIGNED: the host checked the observation buffer's 16-byte alignment for this kernel; every
          // group's run then starts on a 16-byte boundary, so the value-by-value fallback is not compiled)
          if (P::ALIGNED || ((total & 1) == 0 && (reinterpret_cast<unsigned long long>(gobs) & 15) == 0)) {
            double2* g2 = reinterpret_cast<double2*>(gobs);
            if (IMENV_SLAB_BATCH && cnt == GS) {   // a whole group (as the float32 write-out below)
              constexpr int QT = row * GS / 2;
              auto rq = [&](int q) { return make_double2(at(so, 2 * q), at(so, 2 * q + 1)); };
              if constexpr (IMENV_WT_STORE) {
                const auto rs = wt_rsrc(uniform_ptr(gobs));
                slab_copy<QT, GS>(gl, rq, [&](int q, const double2& v) { wt_store16(rs, q * 16, v); });
              } else {
                slab_copy<QT, GS>(gl, rq, [&](int q, const double2& v) { store16<IMENV_NT_STORE>(g2 + q, v); });
              }
            } else if constexpr (IMENV_WT_STORE) {
              const auto rs = wt_rsrc(uniform_ptr(gobs));
              for (int q = gl; q < total / 2; q += GS) wt_store16(rs, q * 16, make_double2(at(so, 2 * q), at(so, 2 * q + 1)));
            } else {
              for (int q = gl; q < total / 2; q += GS)
                store16<IMENV_NT_STORE>(g2 + q, make_double2(at(so, 2 * q), at(so, 2 * q + 1)));
            }
          } else {
            for (int q = gl; q < total; q += GS) gobs[q] = at(so, q);
          }
        }
      }
    }
  } else if constexpr (SROW > 0) {
    // (staged rows: SROW == 3 N for the base layout, as N == NT whenever it is staged)
    if (staged_obs(p)) {
      constexpr int row = SROW;
      auto at = [](const float* so, int q) { return so[(q / row) * SSTR + q % row]; };   // packed -> slab
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int64_t e0 = eb + k * BS + gi * GS;
        if (P::FULL || e0 < n) {
          const int cnt = (P::FULL || (n - e0) >= GS) ? GS : (int)(n - e0);
          const int total = cnt * row;
          float* gobs = static_cast<float*>(A.obs) + e0 * row;
          const float* so = s_obs + k * SLAB + gi * GS * SSTR;
          if (P::ALIGNED || ((total & 3) == 0 && (reinterpret_cast<unsigned long long>(gobs) & 15) == 0)) {
            float4* g4 = reinterpret_cast<float4*>(gobs);
            // 16-byte word q of the group's contiguous output, read from the slab
            auto rq = [&](int q) -> float4 {
              if constexpr (SSTR == row) return reinterpret_cast<const float4*>(so)[q];
              else if constexpr (row % 4 == 0 && SSTR % 4 == 0)   // (q / R) * SSTR + (q % R) * 4, R = row / 4
                return *reinterpret_cast<const float4*>(so + 4 * q + (SSTR - row) * (q / (row / 4)));
              else return make_float4(at(so, 4 * q), at(so, 4 * q + 1), at(so, 4 * q + 2), at(so, 4 * q + 3));
            };
            if (IMENV_SLAB_BATCH && cnt == GS) {
              // a whole group: QT words at compile time, every LDS read of a batch issued before its
              // first store (one LDS wait per batch instead of one per word)
              constexpr int QT = row * GS / 4;
              if constexpr (IMENV_WT_STORE) {
                const auto rs = wt_rsrc(uniform_ptr(gobs));
                slab_copy<QT, GS>(gl, rq, [&](int q, const float4& v) { wt_store16(rs, q * 16, v); });
              } else {
                slab_copy<QT, GS>(gl, rq, [&](int q, const float4& v) { store16<IMENV_NT_STORE>(g4 + q, v); });
              }
            } else if constexpr (IMENV_WT_STORE) {
              const auto rs = wt_rsrc(uniform_ptr(gobs));
              if constexpr (SSTR == row) {
                const float4* s4 = reinterpret_cast<const float4*>(so);
                for (int q = gl; q < total / 4; q += GS) wt_store16(rs, q * 16, s4[q]);
              } else if constexpr (row % 4 == 0 && SSTR % 4 == 0) {
                for (int q = gl; q < total / 4; q += GS)
                  wt_store16(rs, q * 16, *reinterpret_cast<const float4*>(so + (q / (row / 4)) * SSTR + (q % (row / 4)) * 4));
              } else {
                for (int q = gl; q < total / 4; q += GS)
                  wt_store16(rs, q * 16, make_float4(at(so, 4 * q), at(so, 4 * q + 1), at(so, 4 * q + 2), at(so, 4 * q + 3)));
              }
            } else if constexpr (SSTR == row) {
              const float4* s4 = reinterpret_cast<const float4*>(so);
              for (int q = gl; q < total / 4; q += GS) store16<IMENV_NT_STORE>(g4 + q, s4[q]);
            } else if constexpr (row % 4 == 0 && SSTR % 4 == 0) {
              for (int q = gl; q < total / 4; q += GS)
                store16<IMENV_NT_STORE>(g4 + q, *reinterpret_cast<const float4*>(so + (q / (row / 4)) * SSTR +
                                                                                  (q % (row / 4)) * 4));
            } else {
              for (int q = gl; q < total / 4; q += GS)
                store16<IMENV_NT_STORE>(g4 + q, make_float4(at(so, 4 * q), at(so, 4 * q + 1), at(so, 4 * q + 2),
                                                            at(so, 4 * q + 3)));
            }
          } else {
            for (int q = gl; q < total; q += GS) gobs[q] = at(so, q);
          }
        }
      }
    }
  }
  if constexpr (IMENV_STAMPS) {
    stamp[5] = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp[6] = __builtin_amdgcn_s_memrealtime();
    stamp[7] = ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) << 32) | blockIdx.x;  // XCC id
    if (A.stamps && (tid & 63) == 0) {
      uint64_t* o = A.stamps + ((int64_t)blockIdx.x * (BS / 64) + tid / 64) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = stamp[k];
    }
  }
}

// ---------------------------------------------------------------- fused base-stock rollout
// One thread = one (policy, scenario) episode of T periods: base_restock_policy.py:24-45
// (dfo_func) with the order-up-to policy of :4-21, evaluated through the same step_core as the
// step kernel. State lives in registers for the whole episode; the lead-time queue (node i's d_i
// in-transit slots) lives in LDS as [slot][thread] int32 (a wave's access is 64 consecutive
// dwords: conflict-free), as do the Poisson table and the pmf weights. Metrics per episode:
//   RETURN     sum_t reward, accumulated as the reference's eval loop does (inv_management.py:226-231)
//   OBJECTIVE  dfo_func: -1/T * np.sum(pmf(customer_demand) * rewards), in np.sum's pairwise order
//              over the flattened [R][T] products (base_restock_policy.py:41-45). The products of
//              retailer row r come after all of row r-1 in that order, so with R > 1 retailers the
//              episode is replayed R times (pass r adds row r; the replay is deterministic): no
//              per-thread buffer of R*T terms, full occupancy.
//   INVENTORY / BACKLOG  sum_t sum_i of the post-step state; CUSTOMER_BACKLOG  sum_t of the
//              retailers' backlog (inv_management.py:589-592)
// Each block (one policy, BS scenarios) then reduces every metric with wavefront shuffles + LDS to
// (sum, M2 about the block mean, count): the stats kernel merges blocks with Chan's pairwise update
// (stable, deterministic).
// Poisson inversion by an indexed search (Chen & Asau): guide[g] = #{thresholds <= g * 2^22}, then a
// short scan; equals the compare-and-count of poisson_draw (searchsorted right) for every w.
__device__ __forceinline__ int poisson_guided(uint32_t w, const uint32_t* __restrict__ thr,
                                              const uint16_t* __restrict__ guide, int len) {
  int k = guide[w >> (32 - IMENV_GUIDE_BITS)];
  while (k < len && w >= thr[k]) ++k;
  return k;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over the block's threads: wave shuffles, then the waves' sums in a fixed order (deterministic).
// Every thread gets the result. s_red holds BS / 64 doubles.
template <int BS>
__device__ __forceinline__ double block_sum(double v, double* s_red) {
  const int tid = threadIdx.x;
  const double w = wave_sum(v);
  if ((tid & 63) == 0) s_red[tid >> 6] = w;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int k = 0; k < BS / 64; ++k) r += s_red[k];
  __syncthreads();
  return r;
}

// TBUF (trees, R > 1 retailers): 0 replays the episode once per retailer row (above); > 0 runs it once
// and parks the terms of rows 1..R-1 in A.terms as [block][(r - 1) * T + t][thread] (TBUF = (R - 1) * T
// doubles per thread: each block's scratch is one contiguous run, each wave store 512 contiguous
// bytes), then adds them in index order after row 0's: the same np.sum order, one pass.
//
// ACT selects where the actions come from:
//   ROLL_BASE_STOCK    the order-up-to policy above (A.policy [P][N])
//   ROLL_PLAN_SHARED   an open-loop plan per policy row, A.plan [P][T][N]: every scenario of block row
//                      `pol` replays the same actions (wave-uniform address: one broadcast load)
//   ROLL_PLAN_EPISODE  a plan per episode, A.plan [T][P][S][N]: the LP scripts' replay, where the plan
//                      of demand scenario j is solved for that scenario (SHLP_8.py:737-766). Period
//                      t+1's row is loaded while period t computes.
// Plan actions go through decode_orders exactly as step() decodes its action argument. The plan
// replays' customer backlog is node 0's backlog, as every LP script sums it (s[0, 1],
// SHLP_8.py:754, SHLP_div1.py:587); base-stock rollouts keep the retailers' sum.
constexpr int ROLL_BASE_STOCK = 0, ROLL_PLAN_SHARED = 1, ROLL_PLAN_EPISODE = 2;

template <class P, bool OBJ, int TBUF = 0, int ACT = ROLL_BASE_STOCK>
__device__ __forceinline__ void rollout_body(const P& p, const RolloutArgs& A, const SpecDev* __restrict__ sp,
                                             uint32_t* s_thr, uint16_t* s_guide, int32_t* s_ring, double* s_pmf,
                                             int pmf_lds, double* s_red) {
  static_assert(ACT == ROLL_BASE_STOCK || (!OBJ && TBUF == 0), "plan rollouts have no dfo objective");
  constexpr int NT = P::NT;
  constexpr int BS = P::BS;
  const int tid = threadIdx.x;
  const int N = p.N();
  const int T = p.T();
  const int R = p.num_retailers();
  const int64_t pol = (int64_t)blockIdx.x / A.bpp;
  const int64_t sb = (int64_t)blockIdx.x - pol * A.bpp;
  const int64_t s = sb * BS + tid;
  const bool valid = s < A.S;
  const int64_t sl = valid ? s : A.S - 1;
  const uint32_t gid = A.scen_offset + (uint32_t)sl;
  const uint32_t ep = A.episode;
  const uint64_t seed = p.seed();
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const bool draw = p.demand_layout() == IMENV_LAYOUT_DRAW;   // JIT flag: no table
  const bool poisson = draw && p.demand_dist() == IMENV_DEMAND_POISSON;
  const int n_thr = sp->table_len;
  if (poisson) {
    for (int k = tid; k < n_thr; k += BS) s_thr[k] = sp->table[k];
    for (int k = tid; k < (1 << IMENV_GUIDE_BITS); k += BS) s_guide[k] = sp->guide[k];
  }
  const int pmf_n = A.pmf_len < pmf_lds ? A.pmf_len : pmf_lds;
  if constexpr (OBJ) {
    for (int k = tid; k < pmf_n; k += BS) s_pmf[k] = A.pmf[k];
  }
  __syncthreads();

  double lvl[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) lvl[i] = (ACT == ROLL_BASE_STOCK && i < N) ? A.policy[pol * N + i] : 0.0;
  // Per-period inputs read from memory — the plan row (action words; float64: two per node) and the
  // host demand table's entries — are loaded one period ahead: their HBM latency runs under a
  // period of arithmetic. (Two periods ahead measured no faster: tools/bench_plan.py runs at
  // 4.5-4.8 TB/s either way, the step kernel's level; it only costs registers.)
  constexpr int AW = P::act_f64() ? 2 * NT : NT;
  uint32_t pw[AW];
  int dm[NT];
  const int64_t PS = A.P * A.S;
  const int64_t ep_row = pol * A.S + sl;            // this episode's row in a [T][P][S][N] plan
  auto load_inputs = [&](const int t, uint32_t (&w)[AW], int (&dmt)[NT]) {
    if constexpr (ACT == ROLL_PLAN_EPISODE) {
      const int64_t off = ((int64_t)t * PS + ep_row) * NT;
      if constexpr (P::act_f64()) load_words<8 * NT>(static_cast<const double*>(A.plan) + off, w);
      else load_words<4 * NT>(static_cast<const float*>(A.plan) + off, w);
    } else if constexpr (ACT == ROLL_PLAN_SHARED) {
      const int64_t off = (pol * T + t) * NT;
#pragma unroll
      for (int q = 0; q < AW; ++q) w[q] = static_cast<const uint32_t*>(A.plan)[(P::act_f64() ? 2 : 1) * off + q];
    }
    if (!draw) {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int r = (i < N) ? p.retailer_slot(i) : -1;
        dmt[i] = r >= 0 ? A.demand[((int64_t)t * R + r) * A.S + sl] : 0;
      }
    }
  };

  const int n_terms = R * T;                       // np.sum over prob[R][T] * rewards[T]
  const int full = n_terms >= 8 ? n_terms - (n_terms % 8) : 0;
  double ret = 0.0;
  double acc8[8], tail[7];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc8[j] = -0.0;      // -0.0 + x == x for every x: "+=" acts as the first assignment
#pragma unroll
  for (int j = 0; j < 7; ++j) tail[j] = 0.0;
  int64_t inv_s = 0, bl_s = 0, cbl_s = 0;

  const int passes = (OBJ && TBUF == 0) ? R : 1;
  double* __restrict__ my_terms = TBUF > 0 ? A.terms + (int64_t)blockIdx.x * (TBUF * BS) + tid : nullptr;
  // one term into np.sum's pairwise accumulators: 8 interleaved partial sums over the first `full`
  // indices, the rest kept for the sequential tail (NumPy's non-recursive block, n < 128)
  // Terms arrive in index order 0, 1, 2, ... (each pass adds its row's T periods in order; TBUF adds
  // rows 1.. after row 0), so accumulator idx & 7 is always the one at the front: add there and rotate
  // the eight by one (1 add + 7 moves). After `full` (a multiple of 8) terms they are back in place.
  // A (q == idx & 7) select over the eight would cost 8 adds + 16 v_cndmask per term.
  auto add_term = [&](const int idx, const double term) {
    if (idx < full) {
      const double a0 = acc8[0] + term;
#pragma unroll
      for (int q = 0; q < 7; ++q) acc8[q] = acc8[q + 1];
      acc8[7] = a0;
    } else {
      switch (idx - full) {
        case 0: tail[0] = term; break;
        case 1: tail[1] = term; break;
        case 2: tail[2] = term; break;
        case 3: tail[3] = term; break;
        case 4: tail[4] = term; break;
        case 5: tail[5] = term; break;
        default: tail[6] = term; break;
      }
    }
  };
#pragma unroll 1
  for (int pass = 0; pass < passes; ++pass) {
    int inv[NT], bl[NT], ou[NT], btoc[NT], cin[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      inv[i] = (i < N) ? p.init_inv(i) : 0;     // IM_env.py:221-224
      bl[i] = ou[i] = btoc[i] = cin[i] = 0;
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
      if (i < N)
        for (int k = 0; k < p.delay(i); ++k) s_ring[(p.ring_off(i) + k) * BS + tid] = 0;
    load_inputs(0, pw, dm);

    uint4 rb_dem[NT], rb_dbl[NT], rb_zero[NT];   // one Philox block per 4 periods
    uint4 rb_delay[(NT + 3) / 4];                 // noisy delay: one block per 4 nodes per period
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
      const int tw = t & 3;
      if (tw == 0 && draw) {
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          const int r = (i < N) ? p.retailer_slot(i) : -1;
          if (r >= 0) {
            rb_dem[i] = rng_block(gid, ep, t, STREAM_DEMAND, r, k0, k1);
            if (p.noisy_demand()) {
              rb_dbl[i] = rng_block(gid, ep, t, STREAM_ND_DOUBLE, r, k0, k1);
              rb_zero[i] = rng_block(gid, ep, t, STREAM_ND_ZERO, r, k0, k1);
            }
          }
        }
      }
      if (p.noisy_delay()) {
#pragma unroll
        for (int g = 0; g < (NT + 3) / 4; ++g)
          if (4 * g < N) rb_delay[g] = rng_node_block(gid, ep, t, STREAM_NOISY_DELAY, g, k0, k1);
      }
      int cust[NT], arr[NT], order[NT];
      bool defer[NT];
      double x[NT];
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        cust[i] = 0;
        defer[i] = false;
        arr[i] = 0;
        x[i] = 0.0;
        order[i] = 0;
        if (i < N) {
          const int r = p.retailer_slot(i);
          if (r >= 0) {
            int cd;
            if (!draw) {
              cd = dm[i];
            } else {
              const uint32_t w = word_of(rb_dem[i], tw);
              if (poisson) {
                cd = poisson_guided(w, s_thr, s_guide, n_thr);
              } else {
                const uint64_t rng = (uint64_t)(p.uniform_high() - p.uniform_low());
                cd = p.uniform_low() + (int)(((uint64_t)w * rng) >> 32);
              }
              if (p.noisy_demand()) {     // IM_div_env.py:246-255: double, then zero
                if ((uint64_t)word_of(rb_dbl[i], tw) < A.noisy_demand_thr32) cd = 2 * cd;
                if ((uint64_t)word_of(rb_zero[i], tw) < A.noisy_demand_thr32) cd = 0;
              }
            }
            cust[i] = cd;
          }
          const int d = p.delay(i);
          if (t >= d) arr[i] = s_ring[(p.ring_off(i) + t % d) * BS + tid];
          if (p.noisy_delay() && t >= d) defer[i] = (uint64_t)word_of(rb_delay[i >> 2], i & 3) < A.noisy_delay_thr32;
          if constexpr (ACT == ROLL_BASE_STOCK) {
            // base_stock_policy (base_restock_policy.py:12-20): order up to lvl from the echelon position
            // inv + order_u - backlog (integers: exact, as the reference's float64 sum of integers),
            // min(order_max, max(policy - position, 0)); then the env's decode
            const double om = (double)p.order_max(i);
            const double xa = fmin(om, fmax(lvl[i] - (double)(inv[i] + ou[i] - bl[i]), 0.0));
            if (p.std_actions()) x[i] = xa;
            else order[i] = (int)rint(xa);   // unstandardised: the decode's clip is a no-op on [0, om]
          } else if constexpr (P::act_f64()) {
            x[i] = __hiloint2double((int)pw[2 * i + 1], (int)pw[2 * i]);
          } else {
            x[i] = (double)__uint_as_float(pw[i]);   // float32 plans promote exactly, as step() does
          }
        }
      }
      if (t + 1 < T) load_inputs(t + 1, pw, dm);   // period t + 1's loads under this period's work
      if (ACT != ROLL_BASE_STOCK || p.std_actions()) decode_orders(p, x, order);
      int dem[NT], acq[NT], ship[NT], sto[NT], cout[NT], push[NT];
      double prof[NT];
      double rew;
      bool split_ok;
      step_core(p, t, order, cust, defer, arr, cin, inv, bl, ou, btoc, dem, acq, ship, sto, cout, push, prof,
                rew, split_ok);
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (i < N) {
          const int d = p.delay(i);
          s_ring[(p.ring_off(i) + t % d) * BS + tid] = push[i];
          cin[i] = cout[i];
        }
      }
      if (pass == 0) {
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          if (i < N) {
            inv_s += inv[i];
            bl_s += bl[i];
            if (ACT == ROLL_BASE_STOCK ? p.retailer_slot(i) >= 0 : i == 0) cbl_s += bl[i];
          }
        }
        ret += rew;
        // the LP scripts' per-step record, profit[j, t] = r (SHLP_8.py:751): one coalesced row per period
        if (ACT != ROLL_BASE_STOCK && A.rewards && valid) A.rewards[(int64_t)t * PS + ep_row] = rew;
      }
      if constexpr (OBJ) {
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          const int r = (i < N) ? p.retailer_slot(i) : -1;
          if (TBUF > 0 ? r >= 0 : r == pass) {
            const int k = cust[i];
            const double w = (k >= 0 && k < pmf_n) ? s_pmf[k] : ((k >= pmf_n && k < A.pmf_len) ? A.pmf[k] : 0.0);
            const double term = w * rew;
            if (TBUF > 0 && r > 0) my_terms[((r - 1) * T + t) * BS] = term;   // added after row 0
            else add_term(r * T + t, term);   // row-major [R][T]: this pass's terms arrive in index order
          }
        }
      }
    }
  }

  if constexpr (OBJ && TBUF > 0) {
#pragma unroll 1
    for (int idx = T; idx < n_terms; ++idx) add_term(idx, my_terms[(idx - T) * BS]);
  }

  double obj = 0.0;
  if constexpr (OBJ) {
    double sum = (n_terms >= 8) ? ((acc8[0] + acc8[1]) + (acc8[2] + acc8[3])) + ((acc8[4] + acc8[5]) + (acc8[6] + acc8[7]))
                                : 0.0;
#pragma unroll
    for (int q = 0; q < 7; ++q)
      if (q < n_terms - full) sum += tail[q];
    obj = (-1.0 / (double)T) * sum;               // -1 / env.num_periods * np.sum(...)
  }

  const double v[IMENV_NUM_STATS] = {ret, obj, (double)inv_s, (double)bl_s, (double)cbl_s};
  if (A.ep && valid) {
#pragma unroll
    for (int m = 0; m < IMENV_NUM_STATS; ++m) A.ep[m * PS + pol * A.S + s] = v[m];
  }
  // per-block (sum, M2 about the block mean, count) of every metric
  const int64_t rem = A.S - sb * BS;
  const double nb = (double)(rem < BS ? rem : BS);
#pragma unroll
  for (int m = 0; m < IMENV_NUM_STATS; ++m) {
    const double sm = block_sum<BS>(valid ? v[m] : 0.0, s_red);
    const double mb = sm / nb;
    const double dv = valid ? v[m] - mb : 0.0;
    const double m2 = block_sum<BS>(dv * dv, s_red);
    if (tid == 0) {
      double* o = A.partial + (((int64_t)m * A.P + pol) * A.bpp + sb) * 3;
      o[0] = sm;
      o[1] = m2;
      o[2] = nb;
    }
  }
}

// obs staging buffer size (floats) for a policy
template <class P>
constexpr int stage_floats() {
  return stage_row<P>() > 0 ? P::EPT * P::BS * stage_stride<P>() * (P::OBS_STAGE64 ? 2 : 1) : 4;
}

// Kernel template for any policy whose constructor takes (spec, args).
template <class P>
__global__ void __launch_bounds__(P::BS) imenv_step_kernel(const SpecDev* __restrict__ sp, const StepArgs A) {
  __shared__ uint32_t s_tab[P::TAB_LDS];
  __shared__ __attribute__((aligned(16))) float s_obs[stage_floats<P>()];
  const P p(sp, A);
  step_body(p, A, s_tab, s_obs);
}

#ifndef __HIPCC_RTC__
struct LaunchCfg {
  int mc;          // 0, 4, 8
  bool base;
  int es;          // state element bytes 1 / 2 / 4
  unsigned grid;   // number of 256-env blocks
  hipStream_t stream;
};

template <int NT>
void launch_step_nt(const LaunchCfg& c, const SpecDev* sp, const StepArgs& A);
#endif

}  // namespace imenv
