// imenv_jit.hip — hipRTC specialisation of the step kernel (see imenv_jit.h).
//
// The generated translation unit is just a policy class (JitSpec) plus a 5-line kernel calling the
// same step_body<P> as the ahead-of-time kernels, so both paths share one restatement of the
// reference's step() and are tested against the same oracle. The device sources are embedded at
// build time (imenv_rtc_src.inc, written by __graft_entry__.build()).
#include <hip/hiprtc.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <sstream>
#include <unordered_map>

#include "imenv_jit.h"
#include "imenv_rtc_src.inc"   // kRtcDeviceH (imenv_device.h), kRtcImenvH (imenv.h)

namespace imenv {
namespace {

std::string dlit(double x) {
  if (std::isnan(x)) return "(__builtin_nan(\"\"))";
  if (std::isinf(x)) return x > 0 ? "(__builtin_huge_val())" : "(-__builtin_huge_val())";
  char buf[64];
  std::snprintf(buf, sizeof buf, "(%a)", x);   // hex float: exact
  return buf;
}

// `static constexpr T name(int i)` as a switch over the non-default entries: folds to an immediate
// for any constant argument (every call site in step_body is inside a fully unrolled loop).
template <typename F>
void emit1(std::ostream& o, const char* type, const char* name, int n, F val, const std::string& dflt) {
  o << "  __device__ static constexpr " << type << " " << name << "(int i) { switch (i) {";
  for (int i = 0; i < n; ++i) {
    const std::string v = val(i);
    if (v != dflt) o << " case " << i << ": return " << v << ";";
  }
  o << " default: return " << dflt << "; } }\n";
}

template <typename F>
void emit2(std::ostream& o, const char* type, const char* name, int n0, int n1, F val, const std::string& dflt) {
  o << "  __device__ static constexpr " << type << " " << name << "(int i, int j) { switch (i * 256 + j) {";
  for (int i = 0; i < n0; ++i)
    for (int j = 0; j < n1; ++j) {
      const std::string v = val(i, j);
      if (v != dflt) o << " case " << (i * 256 + j) << ": return " << v << ";";
    }
  o << " default: return " << dflt << "; } }\n";
}

std::string ilit(long long v) { return std::to_string(v); }
const char* blit(bool b) { return b ? "true" : "false"; }

constexpr int kInlineTable = 64;
constexpr int kRolloutPmfLds = 256;  // pmf weights staged in LDS (the rest, if any, read from memory)   // Poisson tables up to this length become a compare-sum

// Threads (= envs) per block of the JIT kernel: 256 measured best for the C2 kernel (25.8 us vs
// 26.3 us at 512 and 27.6 us at 1024, profiles/r01); IMENV_JIT_BS overrides (64..1024, multiple of 64).
int jit_block_size() {
  int bs = 256;
  if (const char* v = std::getenv("IMENV_JIT_BS")) bs = std::atoi(v);
  if (bs < 64 || bs > 1024 || bs % 64) bs = 256;
  return bs;
}

// Observation rows are staged in LDS when a block's slab fits kStageLds bytes. The base [N][3] row
// (N <= 8) is always staged, so the block size halves (down to 64) until its slab fits, also under
// IMENV_JIT_BS: a slab over the static LDS limit would fail the hipRTC compile. General rows: the
// block size halves (256 -> 128 -> 64, unless IMENV_JIT_BS is set) until the slab fits, so wide rows
// (8 stages with in-transit features, 2-level trees with shared-network ids) keep coalesced float4
// stores at 4+ waves per SIMD instead of falling back to strided scalar stores; a general row that
// still does not fit is stored directly (jit_obs_row = 0).
// vbytes: 4 (float32 observations) or 8 (float64, staged as doubles); ept: envs per thread.
constexpr int kStageLds = 48 * 1024;

int general_row(const SpecDev& d, bool base) { return base ? 0 : d.s.num_nodes * d.s.num_features; }
// the row the step kernel stages (imenv_device.h stage_row) and its padded LDS stride (stage_stride)
int staged_row(const SpecDev& d, bool base) {
  return base ? (d.s.num_nodes <= 8 ? 3 * d.s.num_nodes : 0) : general_row(d, base);
}
int staged_stride(int row, int vbytes) {   // = imenv_device.h stage_stride
  if (row <= 0) return row;
  if (vbytes == 8) return row % 2 == 0 ? row + 1 : row;
  return row % 8 == 0 ? row + 4 : row;
}
int64_t slab_bytes(const SpecDev& d, bool base, int bs, int vbytes, int ept) {
  return (int64_t)bs * ept * staged_stride(staged_row(d, base), vbytes) * vbytes;
}

// small: the handle's launch has at most two waves per SIMD (JitFlags::small_blocks). One generation
// of waves then runs load, compute and store in lockstep; 64-env blocks (one wave, no slab barrier
// across waves) measured 5.94 -> 5.78 us for C4 at 131,072 envs and 4.32 -> 4.26 us for C2 at
// 131,072, while at 262,144+ envs they were slower (C3 +5%, C2 at 2^20 +4%; profiles/r03/ab_blocks_*).
int jit_step_block_size(const SpecDev& d, bool base, int vbytes, int ept, bool small = false) {
  int bs = (small && !std::getenv("IMENV_JIT_BS")) ? 64 : jit_block_size();
  if (staged_row(d, base) > 0 && (base || !std::getenv("IMENV_JIT_BS")))
    while (bs > 64 && slab_bytes(d, base, bs, vbytes, ept) > kStageLds) bs /= 2;
  return bs;
}

int jit_obs_row(const SpecDev& d, bool base, int bs, int vbytes) {
  const int row = general_row(d, base);
  return (row > 0 && slab_bytes(d, base, bs, vbytes, 1) <= kStageLds) ? row : 0;
}

// Envs per thread of the JIT step kernel (step_body). 1: with two envs per thread the footprint probe
// gets 5% faster (tools/probe3.py: 19.35 vs 20.42 us at C2 size), but the real kernel gets slower
// (23.4 vs 21.0 us: twice the registers, a 24 KiB obs slab per block), profiles/r01/probe3_u8_floor.log.
// IMENV_JIT_EPT=2 selects it (only for the staged float32 base-observation layout, N <= 8).
int jit_envs_per_thread(const SpecDev& d, bool base, bool obs_f64) {
  int ept = 1;
  if (const char* v = std::getenv("IMENV_JIT_EPT")) ept = std::atoi(v) == 2 ? 2 : 1;
  if (!(base && d.s.num_nodes <= 8) || obs_f64) ept = 1;
  return ept;
}

// The reference's observation value a + (v * (b - a)) / den (IM_env.py:435-444), in the same IEEE
// double expression as the device's obs_map (both built with -ffp-contract=off).
double ref_obs(const ImEnvSpec& s, int g, int i, int v) {
  double x = (double)v;
  if (s.group_mode[g] == IMENV_OBS_CLAMP_SCALED) x = std::fmin(x, s.group_clip[g][i]);
  return s.a + (x * (s.b - s.a)) / s.group_den[g][i];
}

std::string flit(float x) {
  char buf[64];
  std::snprintf(buf, sizeof buf, "(%af)", (double)x);
  return buf;
}

// Observation hooks. The generator tries cheap closed forms for every scaled (group, node) and keeps
// one only if it reproduces the reference expression bit for bit at EVERY raw value the observation
// can see (exhaustive check here, on the host). That range is [0, vbound], the bound validate_and_derive
// proves for every state value (capacities, capped or T-period backlog, demand, shipments + split
// overshoot, node ids); a clamped group (MAIM_div's in-transit slots) is clamped first. When the whole
// proven range is verified (up to kVerifyMax values) the form is emitted without a range guard, so
// the kernel spends no compare-and-branch per value; otherwise it is guarded by the tabulated range and
// values outside it take the reference expression (an IEEE double division: exact for every value).
constexpr int64_t kVerifyMax = 1 << 16;

// The raw values an observation can read are state values, so they lie in [0, vbound]: vbound is
// imenv_capi.hip's state_bound, the maximum over every node of inventory / initial inventory, the capped
// or T-period backlog, the demand bound, order_max and a shipment (backlog + demand + the split's
// overshoot), and at least N (node ids). An unguarded closed form is emitted only when the whole of
// [0, vbound] was verified here; otherwise the guarded form, exact for every value.

void emit_obs_hooks(std::ostream& o, const SpecDev& d) {
  const ImEnvSpec& s = d.s;
  const bool use = !(std::getenv("IMENV_JIT_OBS") && std::string(std::getenv("IMENV_JIT_OBS")) == "lut");
  std::ostringstream c32, c64;
  for (int g = 0; g < IMENV_NUM_GROUPS && use; ++g) {
    const int mode = s.group_mode[g];
    if (mode != IMENV_OBS_SCALED && mode != IMENV_OBS_CLAMP_SCALED) continue;
    for (int i = 0; i < s.num_nodes; ++i) {
      const int mx = d.lut_max[g][i];
      if (mx < 0) continue;
      const double d1 = (s.b - s.a) / s.group_den[g][i];
      const float c1 = (float)d1, c0 = (float)s.a;
      // the range to verify: the proven bound, or the clamp when that is smaller and integral
      const double clip = s.group_clip[g][i];
      const bool clamp = mode == IMENV_OBS_CLAMP_SCALED;
      const bool int_clip = clamp && clip >= 0.0 && clip == std::floor(clip) && clip < (double)kVerifyMax;
      int64_t hi = d.vbound;
      bool full = hi <= kVerifyMax;
      if (clamp) {
        if (int_clip) { hi = (int64_t)clip; full = true; }   // every value is clamped to clip first
        else full = false;
      }
      if (!full) hi = mx;
      // k4: all-float32 correctly rounded division of the integer numerator m = v * (b - a) + a * den by den
      // (one Newton-Markstein correction), when a, b - a and den are integers and |m| stays below 2^24
      const double den = s.group_den[g][i];
      const bool ints = s.a == std::floor(s.a) && (s.b - s.a) == std::floor(s.b - s.a) && den == std::floor(den) &&
                        den >= 1.0 && den < 16777216.0 && std::fabs(s.a) < 65536.0 && std::fabs(s.b - s.a) < 65536.0;
      const long long B4 = ints ? (long long)(s.b - s.a) : 0, A4 = ints ? (long long)(s.a * den) : 0;
      const float rc4 = (float)(1.0 / den), den4 = (float)den;
      bool k1 = true, k2 = true, k3 = true, k4 = ints, q1 = true, q2 = true, q3 = den != 0.0 && std::isfinite(den);
      const double rc64 = 1.0 / den;
      for (int64_t v = 0; v <= hi; ++v) {
        const double e = ref_obs(s, g, i, (int)v);
        const float e32 = (float)e;
        if (k4) {
          const long long m = v * B4 + A4;
          if (m <= -16777216 || m >= 16777216) {
            k4 = false;
          } else {
            const float mf = (float)m;
            const float q0 = mf * rc4;
            const float r4 = std::fmaf(std::fmaf(-q0, den4, mf), rc4, q0);
            k4 = std::memcmp(&r4, &e32, 4) == 0;
          }
        }
        const float r1 = std::fmaf((float)v, c1, c0);
        const float r2 = (float)std::fma((double)v, d1, s.a);
        const float r3 = (float)((double)v * d1 + s.a);
        k1 = k1 && std::memcmp(&r1, &e32, 4) == 0;
        k2 = k2 && std::memcmp(&r2, &e32, 4) == 0;
        k3 = k3 && std::memcmp(&r3, &e32, 4) == 0;
        const double s1 = std::fma((double)v, d1, s.a);
        const double s2 = (double)v * d1 + s.a;
        q1 = q1 && std::memcmp(&s1, &e, 8) == 0;
        q2 = q2 && std::memcmp(&s2, &e, 8) == 0;
        if (q3) {   // the reference expression with its division by one Newton-Markstein correction
          const double tv = clamp ? std::fmin((double)v, clip) * (s.b - s.a) : (double)v * (s.b - s.a);
          const double t0 = tv * rc64;
          const double s3 = s.a + std::fma(std::fma(-t0, den, tv), rc64, t0);
          q3 = std::memcmp(&s3, &e, 8) == 0;
        }
      }
      // guard (partial verification) or clamp (clamped group verified up to its integral clip)
      std::string pre;
      if (!full) pre = "if ((unsigned)v <= " + std::to_string(mx) + "u) ";
      else if (int_clip) pre = "v = v < " + std::to_string((long long)clip) + " ? v : " + std::to_string((long long)clip) + "; ";
      const std::string ret = full ? "return " : "return ";
      const std::string tail = full ? ";\n" : "; break;\n";
      const std::string cs = "    case " + std::to_string(g * 256 + i) + ": ";
      // no verified closed form: the reference expression itself (IEEE double division: exact for every
      // v), not a table gather (a dependent gather per value made float64 observations 4-10x slower)
      const std::string direct = "imenv::obs_map(" + std::to_string(mode) + ", (double)v, " + dlit(s.a) + ", " +
                                 dlit(s.b - s.a) + ", " + dlit(s.group_den[g][i]) + ", " +
                                 dlit(s.group_clip[g][i]) + ")";
      if (k1) c32 << cs << pre << ret << "__builtin_fmaf((float)v, " << flit(c1) << ", " << flit(c0) << ")" << tail;
      else if (k4)
        c32 << cs << pre << "{ const float m = (float)(v * " << B4 << " + (" << A4 << ")); const float q0 = m * "
            << flit(rc4) << "; return __builtin_fmaf(__builtin_fmaf(-q0, " << flit(den4) << ", m), " << flit(rc4)
            << ", q0); }" << (full ? "\n" : " break;\n");
      else if (k2) c32 << cs << pre << ret << "(float)__builtin_fma((double)v, " << dlit(d1) << ", " << dlit(s.a) << ")" << tail;
      else if (k3) c32 << cs << pre << ret << "(float)((double)v * " << dlit(d1) << " + " << dlit(s.a) << ")" << tail;
      else c32 << cs << "return (float)" << direct << ";\n";
      if (q1) c64 << cs << pre << ret << "__builtin_fma((double)v, " << dlit(d1) << ", " << dlit(s.a) << ")" << tail;
      else if (q2) c64 << cs << pre << ret << "(double)v * " << dlit(d1) << " + " << dlit(s.a) << tail;
      else if (q3)
        c64 << cs << pre << "{ const double tv = (double)v * " << dlit(s.b - s.a) << "; const double t0 = tv * " << dlit(rc64)
            << "; return " << dlit(s.a) << " + __builtin_fma(__builtin_fma(-t0, " << dlit(den) << ", tv), " << dlit(rc64)
            << ", t0); }" << (full ? "\n" : " break;\n");
      else c64 << cs << "return " << direct << ";\n";
    }
  }
  o << "  __device__ float obs32(int g, int i, int v, const float* __restrict__ lut) const {\n"
       "#if (IMENV_ABLATE & 4)\n    return (float)v;   // diagnostic ablation (imenv_device.h)\n#endif\n"
       "    switch (g * 256 + i) {\n"
    << c32.str()
    << "    default: break;\n    }\n    return imenv::obs_value32(*this, lut, g, i, v);\n  }\n";
  o << "  __device__ double obs64(int g, int i, int v, const double* __restrict__ lut) const {\n"
       "    switch (g * 256 + i) {\n"
    << c64.str()
    << "    default: break;\n    }\n    return imenv::obs_value64(*this, lut, g, i, v);\n  }\n";
}

}  // namespace

namespace {
// The JitSpec policy class: every accessor step_body / rollout_body use, as a constexpr.
void emit_policy(std::ostream& o, const SpecDev& d, int maxc, bool base, const JitFlags& f, int bs, int ept) {
  const ImEnvSpec& s = d.s;
  const int N = s.num_nodes;
  const int F = s.num_features;
  // history rows are kept only when an observation reads an entry older than this step (index >= 1;
  // entry 0 is this step's demand / order, in registers); the same rule allocates them (imenv_capi.hip)
  bool uses_hist = false, has_td = false;
  for (int k = 0; k < F; ++k) {
    if ((s.feat_group[k] == IMENV_G_DEMAND_HIST || s.feat_group[k] == IMENV_G_ORDER_HIST) && s.feat_index[k] >= 1)
      uses_hist = true;
    if (s.feat_group[k] == IMENV_G_TRANSIT) has_td = true;
  }
  // general observation rows staged in LDS and written as contiguous float4 / double2 runs (jit_obs_row)
  const int obs_row = jit_obs_row(d, base, bs, f.obs_f64 ? 8 : 4);
  const bool inline_tab = d.table_len <= kInlineTable;
  if (f.stream_store) o << "#define IMENV_NT_STORE 1\n";
  if (f.wt_obs) o << "#define IMENV_WT_STORE 1\n";
  if (f.wt_state) o << "#define IMENV_WT_STATE 1\n";
  o << "#include \"imenv_device.h\"\n"
       "// generated by imenv_jit.hip: every spec value is a compile-time constant\n"
       "struct JitSpec {\n";
  o << "  static constexpr int NT = " << N << ";\n"
    << "  static constexpr int MC = " << maxc << ";\n"
    << "  static constexpr bool BASE = " << blit(base) << ";\n"
    << "  static constexpr bool EXACT = true;\n"
    << "  static constexpr bool JIT = true;\n"
    << "  static constexpr int TAB_LDS = " << (inline_tab ? 1 : IMENV_TABLE_MAX) << ";\n"
    << "  static constexpr int BS = " << bs << ";\n"
    << "  static constexpr int EPT = " << ept << ";\n"
    << "  static constexpr int RING = " << d.ring_total << ";\n"
    << "  static constexpr int OBS_ROW = " << obs_row << ";\n"
    << "  static constexpr bool OBS_STAGE64 = " << blit(f.obs_f64) << ";\n"
    << "  static constexpr int NBT = " << d.num_bto << ";\n"
    << "  static constexpr int RECW = " << d.rec_bytes / 4 << ";\n"
    << "  static constexpr bool DTAB = " << blit(d.dtab_es > 0 && f.demand_layout == IMENV_LAYOUT_DRAW) << ";\n"
    << "  static constexpr int TD_PRE = " << (has_td && d.dmax > 1 ? d.dmax - 1 : 0) << ";\n"
    << "  static constexpr bool XCD_REMAP = " << blit(f.small_blocks) << ";\n"
    << "  static constexpr bool FULL = " << blit(f.full) << ";\n"
    << "  static constexpr bool INFO = " << blit(f.info) << ";\n"
    << "  static constexpr bool ALIGNED = " << blit(f.aligned) << ";\n"
    << "  using ST = " << (d.es == 1 ? "uint8_t" : d.es == 2 ? "int16_t" : "int32_t") << ";\n"
    << "  const imenv::SpecDev* __restrict__ sp;\n"
    << "  template <class X> __device__ JitSpec(const imenv::SpecDev* __restrict__ s, const X&) : sp(s) {}\n";
  auto sc = [&](const char* type, const char* name, const std::string& v) {
    o << "  __device__ static constexpr " << type << " " << name << "() { return " << v << "; }\n";
  };
  sc("int", "N", ilit(N));
  sc("int", "T", ilit(s.num_periods));
  sc("int", "np", ilit(d.np));
  sc("int", "D", ilit(d.dmax));
  sc("int", "factory", ilit(d.factory));
  sc("int", "num_retailers", ilit(s.num_retailers));
  sc("int", "prev_length", ilit(s.prev_length));
  sc("int", "num_features", ilit(F));
  sc("int", "num_split", ilit(d.num_split));
  sc("int", "nb", ilit(d.num_bto));
  sc("int", "rec_words", ilit(d.rec_bytes / 4));
  sc("int", "bto_es", ilit(d.bto_es));
  sc("int", "dtab_es", ilit(d.dtab_es));
  sc("bool", "std_actions", blit(s.standardise_actions != 0));
  sc("bool", "clip_round", blit(s.decode_mode == IMENV_DECODE_CLIP_ROUND));
  sc("double", "a", dlit(s.a));
  sc("double", "bma", dlit(s.b - s.a));
  sc("double", "inv_bma", dlit(d.inv_bma));
  sc("int", "reward_mode", ilit(s.reward_mode));
  sc("double", "inv_n", dlit(d.inv_n));
  sc("int", "demand_dist", ilit(s.demand_dist));
  sc("int", "uniform_low", ilit(s.uniform_low));
  sc("int", "uniform_high", ilit(s.uniform_high));
  sc("uint64_t", "seed", std::to_string((unsigned long long)s.seed) + "ull");
  sc("bool", "act_f64", blit(f.act_f64));
  sc("bool", "obs_f64", blit(f.obs_f64));
  sc("int", "demand_layout", ilit(f.demand_layout));
  sc("bool", "noisy_delay", blit(f.noisy_delay));
  sc("bool", "noisy_demand", blit(f.noisy_demand));
  sc("bool", "has_delay_u", blit(f.has_delay_u));
  sc("bool", "uses_hist", blit(uses_hist));
  sc("bool", "has_metrics", blit(f.metrics));
  auto I = [](const int32_t* a) { return [a](int i) { return ilit(a[i]); }; };
  auto Dd = [](const double* a) { return [a](int i) { return dlit(a[i]); }; };
  emit1(o, "int", "delay", N, I(s.delay), "1");
  emit1(o, "int", "ring_off", N, I(d.ring_off), "0");
  emit1(o, "int", "init_inv", N, I(s.init_inv), "0");
  emit1(o, "int", "inv_max", N, I(s.inv_max), "0");
  emit1(o, "int", "order_max", N, I(s.order_max), "0");
  emit1(o, "int", "backlog_cap", N, I(s.backlog_cap), "-1");
  emit1(o, "int", "retailer_slot", N, I(s.retailer_slot), "-1");
  emit1(o, "int", "demand_parent", N, I(s.demand_parent), "-1");
  emit1(o, "int", "single_parent", N, I(d.single_parent), "-1");
  emit1(o, "int", "split_child", N, I(d.split_child), "0");
  emit1(o, "int", "bto_slot", N, I(d.bto_slot), "-1");
  emit1(o, "int", "split_node", d.num_split, I(d.split_node), "0");
  emit1(o, "int", "num_children", N, I(s.num_children), "0");
  emit1(o, "double", "sell", N, Dd(s.sell_price), "(0.0)");
  emit1(o, "double", "buy", N, Dd(s.buy_price), "(0.0)");
  emit1(o, "double", "stock_cost", N, Dd(s.stock_cost), "(0.0)");
  emit1(o, "double", "backlog_cost", N, Dd(s.backlog_cost), "(0.0)");
  emit1(o, "double", "inv_target", N, Dd(s.inv_target), "(0.0)");
  emit1(o, "int", "group_mode", IMENV_NUM_GROUPS, I(s.group_mode), "0");
  emit1(o, "int", "feat_group", F, I(s.feat_group), "0");
  emit1(o, "int", "feat_index", F, I(s.feat_index), "0");
  emit2(o, "int", "child", N, IMENV_MAX_CHILDREN, [&](int p, int k) { return ilit(s.children[p][k]); }, "0");
  emit2(o, "int", "split_limit", N, 4, [&](int p, int q) { return ilit(s.split_limit[p][q]); }, "0");
  emit2(o, "double", "group_den", IMENV_NUM_GROUPS, N, [&](int g, int i) { return dlit(s.group_den[g][i]); },
        "(1.0)");
  emit2(o, "double", "group_clip", IMENV_NUM_GROUPS, N, [&](int g, int i) { return dlit(s.group_clip[g][i]); },
        "(0.0)");
  emit2(o, "int", "lut_max", IMENV_NUM_GROUPS, N, [&](int g, int i) { return ilit(d.lut_max[g][i]); }, "-1");
  emit2(o, "int", "lut_off", IMENV_NUM_GROUPS, N, [&](int g, int i) { return ilit(d.lut_off[g][i]); }, "0");
  emit_obs_hooks(o, d);
  if (inline_tab) {
    // count of thresholds <= w == searchsorted(table, w, 'right') for the sorted table. The thresholds
    // are sorted, so once w < thr[K] every later term is 0: the first K thresholds are always counted,
    // the rest only when some lane of the wave has w >= thr[K] (a wave-uniform branch). K is the first
    // index whose tail probability 1 - thr[K] / 2^32 is <= 2^-10 (Poisson(5): K = 13 of 24), so a
    // 64-lane wave takes the tail about 6% of the time and skips ~45% of the compares otherwise.
    int K = d.table_len;
    for (int k = 0; k < d.table_len; ++k)
      if (4294967296.0 - (double)d.table[k] <= 4294967296.0 / 1024.0) { K = k; break; }
    o << "  __device__ static int poisson_draw(uint32_t w, const uint32_t*) {\n    int k = 0;\n";
    for (int k = 0; k < std::min(K, d.table_len); ++k) o << "    k += (w >= " << d.table[k] << "u) ? 1 : 0;\n";
    if (K < d.table_len) {
      o << "    if (__builtin_amdgcn_ballot_w64(w >= " << d.table[K] << "u) != 0) {\n";
      for (int k = K; k < d.table_len; ++k) o << "      k += (w >= " << d.table[k] << "u) ? 1 : 0;\n";
      o << "    }\n";
    }
    o << "    return k;\n  }\n"
         "  __device__ static void stage_tables(uint32_t*, bool) {}\n";
  } else {
    o << "  __device__ static int poisson_draw(uint32_t w, const uint32_t* s_tab) {\n"
         "    int lo = 0, hi = "
      << d.table_len
      << ";\n"
         "    while (lo < hi) { const int mid = (lo + hi) >> 1; if (w >= s_tab[mid]) lo = mid + 1; else hi = mid; }\n"
         "    return lo;\n  }\n"
         "  __device__ void stage_tables(uint32_t* s_tab, bool poisson) const {\n"
         "    if (poisson) { for (int k = threadIdx.x; k < "
      << d.table_len << "; k += BS) s_tab[k] = sp->table[k]; __syncthreads(); }\n  }\n";
  }
  o << "};\n\n";
}
}  // namespace

namespace {
// Extra hipRTC options (IMENV_JIT_OPTS, tuning experiments such as -DIMENV_BUF_LOAD=1) change the kernel
// without changing the spec or the flags, so a hash of them goes into the kernel's name and its tag:
// a kernel trace or a PMC summary of an experiment never matches the production kernel's. Diagnostic
// switches (IMENV_ABLATE gives WRONG results on purpose; IMENV_STAMPS writes phase stamps) are refused
// unless IMENV_DIAG=1 is set too, and their tag starts "jit-diag:" (bench.py and tools/pmc_summary.py
// reject such kernels).
std::string jit_extra_opts() {
  const char* v = std::getenv("IMENV_JIT_OPTS");
  return v ? std::string(v) : std::string();
}
uint32_t fnv1a(const std::string& x) {
  uint32_t h = 2166136261u;
  for (char c : x) h = (h ^ (uint8_t)c) * 16777619u;
  return h;
}
bool diag_opts(const std::string& x) {
  return x.find("IMENV_ABLATE") != std::string::npos || x.find("IMENV_STAMPS") != std::string::npos;
}
// "", or "_opt_<hash>" / "_diag_<hash>" for a kernel built with extra options
std::string opts_suffix() {
  const std::string x = jit_extra_opts();
  if (x.find_first_not_of(" \t") == std::string::npos) return "";
  char b[32];
  std::snprintf(b, sizeof b, "_%s_%08x", diag_opts(x) ? "diag" : "opt", fnv1a(x));
  return b;
}
}  // namespace

// the streaming- and write-through-store variants, and float64-observation kernels, have names of their
// own, so kernel traces and PMC summaries never average them with another variant
static std::string jit_kernel_name(const JitFlags& f) {
  return std::string(f.stream_store ? "imenv_step_jit_nt" : (f.wt_obs || f.wt_state) ? "imenv_step_jit_wt"
                                                                                     : "imenv_step_jit") +
         (f.obs_f64 ? "_o64" : "") + opts_suffix();
}

// the tag's prefix: "jit:", or "jit-diag:" for a diagnostic build
static const char* tag_prefix() { return diag_opts(jit_extra_opts()) ? "jit-diag:" : "jit:"; }

// a diagnostic build needs IMENV_DIAG=1 (never taken by accident from a stray IMENV_JIT_OPTS)
static bool diag_refused(std::string& msg) {
  const std::string x = jit_extra_opts();
  if (!diag_opts(x)) return false;
  const char* d = std::getenv("IMENV_DIAG");
  if (d && std::atoi(d) != 0) return false;
  msg = "IMENV_JIT_OPTS='" + x + "' builds a diagnostic kernel (IMENV_ABLATE / IMENV_STAMPS); set IMENV_DIAG=1 to allow it";
  return true;
}

std::string jit_source(const SpecDev& d, int maxc, bool base, const JitFlags& f) {
  std::ostringstream o;
  const int ept = jit_envs_per_thread(d, base, f.obs_f64);
  emit_policy(o, d, maxc, base, f, jit_step_block_size(d, base, f.obs_f64 ? 8 : 4, ept, f.small_blocks), ept);
  // The arguments a wave needs first lead the signature as scalars, so that with kernel-argument
  // preloading (jit_options) they arrive in SGPRs at wave launch: the loads of actions and state
  // issue without waiting for a scalar load of the argument segment (tools/probe_launch.py: 0.30-0.37 us
  // of a 3.5-4 us launch at 131,072 envs). StepArgs (~360 bytes, not preloadable) follows for the rest.
  o << "extern \"C\" __global__ void __launch_bounds__(JitSpec::BS)\n"
    << jit_kernel_name(f)
    << "(const void* __restrict__ act, void* __restrict__ state, void* __restrict__ aux, void* __restrict__ obs,\n"
       "    double* __restrict__ rew, int t, unsigned n32, unsigned long long ring_pack,\n"
       "    const imenv::SpecDev* __restrict__ sp,\n"
       "    const imenv::StepArgs A0) {\n"
       "  __shared__ uint32_t s_tab[JitSpec::TAB_LDS];\n"
       "  __shared__ __attribute__((aligned(16))) float s_obs[imenv::stage_floats<JitSpec>()];\n"
       "  imenv::StepArgs A = A0;\n"
       "  A.actions = act; A.net = state; A.obs = obs; A.reward = rew; A.t = t; A.n = (int64_t)n32;\n"
       "  // the third hot argument: the drawn-demand table when the handle has one (the episode word then comes\n"
       "  // with the struct), else the episode word\n"
       "  if constexpr (JitSpec::DTAB) A.dtab = aux; else A.episode = static_cast<const uint32_t*>(aux);\n"
       "  if constexpr (JitSpec::RECW > 0) {   // state records: byte i of ring_pack = node i's slot byte\n"
       "#pragma unroll\n"
       "    for (int i = 0; i < JitSpec::NT; ++i) A.ring_at[i] = (int64_t)((ring_pack >> (8 * i)) & 0xFFull);\n"
       "  }\n"
       "  const JitSpec p(sp, A);\n"
       "  imenv::step_body(p, A, s_tab, s_obs);\n"
       "}\n";
  return o.str();
}

namespace {
std::mutex g_mu;

// FNV-1a over the embedded device header (imenv_device.h): identifies the kernel body in tags
unsigned device_src_hash() {
  uint32_t h = 2166136261u;
  for (const char* c = kRtcDeviceH; *c; ++c) h = (h ^ (uint8_t)*c) * 16777619u;
  return h;
}
std::unordered_map<std::string, std::shared_ptr<const std::vector<char>>> g_code;

// Kernel-argument preloading (gfx950): the leading scalar arguments of a kernel are written into SGPRs
// when its waves launch. IMENV_JIT_PRELOAD=0 turns it off (A/B).
bool jit_preload() {
  const char* v = std::getenv("IMENV_JIT_PRELOAD");
  return !(v && std::atoi(v) == 0);
}

std::vector<std::string> jit_options(const std::string& arch) {
  std::vector<std::string> v = {"--offload-arch=" + arch, "-O3", "-std=c++17", "-ffp-contract=off"};
  if (jit_preload()) {
    v.push_back("-mllvm");
    v.push_back("-amdgpu-kernarg-preload-count=16");
  }
  if (const char* extra = std::getenv("IMENV_JIT_OPTS")) {   // tuning experiments, e.g. -DFOO=1
    std::istringstream is(extra);
    std::string w;
    while (is >> w) v.push_back(w);
  }
  return v;
}
}  // namespace

std::shared_ptr<const std::vector<char>> jit_compile(const std::string& src, const std::string& arch,
                                                     std::string& msg) {
  const std::vector<std::string> opts = jit_options(arch);
  std::string key = src;
  for (const auto& s : opts) key += "\n//" + s;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_code.find(key);
    if (it != g_code.end()) return it->second;
  }
  hiprtcProgram prog;
  const char* hdr_src[2] = {kRtcDeviceH, kRtcImenvH};
  const char* hdr_names[2] = {"imenv_device.h", "imenv.h"};
  hiprtcResult r = hiprtcCreateProgram(&prog, src.c_str(), "imenv_step_jit.hip", 2, hdr_src, hdr_names);
  if (r != HIPRTC_SUCCESS) {
    msg = std::string("hiprtcCreateProgram: ") + hiprtcGetErrorString(r);
    return nullptr;
  }
  std::vector<const char*> copts;
  for (const auto& s : opts) copts.push_back(s.c_str());
  r = hiprtcCompileProgram(prog, (int)copts.size(), copts.data());
  if (r != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    msg = std::string("hiprtcCompileProgram: ") + hiprtcGetErrorString(r) + "\n" + log;
    return nullptr;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  auto code = std::make_shared<std::vector<char>>(cs);
  hiprtcGetCode(prog, code->data());
  hiprtcDestroyProgram(&prog);
  if (const char* dir = std::getenv("IMENV_JIT_DUMP")) {   // inspection: <dir>/imenv_jit_<hash>.{hip,co}
    char base[512];
    std::snprintf(base, sizeof base, "%s/imenv_jit_%016zx", dir, std::hash<std::string>()(key));
    if (FILE* fp = std::fopen((std::string(base) + ".hip").c_str(), "w")) {
      std::fwrite(src.data(), 1, src.size(), fp);
      std::fclose(fp);
    }
    if (FILE* fp = std::fopen((std::string(base) + ".co").c_str(), "wb")) {
      std::fwrite(code->data(), 1, code->size(), fp);
      std::fclose(fp);
    }
  }
  std::lock_guard<std::mutex> lk(g_mu);
  auto ins = g_code.emplace(key, code);
  return ins.first->second;
}

namespace {
bool load_module(const std::string& src, const std::string& arch, const char* fn_name, JitKernel& out,
                 std::string& msg) {
  auto code = jit_compile(src, arch, msg);
  if (!code) return false;
  hipModule_t mod = nullptr;
  hipError_t e = hipModuleLoadData(&mod, code->data());
  if (e != hipSuccess) {
    msg = std::string("hipModuleLoadData: ") + hipGetErrorString(e);
    return false;
  }
  hipFunction_t fn = nullptr;
  e = hipModuleGetFunction(&fn, mod, fn_name);
  if (e != hipSuccess) {
    (void)hipModuleUnload(mod);
    msg = std::string("hipModuleGetFunction: ") + hipGetErrorString(e);
    return false;
  }
  out.mod = mod;
  out.fn = fn;
  return true;
}
}  // namespace

bool jit_load(const SpecDev& d, int maxc, bool base, const JitFlags& f, const std::string& arch, JitKernel& out,
              std::string& msg) {
  if (diag_refused(msg)) return false;
  const std::string src = jit_source(d, maxc, base, f);
  if (!load_module(src, arch, jit_kernel_name(f).c_str(), out, msg)) return false;
  out.ept = jit_envs_per_thread(d, base, f.obs_f64);
  out.bs = jit_step_block_size(d, base, f.obs_f64 ? 8 : 4, out.ept, f.small_blocks);
  char tag[224];
  // dev=: hash of the device-code header, so a profile of an older kernel body never matches this one;
  // the kernel name carries the hash of any extra compile options
  // rec=: state records (imenv_capi.hip rec_bytes_for), so a profile of the row layout never matches;
  // kpre=: the hot arguments preloaded into SGPRs (a different code object, with its own profiles)
  std::snprintf(tag, sizeof tag, "%s%s[N=%d,MC=%d,base=%d,es=%d,flags=0x%x,bs=%d,ept=%d,%s%s%zuB,dev=%08x]",
                tag_prefix(), jit_kernel_name(f).c_str(), d.s.num_nodes, maxc, base ? 1 : 0, d.es, f.key(), out.bs,
                out.ept, d.rec_bytes ? (d.rec_bytes == 16 ? "rec=16," : "rec=32,") : "",
                jit_preload() ? "kpre=16," : "", src.size(), device_src_hash());
  out.tag = tag;
  return true;
}

hipError_t jit_launch(const JitKernel& k, hipStream_t st, const SpecDev* sp, const StepArgs& A) {
  const SpecDev* spv = sp;
  StepArgs av = A;
  const void* act = A.actions;
  void* state = A.net;
  void* aux = A.dtab ? A.dtab : const_cast<uint32_t*>(A.episode);   // (see jit_source: JitSpec::DTAB)
  void* obs = A.obs;
  double* rew = A.reward;
  int t = A.t;
  unsigned n32 = (unsigned)A.n;         // n <= 2^31 (imenv_create)
  unsigned long long ring_pack = 0;   // state records: node i's ring byte (< 32) in byte i
  for (int i = 0; i < 8; ++i) ring_pack |= (unsigned long long)(A.ring_at[i] & 0xFF) << (8 * i);
  void* args[] = {&act, &state, &aux, &obs, &rew, &t, &n32, &ring_pack, &spv, &av};
  const int64_t per_block = (int64_t)k.bs * k.ept;
  const unsigned grid = (unsigned)((A.n + per_block - 1) / per_block);
  return hipModuleLaunchKernel(k.fn, grid, 1, 1, (unsigned)k.bs, 1, 1, 0, st, args, nullptr);
}

// ---------------------------------------------------------------- fused base-stock rollout
int rollout_term_slots(const SpecDev& d, const RolloutFlags& f) {
  // trees with R > 1 retailer rows: park rows 1..R-1 of the objective's terms in a global scratch and
  // run the episode once (rollout_body TBUF); 0 = replay once per row (IMENV_ROLLOUT_REPLAY=1 forces
  // it, for A/B)
  if (!f.objective || d.s.num_retailers <= 1) return 0;
  if (const char* v = std::getenv("IMENV_ROLLOUT_REPLAY"))
    if (std::atoi(v) != 0) return 0;
  return (d.s.num_retailers - 1) * d.s.num_periods;
}

int rollout_block_size(const SpecDev& d, const RolloutFlags&) {
  // LDS per block: the in-transit queue (int32 per slot per thread), the Poisson table, the pmf
  // weights and the reduction scratch. 256 threads unless the queue is long.
  for (int bs : {256, 128, 64})
    if (bs * 4 * d.ring_total + 4 * IMENV_TABLE_MAX + 2 * (1 << IMENV_GUIDE_BITS) + 8 * kRolloutPmfLds + 8 * 4 <= 65536)
      return bs;
  return 0;
}

std::string jit_rollout_source(const SpecDev& d, int maxc, const RolloutFlags& f, int bs) {
  JitFlags jf;
  jf.noisy_delay = f.noisy_delay;
  jf.noisy_demand = f.noisy_demand;
  jf.demand_layout = f.table ? IMENV_LAYOUT_PER_ENV : IMENV_LAYOUT_DRAW;
  jf.act_f64 = f.act_f64;
  std::ostringstream o;
  emit_policy(o, d, maxc, false, jf, bs, 1);
  const int pmf = f.objective ? kRolloutPmfLds : 1;
  const int tb = rollout_term_slots(d, f);
  o << "extern \"C\" __global__ void __launch_bounds__(JitSpec::BS)\n"
    << "imenv_rollout_jit" << opts_suffix() << "(const imenv::SpecDev* __restrict__ sp, const imenv::RolloutArgs A) {\n"
       "  __shared__ uint32_t s_thr["
    << (d.s.demand_dist == IMENV_DEMAND_POISSON && !f.table ? IMENV_TABLE_MAX : 1)
    << "];\n"
       "  __shared__ uint16_t s_guide["
    << (d.s.demand_dist == IMENV_DEMAND_POISSON && !f.table ? (1 << IMENV_GUIDE_BITS) : 1)
    << "];\n"
       "  __shared__ int32_t s_ring[JitSpec::RING * JitSpec::BS];\n"
       "  __shared__ double s_pmf["
    << pmf
    << "];\n"
       "  __shared__ double s_red[JitSpec::BS / 64];\n"
       "  const JitSpec p(sp, A);\n"
       "  imenv::rollout_body<JitSpec, "
    << blit(f.objective) << ", " << tb << ", " << f.act << ">(p, A, sp, s_thr, s_guide, s_ring, s_pmf, " << pmf
    << ", s_red);\n"
       "}\n";
  return o.str();
}

bool jit_rollout_load(const SpecDev& d, int maxc, const RolloutFlags& f, const std::string& arch, JitKernel& out,
                      std::string& msg) {
  const int bs = rollout_block_size(d, f);
  if (bs == 0) {
    msg = "rollout: the in-transit queue exceeds 64 KiB of LDS at 64 threads per block";
    return false;
  }
  if (diag_refused(msg)) return false;
  const std::string src = jit_rollout_source(d, maxc, f, bs);
  const std::string name = "imenv_rollout_jit" + opts_suffix();
  if (!load_module(src, arch, name.c_str(), out, msg)) return false;
  out.bs = bs;
  char tag[224];
  std::snprintf(tag, sizeof tag, "%s%s[N=%d,MC=%d,es=%d,flags=0x%x,bs=%d,tb=%d,%zuB,dev=%08x]", tag_prefix(),
                name.c_str(), d.s.num_nodes, maxc, d.es, f.key(), bs, rollout_term_slots(d, f), src.size(),
                device_src_hash());
  out.tag = tag;
  return true;
}

hipError_t jit_rollout_launch(const JitKernel& k, hipStream_t st, const SpecDev* sp, const RolloutArgs& A) {
  const SpecDev* spv = sp;
  RolloutArgs av = A;
  void* args[] = {&spv, &av};
  const unsigned grid = (unsigned)(A.P * A.bpp);
  return hipModuleLaunchKernel(k.fn, grid, 1, 1, (unsigned)k.bs, 1, 1, 0, st, args, nullptr);
}

}  // namespace imenv
