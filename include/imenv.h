/*
 * imenv.h — C ABI of the MI355X-native vectorised inventory-management env.
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json
 * (north_star): the reset()/step() dynamics of the reference's four env classes
 *
 *   environments/IM_env.py        InvManagement.reset/step          (:164-229, :287-360)
 *   environments/MAIM_env.py      MultiAgentInvManagement.reset/step (:176-240, :330-411)
 *   environments/IM_div_env.py    InvManagementDiv.reset/step        (:201-302, :361-549)
 *   environments/MAIM_div_env.py  MultiAgentInvManagementDiv.reset/step (:240-341, :441-630)
 *
 * batched over n_envs independent envs that advance in lockstep. The reference
 * is pure Python, so there is no FFI to mirror line by line; each entry point
 * below names the reference method it replaces. Host-side adaptors that
 * re-expose the reference's gym/RLlib surface over this ABI live in
 * marl-for-im_amd/imenv (ctypes), see INTEGRATION.md.
 *
 * Conventions
 *  - Plain C types only. Every buffer argument is a DEVICE pointer owned by the
 *    caller unless stated otherwise; the handle owns its state buffers.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream). All
 *    calls are stream-ordered and asynchronous unless stated otherwise.
 *  - Return value: IMENV_OK (0) or a negative IMENV_E_* code; the message is
 *    available from imenv_last_error() (thread-local). No exceptions cross the ABI.
 *  - One handle per (process, GPU); not thread-safe per handle.
 *
 * Node indexing is the reference's own: serial envs use stage 0 = retailer,
 * stage N-1 = factory; tree envs use node 0 = factory (root), leaves = retailers.
 */
#ifndef IMENV_H
#define IMENV_H

#ifndef __HIPCC_RTC__   /* hipRTC builds of the step kernel bring their own fixed-width types */
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define IMENV_ABI_VERSION 1

#define IMENV_MAX_NODES 16
#define IMENV_MAX_CHILDREN 8
#define IMENV_MAX_FEATURES 64
#define IMENV_MAX_HIST 8
#define IMENV_MAX_DELAY 64
#define IMENV_MAX_PERIODS 100000

/* status codes */
#define IMENV_OK 0
#define IMENV_E_INVALID -1      /* bad argument / spec (reference: Exception / assert at __init__) */
#define IMENV_E_UNSUPPORTED -2  /* valid in the reference but not supported by this build */
#define IMENV_E_HIP -3          /* HIP runtime error */
#define IMENV_E_DONE -4         /* step() past num_periods (reference: IndexError) */
#define IMENV_E_NOT_RESET -5    /* step() before the first reset() */
#define IMENV_E_SPLIT_LOOP -6   /* an env tripped the divergent split's "Infinite Loop" guard */

/* env class whose semantics the spec encodes (documentation + validation only;
 * every behavioural difference is spelled out in the spec fields) */
#define IMENV_KIND_IM 0
#define IMENV_KIND_MAIM 1
#define IMENV_KIND_IM_DIV 2
#define IMENV_KIND_MAIM_DIV 3

/* order decode: IM / IM_div clip then round (IM_env.py:299-300);
 * MAIM / MAIM_div round then clip (MAIM_env.py:343-347) */
#define IMENV_DECODE_CLIP_ROUND 0
#define IMENV_DECODE_ROUND_CLIP 1

/* reward: single-agent np.sum(profit) in NumPy's summation order (IM_env.py:372);
 * multi-agent shared (0 + p0 + ... + pN-1) / N (MAIM_env.py:418-434);
 * multi-agent independent profit per agent (MAIM_env.py:428-429) */
#define IMENV_REWARD_SUM 0
#define IMENV_REWARD_SHARED_MEAN 1
#define IMENV_REWARD_INDEPENDENT 2

/* observation feature groups (IM_env.py:231-285 etc.) */
#define IMENV_G_INV 0
#define IMENV_G_BACKLOG 1
#define IMENV_G_ORDER_U 2
#define IMENV_G_DEMAND_HIST 3   /* index j: demand at period t-1-j (0 when j >= t) */
#define IMENV_G_ORDER_HIST 4    /* index j: order at period t-1-j (0 when j >= t) */
#define IMENV_G_TRANSIT 5       /* index k: in-transit amount arriving at t+k ("time_dependent_state") */
#define IMENV_G_NODE_ID 6       /* share_network agent id (MAIM_div_env.py:434-435) */
#define IMENV_G_ZERO 7          /* always 0 (MAIM unstandardised history slots) */
#define IMENV_NUM_GROUPS 8

/* how a group's raw value v becomes an observation */
#define IMENV_OBS_ZERO 0
#define IMENV_OBS_RAW 1           /* v */
#define IMENV_OBS_SCALED 2        /* a + (v * (b - a)) / den   (rescale, IM_env.py:435-444) */
#define IMENV_OBS_CLAMP_SCALED 3  /* a + (min(v, clip) * (b - a)) / den  (MAIM_div_env.py:405-411) */

/* what reset() draws when the caller passes no demand (spec.demand_dist) */
#define IMENV_DEMAND_CUSTOM 1    /* the caller must pass a table (the reference's "custom") */
#define IMENV_DEMAND_POISSON 2   /* in-kernel Philox4x32-10 + inversion, Poisson(mu) */
#define IMENV_DEMAND_UNIFORM 3   /* in-kernel Philox4x32-10, randint[low, high) */

/* imenv_reset demand_layout */
#define IMENV_LAYOUT_DRAW 0      /* demand == NULL: draw per spec.demand_dist (+ noisy demand) */
#define IMENV_LAYOUT_PER_ENV 1   /* device int32 [T][R][n]: reset(customer_demand=...) per env */
#define IMENV_LAYOUT_BROADCAST 2 /* device int32 [T][R]: one custom table for every env (+ noisy demand) */

/* dtypes */
#define IMENV_F32 0
#define IMENV_F64 1

typedef struct ImEnvSpec {
  int32_t abi_version;          /* = IMENV_ABI_VERSION */
  int32_t kind;                 /* IMENV_KIND_* */
  int32_t num_nodes;            /* N <= IMENV_MAX_NODES */
  int32_t num_periods;          /* T */

  /* topology: parent[i] = upstream node (-1 for the factory); children in the
   * reference's iteration order (connections[p] list order, IM_div_env.py:415) */
  int32_t parent[IMENV_MAX_NODES];
  int32_t num_children[IMENV_MAX_NODES];
  int32_t children[IMENV_MAX_NODES][IMENV_MAX_CHILDREN];
  /* demand_parent[c]: node whose demand includes c's order (-1: none). Serial:
   * c+1; tree: parent if c > parent (IM_div_env.py:383-387 scans j >= i) */
  int32_t demand_parent[IMENV_MAX_NODES];
  /* retailer_slot[i]: row of the customer-demand table for retailer i, else -1 */
  int32_t retailer_slot[IMENV_MAX_NODES];
  int32_t num_retailers;

  int32_t delay[IMENV_MAX_NODES];       /* lead time, >= 1 in this build */
  /* integral capacities (the reference keeps them as float64) */
  int32_t init_inv[IMENV_MAX_NODES];
  int32_t inv_max[IMENV_MAX_NODES];
  int32_t order_max[IMENV_MAX_NODES];
  int32_t backlog_cap[IMENV_MAX_NODES]; /* -1 = uncapped */
  /* divergent split guard limits (IM_div_env.py:424,449,483,497): rounds > limit trips */
  int32_t split_limit[IMENV_MAX_NODES][4];

  double sell_price[IMENV_MAX_NODES];   /* serial price[i]; tree stage+2 */
  double buy_price[IMENV_MAX_NODES];    /* serial price[i+1]; tree stage+1 */
  double stock_cost[IMENV_MAX_NODES];
  double backlog_cost[IMENV_MAX_NODES];
  double inv_target[IMENV_MAX_NODES];

  /* action decode */
  int32_t standardise_actions;  /* 1: order = rev_scale(x), else x */
  int32_t decode_mode;          /* IMENV_DECODE_* */
  double a, b;                  /* scaling interval (rescale / rev_scale) */

  int32_t reward_mode;          /* IMENV_REWARD_* */

  /* observation: num_features entries of (group, index); per group a mode and
   * a per-node denominator (and clip for CLAMP_SCALED) */
  int32_t num_features;
  int32_t feat_group[IMENV_MAX_FEATURES];
  int32_t feat_index[IMENV_MAX_FEATURES];
  int32_t group_mode[IMENV_NUM_GROUPS];
  double group_den[IMENV_NUM_GROUPS][IMENV_MAX_NODES];
  double group_clip[IMENV_NUM_GROUPS][IMENV_MAX_NODES];
  int32_t prev_length;          /* L: history depth kept for DEMAND/ORDER_HIST */

  /* demand */
  int32_t demand_dist;          /* IMENV_DEMAND_*: what reset() draws with IMENV_LAYOUT_DRAW */
  double poisson_mu;
  int32_t uniform_low, uniform_high;
  int32_t noisy_demand;         /* div envs: double w.p. thr, then zero w.p. thr (IM_div_env.py:246-255) */
  double noisy_demand_threshold;
  int32_t noisy_delay;          /* initial latch (div envs read it from config, IM_div_env.py:50-51) */
  double noisy_delay_threshold;
  uint64_t seed;                /* Philox key */
} ImEnvSpec;

typedef struct ImEnv ImEnv;

/* Optional per-step outputs (the reference's `info` dict, IM_env.py:345-350 and
 * MAIM_env.py:399-409, plus the split state). Any pointer may be NULL.
 * int32 [n][N] unless noted. */
typedef struct ImEnvInfo {
  int32_t* order;        /* 'actual order' (order_r[t]) */
  int32_t* demand;       /* demand[t] */
  int32_t* acquisition;  /* acquisition[t] */
  int32_t* ship;         /* ship[t] */
  double* profit;        /* double [n][N] */
  int32_t* ship_to;      /* amount shipped INTO node c at t (ship_to_list[t][parent][c]) */
  int32_t* backlog_to;   /* backlog_to[parent][c] after the step (0 unless parent splits) */
} ImEnvInfo;

/* Per-episode metrics of a fused base-stock rollout (imenv_base_stock_rollout) */
#define IMENV_STAT_RETURN 0            /* sum_t reward (eval loop, inv_management.py:222-232) */
#define IMENV_STAT_OBJECTIVE 1         /* dfo_func: -1/T * np.sum(pmf(customer_demand) * rewards)
                                        * (base_restock_policy.py:24-45) */
#define IMENV_STAT_INVENTORY 2         /* sum_t sum_i inventory after the step (inv_management.py:589-591) */
#define IMENV_STAT_BACKLOG 3           /* sum_t sum_i backlog after the step */
#define IMENV_STAT_CUSTOMER_BACKLOG 4  /* sum_t backlog of the retailers (inv_management.py:592: bl[0]) */
#define IMENV_NUM_STATS 5

/* Batched episodes of the order-up-to policy (base_restock_policy.py:4-21) run entirely on the
 * device: num_policies x num_scenarios independent episodes of num_periods steps, each reset to
 * period 0 and stepped with actions = min(order_max, max(policy - (inv + order_u - backlog), 0)).
 * All pointers are device pointers. */
typedef struct ImEnvRollout {
  const double* policy;       /* [P][N] order-up-to level per node (float64, finite) */
  int64_t num_policies;       /* P >= 1 */
  int64_t num_scenarios;      /* S >= 1: demand scenarios (episodes) per policy */
  /* customer demand int32 [T][R][S] (reset(customer_demand=...) per scenario, the same table for
   * every policy), or NULL: drawn in-kernel per spec.demand_dist (+ noisy demand), Philox keyed by
   * (spec.seed, scenario_offset + s, episode) exactly like imenv_reset's draws for env id s */
  const int32_t* demand;
  int64_t scenario_offset;
  int64_t episode;            /* Philox counter word (>= 0) */
  /* dfo_func weights: demand_pmf[k] = env.dist.pmf(k) for k < pmf_len (values outside -> 0).
   * NULL: no objective (IMENV_STAT_OBJECTIVE reads 0). Needs num_retailers * T <= 128. */
  const double* demand_pmf;
  int32_t pmf_len;
  int32_t noisy_delay;        /* reset(noisy_delay=True, noisy_delay_threshold) (IM_env.py:180-182) */
  double noisy_delay_threshold;
  double* episode_stats;      /* out [IMENV_NUM_STATS][P][S], or NULL (then only policy_stats) */
  double* policy_stats;       /* out [P][IMENV_NUM_STATS][2]: np.mean, np.std over the S episodes, or NULL */
} ImEnvRollout;

/* Open-loop plan replay (imenv_plan_rollout): the LP scripts' evaluation loop, e.g. SHLP_8.py:737-766
 * (also SHLP*.py, DSHLP*.py, Oracle*.py, DecLP.py, Distributed*_LP.py): per demand scenario
 *   s = env.reset(customer_demand=d); step(plan[t]) for t < T;
 *   lp_reward += r; total_inventory += sum(s[:, 0]); total_backlog += sum(s[:, 1]);
 *   customer_backlog += s[0, 1]; profit[j, t] = r
 * for num_plans x num_scenarios episodes in one launch (state in registers, lead-time queue in LDS).
 * The inventory / backlog sums are of the state (= the scripts' observation sums, since every LP
 * script runs with standardise_state False). */
#define IMENV_PLAN_SHARED 0        /* actions [P][T][N]: plan p is replayed on every scenario */
#define IMENV_PLAN_PER_EPISODE 1   /* actions [T][P][S][N]: each (plan row, scenario) episode has its own
                                    * actions (an LP solved per demand scenario) */
typedef struct ImEnvPlanRollout {
  const void* actions;        /* device, action_dtype, layout plan_layout; decoded as step() decodes */
  int32_t action_dtype;       /* IMENV_F32 / IMENV_F64 */
  int32_t plan_layout;        /* IMENV_PLAN_* */
  int64_t num_plans;          /* P >= 1 */
  int64_t num_scenarios;      /* S >= 1 */
  const int32_t* demand;      /* customer demand int32 [T][R][S] or NULL (drawn, as ImEnvRollout.demand) */
  int64_t scenario_offset;
  int64_t episode;
  int32_t noisy_delay;        /* reset(noisy_delay=True, noisy_delay_threshold) */
  int32_t pad_;
  double noisy_delay_threshold;
  double* rewards;            /* out double [T][P][S]: the per-step reward (profit[j, t]), or NULL */
  double* episode_stats;      /* out [IMENV_NUM_STATS][P][S] (OBJECTIVE reads 0; CUSTOMER_BACKLOG is node 0's
                               * backlog, s[0, 1]), or NULL */
  double* policy_stats;       /* out [P][IMENV_NUM_STATS][2]: np.mean, np.std over the S episodes, or NULL */
} ImEnvPlanRollout;

/* Replaces the constructors: InvManagement.__init__ (IM_env.py:7-162),
 * MultiAgentInvManagement.__init__ (MAIM_env.py:8-173), InvManagementDiv.__init__
 * (IM_div_env.py:9-199), MultiAgentInvManagementDiv.__init__ (MAIM_div_env.py:9-237).
 * The caller derives the spec from the reference config dict (imenv/spec.py).
 * env_offset = global id of this handle's first env (RNG key; sharding). */
int imenv_create(const ImEnvSpec* spec, int64_t n_envs, int64_t env_offset, int device, ImEnv** out);

/* Replaces reset(customer_demand=None, noisy_delay=False, noisy_delay_threshold=0)
 * (IM_env.py:164-229 and siblings). Writes the period-0 observation to obs
 * ([n][N][F], obs_dtype). demand / demand_layout: IMENV_LAYOUT_* above (the
 * table is copied; the caller may free it after the call is stream-ordered).
 * Noisy demand (div envs, IM_div_env.py:246-255) applies to drawn and broadcast
 * demand only, as in the reference (not to demand passed per env).
 * noisy_delay != 0 latches noisy delay with the given threshold, as the reference
 * does (IM_env.py:180-182). delay_uniforms: optional device double [T][N][n] —
 * host-fed uniforms for the noisy-delay draw (u <= threshold; bit-exact parity
 * path); NULL = in-kernel Philox. episode: Philox counter word for this
 * episode; pass -1 to auto-increment (first reset -> 0). */
int imenv_reset(ImEnv* env, const int32_t* demand, int demand_layout, int noisy_delay,
                double noisy_delay_threshold, const double* delay_uniforms, int64_t episode, void* obs,
                int obs_dtype, void* stream);

/* Replaces step(action) / step(action_dict) (IM_env.py:287-360 and siblings).
 * actions: device [n][N] (action_dtype IMENV_F32 / IMENV_F64; f32 is promoted to
 * f64 before decoding, as the reference's ndarray path does). obs: [n][N][F]
 * (obs_dtype). reward: double [n] (SUM / SHARED_MEAN) or [n][N] (INDEPENDENT).
 * info: optional. done_out (HOST int*, may be NULL) receives period >= T. */
int imenv_step(ImEnv* env, const void* actions, int action_dtype, void* obs, int obs_dtype,
               double* reward, const ImEnvInfo* info, int32_t* done_out, void* stream);

/* Replaces dfo_func(policy, env, demand) (base_restock_policy.py:24-45) and the base-stock
 * evaluation loop (inv_management.py:222-232) for many policies and scenarios at once: one fused
 * launch (state in registers, lead-time queue in LDS, wavefront reductions of the metrics) plus a
 * small deterministic reduction launch for policy_stats. Scalar-reward specs only (IMENV_REWARD_SUM /
 * SHARED_MEAN). Independent of the handle's own env state (it may be mid-episode); uses its spec,
 * device and kernel cache. Always runs a hipRTC-specialised kernel (IMENV_E_UNSUPPORTED without it). */
int imenv_base_stock_rollout(ImEnv* env, const ImEnvRollout* args, void* stream);

/* Replaces the LP scripts' plan replay loop (SHLP_8.py:737-766 and the scripts listed at
 * ImEnvPlanRollout) for P plans x S scenarios in one fused launch (+ the stats reduction when
 * policy_stats is given). Scalar-reward specs only. Like imenv_base_stock_rollout, independent of the
 * handle's own env state; always hipRTC-specialised (IMENV_E_UNSUPPORTED without it). */
int imenv_plan_rollout(ImEnv* env, const ImEnvPlanRollout* args, void* stream);

/* Evaluation-harness metrics (inv_management.py:567-606, MA_inv_management.py:517-587,
 * MA_inv_management_div.py): with a buffer attached, every step() adds, per env, into row e of
 * acc (device double [n][4 + N], caller-owned; period 0 restarts each row from zero):
 *   [0] episode reward: += reward (IM / IM_div), or += each agent's reward in agent order (MA)
 *   [1] total inventory: += sum over agents of rev_scale(obs[m][0], 0, inv_max[m], a, b)
 *   [2] total backlog:   += sum over agents of rev_scale(obs[m][1], 0, inv_max[m], a, b)
 *   [3] customer backlog: += rev_scale(obs[0][1], 0, inv_max[0], a, b)
 *   [4 + m] stage reward: += profit[m]
 * from the float64 observation, in the harness's own summation order. NULL detaches. */
#define IMENV_METRIC_RETURN 0
#define IMENV_METRIC_INVENTORY 1
#define IMENV_METRIC_BACKLOG 2
#define IMENV_METRIC_CUSTOMER_BACKLOG 3
#define IMENV_METRIC_STAGE_PROFIT 4
int imenv_set_episode_metrics(ImEnv* env, double* acc);

/* np.mean / np.std (population) of each column of a device float64 [rows][cols] matrix into
 * out (device double [cols][2]) — e.g. the harness metrics above over n test episodes. */
int imenv_column_stats(const double* x, int64_t rows, int32_t cols, double* out, void* stream);

/* Centralised-critic observations: replaces central_critic_observer (models/CC_Model.py:196-214)
 * plus the opponent actions FillInActions writes (:165-193; CC_inv_management.py:394-407 in the
 * evaluation loop), flattened in RLlib's order for the Dict space of CC_inv_management.py:137-141
 * (keys sorted: opponent_action, opponent_obs, own_obs). For rows = n envs x num_agents agents:
 *   out[e][m] = [clip(actions[e][o], clip_lo, clip_hi) for o != m]
 *               [obs[e][o][0:F] for o != m] [obs[e][m][0:F]]        (o ascending)
 * obs: device [n][N][F] (obs_dtype), actions: device [n][N] (action_dtype) or NULL (zeros, as
 * central_critic_observer leaves them), out: device [n][N][N*F + N - 1] (obs_dtype). Works on any
 * row batch (e.g. a [T*n] rollout buffer); no env handle needed. The rows are written with
 * non-temporal stores (a later training pass reads them); IMENV_CC_NT=0 in the environment selects
 * plain stores. */
int imenv_cc_observation(int64_t n, int32_t num_agents, int32_t num_features, const void* obs, int obs_dtype,
                         const void* actions, int action_dtype, double clip_lo, double clip_hi, void* out,
                         void* stream);

/* Generalised advantage estimation over a device rollout buffer: replaces the compute_advantages
 * call of the trainers' postprocessing (models/CC_Policy.py:238-250; RLlib 1.5 compute_advantages
 * with use_gae, discount_cumsum = scipy lfilter; gamma 0.99 / lambda 0.95 at utils.py:19-23).
 * rewards / values: device [T][n] (float32 or float64), last_value: device [n] bootstrap value
 * (value_dtype) or NULL for completed episodes (last_r = 0). Outputs float32 [T][n]: advantages and,
 * if not NULL, value_targets = advantages + values. Arithmetic follows the reference's NumPy / SciPy
 * dtypes and operation order (float64, or float32 deltas with a float32 bootstrap; imenv_gae_kernel).
 * Outputs are written with non-temporal stores; IMENV_GAE_NT=0 selects plain stores. */
int imenv_gae(int64_t n, int32_t T, const void* rewards, int reward_dtype, const void* values, int value_dtype,
              const void* last_value, double gamma, double lambda, float* advantages, float* value_targets,
              void* stream);

/* State the reference's callers read directly (base_restock_policy.py:12:
 * env.inv/order_u/backlog[env.period]). Copies int32 [N][n] SoA into the given
 * device buffers (any may be NULL); *period (HOST) receives the current period. */
int imenv_get_state(ImEnv* env, int32_t* inv, int32_t* backlog, int32_t* order_u, int32_t* period,
                    void* stream);

/* Divergent-split guard trips ("Infinite Loop 1-4", MAIM_div_env.py:505-575):
 * per-env flags (device uint32 [n], may be NULL) and, synchronously, the OR of
 * all flags since the last reset into *any_out (HOST). */
int imenv_get_errors(ImEnv* env, uint32_t* flags, uint32_t* any_out, void* stream);

/* Shapes: number of nodes, observation features per node, customer-demand rows. */
int imenv_dims(const ImEnv* env, int32_t* num_nodes, int32_t* num_features, int32_t* num_retailers,
               int32_t* num_periods);

/* Inversion table used for in-kernel Poisson draws (uint32 thresholds, HOST
 * buffer of capacity `cap`); *len_out receives the table length. */
int imenv_poisson_table(const ImEnv* env, uint32_t* out, int32_t cap, int32_t* len_out);

/* Packed state layout chosen at create: element bytes (1 = uint8 / 2 = int16 when
 * the spec's bounds prove every state value fits in 0..255 / 32767, else 4), row length per env, and the rows of the
 * in-transit ring (one row of n envs per node and lead-time slot: the sum of the delays). */
int imenv_state_layout(const ImEnv* env, int32_t* elem_bytes, int32_t* row_len, int32_t* ring_depth);

/* Divergent split state layout (trees, IM_div_env.py:396-502 / MAIM_div_env.py:476-579 backlog_to):
 * the number of split children (nodes whose parent ships to more than one child; only they carry a
 * backlog_to) and its element bytes (2 = int16 when num_periods x the children's order_max fits 32767,
 * else 4). 0 children for serial chains. */
int imenv_split_layout(const ImEnv* env, int32_t* num_split_children, int32_t* elem_bytes);

/* Drawn-demand layout (IMENV_LAYOUT_DRAW, IM_env.py:194-200 / IM_div_env.py:235-255 demand draws): 0 when
 * every step draws its own period's demand, else the element bytes (1 = uint8, 2 = int16, 4 = int32) of a
 * [num_periods][num_retailers][n] table through which the step at t % 4 == 0 hands the demand of periods
 * t+1..t+3 (the rest of its Philox block; same values) to the next three steps. Chosen at imenv_create for
 * small single-retailer handles (<= 131,072 envs; IMENV_DTAB / IMENV_DTAB_MAX_ENVS override). */
int imenv_draw_layout(const ImEnv* env, int32_t* elem_bytes);

/* Host-fed noisy-delay uniforms for ONE period (device double [N][n]) written into the table that
 * reset(delay_uniforms=...) fills, so a caller can draw them lazily, step by step, in the
 * reference's order (np.random.uniform per node, factory first, IM_env.py:384-407) and keep its
 * host RNG stream identical to the reference even across mid-episode resets. period must be >= the
 * current period. Rows never written read as 1.0. Switches the handle to host-fed uniforms until
 * the next reset() without a table. */
int imenv_set_delay_uniforms(ImEnv* env, int32_t period, const double* u, void* stream);

/* Step-kernel selection. mode 1 (the default; IMENV_JIT=0 in the environment makes 0 the
 * default): step() runs a kernel compiled at run time with hipRTC for this spec, every spec value
 * a compile-time constant (first step per dtype/layout combination pays ~1 s of compilation;
 * cached per process). mode 0: the ahead-of-time kernels, which read the spec from device memory.
 * Both compute the same function; a JIT failure sends that dtype/layout combination (only) to the
 * mode-0 kernels and is reported by imenv_kernel_info (IMENV_JIT_STRICT=1 turns it into an
 * IMENV_E_UNSUPPORTED from step()); set_jit(1) retries failed combinations. */
int imenv_set_jit(ImEnv* env, int mode);

/* Store policy of the step kernel's output stores (hipRTC kernels; the ahead-of-time kernels always
 * use plain stores). Results are identical under every policy; no reference counterpart (a
 * performance knob of this implementation).
 *  IMENV_STORE_DEFAULT: observation and reward stores write-through (cache policy sc1: written to
 *    memory at once, nothing left dirty in L2 for the end-of-launch write-back, which otherwise
 *    costs ~bytes / 6 TB/s at every dependent launch boundary); the state rows too when a launch's
 *    observation + reward bytes are at most 24 MiB (small batches: L2 is 32 MiB), else plain.
 *  IMENV_STORE_STREAM: non-temporal observation / reward stores (outputs bound for a rollout buffer
 *    read much later).
 *  IMENV_STORE_PLAIN: plain cached stores everywhere (the round-2 default).
 *  IMENV_STORE_WRITETHROUGH: write-through for observations, rewards and state rows at any size. */
#define IMENV_STORE_DEFAULT 0
#define IMENV_STORE_STREAM 1
#define IMENV_STORE_PLAIN 2
#define IMENV_STORE_WRITETHROUGH 3
int imenv_set_store_policy(ImEnv* env, int policy);

/* NUL-terminated description of the kernel the last step() launched, truncated to len bytes. */
int imenv_kernel_info(const ImEnv* env, char* buf, int64_t len);

/* Diagnostics (no device needed): generate and compile with hipRTC the specialised step kernel of
 * `spec` for `arch` (e.g. "gfx950"); flags = bit0 f64 actions, bit1 f64 obs, bit2 noisy delay,
 * bit3 noisy demand, bit4 host-fed delay uniforms, bits 5-9 demand layout, bit10 episode metrics, bit11
 * streaming stores (IMENV_STORE_STREAM), bit13 write-through observation / reward stores, bit14
 * write-through state rows. With bit 12 set it
 * compiles the rollout kernel instead: bit13 demand table, bit14 noisy delay, bit15 noisy
 * demand, bit16 objective, bits 17-18 action source (0 base-stock, 1 shared plan, 2 per-episode
 * plan), bit19 float64 plan actions. `log` receives "ok" or
 * the compiler log. */
int imenv_jit_check(const ImEnvSpec* spec, const char* arch, uint32_t flags, char* log, int64_t log_len);

/* Diagnostics: per-wave phase timestamps of the last step() launched by a kernel built with
 * -DIMENV_STAMPS=1 (IMENV_JIT_OPTS) on a handle created with IMENV_STAMPS=1 in the environment:
 * 8 uint64 per wave (s_memrealtime, 100 MHz: entry, loads issued, loads landed, computed, slab
 * barrier passed, stores issued, stores acknowledged; then XCC id << 32 | block). Copies up to cap
 * values to HOST memory (synchronous); *count receives the buffer length (0: no stamps). */
int imenv_debug_stamps(ImEnv* env, uint64_t* out, int64_t cap, int64_t* count);

void imenv_destroy(ImEnv* env);

const char* imenv_last_error(void);

int imenv_abi_version(void);

/* sizeof(ImEnvSpec) as compiled into the library (binding layout check). */
int64_t imenv_spec_size(void);

#ifdef __cplusplus
}
#endif

#endif /* IMENV_H */
