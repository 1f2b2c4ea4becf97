"""VectorInvEnv — a batch of n independent inventory envs resident in HBM.

Python host over the C ABI (include/imenv.h). All buffers are torch tensors on
the HIP device; every call is enqueued on the current torch stream of that
device, so it composes with a torch policy without synchronisation. The envs
advance in lockstep (all share the period t, as every reference env has a
fixed horizon and no auto-reset).

    env = VectorInvEnv("MAIM", env_config, n_envs=1 << 20)
    obs = env.reset()                      # [n, N, F] float32, period 0
    obs, reward, done, info = env.step(actions)   # actions [n, N] in [a, b]

This replaces, batched, the reference's reset()/step() of the four env classes
(environments/IM_env.py:164-360, MAIM_env.py:176-411, IM_div_env.py:201-549,
MAIM_div_env.py:240-630). There is no CPU fallback: construction fails loudly
without a HIP device or without libimenv.so.
"""
import ctypes
from ctypes import byref, c_int32, c_uint32, c_void_p

import numpy as np
import torch

from . import _native as nat
from .spec import HostSpec, build_spec

_FLOATS = (torch.float32, torch.float64)


class VectorInvEnv:
    def __init__(self, kind_or_spec, config=None, n_envs=1, device=None, env_offset=0,
                 obs_dtype=torch.float32):
        self.spec = kind_or_spec if isinstance(kind_or_spec, HostSpec) else build_spec(kind_or_spec, config or {})
        if not torch.cuda.is_available():
            raise nat.ImEnvNativeError("VectorInvEnv needs a HIP device; there is no CPU fallback")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.n = int(n_envs)
        self.env_offset = int(env_offset)
        if obs_dtype not in (torch.float32, torch.float64):
            raise ValueError("obs_dtype must be float32 or float64")
        self.obs_dtype = obs_dtype
        self.lib = nat.load()
        self._c = self.spec.to_c()
        h = c_void_p()
        nat.check(self.lib.imenv_create(byref(self._c), self.n, self.env_offset, self.device.index, byref(h)),
                  "imenv_create")
        self._h = h
        self.N = self.spec.num_nodes
        self.F = self.spec.num_features
        self.R = self.spec.num_retailers
        self.T = self.spec.num_periods
        self.period = 0
        self.episode = -1
        self._keep = []
        self._done = c_int32(0)
        self._done_ref = byref(self._done)
        self.noisy_delay = bool(self.spec.noisy_delay)   # latched by reset(noisy_delay=True), as the C handle

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        # the raw handle of the current stream (the public torch.cuda.current_stream() builds a Stream
        # object per call: a few microseconds of the per-step host cost)
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:
            return c_void_p(raw(self.device.index))
        return c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _obs_code(self, dtype):
        return nat.F64 if dtype == torch.float64 else nat.F32

    def _out(self, t, shape, dtypes, what):
        """A caller-owned output buffer the kernel writes in place: checked before any launch (a
        wrong-sized buffer would be written out of bounds), else a fresh tensor."""
        if t is None:
            return torch.empty(shape, dtype=dtypes[0], device=self.device)
        if not torch.is_tensor(t) or t.device != self.device or t.dtype not in dtypes or \
                t.shape != shape or not t.is_contiguous():
            raise ValueError("%s must be a contiguous %s tensor of shape %s on %s (got %s)" % (
                what, "/".join(str(d) for d in dtypes), tuple(shape), self.device,
                (tuple(t.shape), t.dtype, t.device, t.is_contiguous()) if torch.is_tensor(t) else type(t)))
        return t

    def reward_shape(self):
        return (self.n, self.N) if self.spec.reward_mode == nat.REWARD_INDEPENDENT else (self.n,)

    def _demand_tensor(self, customer_demand):
        """-> (device int32 tensor, layout). Per-env [n,T] / [n,R,T] or broadcast [T] / [R,T]."""
        cd = torch.as_tensor(np.asarray(customer_demand) if not torch.is_tensor(customer_demand)
                             else customer_demand)
        cd = cd.to(device=self.device, dtype=torch.int32)
        T, R, n = self.T, self.R, self.n
        if cd.shape[-1] < T:
            raise ValueError("customer demand shorter than num_periods")
        cd = cd[..., :T]
        per_env = cd.dim() == (2 if self.spec.serial else 3)
        if per_env:
            # per env: serial [n, T] -> [T, 1, n]; tree [n, R, T] -> [T, R, n]
            if cd.dim() == 2:
                cd = cd[:, None, :]
            if cd.shape[0] != n or cd.shape[1] != R:
                raise ValueError("per-env demand must be [n, T] (serial) or [n, R, T] (tree)")
            return cd.permute(2, 1, 0).contiguous(), nat.LAYOUT_PER_ENV
        if cd.dim() == 1:
            cd = cd[None, :]
        if cd.dim() != 2 or cd.shape[0] != R:
            raise ValueError("broadcast demand must be [T] (serial) or [R, T] (tree)")
        return cd.t().contiguous(), nat.LAYOUT_BROADCAST

    # ------------------------------------------------------------------ API
    def reset(self, customer_demand=None, noisy_delay=False, noisy_delay_threshold=0.0,
              delay_uniforms=None, episode=None, obs_out=None):
        """reset(customer_demand=None, noisy_delay=False, noisy_delay_threshold=0) (IM_env.py:164).

        customer_demand: per-env [n, T] (serial) / [n, R, T] (tree), or one table [T] / [R, T]
        for every env; None draws from the spec's distribution in-kernel (Philox, keyed by
        (seed, global env id, episode)). delay_uniforms: [n, T, N] float64 host-fed uniforms
        for noisy delay (bit-exact parity), None = in-kernel draws.
        """
        keep = []
        dptr, layout = None, nat.LAYOUT_DRAW
        if customer_demand is not None:
            d, layout = self._demand_tensor(customer_demand)
            keep.append(d)
            dptr = d.data_ptr()
        elif self.spec.demand_dist == "custom":
            d, layout = self._demand_tensor(self.spec.custom_demand)
            keep.append(d)
            dptr = d.data_ptr()
        uptr = None
        if delay_uniforms is not None:
            u = torch.as_tensor(delay_uniforms).to(device=self.device, dtype=torch.float64)
            if tuple(u.shape) != (self.n, self.T, self.N):
                raise ValueError("delay_uniforms must be [n, T, N]")
            u = u.permute(1, 2, 0).contiguous()
            keep.append(u)
            uptr = u.data_ptr()
        obs = self._out(obs_out, (self.n, self.N, self.F), (self.obs_dtype, torch.float32, torch.float64), "obs_out")
        ep = -1 if episode is None else int(episode)
        nat.check(self.lib.imenv_reset(self._h, dptr, layout, int(bool(noisy_delay)), float(noisy_delay_threshold),
                                       uptr, ep, obs.data_ptr(), self._obs_code(obs.dtype), self._stream()),
                  "imenv_reset")
        self._keep = keep          # the copies are stream-ordered; keep sources alive one call
        self.noisy_delay = self.noisy_delay or bool(noisy_delay)
        self.period = 0
        self.episode = self.episode + 1 if episode is None else int(episode)
        return obs

    def set_delay_uniforms(self, period, u):
        """Host-fed noisy-delay uniforms [n, N] (float64) for one period (imenv_set_delay_uniforms)."""
        t = torch.as_tensor(u).to(device=self.device, dtype=torch.float64).reshape(self.n, self.N).t().contiguous()
        nat.check(self.lib.imenv_set_delay_uniforms(self._h, int(period), t.data_ptr(), self._stream()),
                  "imenv_set_delay_uniforms")
        self._keep_u = t

    def rollout_stepper(self, actions, obs_out, reward_out):
        """A launcher for step() over a rollout buffer whose tensors are validated once, here:
        actions [T, n, N] float32 / float64, obs_out [T + 1, n, N, F] (row t + 1 receives the
        observation after step t; row 0 is for reset(obs_out=obs_out[0])) or [T, n, N, F] (row t),
        reward_out [T] + reward_shape(), all contiguous on this device. stepper(t) then launches the
        step of period t with precomputed pointers on the current stream: one C call and no tensor
        checks, for batches small enough that step()'s per-call host work (~9 us) would exceed the
        kernel. t must be the handle's current period (0 after reset()). Returns done (period >= T)
        like step(). Same kernels, same results as step(). The stepper writes into the tensors given
        here for its whole life (their pointers are taken now): rebinding a buffer means a new
        stepper. Stepping past the horizon raises like step() does (IMENV_E_DONE)."""
        T, n, N, F = self.T, self.n, self.N, self.F
        ok = (torch.is_tensor(actions) and actions.device == self.device and actions.dtype in _FLOATS
              and actions.is_contiguous() and tuple(actions.shape) == (T, n, N))
        if not ok:
            raise ValueError("actions must be a contiguous float32/float64 [%d, %d, %d] tensor on %s" % (T, n, N, self.device))
        if not (torch.is_tensor(obs_out) and obs_out.device == self.device and obs_out.dtype in _FLOATS and
                obs_out.is_contiguous() and tuple(obs_out.shape[1:]) == (n, N, F) and obs_out.shape[0] in (T, T + 1)):
            raise ValueError("obs_out must be a contiguous float32/float64 [%d or %d, %d, %d, %d] tensor on %s"
                             % (T + 1, T, n, N, F, self.device))
        rshape = (T,) + self.reward_shape()
        self._out(reward_out, rshape, (torch.float64,), "reward_out")
        shift = 1 if obs_out.shape[0] == T + 1 else 0
        a_ptr = [actions[t].data_ptr() for t in range(T)]
        o_ptr = [obs_out[t + shift].data_ptr() for t in range(T)]
        r_ptr = [reward_out[t].data_ptr() for t in range(T)]
        adt = nat.F64 if actions.dtype == torch.float64 else nat.F32
        odt = nat.F64 if obs_out.dtype == torch.float64 else nat.F32
        lib, h, done, done_ref, stream = self.lib.imenv_step, self._h, self._done, self._done_ref, self._stream
        keep = (actions, obs_out, reward_out)

        def stepper(t):
            if t >= T:
                raise ValueError("stepper(%d): past the horizon of %d periods (reset first)" % (t, T))
            if t != self.period:
                raise ValueError("stepper(%d) at period %d: the kernel steps the handle's own period" % (t, self.period))
            rc = lib(h, a_ptr[t], adt, o_ptr[t], odt, r_ptr[t], None, done_ref, stream())
            if rc:
                nat.check(rc, "imenv_step")
            self.period += 1
            return bool(done.value)

        stepper.buffers = keep      # the tensors stay alive as long as the stepper
        return stepper

    def step(self, actions, obs_out=None, reward_out=None, info=False, info_out=None):
        """step(action) (IM_env.py:287-360): actions [n, N] (or [n*N]) in the spec's action units.

        info=True returns the info tensors (order, demand, acquisition, ship, profit, ship_to,
        backlog_to, each [n, N]); info_out: a dict of caller-owned contiguous tensors of those names
        ([n, N], int32 / float64 profit) the kernel writes instead (no allocation per step)."""
        a = actions
        # fast path: a contiguous float device tensor of n*N values is passed as is
        if not (torch.is_tensor(a) and a.device == self.device and a.dtype in _FLOATS and a.is_contiguous() and
                a.numel() == self.n * self.N):
            a = a if torch.is_tensor(a) else torch.as_tensor(np.asarray(a))
            if a.device != self.device or a.dtype not in _FLOATS:
                a = a.to(device=self.device, dtype=torch.float64 if a.dtype == torch.float64 else torch.float32)
            a = a.reshape(self.n, self.N).contiguous()
        obs = self._out(obs_out, (self.n, self.N, self.F), (self.obs_dtype, torch.float32, torch.float64), "obs_out")
        rew = self._out(reward_out, self.reward_shape(), (torch.float64,), "reward_out")
        inf = None
        iptr = None
        if info or info_out is not None:
            if info_out is not None:
                inf = {k: self._out(info_out[k], (self.n, self.N),
                                    (torch.float64 if k == "profit" else torch.int32,), "info_out[%s]" % k)
                       for k in ("order", "demand", "acquisition", "ship", "profit", "ship_to", "backlog_to")}
            else:
                z = lambda dt: torch.empty((self.n, self.N), dtype=dt, device=self.device)
                inf = dict(order=z(torch.int32), demand=z(torch.int32), acquisition=z(torch.int32),
                           ship=z(torch.int32), profit=z(torch.float64), ship_to=z(torch.int32),
                           backlog_to=z(torch.int32))
            ci = nat.ImEnvInfo(*[inf[k].data_ptr() for k in ("order", "demand", "acquisition", "ship",
                                                               "profit", "ship_to", "backlog_to")])
            iptr = byref(ci)
        done = self._done
        rc = self.lib.imenv_step(self._h, a.data_ptr(), nat.F64 if a.dtype == torch.float64 else nat.F32,
                                 obs.data_ptr(), nat.F64 if obs.dtype == torch.float64 else nat.F32, rew.data_ptr(),
                                 iptr, self._done_ref, self._stream())
        if rc:
            nat.check(rc, "imenv_step")
        self._keep = [a]
        self.period += 1
        return obs, rew, bool(done.value), inf

    def state(self, out=None):
        """inv / backlog / order_u at the current period as [n, N] int32 (base_restock_policy.py:12).
        out: three caller-owned contiguous int32 [N, n] tensors to write instead (no allocation)."""
        if out is not None:
            bufs = [self._out(b, (self.N, self.n), (torch.int32,), "state out") for b in out]
        else:
            bufs = [torch.empty((self.N, self.n), dtype=torch.int32, device=self.device) for _ in range(3)]
        p = c_int32()
        nat.check(self.lib.imenv_get_state(self._h, bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr(),
                                           byref(p), self._stream()), "imenv_get_state")
        return dict(inv=bufs[0].t(), backlog=bufs[1].t(), order_u=bufs[2].t(), period=p.value)

    def errors(self):
        """Per-env split-guard flags ("Infinite Loop", MAIM_div_env.py:505-575) and their OR (syncs)."""
        flags = torch.empty(self.n, dtype=torch.int32, device=self.device)
        anyv = c_uint32()
        nat.check(self.lib.imenv_get_errors(self._h, flags.data_ptr(), byref(anyv), self._stream()),
                  "imenv_get_errors")
        return flags, int(anyv.value)

    def attach_metrics(self, enable=True):
        """Accumulate the reference evaluation harness's per-episode metrics in every step()
        (imenv_set_episode_metrics): episode reward, total inventory / backlog, customer backlog and
        per-stage reward, per env, as inv_management.py:567-606 / MA_inv_management.py:517-587 do."""
        if enable:
            self._metrics = torch.zeros((self.n, 4 + self.N), dtype=torch.float64, device=self.device)
            ptr = self._metrics.data_ptr()
        else:
            self._metrics, ptr = None, None
        nat.check(self.lib.imenv_set_episode_metrics(self._h, ptr), "imenv_set_episode_metrics")

    def metrics(self):
        """Per-env sums since the last reset: {name: [n]} plus "stage_reward" [n, N] (device tensors)."""
        m = getattr(self, "_metrics", None)
        if m is None:
            raise RuntimeError("attach_metrics() first")
        out = {k: m[:, j] for j, k in enumerate(nat.METRIC_NAMES)}
        out["stage_reward"] = m[:, 4:]
        return out

    def metrics_stats(self):
        """np.mean / np.std over the n envs of every metric column: [4 + N, 2] (imenv_column_stats)."""
        m = getattr(self, "_metrics", None)
        if m is None:
            raise RuntimeError("attach_metrics() first")
        out = torch.empty((m.shape[1], 2), dtype=torch.float64, device=self.device)
        nat.check(self.lib.imenv_column_stats(m.data_ptr(), m.shape[0], m.shape[1], out.data_ptr(), self._stream()),
                  "imenv_column_stats")
        return out

    def poisson_table(self):
        ln = c_int32()
        nat.check(self.lib.imenv_poisson_table(self._h, None, 0, byref(ln)), "imenv_poisson_table")
        buf = (ctypes.c_uint32 * max(ln.value, 1))()
        nat.check(self.lib.imenv_poisson_table(self._h, buf, ln.value, byref(ln)), "imenv_poisson_table")
        return np.array(buf[:ln.value], dtype=np.uint64)

    def state_layout(self):
        """(element bytes, packed row length, in-transit ring rows = sum of delays) of the HBM state."""
        eb, rl, rd = c_int32(), c_int32(), c_int32()
        nat.check(self.lib.imenv_state_layout(self._h, byref(eb), byref(rl), byref(rd)), "imenv_state_layout")
        return eb.value, rl.value, rd.value

    def split_layout(self):
        """(split children carrying a backlog_to, its element bytes) of the HBM split state."""
        nb, eb = c_int32(), c_int32()
        nat.check(self.lib.imenv_split_layout(self._h, byref(nb), byref(eb)), "imenv_split_layout")
        return nb.value, eb.value

    def draw_layout(self):
        """Element bytes of the drawn-demand table (IMENV_LAYOUT_DRAW) through which the step at t % 4 == 0
        hands periods t+1..t+3 to the next three steps, or 0 when every step draws its own period's demand
        (imenv_draw_layout)."""
        eb = c_int32()
        nat.check(self.lib.imenv_draw_layout(self._h, byref(eb)), "imenv_draw_layout")
        return eb.value

    def step_traffic(self, action_bytes=4, obs_bytes=4, host_demand=False, metrics=False, handover=False):
        """Algorithmic HBM bytes of one step() per env: (steady state, average over an episode)."""
        per = self.step_traffic_per_period(action_bytes, obs_bytes, host_demand, metrics, handover)
        return per[-1], float(np.mean(per))

    def step_traffic_per_period(self, action_bytes=4, obs_bytes=4, host_demand=False, metrics=False, handover=False):
        """Algorithmic HBM bytes of the step() at period t per env, for t = 0 .. T-1.

        The minimal traffic of this handle's layout: actions; the net-inventory
        (inv - backlog) and order_u rows read + written (no read at t = 0: the initial state is
        implicit); node i's arrival read
        (only once t >= d_i) and departure written; the time-dependent observation's other in-transit
        slots; int32 noisy-delay carry and divergent backlog_to rows; the demand / order history rows
        (written every step, read for the features j >= 1); the observation; the reward; optional
        host-fed demand and harness-metric rows. `handover=True` adds the drawn-demand table's bytes
        (draw_layout: periods t+1..t+3 written at t % 4 == 0, read at the other periods): traffic of an
        implementation choice, like the state record's unused slots, so not part of the algorithmic
        figure the roofline is priced on (bench.py reports it beside it).
        """
        es, NP, _ = self.state_layout()
        s = self.spec
        N, T = s.num_nodes, s.num_periods
        d = [int(x) for x in s.delay]
        nbto, bto_es = self.split_layout()
        dtab_es = self.draw_layout() if handover and not host_demand else 0
        split = nbto > 0
        hist = any(g in (nat.G_DEMAND_HIST, nat.G_ORDER_HIST) and j >= 1 for g, j in s.features)
        per = []
        # noisy-delay carry rows: int16 beside uint8 state, else int32, padded to 4 bytes (CarryOf /
        # row_len in imenv_device.h); divergent backlog_to rows: the split children's only, int16 or int32
        # (BtoRow), padded to 4 bytes
        cb = 2 if es == 1 else 4
        carry_row = cb * (((N + 1) & ~1) if cb == 2 else N)
        bto_row = bto_es * (((nbto + 1) & ~1) if bto_es == 2 else nbto)
        for t in range(T):
            b = N * action_bytes + 2 * NP * es + (2 * NP * es if t > 0 else 0)
            b += es * sum(1 for i in range(N) if t >= d[i]) + N * es
            for on, row in ((self.noisy_delay, carry_row), (split, bto_row)):
                if on:
                    b += row + (row if t > 0 else 0)
            if hist:
                b += 2 * NP * es
            for g, j in s.features:
                if g in (nat.G_DEMAND_HIST, nat.G_ORDER_HIST) and j >= 1 and t - j >= 0:
                    b += NP * es
                elif g == nat.G_TRANSIT:
                    b += es * sum(1 for i in range(N) if j < d[i] - 1 and t + 1 + j - d[i] >= 0)
            b += N * s.num_features * obs_bytes
            b += 8 * N if s.reward_mode == nat.REWARD_INDEPENDENT else 8
            if host_demand:
                b += 4 * s.num_retailers
            if dtab_es:
                b += dtab_es * s.num_retailers * (sum(1 for w in (1, 2, 3) if t + w < T) if t % 4 == 0 else 1)
            if metrics:
                b += 16 * (4 + N) - (8 * (4 + N) if t == 0 else 0)
            per.append(b)
        return per

    STORE_POLICIES = ("default", "stream", "plain", "writethrough")

    def set_store_policy(self, policy):
        """Store policy of the step kernel's outputs (imenv.h); same results under all:
        "default": write-through observation / reward stores (nothing left dirty in L2 for the
        end-of-launch write-back), the state rows too for batches whose outputs fit in L2;
        "stream": non-temporal stores (outputs read much later, e.g. a rollout buffer);
        "plain": plain cached stores; "writethrough": write-through for every store."""
        codes = dict(zip(self.STORE_POLICIES, (nat.STORE_DEFAULT, nat.STORE_STREAM, nat.STORE_PLAIN,
                                               nat.STORE_WRITETHROUGH)))
        if policy not in codes:
            raise ValueError("store policy must be one of %s" % (self.STORE_POLICIES,))
        nat.check(self.lib.imenv_set_store_policy(self._h, codes[policy]), "imenv_set_store_policy")

    def set_jit(self, mode):
        """1: hipRTC kernel specialised for this spec (default); 0: ahead-of-time kernels."""
        nat.check(self.lib.imenv_set_jit(self._h, int(mode)), "imenv_set_jit")

    def kernel_info(self):
        """Description of the kernel the last step() launched (and any JIT failure)."""
        buf = ctypes.create_string_buffer(512)
        nat.check(self.lib.imenv_kernel_info(self._h, buf, len(buf)), "imenv_kernel_info")
        return buf.value.decode()

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.device)
            self.lib.imenv_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
