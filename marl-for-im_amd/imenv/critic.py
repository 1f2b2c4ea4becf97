"""Centralised-critic observations on the GPU (models/CC_Model.py, CC_inv_management.py).

``cc_observation(obs, actions)`` builds, for every env and agent, what the reference's
central_critic_observer (CC_Model.py:196-214) and FillInActions callback (:165-193) produce for the
centralised-critic PPO trainers, in RLlib's flattened Dict order (opponent_action, opponent_obs,
own_obs; gym sorts the keys of the space declared at CC_inv_management.py:137-141):

    obs [B, N, F] (+ actions [B, N])  ->  [B, N, N*F + N - 1]

B is any batch of env rows: one step's [n] envs, or a whole [T, n] rollout buffer flattened.
``split_cc_observation`` gives back the three dict entries as views.
"""
import torch

from . import _native as nat


def cc_observation(obs, actions=None, clip=(-1.0, 1.0), out=None):
    if obs.dim() < 3:
        raise ValueError("obs must be [..., N, F]")
    lead = obs.shape[:-2]
    N, F = obs.shape[-2], obs.shape[-1]
    if N < 2:
        raise ValueError("a centralised critic needs at least 2 agents")
    if obs.dtype not in (torch.float32, torch.float64) or not obs.is_cuda:
        raise ValueError("obs must be a float32/float64 device tensor")
    o = obs.contiguous().reshape(-1, N, F)
    B = o.shape[0]
    a = None
    if actions is not None:
        a = actions.to(device=obs.device).contiguous().reshape(B, N)
        if a.dtype not in (torch.float32, torch.float64):
            a = a.to(torch.float64)
    W = N * F + N - 1
    if out is None:
        out = torch.empty((B, N, W), dtype=obs.dtype, device=obs.device)
    elif (out.dtype != obs.dtype or out.device != obs.device or not out.is_contiguous() or
          out.numel() != B * N * W):
        raise ValueError("out must be a contiguous %s tensor of %d x %d x %d values on %s"
                         % (obs.dtype, B, N, W, obs.device))
    lib = nat.load()
    st = torch.cuda.current_stream(obs.device).cuda_stream
    nat.check(lib.imenv_cc_observation(B, N, F, o.data_ptr(), nat.F64 if o.dtype == torch.float64 else nat.F32,
                                       a.data_ptr() if a is not None else None,
                                       nat.F64 if (a is None or a.dtype == torch.float64) else nat.F32,
                                       float(clip[0]), float(clip[1]), out.data_ptr(), st), "imenv_cc_observation")
    return out.reshape(*lead, N, N * F + N - 1)


def split_cc_observation(cc, num_features):
    """[..., N, N*F + N - 1] -> dict(opponent_action, opponent_obs, own_obs) views."""
    N, F = cc.shape[-2], int(num_features)
    return {"opponent_action": cc[..., :N - 1], "opponent_obs": cc[..., N - 1:(N - 1) * (F + 1)],
            "own_obs": cc[..., (N - 1) * (F + 1):]}
