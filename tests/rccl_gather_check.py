"""Helper of tests/test_rccl_gpu.py (run as its own process): the per-step all-gather of bench.py's
N-rank line (imenv.shard.StepGather) over a one-rank "nccl" (RCCL) process group on one MI355X.

Handle A steps C2 envs straight into StepGather's double-buffered send buffers, with each step's
collective in flight on RCCL's stream under the next step (bench.py's timed_gather sequence); handle
B, same envs and actions, steps into plain buffers. Every gathered step must equal B's outputs bit for
bit, which checks the stream ordering of the pipeline (the env never overwrites a buffer whose
collective is still reading it, and result(t) waits for collective t) with RCCL itself. Prints one
JSON line.
"""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd")]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import torch
    import torch.distributed as dist
    from bench import C2_CONFIG
    from imenv import VectorInvEnv
    from imenv.shard import StepGather

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    a = VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev)
    b = VectorInvEnv("MAIM", C2_CONFIG, n_envs=n, device=dev)
    T = a.T
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    acts = torch.rand((2 * T, n, a.N), generator=g, device=dev) * 2.2 - 1.1
    obs_b = torch.empty((n, a.N, a.F), dtype=torch.float32, device=dev)
    rew_b = torch.empty(b.reward_shape(), dtype=torch.float64, device=dev)
    gth = StepGather(obs_b, rew_b)
    steps = mismatches = 0
    prev = None
    for s in range(2 * T):
        t = s % T
        if t == 0:
            a.reset()
            b.reset()
        a.step(acts[s], obs_out=gth.obs_out(s), reward_out=gth.reward_out(s))
        gth.start(s)
        b.step(acts[s], obs_out=obs_b, reward_out=rew_b)
        want = (obs_b.clone(), rew_b.clone())
        if prev is not None:         # step s-1's collective completed under step s
            o, r = gth.result(s - 1)
            mismatches += int(not (torch.equal(o, prev[0]) and torch.equal(r, prev[1])))
            steps += 1
        prev = want
    o, r = gth.result(2 * T - 1)
    mismatches += int(not (torch.equal(o, prev[0]) and torch.equal(r, prev[1])))
    steps += 1
    torch.cuda.synchronize(dev)
    print(json.dumps({"backend": dist.get_backend(), "collective": "all_gather_into_tensor" if gth._into else "list",
                      "world": dist.get_world_size(), "n_envs": n, "steps": steps, "mismatches": mismatches}),
          flush=True)
    a.close()
    b.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
