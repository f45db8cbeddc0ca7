"""Times the reference's own PPO iteration (imported from /root/reference, CPU, as tests/golden/make_golden.py does)
next to oracle/torch_cpu_ppo.py's restatement on the same threads -- the cross-check behind bench.py's cpu_baseline.
Build-host only (reads /root/reference): python scripts/ref_cpu_timing.py [N] [threads]."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from make_golden import _RowDict, import_reference  # noqa: E402
from oracle import torch_cpu_ppo  # noqa: E402


def reference_iteration(N, O=48, A=12, T=24):
    PPO, ActorCritic, _ = import_reference("/root/reference")
    torch.manual_seed(0)
    obs = _RowDict({"policy": torch.randn(N, O)}, batch_size=[N], device="cpu")
    groups = {"policy": ["policy"], "critic": ["policy"]}
    pol = ActorCritic(obs, groups, A, actor_hidden_dims=[256] * 3, critic_hidden_dims=[256] * 3)
    alg = PPO(pol, device="cpu")
    alg.init_storage("rl", N, T, obs, [A])
    g = torch.Generator().manual_seed(1)
    t0 = time.perf_counter()
    with torch.inference_mode():
        for _ in range(T):
            alg.act(obs)
            obs = _RowDict({"policy": torch.randn(N, O, generator=g)}, batch_size=[N], device="cpu")
            rew = torch.randn(N, generator=g)
            dones = (torch.rand(N, generator=g) < 0.02).long()
            alg.process_env_step(obs, rew, dones, {"time_outs": torch.zeros(N)})
    t1 = time.perf_counter()
    with torch.inference_mode():
        alg.compute_returns(obs)
    t2 = time.perf_counter()
    alg.update()
    t3 = time.perf_counter()
    return {"rollout": round(t1 - t0, 3), "returns": round(t2 - t1, 3), "update": round(t3 - t2, 3),
            "env_steps_per_s": round(N * T / (t3 - t0), 1)}


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    th = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    torch.set_num_threads(th)
    ref = reference_iteration(N)
    rate, secs, parts = torch_cpu_ppo.time_iterations(N, iters=1, warmup=0, threads=th)
    print({"N": N, "threads": th, "reference": ref,
           "port": {"env_steps_per_s": round(rate, 1), **parts["seconds"]}})


if __name__ == "__main__":
    main()
