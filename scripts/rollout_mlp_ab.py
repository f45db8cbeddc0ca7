"""The rollout step's policy half (PPO.act: the captured act graph of modules/act_graph.py) with the one-launch forward
(rollout_mlp.hip) against the layer-by-layer launches (RSLRL_ROLLOUT_MLP=0), alternated in one process on C3's
networks: HIP-event time per step at the given env counts.

    python scripts/rollout_mlp_ab.py --num-envs 16384 65536 --steps 240 --rounds 3 --out gpurun_out/rollout_mlp_ab.json
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd.modules import ActorCritic  # noqa: E402
from rsl_rl_amd.modules.act_graph import RolloutActGraph  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, nargs="+", default=[16384, 65536])
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--modes", nargs="+", default=["0", "1"], help="0: layer by layer; 1: rslrl_rollout_mlp_pair")
    ap.add_argument("--out", default="gpurun_out/rollout_mlp_ab.json")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    out = {"note": __doc__.strip().splitlines()[0], "runs": []}
    for n in a.num_envs:
        torch.manual_seed(0)
        obs = {"policy": torch.randn(n, 48, device=dev)}
        pol = ActorCritic(obs, {"policy": ["policy"], "critic": ["policy"]}, 12, actor_hidden_dims=[256, 256, 256],
                          critic_hidden_dims=[256, 256, 256], actor_obs_normalization=True,
                          critic_obs_normalization=True).to(dev)
        pol.update_normalization(obs)
        res, hres = {m: [] for m in a.modes}, {m: [] for m in a.modes}
        for r in range(a.rounds):
            for mode in (a.modes if r % 2 == 0 else a.modes[::-1]):
                fused_mlp._ROLLOUT_MLP = mode != "0"
                g = RolloutActGraph(pol) if a.graph else None
                with torch.inference_mode(), fused_mlp.frozen_weights():
                    for _ in range(4):  # eager, capture, replays
                        if g is None or g(obs) is None:
                            pol.act_and_evaluate(obs)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    t0 = time.perf_counter()
                    for _ in range(a.steps):
                        if g is None or g(obs) is None:
                            pol.act_and_evaluate(obs)
                    host = (time.perf_counter() - t0) * 1e6 / a.steps
                    e1.record()
                    torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.steps
                res[mode].append(us)
                hres[mode].append(host)
                print(json.dumps({"num_envs": n, "round": r, "rollout_mlp": mode, "us_per_step": round(us, 2),
                                  "host_us_per_step": round(host, 2), "graph_used": bool(g is not None and g._graph is not None)}),
                      flush=True)
        summ = {("layer_by_layer" if m == "0" else "one_launch"): {"us_per_step": [round(x, 2) for x in v],
                                                          "median": round(statistics.median(v), 2),
                                                          "host_us_per_step_median": round(statistics.median(hres[m]), 2)}
                for m, v in res.items() if v}
        out["runs"].append({"num_envs": n, "steps": a.steps, "graph": bool(a.graph), **summ})
        print(json.dumps(out["runs"][-1]), flush=True)
    fused_mlp._ROLLOUT_MLP = True
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
