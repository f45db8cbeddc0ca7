"""The rollout's act() replayed as a captured HIP graph (modules/act_graph.py) against the eager calls: the same
actions, values, log-probs and storage contents bit for bit over whole training iterations (the sample draws from
the default CUDA generator in the same order), and the same parameters after the updates."""

import contextlib
import io

import pytest
import torch

from rsl_rl_amd.env import SyntheticVecEnv
from rsl_rl_amd.runners import OnPolicyRunner

pytestmark = pytest.mark.gpu


def _cfg(hidden, timeouts=False):
    return {"num_steps_per_env": 8, "save_interval": 10**9, "obs_groups": {"policy": ["policy"], "critic": ["policy"]},
            "policy": {"class_name": "ActorCritic", "activation": "elu", "actor_hidden_dims": hidden,
                       "critic_hidden_dims": hidden, "init_noise_std": 1.0},
            "algorithm": {"class_name": "PPO", "num_learning_epochs": 2, "num_mini_batches": 2}}


def _run(graph: bool, monkeypatch, dev, hidden, n_envs, iters=3):
    monkeypatch.setenv("RSLRL_ACT_GRAPH", "1" if graph else "0")
    torch.manual_seed(7)
    env = SyntheticVecEnv(n_envs, 48, 12, device=dev, seed=3, timeout_prob=0.2)
    with contextlib.redirect_stdout(io.StringIO()):
        runner = OnPolicyRunner(env, _cfg(hidden), log_dir=None, device=dev)
        snaps = []
        for _ in range(iters):
            runner.learn(1)
            st = runner.alg.storage
            snaps.append({k: getattr(st, k).clone() for k in ("actions", "values", "actions_log_prob", "rewards")})
    params = [p.detach().clone() for p in runner.alg.policy.parameters()]
    return snaps, params, runner.alg._act_graph


@pytest.mark.parametrize("hidden,n_envs", [([256, 256, 256], 4096), ([64, 64], 1000)])
def test_graphed_rollout_matches_eager(hidden, n_envs, cuda_device, monkeypatch):
    eager, p_eager, _ = _run(False, monkeypatch, cuda_device, hidden, n_envs)
    graphed, p_graph, g = _run(True, monkeypatch, cuda_device, hidden, n_envs)
    assert g is not None and g._graph is not None, "the graph was not captured"
    assert g._direct, "the env's observation ring should be read by direct graphs"
    for a, b in zip(eager, graphed):
        for k in a:
            assert torch.equal(a[k], b[k]), k
    for a, b in zip(p_eager, p_graph):
        assert torch.equal(a, b)


def test_act_graph_sees_a_replaced_submodule(cuda_device):
    """The graph's configuration key lists the policy's modules once; replacing a submodule after capture (a new
    output layer with other weights) must be seen: the next step runs with the new layer, as the eager act() does."""
    from rsl_rl_amd.modules import ActorCritic
    from rsl_rl_amd.modules.act_graph import RolloutActGraph

    torch.manual_seed(0)
    obs = {"policy": torch.randn(4096, 48, device=cuda_device)}
    pol = ActorCritic(obs, {"policy": ["policy"], "critic": ["policy"]}, 12, actor_hidden_dims=[256, 256, 256],
                      critic_hidden_dims=[256, 256, 256]).to(cuda_device)
    g = RolloutActGraph(pol)
    with torch.inference_mode():
        for _ in range(3):  # eager, capture, replay
            if g(obs) is None:
                pol.act_and_evaluate(obs)
        assert g._graph is not None
        new = torch.nn.Linear(256, 12).to(cuda_device)
        pol.actor[-1] = new  # a replaced module: its parent's children change
        torch.cuda.manual_seed(5)
        res = g(obs)
        if res is None:
            res = pol.act_and_evaluate(obs)
        mean_g = pol.action_mean.clone()
        torch.cuda.manual_seed(5)
        pol.act(obs)
        assert torch.equal(mean_g, pol.action_mean)


def test_direct_graphs_read_recurring_observation_buffers(cuda_device):
    """Observation buffers that recur get copy-free graphs (act_graph._direct_graph): a step that reads two alternating
    buffers (rewritten between steps, as an env's ring is) and, in between, fresh tensors gives the eager
    act_and_evaluate's actions, values and mean bit for bit, and the direct graphs are the ones replayed."""
    from rsl_rl_amd.modules import ActorCritic
    from rsl_rl_amd.modules.act_graph import RolloutActGraph
    from rsl_rl_amd.networks import fused_mlp

    torch.manual_seed(0)
    dev = cuda_device
    bufs = [torch.empty(4096, 48, device=dev) for _ in range(2)]
    pol = ActorCritic({"policy": bufs[0]}, {"policy": ["policy"], "critic": ["policy"]}, 12,
                      actor_hidden_dims=[256, 256, 256], critic_hidden_dims=[256, 256, 256]).to(dev)
    g = RolloutActGraph(pol)
    gen = torch.Generator(device=dev).manual_seed(1)
    with torch.inference_mode(), fused_mlp.frozen_weights():
        for step in range(30):
            fresh = step in (7, 8)
            x = torch.randn(4096, 48, device=dev, generator=gen)
            if fresh:
                obs = {"policy": x}
            else:
                bufs[step % 2].copy_(x)
                obs = {"policy": bufs[step % 2]}
            torch.cuda.manual_seed(100 + step)
            res = g(obs)
            if res is None:
                res = pol.act_and_evaluate(obs)
            a, v, mu = res[0].clone(), res[1].clone(), pol.action_mean.clone()
            torch.cuda.manual_seed(100 + step)
            a_ref, v_ref = pol.act_and_evaluate({"policy": x.clone()})
            assert torch.equal(a, a_ref) and torch.equal(v, v_ref) and torch.equal(mu, pol.action_mean), step
    assert {k[0] for k in g._direct} >= {b.data_ptr() for b in bufs}, "both recurring buffers should have a direct graph"


def test_direct_graph_actions_are_fresh_tensors(cuda_device):
    """A direct graph writes the actions into the step's freshly allocated tensor: actions a caller keeps are never
    overwritten by later steps (their block is not handed out again while they live), and steps whose actions were
    dropped reuse the blocks (the direct graphs replay)."""
    from rsl_rl_amd.modules import ActorCritic
    from rsl_rl_amd.modules.act_graph import RolloutActGraph
    from rsl_rl_amd.networks import fused_mlp

    torch.manual_seed(0)
    dev = cuda_device
    buf = torch.randn(4096, 48, device=dev)
    pol = ActorCritic({"policy": buf}, {"policy": ["policy"], "critic": ["policy"]}, 12,
                      actor_hidden_dims=[256, 256, 256], critic_hidden_dims=[256, 256, 256]).to(dev)
    g = RolloutActGraph(pol)
    kept = []
    with torch.inference_mode(), fused_mlp.frozen_weights():
        actions = None
        for step in range(16):
            buf.normal_()
            res = g({"policy": buf})
            actions = res[0] if res is not None else pol.act_and_evaluate({"policy": buf})[0]
            if step in (9, 12):
                kept.append((actions, actions.clone()))
        torch.cuda.synchronize()
    for a, snap in kept:
        assert torch.equal(a, snap)
    assert g._direct, "no direct graph was captured"
    assert len(g._direct) <= RolloutActGraph.kMaxDirect
