"""The policy half of a rollout step as one captured HIP graph (ppo.py:129-140: act -> actor and critic forwards,
the Normal sample; on_policy_runner.py:103-109 calls it once per env step).

Eagerly, ActorCritic.act_and_evaluate issues ~20 host calls per step (the B-image build, the paired MLP launches
through ctypes, the Normal sample's four torch ops): ~100 us of host time that the GPU waits out when a GPU holds
few envs (the strong-scaling shares of config C4).  Here the same calls are captured once per configuration into a
torch.cuda.CUDAGraph and replayed: the observation is copied into the graph's static input, the graph replays, and
the outputs are the graph's static tensors (the actions are cloned, so a caller may keep them).  Two graphs per
configuration: one with the B-image build of the weights (replayed at the first step of each rollout -- each entry
into an outermost fused_mlp.frozen_weights() scope -- so parameters updated in place between rollouts are picked
up, and at every step outside such a scope) and one without it, reading the images the first one wrote (the other
23 steps of a rollout).

Same values and the same random stream as the eager calls: the sample's standard normals are drawn eagerly into a
static buffer right before each replay (the same normal_() on the same [N, A] shape from the default generator as
the eager step draws -- outside the graph, so a replay does not need the two generator-state fill launches of a
captured draw), and the graph scales and shifts them (inside the one-launch forward when it runs); tests/
test_gpu_act_graph.py compares a graphed and an eager rollout bitwise.

Observation buffers that recur (an env that writes its observations into a few persistent buffers -- the synthetic
env's ring of three, a simulator's obs buffer) get graphs of their own that read the buffer in place: the step draws
its normals into a fresh tensor (the caching allocator hands the same few blocks back once the caller drops earlier
actions), and a (observation pointers, fresh-tensor pointer) set seen twice is captured as a "direct" graph of the
image-free step (reading the image graph's images) that reads the observations and writes the actions in place into
that fresh tensor -- one draw + one replay per step, without the copy into the static input or the actions' clone.
A direct graph is replayed only while the observation tensors sit at exactly the pointers it was captured on (same
shapes and strides: the configuration key), i.e. it reads the step's own observations, and writes only into the
step's own freshly allocated actions; at most kMaxDirect pointer sets per configuration.
The first call of a configuration runs eagerly, the second captures; any capture failure falls back to the eager
path for that configuration.  RSLRL_ACT_GRAPH=0 disables it.
"""

from __future__ import annotations

import contextlib
import os
import warnings

import torch
from torch.distributions import Normal

from .. import kernels
from ..networks import fused_mlp


class RolloutActGraph:
    kMaxDirect = 12  # pointer sets with a direct graph, per configuration

    def __init__(self, policy):
        self.policy = policy
        self._key = None
        self._seen = 0
        self._graph = None
        self._failed = set()
        self._static_in = None
        self._out = None
        self._graph_fwd = None  # the graph without the image build, and its outputs
        self._out_fwd = None
        self._imgs = None  # the image tensors both graphs use (written by the first one's replay)
        self._img_gen = None  # fused_mlp._frozen_gen of the last image build
        self._eps = None  # the sample's standard normals, drawn before each replay
        self._dists = {}  # id(output tuple) -> the Normal over that graph's static mean / scale
        self._groups = None  # the observation groups the step reads
        self._mods = None  # the policy's modules (their parameters and buffers key the configuration)
        self._parents = []  # [(module, its children)] of the modules that have children: a replaced module shows here
        self._tdicts = []  # the modules' parameter and buffer dicts (their entries key the configuration)
        self._img_cache = None  # the image graph's fused_mlp image cache entries (the direct graphs read them)
        self._direct = {}  # observation pointers -> (graph, outputs): the step reading those buffers in place
        self._ptr_seen = {}  # observation pointers -> times seen (a pointer set seen twice gets a direct graph)

    @staticmethod
    def enabled() -> bool:
        return os.environ.get("RSLRL_ACT_GRAPH", "1") != "0"

    def _config(self, obs):
        pol = self.policy
        if self._groups is None:
            self._groups = sorted(set(pol.obs_groups["policy"]) | set(pol.obs_groups["critic"]))
        # the policy's modules, listed once and re-listed when any module's children change: a step reads their
        # parameter / buffer dicts directly (walking the module tree per step was ~20 us of host time at the 16,384-env
        # share, where the rollout was host-bound)
        if self._mods is None or any(tuple(m._modules.values()) != kids for m, kids in self._parents):
            self._mods = list(pol.modules())
            self._parents = [(m, tuple(m._modules.values())) for m in self._mods if m._modules]
            self._tdicts = [d for m in self._mods for d in (m._parameters, m._buffers)]  # the dicts, read per step
        shapes = []
        for g in self._groups:
            t = obs[g]
            if not (isinstance(t, torch.Tensor) and t.is_cuda):
                return None
            shapes.append((g, tuple(t.shape), t.dtype, t.device, t.stride()))
        ptrs = tuple([t.data_ptr() for d in self._tdicts for t in d.values() if t is not None])
        return (tuple(shapes), ptrs, fused_mlp._mode, torch.is_inference_mode_enabled())

    def __call__(self, obs):
        """(actions, values) of the step, with policy.distribution set as act() sets it; None: run eagerly.

        actions is a fresh tensor; values and policy.distribution's mean / scale are the graph's static outputs and
        stay valid only until the next call (policy.distribution is the same Normal object on every step of a graph:
        the replay rewrites its loc / scale in place)."""
        key = self._config(obs)
        if key is None or key in self._failed:
            return None
        if key != self._key:
            self._key, self._seen, self._graph, self._static_in, self._out = key, 0, None, None, None
            self._graph_fwd, self._out_fwd, self._imgs, self._img_gen, self._eps = None, None, None, None, None
            self._dists, self._img_cache, self._direct, self._ptr_seen = {}, None, {}, {}
        if self._graph is None:
            self._seen += 1
            if self._seen < 2:  # the first call of a configuration runs eagerly (lazy initialisations happen there)
                return None
            if not self._capture(obs, key):
                return None
        frozen = fused_mlp._frozen_depth > 0
        current = frozen and self._graph_fwd is not None and self._img_gen == fused_mlp._frozen_gen
        if current and fused_mlp._STEP_FUSION:
            # the sample's normals go into a fresh tensor (the actions the caller receives: no clone); its block
            # recurs once the caller has dropped an earlier step's actions
            eps = torch.empty(self._eps.shape, dtype=self._eps.dtype, device=self._eps.device)
            direct = self._direct_graph(obs, eps)
            if direct is not None:  # the observations are read in place and the actions written in place: no copies
                eps.normal_()  # the draw the eager step makes (same generator, same shape, same order)
                direct[0].replay()
                out = direct[1]
                self.policy.distribution = self._dist(out)
                return eps, out[1]
        if current:
            for g, t in self._static_in.items():
                t.copy_(obs[g])
            self._eps.normal_()
            self._graph_fwd.replay()  # the images of this rollout's weights are current
            out = self._out_fwd
        else:
            for g, t in self._static_in.items():
                t.copy_(obs[g])
            self._eps.normal_()
            self._graph.replay()
            self._img_gen = fused_mlp._frozen_gen if frozen else None
            out = self._out
        actions, values = out[0], out[1]
        # Aliasing contract: actions are cloned (a direct graph's are the step's fresh tensor); the returned values
        # and the distribution's mean / scale ARE the graph's static outputs, valid only until the next call (the next
        # replay overwrites them; the eager path allocates new tensors).  PPO.act keeps them in its transition only until process_env_step copies them into
        # the storage in the same env step.  (A clone of values would add one launch per env step to the
        # host-bound rollout at the 16384-env share.)
        # one Normal per graph output set, built once: its loc / scale ARE the static outputs (a Normal per step cost
        # ~8 us of host time in torch.distributions' broadcast_all on the launch-bound rollout)
        self.policy.distribution = self._dist(out)
        return actions.clone(), values

    def _dist(self, out):
        dist = self._dists.get(id(out))
        if dist is None or dist.loc is not out[2] or dist.scale is not out[3]:
            dist = self._dists[id(out)] = Normal(out[2], out[3])
        return dist

    def _direct_graph(self, obs, eps):
        """The direct graph of the observations' and the sample buffer's pointers (captured at their second
        sighting), or None.  It reads the observations in place and writes the actions into `eps` in place."""
        ptrs = tuple(obs[g].data_ptr() for g in self._groups) + (eps.data_ptr(),)
        hit = self._direct.get(ptrs)
        if hit is not None or self._img_cache is None:
            return hit
        n = self._ptr_seen.get(ptrs, 0) + 1
        if len(self._ptr_seen) >= 64 and ptrs not in self._ptr_seen:  # fresh pointers every step: stop counting
            return None
        self._ptr_seen[ptrs] = n
        if n < 2 or len(self._direct) >= self.kMaxDirect:
            return None
        pol = self.policy
        graph = torch.cuda.CUDAGraph()
        pol._static_eps = eps
        try:
            with _capture_caches() as cache:
                cache.update(self._img_cache)  # the image graph's images: no image build in this graph
                with torch.cuda.graph(graph):
                    _, values = pol.act_and_evaluate({g: obs[g] for g in self._groups})
                    dist = pol.distribution
                    # no reference to the actions (this step's fresh tensor): its block must go back to the allocator
                    out = (None, values, dist.loc, dist.scale)
        except Exception as e:  # noqa: BLE001 -- stay on the copying graph for this pointer set
            self._ptr_seen[ptrs] = -(1 << 30)
            warnings.warn(f"rollout act() direct graph capture failed, copying the observations: {e}")
            return None
        finally:
            pol._static_eps = None
        self._direct[ptrs] = (graph, out)
        return self._direct[ptrs]

    def _capture(self, obs, key) -> bool:
        pol = self.policy
        static_in = {g: obs[g].clone() for g in sorted(set(pol.obs_groups["policy"]) | set(pol.obs_groups["critic"]))}
        graph, graph_fwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        loc = pol.distribution.loc  # the eager first call's distribution: the sample's shape
        eps = torch.empty(loc.shape, dtype=loc.dtype, device=loc.device)
        pol._static_eps = eps
        try:
            with _capture_caches() as cache:
                with torch.cuda.graph(graph):  # image build + forward + sample
                    actions, values = pol.act_and_evaluate(static_in)
                    dist = pol.distribution
                    out = (actions, values, dist.loc, dist.scale)
                imgs = [v[1] for v in cache.values()]
                img_cache = dict(cache)
                out_fwd = None
                if imgs:  # the same step reading the cached images (no image launch in this graph)
                    with torch.cuda.graph(graph_fwd):
                        a2, v2 = pol.act_and_evaluate(static_in)
                        d2 = pol.distribution
                        out_fwd = (a2, v2, d2.loc, d2.scale)
        except Exception as e:  # noqa: BLE001 -- any op that cannot be captured: stay eager for this configuration
            self._failed.add(key)
            warnings.warn(f"rollout act() graph capture failed, running eagerly: {e}")
            return False
        finally:
            pol._static_eps = None
        self._graph, self._static_in, self._out, self._eps = graph, static_in, out, eps
        self._graph_fwd, self._out_fwd, self._imgs = (graph_fwd, out_fwd, imgs) if out_fwd is not None else (None,) * 3
        self._img_cache = dict(img_cache) if out_fwd is not None else None
        self._img_gen = None  # the first replay runs the image build
        return True


@contextlib.contextmanager
def _capture_caches():
    """While capturing: a private frozen-weights image cache (the first graph's image build fills it, the second graph
    reads it), no kernel-timer events; the caller's cache and memo are restored afterwards."""
    depth, en, men = fused_mlp._frozen_depth, kernels.timer.enabled, kernels.timer.mlp_enabled
    cache, memo = dict(fused_mlp._bimage_cache), dict(fused_mlp._pair_memo)
    fused_mlp._bimage_cache.clear()
    fused_mlp._pair_memo.clear()
    fused_mlp._frozen_depth = 1
    kernels.timer.enabled = kernels.timer.mlp_enabled = False
    try:
        yield fused_mlp._bimage_cache
    finally:
        fused_mlp._frozen_depth = depth
        fused_mlp._bimage_cache.clear()
        fused_mlp._bimage_cache.update(cache)
        fused_mlp._pair_memo.clear()
        fused_mlp._pair_memo.update(memo)
        kernels.timer.enabled, kernels.timer.mlp_enabled = en, men
