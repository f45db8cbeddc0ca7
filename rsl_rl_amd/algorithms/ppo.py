"""PPO with the fused HIP loss (rsl_rl/algorithms/ppo.py:19-469).

Constructor, attributes (policy, optimizer, storage, learning_rate, rnd, rnd_optimizer, transition,
intrinsic_rewards, ...) and methods (init_storage, act, process_env_step, compute_returns, update,
broadcast_parameters, reduce_parameters) keep the reference's signatures and semantics.  The update
differs in how each mini-batch is evaluated:

* for the standard ActorCritic the update runs without autograd: the actor and critic forwards keep
  their activations (networks/fused_mlp.train_forward), one fused kernel (kernels.ppo_loss_fwd_bwd)
  computes the KL, the clipped surrogate, the clipped value loss, the entropy and the exact gradients
  d(loss)/d(mean, sigma, V), and the MLP backward kernels write every parameter gradient straight into
  its slot of one contiguous gradient arena (GradArena) -- each parameter's .grad is a view of it;
* under multi-GPU the arena holds, after the gradients, the mini-batch KL: ONE RCCL all-reduce of that
  buffer (SUM, then / world size) averages the gradients and the KL together (ppo.py:271-273 and
  ppo.py:441-469 fused into one collective per mini-batch);
* the adaptive learning rate, the loss statistics, gradient clipping and the Adam step stay on the device
  (kernels.ppo_update_tail, kernels.FusedClipAdam): no host synchronisation per mini-batch.
Any other policy keeps the autograd path (the reference's structure, with the KL appended to the
gradient concatenation of reduce_parameters).

Multi-GPU LR rule: the reference all-reduces kl_mean, lets rank 0 decide, broadcasts the lr as an fp32
tensor and reads it back (ppo.py:272-290).  After the all-reduce every rank holds the same kl_mean, so
each rank applies the same rule locally and rounds the lr through fp32 exactly like the broadcast did:
same learning rates on every rank, no broadcast.
"""

from __future__ import annotations

import os
from itertools import chain

import torch
import torch.nn as nn
import torch.optim as optim

from .. import kernels
from ..modules import ActorCritic
from ..networks import fused_mlp
from ..modules.act_graph import RolloutActGraph
from ..modules.rnd import RandomNetworkDistillation
from ..storage import RolloutStorage
from ..utils import string_to_callable

# RSLRL_FUSED_TAIL=0 (A/B; the same values): the per-mini-batch lr rule / loss sums as their own launch instead of
# inside the clip-and-Adam norm launch
_FUSED_TAIL = os.environ.get("RSLRL_FUSED_TAIL", "1") != "0"


def adapt_learning_rate(learning_rate: float, kl_mean: float, desired_kl: float) -> float:
    """The adaptive schedule of ppo.py:280-284."""
    if kl_mean > desired_kl * 2.0:
        return max(1e-5, learning_rate / 1.5)
    if kl_mean < desired_kl / 2.0 and kl_mean > 0.0:
        return min(1e-2, learning_rate * 1.5)
    return learning_rate


def adapt_learning_rate_device(lr: torch.Tensor, kl_mean: torch.Tensor, desired_kl: float) -> torch.Tensor:
    """ppo.py:280-284 without leaving the device: lr is an fp64 0-d tensor (the reference's Python float),
    kl_mean the fp32 KL; the comparisons happen in fp32 against fp32(2 * kl*) / fp32(kl* / 2), exactly as
    the reference's `tensor > python_float` does."""
    kl = kl_mean.reshape(())
    # Python-float operands: torch compares a fp32 tensor with a wrapped scalar in fp32, like the reference,
    # and no threshold tensor has to be copied to the device (a pageable copy would synchronise)
    down = torch.clamp(lr / 1.5, min=1e-5)
    up = torch.clamp(lr * 1.5, max=1e-2)
    return torch.where(kl > desired_kl * 2.0, down, torch.where((kl < desired_kl / 2.0) & (kl > 0.0), up, lr))


class GradArena:
    """One contiguous fp32 buffer behind every trainable parameter's gradient, followed by `extra` scalar slots (the
    mini-batch KL) that travel in the same all-reduce.  The reference concatenates the gradients in parameters() order
    (policy.parameters(), then the RND predictor's; ppo.py:447-450); here `early` parameters (those whose gradients are
    complete before the rest of the backward, see PPO._early_params) come first, so that the all-reduce can start on
    that prefix while the backward still runs (`early_numel`).  The order of a SUM all-reduce's elements does not change
    any element's sum; every other parameter keeps its relative order (the RND predictor's span stays contiguous)."""

    def __init__(self, params, extra: int, device, early=()):
        self.params = list(params)
        ids = {id(p) for p in early}
        order = [p for p in self.params if id(p) in ids] + [p for p in self.params if id(p) not in ids]
        self.numel = sum(p.numel() for p in self.params)
        self.early_numel = sum(p.numel() for p in order if id(p) in ids)
        self.flat = torch.zeros(self.numel + extra, dtype=torch.float32, device=device)
        slots, off = {}, 0
        for p in order:
            slots[id(p)] = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.views = [slots[id(p)] for p in self.params]
        self._slot = slots
        self.extra = self.flat[self.numel:]

    def matches(self, params) -> bool:
        return len(params) == len(self.params) and all(a is b for a, b in zip(params, self.params))

    def slot(self, p) -> torch.Tensor:
        return self._slot[id(p)]

    def bind(self):
        """Make each parameter's .grad its arena view (the optimizers read and write gradients there)."""
        for p, v in zip(self.params, self.views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def span(self, params) -> torch.Tensor:
        """The contiguous arena range of consecutive parameters (e.g. the RND predictor's)."""
        first, last = self.slot(params[0]), self.slot(params[-1])
        start = first.data_ptr() - self.flat.data_ptr()
        stop = last.data_ptr() - self.flat.data_ptr() + 4 * last.numel()
        return self.flat[start // 4: stop // 4]


class PPO:
    """Proximal Policy Optimization algorithm (https://arxiv.org/abs/1707.06347)."""

    policy: ActorCritic

    def __init__(
        self,
        policy,
        num_learning_epochs=5,
        num_mini_batches=4,
        clip_param=0.2,
        gamma=0.99,
        lam=0.95,
        value_loss_coef=1.0,
        entropy_coef=0.01,
        learning_rate=0.001,
        max_grad_norm=1.0,
        use_clipped_value_loss=True,
        schedule="adaptive",
        desired_kl=0.01,
        device="cpu",
        normalize_advantage_per_mini_batch=False,
        rnd_cfg: dict | None = None,
        symmetry_cfg: dict | None = None,
        multi_gpu_cfg: dict | None = None,
    ):
        self.device = device
        self.is_multi_gpu = multi_gpu_cfg is not None
        if multi_gpu_cfg is not None:
            self.gpu_global_rank = multi_gpu_cfg["global_rank"]
            self.gpu_world_size = multi_gpu_cfg["world_size"]
        else:
            self.gpu_global_rank = 0
            self.gpu_world_size = 1

        if rnd_cfg is not None:
            rnd_lr = rnd_cfg.pop("learning_rate", 1e-3)
            self.rnd = RandomNetworkDistillation(device=self.device, **rnd_cfg)
            self.rnd_optimizer = optim.Adam(self.rnd.predictor.parameters(), lr=rnd_lr)
        else:
            self.rnd = None
            self.rnd_optimizer = None
        self.intrinsic_rewards = None

        if symmetry_cfg is not None:
            use_symmetry = symmetry_cfg["use_data_augmentation"] or symmetry_cfg["use_mirror_loss"]
            if not use_symmetry:
                print("Symmetry not used for learning. We will use it for logging instead.")
            if isinstance(symmetry_cfg["data_augmentation_func"], str):
                symmetry_cfg["data_augmentation_func"] = string_to_callable(symmetry_cfg["data_augmentation_func"])
            if symmetry_cfg["use_data_augmentation"] and not callable(symmetry_cfg["data_augmentation_func"]):
                raise ValueError(
                    "Data augmentation enabled but the function is not callable:"
                    f" {symmetry_cfg['data_augmentation_func']}"
                )
            self.symmetry = symmetry_cfg
        else:
            self.symmetry = None

        self.policy = policy
        self.policy.to(self.device)
        # on a ROCm device Adam runs fused (one kernel per step) and accepts the device-resident lr of update()
        on_gpu = str(device).startswith("cuda")
        self.optimizer = optim.Adam(self.policy.parameters(), lr=learning_rate, fused=True if on_gpu else None)
        # clip_grad_norm_ + optimizer.step() as two launches (kernels.FusedClipAdam, ppo.py:373-374)
        self._clip_adam = (kernels.FusedClipAdam(self.optimizer, max_grad_norm)
                           if on_gpu and kernels.FusedClipAdam.supported(self.optimizer) else None)
        # the RND predictor's optimizer.step() (unclipped, ppo.py:383-384) as one fused launch pair, used when the
        # update runs the RND step on the fused kernels (_rnd_update_plan)
        self._rnd_adam = (kernels.FusedClipAdam(self.rnd_optimizer, 0.0)
                          if on_gpu and self.rnd_optimizer is not None
                          and kernels.FusedClipAdam.supported(self.rnd_optimizer) else None)
        self._act_graph = RolloutActGraph(self.policy) if on_gpu and isinstance(self.policy, ActorCritic) else None
        self.storage: RolloutStorage = None  # type: ignore
        self.transition = RolloutStorage.Transition()

        self.clip_param = clip_param
        self.num_learning_epochs = num_learning_epochs
        self.num_mini_batches = num_mini_batches
        self.value_loss_coef = value_loss_coef
        self.entropy_coef = entropy_coef
        self.gamma = gamma
        self.lam = lam
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.desired_kl = desired_kl
        self.schedule = schedule
        self.learning_rate = learning_rate
        self.normalize_advantage_per_mini_batch = normalize_advantage_per_mini_batch

        self._arena: GradArena | None = None  # gradient arena of the manual update path (see update())
        # while update() runs: the fp64 device scalar that holds the reference's self.learning_rate (decided on the
        # device per mini-batch, read back once at the end); None otherwise.  Read by anything that wants the lr a
        # given optimizer step uses without a host sync point per mini-batch (tests/update_fixtures.py records the
        # lr trace through it)
        self.learning_rate_device = None

    def init_storage(self, training_type, num_envs, num_transitions_per_env, obs, actions_shape):
        self.storage = RolloutStorage(training_type, num_envs, num_transitions_per_env, obs, actions_shape,
                                      self.device)

    # ------------------------------------------------------------------ rollout (ppo.py:129-169)
    def act(self, obs):
        if self.policy.is_recurrent:
            self.transition.hidden_states = self.policy.get_hidden_states()
        pcls = type(self.policy)
        if isinstance(self.policy, ActorCritic) and pcls.act is ActorCritic.act and pcls.evaluate is ActorCritic.evaluate:
            # the actor's and critic's hidden layers batched into one launch each (same values and draws), replayed
            # as one captured HIP graph per configuration (modules/act_graph.py)
            res = None
            if self._act_graph is not None and RolloutActGraph.enabled():
                res = self._act_graph(obs)
            actions, values = res if res is not None else self.policy.act_and_evaluate(obs)
        else:
            actions, values = self.policy.act(obs), self.policy.evaluate(obs)
        self.transition.actions = actions.detach()
        self.transition.values = values.detach()
        self.transition.action_mean = self.policy.action_mean.detach()
        self.transition.action_sigma = self.policy.action_std.detach()
        self.transition.observations = obs
        if not self._fused_rollout():
            self.transition.actions_log_prob = self.policy.get_actions_log_prob(self.transition.actions).detach()
        # else: the log-prob is computed by the fused record kernel in process_env_step
        return self.transition.actions

    def _fused_rollout(self) -> bool:
        return self.storage is not None and self.storage.fused_record_ok(self.transition)

    def _rnd_fused_args(self, obs):
        """Arguments of the RND part of the fused record, or None when the RND module is not of the fused
        form (one hidden ELU layer <= 64 wide, <= 8 outputs, no reward normalisation)."""
        rnd = self.rnd
        if rnd is None or rnd.reward_normalization:
            return None
        nets = []
        for mlp in (rnd.target, rnd.predictor):
            mods = [m for m in mlp]
            lin = [m for m in mods if isinstance(m, torch.nn.Linear)]
            if (len(mods) != 3 or len(lin) != 2 or not isinstance(mods[1], torch.nn.ELU) or mods[1].alpha != 1.0
                    or lin[0].in_features > 64 or lin[0].out_features > 64 or lin[1].out_features > 8):
                return None
            nets.append(lin)
        if nets[0][0].out_features != nets[1][0].out_features:
            return None
        groups = rnd.obs_groups["rnd_state"]
        state = obs[groups[0]] if len(groups) == 1 else torch.cat([obs[g] for g in groups], dim=-1)
        # weight schedule (rnd.py:128-132), evaluated on the host as the reference does
        rnd.update_counter += 1
        if rnd.weight_scheduler is not None:
            rnd.weight = rnd.weight_scheduler(step=rnd.update_counter, **rnd.weight_scheduler_params)
        else:
            rnd.weight = rnd.initial_weight
        args = {"obs": state, "hidden": nets[0][0].out_features, "out": nets[0][1].out_features,
                "target": kernels.pack_rnd_net(rnd.target), "predictor": kernels.pack_rnd_net(rnd.predictor),
                "weight": rnd.weight}
        if rnd.state_normalization:
            sn = rnd.state_normalizer
            args.update(state_mean=sn._mean, state_std=sn._std, state_eps=sn.eps)
        return args

    def process_env_step(self, obs, rewards, dones, extras):
        self.policy.update_normalization(obs)
        if self.rnd:
            self.rnd.update_normalization(obs)
        time_outs = extras.get("time_outs") if isinstance(extras, dict) else None
        if self._fused_rollout():
            # ppo.py:142-169 + rollout_storage.py:77-103 + rnd.py:113-135 in one launch
            rnd_args = self._rnd_fused_args(obs) if self.rnd else None
            extra = None
            if self.rnd and rnd_args is None:  # RND of a form the kernel does not evaluate: PyTorch, then fused add
                extra = self.rnd.get_intrinsic_reward(obs)
                self.intrinsic_rewards = extra
            elif rnd_args is not None:
                self.intrinsic_rewards = torch.empty(rewards.shape[0], dtype=torch.float32, device=rewards.device)
            if time_outs is not None:
                time_outs = time_outs.to(self.device)
            self.storage.add_transition_fused(self.transition, rewards, dones, time_outs, self.gamma,
                                              extra_reward=extra, rnd=rnd_args,
                                              intrinsic_out=self.intrinsic_rewards if rnd_args is not None else None)
        else:
            self.transition.rewards = rewards.clone()
            self.transition.dones = dones
            if self.rnd:
                self.intrinsic_rewards = self.rnd.get_intrinsic_reward(obs)
                self.transition.rewards += self.intrinsic_rewards
            if time_outs is not None:  # bootstrap on time-outs (ppo.py:161-164)
                self.transition.rewards += self.gamma * torch.squeeze(
                    self.transition.values * time_outs.unsqueeze(1).to(self.device), 1
                )
            self.storage.add_transitions(self.transition)
        self.transition.clear()
        self.policy.reset(dones)

    def compute_returns(self, obs):
        last_values = self.policy.evaluate(obs).detach()
        self.storage.compute_returns(last_values, self.gamma, self.lam,
                                     normalize_advantage=not self.normalize_advantage_per_mini_batch)

    # ------------------------------------------------------------------ update (ppo.py:178-422)
    def _trainable_params(self):
        params = list(self.policy.parameters())
        if self.rnd:  # only the predictor receives gradients (the target output is detached)
            params += list(self.rnd.predictor.parameters())
        return [p for p in params if p.requires_grad]

    def grad_arena(self) -> GradArena:
        """The gradient arena over the trainable parameters (+ one KL slot), created on first use and whenever
        the parameter list changes."""
        params = self._trainable_params()
        if self._arena is None or not self._arena.matches(params) or self._arena.flat.device != params[0].device:
            early = self._early_params() if self.is_multi_gpu else ()
            self._arena = GradArena(params, extra=1, device=params[0].device, early=early)
        return self._arena

    def _early_params(self):
        """Parameters whose gradients the manual backward completes before its last layer: every Linear of the actor
        and the critic but the first (the paired backward runs the output layers, then the hidden layers from the top;
        the first layers' weight gradients come last).  With RSLRL_OVERLAP_ALLREDUCE=1 their arena prefix is
        all-reduced while the first layers' backward runs.  Off by default since round 6: on RCCL at
        world 1 the two collectives cost what the single one does (profiles/r6_overlap_ab.json), and at world > 1 the
        fused backward holds every CU's registers and LDS (one 256-VGPR workgroup per CU), so the collective's kernel
        cannot co-run with it anyway -- the split only doubles the latency-bound calls."""
        if os.environ.get("RSLRL_OVERLAP_ALLREDUCE", "0") != "1" or not isinstance(self.policy, ActorCritic):
            return ()
        out = []
        for net in (self.policy.actor, self.policy.critic):
            lins = [m for m in net.modules() if isinstance(m, nn.Linear)]
            for m in lins[1:]:
                out += [m.weight, m.bias]
        return out

    def _sync_kl_and_lr(self, kl_mean: torch.Tensor):
        """KL all-reduce + adaptive lr + fp32 lr rounding under multi-GPU (ppo.py:271-294), host version
        (one device read-back); the update keeps the lr on the device instead (kernels.ppo_update_tail)."""
        if self.is_multi_gpu:
            torch.distributed.all_reduce(kl_mean, op=torch.distributed.ReduceOp.SUM)
            kl_mean /= self.gpu_world_size
        kl = kl_mean.item()
        self.learning_rate = adapt_learning_rate(self.learning_rate, kl, self.desired_kl)
        if self.is_multi_gpu:
            self.learning_rate = torch.tensor(self.learning_rate, dtype=torch.float32).item()
        for param_group in self.optimizer.param_groups:
            param_group["lr"] = self.learning_rate
        return kl

    def update(self):  # noqa: C901
        if self.symmetry:
            raise NotImplementedError(
                "symmetry augmentation / mirror loss (ppo.py:226-244, :318-348) is outside the MI355X PPO "
                "hot-path scope (SURVEY.md §2)"
            )
        if self.policy.is_recurrent:
            raise NotImplementedError("recurrent policies are outside the MI355X PPO hot-path scope (SURVEY.md §2)")
        adaptive = self.desired_kl is not None and self.schedule == "adaptive"
        dev = self.storage.values.device
        if self._clip_adam is not None:
            self._clip_adam.adopt_loaded_state()  # a checkpoint of a non-fused Adam may have been loaded
        sums = torch.zeros(4, dtype=torch.float64, device=dev)  # value, surrogate, entropy, rnd
        stats_buf = torch.empty(8, dtype=torch.float32, device=dev)
        # device-resident lr (needs an optimizer that takes a tensor lr: fused / capturable Adam)
        device_lr = adaptive and dev.type == "cuda" and self._optimizer_takes_tensor_lr()
        # torch.full, not torch.tensor: a fill launch instead of a pageable host-to-device copy, which would block the
        # host until the rollout's kernels have drained (the GPU then idles through the update's host prologue)
        lr_dev = torch.full((), self.learning_rate, dtype=torch.float64, device=dev) if device_lr else None
        self.learning_rate_device = lr_dev  # the reference's self.learning_rate during update() (fp64, device)
        lr32 = None
        if device_lr:  # the optimizer reads the lr as this fp32 device tensor (written by ppo_update_tail)
            lr32 = torch.full((), self.learning_rate, dtype=torch.float32, device=dev)
            for param_group in self.optimizer.param_groups:
                param_group["lr"] = lr32
        manual = None  # decided at the first mini-batch (needs the observation batch)
        arena = None
        # the predictor's trainable parameters: the same filter as _trainable_params, so that they are exactly the
        # arena's RND span
        rnd_params = [p for p in self.rnd.predictor.parameters() if p.requires_grad] if self.rnd else []
        rnd_fused = None  # decided at the first mini-batch (needs the observation batch and the arena)
        # RND target embedding per mini-batch slice of this update's gathered storage, keyed by the slice's index
        # within an epoch: every epoch walks the same permutation's slices in the same order
        target_cache = {}

        generator = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
        for mb_index, (
            obs_batch,
            actions_batch,
            target_values_batch,
            advantages_batch,
            returns_batch,
            old_actions_log_prob_batch,
            old_mu_batch,
            old_sigma_batch,
            hid_states_batch,
            masks_batch,
        ) in enumerate(generator):
            if manual is None:
                manual = (isinstance(self.policy, ActorCritic) and self.policy.manual_update_ok(obs_batch)
                          and all(p.requires_grad for p in self.policy.parameters()))
                if manual:
                    arena = self.grad_arena()
                    arena.bind()
            loss_kw = dict(clip_param=self.clip_param, value_loss_coef=self.value_loss_coef,
                           entropy_coef=self.entropy_coef, use_clipped_value_loss=self.use_clipped_value_loss,
                           compute_kl=adaptive, normalize_advantage=self.normalize_advantage_per_mini_batch,
                           stats=stats_buf)
            if manual:
                # forward, fused loss and backward without autograd; gradients land in the arena
                # (ppo.py:246-253 forward, :221-223 + :259-315 loss, :367-368 backward)
                with torch.no_grad():
                    side = self._side_stream(dev)
                    # the critic's last launch also runs d(value loss)/dV and the value head's backward (the same
                    # values as the loss kernel's d/dV followed by the output-layer backward)
                    vh = fused_mlp.ValueHead(target_values_batch, returns_batch, self.clip_param, self.value_loss_coef,
                                             self.use_clipped_value_loss)
                    # the actor's last launch may also run the loss and the output layer's backward (shared std, no
                    # per-mini-batch advantage normalisation): the same statistics and d sigma as the loss kernel
                    ah = None
                    if (not self.normalize_advantage_per_mini_batch and not self.policy.state_dependent_std
                            and actions_batch.shape[-1] == fused_mlp.ACTOR_HEAD_ACTIONS):
                        ah_gs = (arena.slot(self.policy.std) if self.policy.noise_std_type == "scalar"
                                 else torch.empty(actions_batch.shape[-1], device=dev, dtype=torch.float32))
                        ah = fused_mlp.ActorHead(
                            actions_batch, old_actions_log_prob_batch, advantages_batch, target_values_batch,
                            returns_batch, old_mu_batch, old_sigma_batch, None, clip_param=self.clip_param,
                            value_loss_coef=self.value_loss_coef, entropy_coef=self.entropy_coef,
                            use_clipped=self.use_clipped_value_loss, compute_kl=adaptive, grad_sigma=ah_gs,
                            stats=stats_buf)
                    mean, sigma, value_batch, tape = self.policy.train_forward(obs_batch, side_stream=side,
                                                                               value_head=vh, actor_head=ah)
                    if ah is not None and ah.done:  # loss and d loss / d mu ran inside the actor's launch
                        stats, g_mean, g_sigma, g_value = stats_buf, mean, ah.grad_sigma, value_batch
                    else:
                        g_mean, g_sigma = self.policy.train_grad_buffers(mean, sigma)
                        if g_sigma is None:  # shared std: d sigma reduced by the loss kernel, into the std's slot
                            g_sigma = (arena.slot(self.policy.std) if self.policy.noise_std_type == "scalar"
                                       else torch.empty_like(sigma))
                        # the value head's gradient: a contiguous [B, 1] (the critic's fused output-layer backward
                        # reads its 1-wide rows as they are; a strided column of a padded buffer cost the loss ~2 us)
                        stats, g_mean, g_sigma, g_value = kernels.ppo_loss_fwd_bwd(
                            mean, sigma, value_batch, actions_batch, old_actions_log_prob_batch, advantages_batch,
                            target_values_batch, returns_batch, old_mu_batch, old_sigma_batch, grad_mu=g_mean,
                            grad_sigma=g_sigma, **loss_kw)
                    early_work = []
                    if self.is_multi_gpu and arena.early_numel:
                        def on_early(buf=arena.flat[:arena.early_numel]):
                            # the early prefix's gradients are enqueued: its all-reduce starts now and overlaps the
                            # first layers' backward (the collective's stream waits for this point of ours)
                            early_work.append(torch.distributed.all_reduce(buf, op=torch.distributed.ReduceOp.SUM,
                                                                           async_op=True))
                    else:
                        on_early = None
                    self.policy.train_backward(tape, g_mean, g_sigma, g_value, sigma, arena.slot, side_stream=side,
                                               on_early=on_early)
                    del tape
            else:
                # autograd path for any other policy (ppo.py:246-253, :367-372)
                if hasattr(self.policy, "action_distribution_params"):
                    mean, sigma = self.policy.action_distribution_params(obs_batch)
                else:
                    self.policy.act(obs_batch, masks=masks_batch, hidden_states=hid_states_batch[0])
                    mean, sigma = self.policy.action_mean, self.policy.action_std
                value_batch = self.policy.evaluate(obs_batch, masks=masks_batch, hidden_states=hid_states_batch[1])
                stats, g_mean, g_sigma, g_value = kernels.ppo_loss_fwd_bwd(
                    mean, sigma, value_batch, actions_batch, old_actions_log_prob_batch, advantages_batch,
                    target_values_batch, returns_batch, old_mu_batch, old_sigma_batch, **loss_kw)
                for p in self.policy.parameters():  # optimizer.zero_grad() (set_to_none)
                    p.grad = None
                outs, grads = [mean, value_batch], [g_mean, g_value]
                if sigma.requires_grad:
                    outs.append(sigma)
                    grads.append(g_sigma)
                torch.autograd.backward(outs, grads)

            # RND loss (ppo.py:352-363, :369-371)
            if self.rnd and rnd_fused is None:
                rnd_fused = self._rnd_update_plan(obs_batch, rnd_params, arena if manual else None)
            if self.rnd and rnd_fused:
                # one launch pair: predictor forward, detached target (computed in the first epoch, then read from
                # the per-update cache -- its weights and inputs do not change within update()), MSE, backward
                # straight into the predictor's arena span; the loss statistic accumulates into sums[3]
                self._rnd_update_fused(obs_batch, arena.span(rnd_params), sums, target_cache,
                                       mb_index % self.num_mini_batches)
            elif self.rnd:
                with torch.no_grad():
                    rnd_state_batch = self.rnd.get_rnd_state(obs_batch)
                    rnd_state_batch = self.rnd.state_normalizer(rnd_state_batch)
                predicted_embedding = self.rnd.predictor(rnd_state_batch)
                target_embedding = self.rnd.target(rnd_state_batch).detach()
                rnd_loss = nn.functional.mse_loss(predicted_embedding, target_embedding)
                if manual:  # zeroed arena range + autograd's in-place accumulation = fresh gradients
                    if rnd_params:
                        arena.span(rnd_params).zero_()
                else:
                    for p in rnd_params:
                        p.grad = None
                rnd_loss.backward()

            # multi-GPU: gradients (+ the KL) averaged over ranks by one all-reduce (ppo.py:271-273, :376)
            kl_src = stats[kernels.STATS_KL:kernels.STATS_KL + 1]
            if self.is_multi_gpu:
                if manual:
                    if adaptive:
                        arena.extra[:1].copy_(kl_src)
                    self._all_reduce_arena(arena, with_kl=adaptive, skip=arena.early_numel if early_work else 0,
                                           pending=early_work)
                    kl_src = arena.extra[:1]
                else:
                    kl_src = kl_src.clone() if adaptive else None
                    self.reduce_parameters(kl_mean=kl_src)

            # adaptive lr + loss statistics (ppo.py:259-294, :387-395)
            if adaptive and device_lr:
                tail = kernels.ppo_tail_args(stats, kl_src, lr_dev, lr32, self.desired_kl, sums,
                                             round_fp32=self.is_multi_gpu)
            else:
                if adaptive:  # host rule; the KL is already averaged over ranks
                    kl = kl_src.item()
                    self.learning_rate = adapt_learning_rate(self.learning_rate, kl, self.desired_kl)
                    if self.is_multi_gpu:
                        self.learning_rate = torch.tensor(self.learning_rate, dtype=torch.float32).item()
                    for param_group in self.optimizer.param_groups:
                        param_group["lr"] = self.learning_rate
                tail = kernels.ppo_tail_args(stats, None, None, None, 0.0, sums)
            fuse_tail = self._clip_adam is not None and _FUSED_TAIL
            if not fuse_tail:
                kernels.ppo_update_tail_args(tail, dev)

            # clip + Adam (ppo.py:373-374); the tail above runs inside the norm launch when fused
            if self._clip_adam is None:
                nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
                self.optimizer.step()
            else:
                self._clip_adam.max_grad_norm = float(self.max_grad_norm)
                self._clip_adam.step(tail=tail if fuse_tail else None)
            if self.rnd_optimizer:
                if rnd_fused and self._rnd_adam is not None:
                    self._rnd_adam.step()  # the reference's unclipped Adam on the predictor (ppo.py:383-384)
                else:
                    self.rnd_optimizer.step()

            # loss statistics stay on the device (ppo.py:387-395): accumulated by ppo_update_tail above
            if self.rnd and not rnd_fused:
                sums[3] += rnd_loss.detach().double()

        num_updates = self.num_learning_epochs * self.num_mini_batches
        # one read-back for the loss means and the device lr (back to a Python float, as the reference keeps it:
        # logging, checkpoints)
        # (+ compute_returns' grid-barrier status word, if its one-launch form ran: nonzero = NaN advantages, raise)
        gae_status = getattr(self.storage, "gae_status", None)
        parts = [sums / num_updates] + ([lr_dev.reshape(1)] if device_lr else [])
        if gae_status is not None:
            parts.append(gae_status.to(sums.dtype))
        host = torch.cat(parts).tolist()
        if device_lr:
            self.learning_rate = host[4]
            self.learning_rate_device = None
            for param_group in self.optimizer.param_groups:
                param_group["lr"] = self.learning_rate
        self.storage.clear()
        if gae_status is not None:
            # the rollout's advantages were NaN, and so are this update's parameters: stop loudly
            self.storage.gae_status = None
            kernels.raise_on_gae_status(gae_status, host[-1])
        loss_dict = {"value_function": host[0], "surrogate": host[1], "entropy": host[2]}
        if self.rnd:
            loss_dict["rnd"] = host[3]
        return loss_dict

    def _rnd_update_plan(self, obs_batch, rnd_params, arena) -> bool:
        """Whether the RND predictor's step runs on the fused kernels (kernels.rnd_update): the manual update's
        gradient arena, Linear-ELU-Linear networks of the kernel's sizes, all four predictor parameters trainable
        (their arena span is then [W1 | b1 | W2 | b2]), an identity or empirical state normaliser, fp32 GPU
        observations, our RolloutStorage (its mini-batches are fixed slices of one gathered buffer per update,
        which the target cache relies on)."""
        from ..networks.normalization import EmpiricalNormalization
        rnd = self.rnd
        if arena is None or not isinstance(self.storage, RolloutStorage):
            return False
        pred, targ = kernels.rnd_linears(rnd.predictor), kernels.rnd_linears(rnd.target)
        if pred is None or targ is None:
            return False
        if [(m.in_features, m.out_features) for m in pred] != [(m.in_features, m.out_features) for m in targ]:
            return False
        if len(rnd_params) != 4 or any(a is not b for a, b in zip(rnd_params, [pred[0].weight, pred[0].bias,
                                                                                pred[1].weight, pred[1].bias])):
            return False
        sn = rnd.state_normalizer
        if not isinstance(sn, (nn.Identity, EmpiricalNormalization)):
            return False
        state = self._rnd_state(obs_batch)
        if state is None or not state.is_cuda or state.dtype != torch.float32 or state.shape[1] != pred[0].in_features:
            return False
        if self._rnd_adam is not None:
            self._rnd_adam.adopt_loaded_state()
        return True

    def _rnd_state(self, obs_batch):
        """The RND state of a mini-batch (rnd.py get_rnd_state) without a copy when it is one observation group."""
        groups = self.rnd.obs_groups["rnd_state"]
        if len(groups) == 1:
            s = obs_batch[groups[0]]
            return s if s.dim() == 2 and s.stride(1) == 1 else None
        return self.rnd.get_rnd_state(obs_batch)

    def _rnd_update_fused(self, obs_batch, grad_span, sums, target_cache, slice_index):
        """slice_index: the mini-batch's slice of the update's permutation (its index within the epoch).  The cache
        is keyed by it, not by the state's address: with several rnd_state groups the state is a fresh torch.cat per
        mini-batch, and the caching allocator hands the next mini-batch's cat the same address."""
        rnd = self.rnd
        state = self._rnd_state(obs_batch)
        B = state.shape[0]
        pred, targ = kernels.rnd_linears(rnd.predictor), kernels.rnd_linears(rnd.target)
        key = (slice_index, B)
        temb = target_cache.get(key)
        compute_target = temb is None
        if compute_target:
            temb = torch.empty(B, targ[1].out_features, dtype=torch.float32, device=state.device)
            target_cache[key] = temb
        kw = {}
        if rnd.state_normalization:
            sn = rnd.state_normalizer
            kw = dict(state_mean=sn._mean.reshape(-1), state_std=sn._std.reshape(-1), state_eps=sn.eps)
        kernels.rnd_update(state, pred, targ if compute_target else None, temb, grad_span, loss_sum=sums[3:4], **kw)

    def _side_stream(self, dev):
        """A second stream for the critic's MLP launches in the manual update (networks/fused_mlp.side_stream;
        opt-in: RSLRL_TWO_STREAMS=1, read per update)."""
        return fused_mlp.side_stream(dev)

    def _optimizer_takes_tensor_lr(self) -> bool:
        d = self.optimizer.defaults
        return bool(d.get("fused") or d.get("capturable"))

    # ------------------------------------------------------------------ multi-GPU (ppo.py:428-469)
    def broadcast_parameters(self):
        """Broadcast model parameters from rank 0 to all ranks."""
        model_params = [self.policy.state_dict()]
        if self.rnd:
            model_params.append(self.rnd.predictor.state_dict())
        torch.distributed.broadcast_object_list(model_params, src=0)
        self.policy.load_state_dict(model_params[0])
        if self.rnd:
            self.rnd.predictor.load_state_dict(model_params[1])

    def _all_reduce_arena(self, arena: GradArena, with_kl: bool, skip: int = 0, pending=()):
        """The gradient collective per mini-batch: SUM all-reduce of the arena's gradients (+ its KL slot), then
        / world size (ppo.py:453-454 for the gradients, :273-274 for the KL).  skip / pending: the first `skip`
        elements were already handed to the asynchronous all-reduce(s) `pending` during the backward (the early
        prefix); the rest is reduced here, then the current stream waits for them before the division."""
        buf = arena.flat[:arena.numel + (1 if with_kl else 0)]
        if skip < buf.numel():
            torch.distributed.all_reduce(buf[skip:], op=torch.distributed.ReduceOp.SUM)
        for w in pending:
            w.wait()
        buf /= self.gpu_world_size

    def reduce_parameters(self, kl_mean: torch.Tensor | None = None):
        """Average gradients across ranks: SUM all-reduce then / world_size (ppo.py:441-469).

        Gradients that are views of the gradient arena (the manual update path) are reduced in place as one
        buffer; otherwise the reference's concatenation / all-reduce / copy-back.  kl_mean: an optional fp32
        1-element tensor appended to the concatenation (averaged in place) so that the KL needs no collective
        of its own."""
        arena = self._arena
        params = self._trainable_params()
        if arena is not None and arena.matches(params) and kl_mean is None and all(
                p.grad is not None and p.grad.data_ptr() == v.data_ptr() for p, v in zip(params, arena.views)):
            self._all_reduce_arena(arena, with_kl=False)
            return
        grads = [p.grad.view(-1) for p in self.policy.parameters() if p.grad is not None]
        if self.rnd:
            grads += [p.grad.view(-1) for p in self.rnd.parameters() if p.grad is not None]
        if kl_mean is not None:
            grads.append(kl_mean.reshape(1).to(grads[0].dtype))
        all_grads = torch.cat(grads)
        torch.distributed.all_reduce(all_grads, op=torch.distributed.ReduceOp.SUM)
        all_grads /= self.gpu_world_size
        if kl_mean is not None:
            kl_mean.copy_(all_grads[-1:].reshape(kl_mean.shape))
            all_grads = all_grads[:-1]
        all_params = self.policy.parameters()
        if self.rnd:
            all_params = chain(all_params, self.rnd.parameters())
        # copy back (ppo.py:464-469) as one multi-tensor copy
        dst = [p.grad.data for p in all_params if p.grad is not None]
        torch._foreach_copy_(dst, [g.view_as(d) for g, d in zip(all_grads.split([d.numel() for d in dst]), dst)])
