"""Gaussian MLP actor + MLP critic (rsl_rl/modules/actor_critic.py:15-195).

Same constructor, attributes, parameter names and behaviour as the reference, so configs and
checkpoints carry over.  In addition `action_distribution_params()` hands the PPO update the raw
(mean, sigma) of the policy without materialising a torch Normal's per-row sigma, so the fused HIP
loss (rsl_rl_amd.kernels.ppo_loss_fwd_bwd) can read a shared [A] sigma and return its gradient
already reduced over the mini-batch.
"""

from __future__ import annotations

import torch
import torch.nn as nn
from torch.distributions import Normal

from .. import kernels
from ..networks import MLP, EmpiricalNormalization
from ..networks import fused_mlp
from ..networks.fused_mlp import fused_mlp_forward_pair


class ActorCritic(nn.Module):
    is_recurrent = False

    def __init__(
        self,
        obs,
        obs_groups,
        num_actions,
        actor_obs_normalization=False,
        critic_obs_normalization=False,
        actor_hidden_dims=[256, 256, 256],
        critic_hidden_dims=[256, 256, 256],
        activation="elu",
        init_noise_std=1.0,
        noise_std_type: str = "scalar",
        state_dependent_std=False,
        **kwargs,
    ):
        if kwargs:
            print("ActorCritic.__init__ got unexpected arguments, which will be ignored: " + str(list(kwargs)))
        super().__init__()
        self.obs_groups = obs_groups
        num_actor_obs = self._group_dim(obs, obs_groups["policy"])
        num_critic_obs = self._group_dim(obs, obs_groups["critic"])
        self.num_actions = num_actions
        self.state_dependent_std = state_dependent_std
        self.noise_std_type = noise_std_type
        if noise_std_type not in ("scalar", "log"):
            raise ValueError(f"Unknown standard deviation type: {noise_std_type}. Should be 'scalar' or 'log'")

        out = [2, num_actions] if state_dependent_std else num_actions
        self.actor = MLP(num_actor_obs, out, actor_hidden_dims, activation)
        self.actor_obs_normalization = actor_obs_normalization
        self.actor_obs_normalizer = EmpiricalNormalization(num_actor_obs) if actor_obs_normalization else nn.Identity()
        print(f"Actor MLP: {self.actor}")
        self.critic = MLP(num_critic_obs, 1, critic_hidden_dims, activation)
        self.critic_obs_normalization = critic_obs_normalization
        self.critic_obs_normalizer = (
            EmpiricalNormalization(num_critic_obs) if critic_obs_normalization else nn.Identity()
        )
        print(f"Critic MLP: {self.critic}")

        if state_dependent_std:
            # the std half of the last layer starts at weight 0 and bias = init std (actor_critic.py:77-86)
            last = self.actor[-2]
            nn.init.zeros_(last.weight[num_actions:])
            init_bias = init_noise_std if noise_std_type == "scalar" else torch.log(torch.tensor(init_noise_std + 1e-7))
            nn.init.constant_(last.bias[num_actions:], init_bias)
        elif noise_std_type == "scalar":
            self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        else:
            self.log_std = nn.Parameter(torch.log(init_noise_std * torch.ones(num_actions)))

        self.distribution = None
        Normal.set_default_validate_args(False)

    @staticmethod
    def _group_dim(obs, groups):
        dim = 0
        for g in groups:
            assert len(obs[g].shape) == 2, "The ActorCritic module only supports 1D observations."
            dim += obs[g].shape[-1]
        return dim

    def reset(self, dones=None):
        pass

    def forward(self):
        raise NotImplementedError

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def _mean_and_std(self, obs, actor_out=None):
        """(mean [B, A], std) with std either the shared [A] parameter-derived vector or per-row [B, A];
        actor_out: the actor's output when it was already computed (act_and_evaluate)."""
        out = self.actor(obs) if actor_out is None else actor_out
        if self.state_dependent_std:
            mean, std = torch.unbind(out, dim=-2)
            if self.noise_std_type == "log":
                std = torch.exp(std)
            return mean, std
        std = self.std if self.noise_std_type == "scalar" else torch.exp(self.log_std)
        return out, std

    def update_distribution(self, obs):
        mean, std = self._mean_and_std(obs)
        self.distribution = Normal(mean, std.expand_as(mean))

    def action_distribution_params(self, obs):
        """Actor forward for the fused PPO loss: returns (mean [B, A], sigma) where sigma is [A] (shared
        std / exp(log_std), gradient flows to the parameter) or [B, A] (state-dependent std).  Also
        leaves `self.distribution` set, as `act()` would, for logging (on_policy_runner.py:208)."""
        obs = self.actor_obs_normalizer(self.get_actor_obs(obs))
        mean, std = self._mean_and_std(obs)
        self.distribution = Normal(mean.detach(), std.detach().expand_as(mean))
        return mean, std

    # ---------------------------------------------------------------- PPO update without autograd
    def manual_update_ok(self, obs) -> bool:
        """The PPO update may drive this policy through train_forward / train_backward: an unmodified
        ActorCritic whose actor and critic are fused Linear+ELU stacks and whose inputs live on a ROCm device."""
        cls = type(self)
        if (cls.action_distribution_params is not ActorCritic.action_distribution_params
                or cls.evaluate is not ActorCritic.evaluate or cls.act is not ActorCritic.act):
            return False
        if not (getattr(self.actor, "_fused", False) and getattr(self.critic, "_fused", False)):
            return False
        groups = self.obs_groups["policy"] + self.obs_groups["critic"]
        return all(obs[g].is_cuda and obs[g].dtype == torch.float32 for g in groups)

    @staticmethod
    def _linears(mlp):
        lin = [m for m in mlp if isinstance(m, nn.Linear)]
        return [m.weight for m in lin], [m.bias for m in lin]

    def train_forward(self, obs, side_stream=None, value_head=None, actor_head=None):
        """The update's forward (ppo.py:246-253) without an autograd graph: returns (mean [B, A], sigma, value
        [B, 1], tape) with sigma the shared [A] std (scalar / exp(log_std)) or the per-row [B, A] std of a
        state-dependent head (strided views of the actor output).  Call under torch.no_grad().

        side_stream: a second stream of the device for the critic's MLP -- the actor's and the critic's launch
        chains are independent, so each fills the other's launch tails; the current stream waits for it before
        returning (the results are the same values either way).

        value_head: a fused_mlp.ValueHead of the mini-batch (target values, returns, value-loss settings): the critic's
        last launch then also computes d(value loss)/dV and the value head's backward (networks/fused_mlp.py
        value_head_fwd_bwd; paired passes only) -- train_backward then takes the critic's gradient from the tape.

        actor_head: a fused_mlp.ActorHead of the mini-batch (with value_head; shared std only): the actor's last launch
        then also runs the PPO loss and the output layer's backward (actor_head_fwd_bwd).  Its `sigma` is set here (the
        std this call returns); actor_head.done tells whether it ran -- the loss statistics and d loss / d sigma are
        then written and train_backward takes the actor's gradient from the tape (g_mean is not read)."""
        a_obs = self.actor_obs_normalizer(self.get_actor_obs(obs))
        c_obs = self.critic_obs_normalizer(self.get_critic_obs(obs))
        a_obs = a_obs if a_obs.is_contiguous() else a_obs.contiguous()
        c_obs = c_obs if c_obs.is_contiguous() else c_obs.contiguous()
        pair = None
        if actor_head is not None:
            if self.state_dependent_std or value_head is None or side_stream is not None:
                actor_head = None
            else:
                std_now = self.std if self.noise_std_type == "scalar" else torch.exp(self.log_std)
                actor_head.sigma = std_now.detach().contiguous()
        if side_stream is None:  # the actor's and the critic's same-shape layers batched into one launch each
            pair = fused_mlp.train_forward_pair(a_obs, *self._linears(self.actor), c_obs, *self._linears(self.critic),
                                                value_head=value_head, actor_head=actor_head)
        if pair is not None:
            y, tape_a, value, tape_c = pair
        elif side_stream is not None:
            main = torch.cuda.current_stream(c_obs.device)
            side_stream.wait_stream(main)
            c_obs.record_stream(side_stream)  # kept by the critic's tape for its backward on the side stream
            with torch.cuda.stream(side_stream):
                value, tape_c = fused_mlp.train_forward(c_obs, *self._linears(self.critic))
        if pair is None:
            y, tape_a = fused_mlp.train_forward(a_obs, *self._linears(self.actor))
        A = self.num_actions
        if self.state_dependent_std:
            mean, raw = y[:, :A], y[:, A:]  # = unbind(Unflatten([2, A])(y), dim=-2)
            std = torch.exp(raw) if self.noise_std_type == "log" else raw
        else:
            mean = y
            std = self.std if self.noise_std_type == "scalar" else torch.exp(self.log_std)
        if pair is None and side_stream is None:
            value, tape_c = fused_mlp.train_forward(c_obs, *self._linears(self.critic))
        elif side_stream is not None:
            main.wait_stream(side_stream)
            value.record_stream(main)  # allocated on the side stream, read by the loss on this one
        self.distribution = Normal(mean, std.expand_as(mean))  # for logging, as act() leaves it
        return mean, std, value, (tape_a, tape_c, y.shape, pair is not None)

    def train_grad_buffers(self, mean, std):
        """(d mean, d sigma) destinations for the fused loss: for a state-dependent head both are the halves of
        one [B, 2A] buffer, the actor output's gradient; otherwise d mean [B, A] and d sigma [A]."""
        B, A = mean.shape
        if self.state_dependent_std:
            dy = torch.empty(B, 2 * A, device=mean.device, dtype=torch.float32)
            return dy[:, :A], dy[:, A:]
        return torch.empty(B, A, device=mean.device, dtype=torch.float32), None

    def train_backward(self, tape, g_mean, g_sigma, g_value, std, slot, side_stream=None, g_value_padded=None,
                       on_early=None):
        """Backward of train_forward given the loss gradients w.r.t. (mean, sigma, value), written into the
        gradient slots `slot(param)` (a gradient arena).  g_sigma: for the shared std the [A] gradient w.r.t.
        sigma (for log_std it is chained through exp here); for a state-dependent head the half of the actor-output
        gradient buffer (train_grad_buffers) the loss kernel wrote.  side_stream: as in train_forward (the
        critic's backward runs there; the current stream waits for it before returning).  g_value_padded: a zero-padded
        [B, 4] buffer whose column 0 is g_value (the loss kernel wrote it there), or None.  on_early: called once the
        gradients of every layer but the first of both networks are enqueued (PPO starts their all-reduce there); on
        the paths that do not split the backward it is called at the end."""
        tape_a, tape_c, y_shape, paired = tape
        if self.state_dependent_std:
            dy = torch.as_strided(g_mean, y_shape, (y_shape[1], 1))  # the [B, 2A] buffer behind both halves
            if self.noise_std_type == "log":  # d raw = d sigma * exp(raw) (ExpBackward: grad * result)
                g_sigma.mul_(std)
        else:
            dy = g_mean
            if self.noise_std_type == "log":
                torch.mul(g_sigma, std, out=slot(self.log_std))
            elif g_sigma.data_ptr() != slot(self.std).data_ptr():
                slot(self.std).copy_(g_sigma)
        def run(mlp, tp, d, d_pad=None):
            ws, bs = self._linears(mlp)
            fused_mlp.train_backward(tp, d, outs=[(slot(w), slot(b)) for w, b in zip(ws, bs)], dy_padded=d_pad)

        if side_stream is None:
            if paired and g_value_padded is None:
                outs = [[(slot(w), slot(b)) for w, b in zip(*self._linears(m))] for m in (self.actor, self.critic)]
                if fused_mlp.train_backward_pair(tape_a, dy, outs[0], tape_c, g_value.reshape(-1, 1), outs[1],
                                                 on_early=on_early):
                    return
            if tape_c.head is not None:
                raise RuntimeError("train_backward: the critic's head ran fused (value_head) but the paired backward "
                                   "does not apply to these gradient destinations")
            run(self.actor, tape_a, dy)
            run(self.critic, tape_c, g_value.reshape(-1, 1), g_value_padded)
            if on_early is not None:
                on_early()
            return
        main = torch.cuda.current_stream(dy.device)
        side_stream.wait_stream(main)
        g_value.record_stream(side_stream)  # written by the loss on this stream, read on the side stream
        with torch.cuda.stream(side_stream):
            run(self.critic, tape_c, g_value.reshape(-1, 1), g_value_padded)
        run(self.actor, tape_a, dy)
        main.wait_stream(side_stream)
        if on_early is not None:
            on_early()

    def act(self, obs, **kwargs):
        obs = self.actor_obs_normalizer(self.get_actor_obs(obs))
        self.update_distribution(obs)
        return self._sample()

    def _sample(self):
        # = self.distribution.sample(): torch.normal(loc, scale) draws normal_(0, 1) and applies
        # .mul_(scale).add_(loc) -- the same values from the same generator stream -- but first checks
        # scale.min() >= 0 with a device-to-host read that stalls the launch queue every env step
        loc, scale = self.distribution.loc, self.distribution.scale
        with torch.no_grad():
            eps = getattr(self, "_static_eps", None)  # a captured rollout graph's standard normals, drawn before replay
            if eps is None or eps.shape != loc.shape:
                eps = torch.empty_like(loc).normal_()
            if (eps.is_cuda and eps.dim() == 2 and eps.is_contiguous() and scale.shape == eps.shape
                    and loc.shape == eps.shape and scale.stride(1) == 1 and loc.stride(1) == 1):
                return kernels.normal_affine_(eps, scale, loc)  # the mul_ + add_ pair in one launch, same bits
            return eps.mul_(scale).add_(loc)

    def act_and_evaluate(self, obs):
        """(act(obs), evaluate(obs)) of the rollout step (ppo.py:155-156) with the actor's and the critic's
        same-shape hidden layers batched into one launch each (networks/fused_mlp.fused_mlp_forward_pair);
        the same values, distribution and generator draws as the two calls.  Falls back to them when the
        pair does not qualify."""
        a_obs = self.actor_obs_normalizer(self.get_actor_obs(obs))
        c_obs = self.critic_obs_normalizer(self.get_critic_obs(obs))
        if not a_obs.is_cuda:
            pair = None
        elif (getattr(self, "_static_eps", None) is not None and not self.state_dependent_std
              and fused_mlp._STEP_FUSION):
            # a captured rollout graph: its standard normals are drawn before the replay, so the forward's launch can
            # also apply the sample (eps * std + mean, _sample's expression) -- one launch less per env step
            std = self.std if self.noise_std_type == "scalar" else torch.exp(self.log_std)
            pair = fused_mlp_forward_pair(self.actor, a_obs, self.critic, c_obs, sample=(self._static_eps, std))
            if pair is not None and pair[2]:
                self.distribution = Normal(pair[0], std.expand_as(pair[0]))
                return self._static_eps, pair[1]
        else:
            pair = fused_mlp_forward_pair(self.actor, a_obs, self.critic, c_obs)
        if pair is None:
            self.update_distribution(a_obs)
            return self._sample(), self.critic(c_obs)
        mean, std = self._mean_and_std(a_obs, actor_out=pair[0])
        self.distribution = Normal(mean, std.expand_as(mean))
        return self._sample(), pair[1]

    def act_inference(self, obs):
        obs = self.actor_obs_normalizer(self.get_actor_obs(obs))
        return self.actor(obs)

    def evaluate(self, obs, **kwargs):
        obs = self.critic_obs_normalizer(self.get_critic_obs(obs))
        return self.critic(obs)

    @staticmethod
    def _concat(obs, groups):
        # a single group is used as is (the reference's torch.cat of one tensor is a pure copy)
        return obs[groups[0]] if len(groups) == 1 else torch.cat([obs[g] for g in groups], dim=-1)

    def get_actor_obs(self, obs):
        return self._concat(obs, self.obs_groups["policy"])

    def get_critic_obs(self, obs):
        return self._concat(obs, self.obs_groups["critic"])

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def update_normalization(self, obs):
        if self.actor_obs_normalization:
            self.actor_obs_normalizer.update(self.get_actor_obs(obs))
        if self.critic_obs_normalization:
            self.critic_obs_normalizer.update(self.get_critic_obs(obs))

    def load_state_dict(self, state_dict, strict=True):
        """Load parameters; returns True (= training resumes), as the reference (actor_critic.py:181-195)."""
        super().load_state_dict(state_dict, strict=strict)
        return True
