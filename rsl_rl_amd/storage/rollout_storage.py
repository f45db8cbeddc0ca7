"""Rollout buffer with the PPO hot path on the GPU (rsl_rl/storage/rollout_storage.py:14-260).

Buffers, shapes, dtypes and the public interface are the reference's ([T, N, ...] per field, dones
uint8, TensorDict observations, Transition, add_transitions, clear, compute_returns,
mini_batch_generator), so PPO code and external callers see the same object.  What changes is how the
two hot functions run:

* compute_returns (:127-149) is one HIP reverse-scan kernel (+ one normalisation kernel) over the
  [T, N] slabs instead of a Python loop of ~320 tiny ATen launches; results are bit-identical to the
  reference for returns and raw advantages.
* mini_batch_generator (:160-203) draws its permutation with torch's CPU randperm semantics (host
  mt19937 Fisher-Yates, bit-exact), uploads it once, and *packs* every field in permuted order with a
  single multi-field gather launch.  Because the reference reuses one permutation for all epochs, each
  mini-batch is then a contiguous slice of the packed buffers: the yielded tensors equal the
  reference's `field.flatten(0, 1)[indices[i*mb:(i+1)*mb]]` exactly, and no epoch re-gathers.

Permutation source: the reference calls `torch.randperm(n, device=self.device)`, i.e. on a GPU it draws
from the device generator with a device-specific algorithm.  Here the permutation always follows the
CPU randperm algorithm on `perm_generator` (default: torch's process-wide CPU generator), which makes it
reproducible under torch.manual_seed and bit-exact with the reference run on CPU.

Transition records (ROCm storages of feed-forward RL with 4-multiple widths): the gathered fields of an
env-step sit side by side in one fp32 record padded to whole 128-byte lines ([T, N, R]; 96 floats at C3):
observation groups, actions, mu and sigma (written by the rollout; `observations[k]`, `actions`, `mu`,
`sigma` are strided views of the records, same shapes and values as the reference's buffers).  The update's
scalars {value, log-prob, return, advantage} of an env-step sit in one 16-byte unit of a contiguous slot array
([T, N, 4]), filled once per update from the contiguous [T, N, 1] scalar buffers (GAE wants those contiguous): by
compute_returns' normalisation pass itself when it normalises (rslrl_compute_returns_slots, coalesced stores), else
by a slot copy at the first mini_batch_generator after it; the gather reads a drawn row's slot beside its record
(rslrl_gather_records_side).  A randomly drawn row then reads its record's own lines plus one 16-byte unit instead
of at least one line per field (2.2x the used bytes with one buffer per field).
RSLRL_RECORD_LAYOUT=0 keeps one buffer per field.

The host draw (1.57M elements at C3: ~4.7 ms, with the GPU idle behind it) is computed ahead: right after a
draw, a worker thread draws the NEXT permutation from a copy of the generator state.  The next
mini_batch_generator uses it only if the generator's state is still exactly that copy (nothing drew from it
in between) and then sets the generator to the post-draw state -- the same permutation and the same
generator state as drawing at that point; otherwise it draws synchronously.
"""

from __future__ import annotations

import os
import threading

import torch

from .. import kernels

# RSLRL_STAGE_PERM=1 (opt-in; the same permutations): the next update's permutation is uploaded at compute_returns on
# a side stream (stage_permutation) instead of at the update's start.  Off by default: it saves 20-100 us of host time
# where the GPU waits, but the same-box A/B at the 16,384-env share read 16.30 / 16.59 / 15.80 M with it against
# 16.55 / 16.53 / 16.56 M without (profiles/r6_stage_perm_ab.json) -- a third stream in the rollout's queue set is
# not worth that spread
_STAGE_PERM = os.environ.get("RSLRL_STAGE_PERM", "0") == "1"
from ..utils import TensorDict


class RolloutStorage:
    class Transition:
        def __init__(self):
            self.observations = None
            self.actions = None
            self.privileged_actions = None
            self.rewards = None
            self.dones = None
            self.values = None
            self.actions_log_prob = None
            self.action_mean = None
            self.action_sigma = None
            self.hidden_states = None

        def clear(self):
            self.__init__()

    def __init__(self, training_type, num_envs, num_transitions_per_env, obs, actions_shape, device="cpu"):
        self.training_type = training_type
        self.device = device
        self.num_transitions_per_env = num_transitions_per_env
        self.num_envs = num_envs
        self.actions_shape = actions_shape
        T, N = num_transitions_per_env, num_envs

        def zeros(*shape, dtype=torch.float32):
            return torch.zeros(*shape, dtype=dtype, device=device)

        self.records = None
        self._rec_plan = None  # kernels.RolloutRecordPlan of the fused rollout step (add_transition_fused)
        self._rec_plan_key = None  # the step signature _rec_plan was built for (a None plan is remembered too)
        self.record_layout = self._record_layout(training_type, obs, actions_shape, device)
        if self.record_layout is not None:
            R, offs = self.record_layout
            self.records = zeros(T, N, R)
            view = lambda name, w: self.records[:, :, offs[name]:offs[name] + w]  # noqa: E731
            self.observations = TensorDict({k: view("obs/" + k, v.shape[-1]) for k, v in obs.items()},
                                           batch_size=[T, N], device=device)
            self.actions = view("actions", actions_shape[0])
            self.mu = view("mu", actions_shape[0])
            self.sigma = view("sigma", actions_shape[0])
            # the update's scalar slot array {value, log-prob, return, advantage}: one contiguous 16-byte unit per
            # env-step, written by compute_returns' normalisation pass and gathered beside each drawn record
            self.slots = zeros(T, N, 4)
        else:
            self.observations = TensorDict({k: zeros(T, *v.shape) for k, v in obs.items()}, batch_size=[T, N],
                                           device=device)
            self.actions = zeros(T, N, *actions_shape)
        self.rewards = zeros(T, N, 1)
        self.dones = zeros(T, N, 1, dtype=torch.uint8)
        if training_type == "distillation":
            self.privileged_actions = zeros(T, N, *actions_shape)
        if training_type == "rl":
            self.values = zeros(T, N, 1)
            self.actions_log_prob = zeros(T, N, 1)
            if self.records is None:
                self.mu = zeros(T, N, *actions_shape)
                self.sigma = zeros(T, N, *actions_shape)
            self.returns = zeros(T, N, 1)
            self.advantages = zeros(T, N, 1)
        self.saved_hidden_states_a = None
        self.saved_hidden_states_c = None
        self.step = 0
        self._fills = 0  # transitions added so far (any path): a slot written before the last one is stale
        self._slot_key = None  # what the slot array was filled from (compute_returns), or None
        self.gae_status = None  # compute_returns' grid-barrier status word (kernels.compute_returns_slots), or None

        # mini-batch machinery (allocated on first use)
        self.perm_generator: torch.Generator | None = None
        self.last_indices: torch.Tensor | None = None  # device int32 permutation of the last generator
        self._packed = None
        self._packed_key = None
        self._perm_bufs = [None, None]  # pinned staging buffers (ping-pong: one may still be uploading)
        self._perm_events = [None, None]
        self._perm_slot = 0
        self._prefetch = None  # (n, state before, state after, slot, worker thread, done[, device copy, its event])
        self._upload_stream = None  # side stream of stage_permutation's upload

    @staticmethod
    def _record_layout(training_type, obs, actions_shape, device):
        """(R, {field: offset}) of the transition record, or None for one buffer per field: RL on a ROCm
        device, 2-D fp32 observation groups (<= 4) and 1-D actions, every width a multiple of 4 (16-byte
        fields), at most 256 used floats."""
        if os.environ.get("RSLRL_RECORD_LAYOUT", "1") == "0":
            return None
        if training_type != "rl" or torch.device(device).type != "cuda" or len(actions_shape) != 1:
            return None
        widths = []
        for k, v in obs.items():
            if v.dim() != 2 or v.dtype != torch.float32 or v.shape[-1] % 4:
                return None
            widths.append(("obs/" + k, v.shape[-1]))
        A = actions_shape[0]
        if A % 4 or len(widths) > 4:
            return None
        widths += [("actions", A), ("mu", A), ("sigma", A)]
        offs, used = {}, 0
        for name, w in widths:
            offs[name] = used
            used += w
        # (round 4: the per-update scalars {value, log-prob, return, advantage} moved out of the record into the
        # contiguous slot array: a 32-byte slot per 384-byte record was written at ~1.6 TB/s, the array at HBM rate)
        if used > 256:
            return None
        return -(-used // 32) * 32, offs

    # ------------------------------------------------------------------ filling (rollout_storage.py:77-125)
    def add_transitions(self, transition: Transition):
        if self.step >= self.num_transitions_per_env:
            raise OverflowError("Rollout buffer overflow! You should call clear() before adding new transitions.")
        t = self.step
        self.observations[t].copy_(transition.observations)
        self.actions[t].copy_(transition.actions)
        self.rewards[t].copy_(transition.rewards.view(-1, 1))
        self.dones[t].copy_(transition.dones.view(-1, 1))
        if self.training_type == "distillation":
            self.privileged_actions[t].copy_(transition.privileged_actions)
        if self.training_type == "rl":
            self.values[t].copy_(transition.values)
            self.actions_log_prob[t].copy_(transition.actions_log_prob.view(-1, 1))
            self.mu[t].copy_(transition.action_mean)
            self.sigma[t].copy_(transition.action_sigma)
        self._save_hidden_states(transition.hidden_states)
        self.step += 1
        self._fills += 1
        self._slot_key = None  # values / log-prob rewritten: the slots are stale

    def fused_record_ok(self, transition) -> bool:
        """The fused rollout record (kernels.rollout_record) covers the RL transition of a feed-forward
        policy on a ROCm device: A <= 64 and fp32 policy outputs."""
        a = transition.actions
        return (self.training_type == "rl" and a is not None and a.is_cuda and a.dim() == 2
                and a.dtype == torch.float32 and a.shape[1] <= 64 and transition.hidden_states in (None, (None, None))
                and len(self.actions_shape) == 1)

    def add_transition_fused(self, transition, rewards, dones, time_outs, gamma, extra_reward=None, rnd=None,
                             intrinsic_out=None):
        """add_transitions + the reward arithmetic of PPO.process_env_step in one launch
        (rollout_storage.py:77-103, ppo.py:147-164): row t receives the observation groups, actions,
        (rewards + extra + r_int) + gamma * values * time_outs, uint8(dones), values, log-prob, mu, sigma."""
        if self.step >= self.num_transitions_per_env:
            raise OverflowError("Rollout buffer overflow! You should call clear() before adding new transitions.")
        t = self.step
        sigma = transition.action_sigma
        if sigma.dim() == 2 and sigma.stride(0) == 0:  # Normal's expand of a shared [A] std
            sigma = sigma[0]
        if self.records is not None and rnd is None and extra_reward is None and intrinsic_out is None:
            # the common step (record layout, no RND): a cached argument struct, only this step's pointers written
            srcs = [transition.observations[k] for k in self.observations.keys()]
            args = (transition.actions, transition.action_mean, sigma, transition.values, rewards, dones, time_outs, srcs,
                    gamma)
            key = kernels.RolloutRecordPlan.signature(sigma, dones, time_outs, srcs, gamma)
            if key != self._rec_plan_key:  # built once per signature (None: the signature has no plan)
                self._rec_plan, self._rec_plan_key = self._record_plan(*args), key
            plan = self._rec_plan
            if plan is not None and plan.fits(*args[:-1]):
                plan.launch(t, *args[:-1])
                self.step += 1
                self._fills += 1
                self._slot_key = None  # written through data_ptr (no _version bump): the slots are stale
                return
        pairs, late = [], []
        for k, dst in self.observations.items():
            src = transition.observations[k]
            ok = (src.dtype == torch.float32 and src.is_cuda and src.dim() == 2 and src.shape[-1] % 4 == 0
                  and src.is_contiguous() and src.data_ptr() % 16 == 0 and dst[t].data_ptr() % 16 == 0
                  and len(pairs) < 4)
            if ok:
                pairs.append((src, dst[t]))
            else:
                late.append((src, dst[t]))  # after the launch: with records it writes every record whole
        kernels.rollout_record(
            t, obs_pairs=pairs, actions=transition.actions, mu=transition.action_mean, sigma=sigma,
            values=transition.values, rewards=rewards, dones=dones, time_outs=time_outs, gamma=gamma,
            out_actions=self.actions[t], out_rewards=self.rewards[t], out_dones=self.dones[t],
            out_values=self.values[t], out_logp=self.actions_log_prob[t], out_mu=self.mu[t], out_sigma=self.sigma[t],
            extra_reward=extra_reward, rnd=rnd, intrinsic_out=intrinsic_out,
            out_records=self.records[t] if self.records is not None else None)
        for src, dst in late:
            dst.copy_(src)
        self.step += 1
        self._fills += 1
        self._slot_key = None  # written through data_ptr (no _version bump): the slots are stale

    def _record_plan(self, actions, mu, sigma, values, rewards, dones, time_outs, srcs, gamma):
        """kernels.RolloutRecordPlan for steps with this one's signature, or None (the general path takes them); each
        step still checks that its own inputs fit the plan (RolloutRecordPlan.fits)."""
        codes = (torch.float32, torch.uint8, torch.bool, torch.int32, torch.int64)
        if len(srcs) > 4 or dones.dtype not in codes or (time_outs is not None and time_outs.dtype not in codes):
            return None
        if not all(s.dtype == torch.float32 and s.is_cuda and s.dim() == 2 and s.shape[-1] % 4 == 0 for s in srcs):
            return None
        outs = {"out_actions": self.actions, "out_rewards": self.rewards, "out_dones": self.dones,
                "out_values": self.values, "out_logp": self.actions_log_prob, "out_mu": self.mu,
                "out_sigma": self.sigma, "out_records": self.records}
        return kernels.RolloutRecordPlan(outs, [self.observations[k] for k in self.observations.keys()],
                                         [s.shape[-1] for s in srcs], self.num_envs, self.actions.shape[-1], gamma,
                                         dones.dtype, time_outs.dtype if time_outs is not None else None,
                                         sigma.dim() == 1, self.device)

    def _save_hidden_states(self, hidden_states):
        if hidden_states is None or hidden_states == (None, None):
            return
        hid_a = hidden_states[0] if isinstance(hidden_states[0], tuple) else (hidden_states[0],)
        hid_c = hidden_states[1] if isinstance(hidden_states[1], tuple) else (hidden_states[1],)
        if self.saved_hidden_states_a is None:
            T = self.num_transitions_per_env
            self.saved_hidden_states_a = [torch.zeros(T, *h.shape, device=self.device) for h in hid_a]
            self.saved_hidden_states_c = [torch.zeros(T, *h.shape, device=self.device) for h in hid_c]
        for i in range(len(hid_a)):
            self.saved_hidden_states_a[i][self.step].copy_(hid_a[i])
            self.saved_hidden_states_c[i][self.step].copy_(hid_c[i])

    def clear(self):
        self.step = 0

    # ------------------------------------------------------------------ GAE (rollout_storage.py:127-149)
    def compute_returns(self, last_values, gamma, lam, normalize_advantage: bool = True):
        self.stage_permutation()  # the next update's permutation, uploaded while the rollout's launches drain
        last_values = last_values.detach()
        if not last_values.is_contiguous():
            last_values = last_values.contiguous()
        if self.records is not None and normalize_advantage:
            # the normalisation pass also writes the slot array {value, log-prob, return, advantage} (coalesced
            # 16-byte units): the mini-batch generator gathers it beside the records (no slot copy per update)
            # the one-launch form's grid-barrier status word: PPO.update reads it with its loss statistics
            self.gae_status = kernels.compute_returns_slots(self.values, self.rewards, self.dones, last_values,
                                                            float(gamma), float(lam), self.returns, self.advantages,
                                                            self.actions_log_prob, self.slots)
            self._slot_key = self._slot_sources()
            return
        self._slot_key = None
        kernels.compute_returns(self.values, self.rewards, self.dones, last_values, float(gamma), float(lam),
                                normalize_advantage, self.returns, self.advantages)

    def _slot_sources(self):
        """What the slot array holds: the transition count and the in-place versions of the four scalar buffers
        (any later add_transitions or in-place write to values / log-prob / returns / advantages invalidates them).

        Invariant: a C-ABI kernel that writes values / log-prob / returns / advantages through data_ptr does not bump
        their torch _version, so every storage method that launches one must set self._slot_key itself (None, or
        the new sources after it rewrote the slots too): add_transitions, add_transition_fused, compute_returns."""
        return (self._fills, self.values._version, self.actions_log_prob._version, self.returns._version,
                self.advantages._version)

    # ------------------------------------------------------------------ distillation (rollout_storage.py:152-157)
    def generator(self):
        if self.training_type != "distillation":
            raise ValueError("This function is only available for distillation training.")
        for i in range(self.num_transitions_per_env):
            yield self.observations[i], self.actions[i], self.privileged_actions[i], self.dones[i]

    # ------------------------------------------------------------------ mini-batches (rollout_storage.py:160-203)
    def _packed_buffers(self, rows: int):
        key = (rows, tuple(self.observations.keys()))
        if self._packed_key != key:
            A = tuple(self.actions_shape)
            dev = self.device
            obs = {k: torch.empty(rows, *v.shape[2:], device=dev) for k, v in self.observations.items()}
            self._packed = {
                "obs": obs,
                "actions": torch.empty(rows, *A, device=dev),
                "values": torch.empty(rows, 1, device=dev),
                "returns": torch.empty(rows, 1, device=dev),
                "actions_log_prob": torch.empty(rows, 1, device=dev),
                "advantages": torch.empty(rows, 1, device=dev),
                "mu": torch.empty(rows, *A, device=dev),
                "sigma": torch.empty(rows, *A, device=dev),
            }
            self._packed_key = key
        return self._packed

    def _gen(self):
        return torch.default_generator if self.perm_generator is None else self.perm_generator

    def _staging(self, slot: int, n: int) -> torch.Tensor:
        """Pinned int32 buffer `slot`, once its previous upload has completed."""
        if self._perm_events[slot] is not None:
            self._perm_events[slot].synchronize()
            self._perm_events[slot] = None
        buf = self._perm_bufs[slot]
        if buf is None or buf.numel() < n:
            buf = torch.empty(n, dtype=torch.int32, pin_memory=True)
            self._perm_bufs[slot] = buf
        return buf

    def _upload(self, host: torch.Tensor, slot: int) -> torch.Tensor:
        dev = torch.empty(host.numel(), dtype=torch.int32, device=self.device)
        dev.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev.device))
        self._perm_events[slot] = ev
        self._perm_slot = slot
        return dev

    def _start_prefetch(self, n: int) -> None:
        gen = self._gen()
        if gen.device.type != "cpu":
            return
        before = gen.get_state()
        after = before.clone()
        slot = self._perm_slot ^ 1
        buf = self._staging(slot, n)
        done = []  # appended to only when the draw returned normally

        def draw():
            kernels.randperm_mt19937_state(n, after, buf)
            done.append(True)

        worker = threading.Thread(target=draw, daemon=True)
        worker.start()
        self._prefetch = (n, before, after, slot, worker, done)

    def stage_permutation(self) -> None:
        """Upload the next update's drawn-ahead permutation now, on a side stream (compute_returns calls this at the
        end of the rollout, where the GPU still has the rollout's last launches queued): the update then finds it on
        the device instead of paying the upload's host time where the GPU waits for its first launches.  Nothing is
        decided here: draw_permutation still checks the generator state and falls back to a synchronous draw."""
        pf = self._prefetch
        if pf is None or len(pf) != 6 or torch.device(self.device).type != "cuda" or not _STAGE_PERM:
            return
        pn, _, _, slot, worker, done = pf
        if worker.is_alive() or not done:
            return
        dev = torch.device(self.device)
        if self._upload_stream is None:
            self._upload_stream = torch.cuda.Stream(dev)
        with torch.cuda.stream(self._upload_stream):
            d = torch.empty(pn, dtype=torch.int32, device=dev)
            d.copy_(self._perm_bufs[slot][:pn], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._upload_stream)
        self._perm_events[slot] = ev  # the pinned buffer is rewritten only after this upload
        self._prefetch = pf + (d, ev)

    def draw_permutation(self, n: int) -> torch.Tensor:
        """Device int32 permutation of range(n) with torch CPU randperm semantics on perm_generator.

        Host mt19937 Fisher-Yates into a pinned staging buffer (or the permutation a worker thread drew ahead
        from the very same generator state), then one async upload on the current stream.
        """
        pf, self._prefetch = self._prefetch, None
        if pf is not None:
            pn, before, after, slot, worker, done = pf[:6]
            worker.join()
            gen = self._gen()
            # the drawn-ahead permutation is used only if its draw succeeded (the state advanced) and the generator
            # still holds the state it was drawn from; otherwise draw synchronously below
            if done and pn == n and not torch.equal(after, before) and torch.equal(gen.get_state(), before):
                gen.set_state(after)
                if len(pf) == 8:  # staged by stage_permutation: already (being) copied to the device
                    d, ev = pf[6], pf[7]
                    cur = torch.cuda.current_stream(d.device)
                    cur.wait_event(ev)
                    d.record_stream(cur)
                    self._perm_slot = slot
                    return d
                return self._upload(self._perm_bufs[slot][:n], slot)
        slot = self._perm_slot ^ 1
        host = kernels.randperm_mt19937(n, self.perm_generator, out=self._staging(slot, n))
        return self._upload(host, slot)

    def mini_batch_generator(self, num_mini_batches, num_epochs=8):
        if self.training_type != "rl":
            raise ValueError("This function is only available for reinforcement learning training.")
        batch_size = self.num_envs * self.num_transitions_per_env
        mini_batch_size = batch_size // num_mini_batches
        rows = num_mini_batches * mini_batch_size
        # permutation (:165) -- drawn lazily at the first next(), like the reference's generator body
        indices = self.draw_permutation(rows)
        self.last_indices = indices
        p = self._packed_buffers(rows)
        if self.records is not None:
            R, offs = self.record_layout
            A = self.actions_shape[0]
            # the scalar fields' final values into the slot array (unless compute_returns already wrote them and
            # nothing changed since), then one gather of the records' used prefixes with each row's slot beside it
            if self._slot_key is None or self._slot_key != self._slot_sources():
                kernels.record_fill_slot(self.slots, 0, 4,
                                         columns=[self.values, self.actions_log_prob, self.returns, self.advantages])
                self._slot_key = self._slot_sources()
            fields = [(offs["obs/" + k], v.shape[-1], p["obs"][k]) for k, v in self.observations.items()]
            fields += [(offs["actions"], A, p["actions"]), (offs["mu"], A, p["mu"]), (offs["sigma"], A, p["sigma"])]
            side = [(0, 1, p["values"]), (1, 1, p["actions_log_prob"]), (2, 1, p["returns"]), (3, 1, p["advantages"])]
            kernels.gather_records_side(self.records, fields, self.slots, side, indices)
        else:
            flat = lambda t: t.flatten(0, 1)  # noqa: E731
            pairs = [(flat(v), p["obs"][k]) for k, v in self.observations.items()]
            pairs += [(flat(self.actions), p["actions"]), (flat(self.values), p["values"]),
                      (flat(self.returns), p["returns"]), (flat(self.actions_log_prob), p["actions_log_prob"]),
                      (flat(self.advantages), p["advantages"]), (flat(self.mu), p["mu"]),
                      (flat(self.sigma), p["sigma"])]
            kernels.gather_rows(pairs, indices)

        prefetch = True
        for _epoch in range(num_epochs):
            for i in range(num_mini_batches):
                if prefetch and (_epoch or i):
                    # the next update's permutation, drawn on a worker thread meanwhile -- started once the first
                    # mini-batch's launches are queued (starting the thread costs ~125 us of host time that the GPU
                    # would otherwise wait out between the gather and the first mini-batch)
                    self._start_prefetch(rows)
                    prefetch = False
                s = slice(i * mini_batch_size, (i + 1) * mini_batch_size)
                obs_batch = TensorDict({k: v[s] for k, v in p["obs"].items()}, batch_size=[mini_batch_size],
                                       device=self.device)
                yield (
                    obs_batch,
                    p["actions"][s],
                    p["values"][s],
                    p["advantages"][s],
                    p["returns"][s],
                    p["actions_log_prob"][s],
                    p["mu"][s],
                    p["sigma"][s],
                    (None, None),
                    None,
                )

    def recurrent_mini_batch_generator(self, num_mini_batches, num_epochs=8):
        raise NotImplementedError(
            "recurrent policies (rollout_storage.py:206-260) are outside the MI355X PPO hot-path scope (SURVEY.md §2)"
        )
