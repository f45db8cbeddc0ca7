"""On-policy runner (rsl_rl/runners/on_policy_runner.py:22-460): the public training entry point.

Construction, learn(), save()/load(), get_inference_policy(), train_mode()/eval_mode(),
add_git_repo_to_log() and the attributes (alg, env, cfg, current_learning_iteration, log_dir) behave as
in the reference; `class_name` strings in the config are resolved against this module's namespace
(ActorCritic, PPO), so reference configs work unchanged.  Multi-GPU: one process per GPU launched by
torchrun, env vars WORLD_SIZE / RANK / LOCAL_RANK, `torch.distributed` with backend "nccl" (RCCL on
ROCm, over xGMI); each rank owns its own environment shard, storage and permutation.

Timing follows the reference (collection = rollout + compute_returns, learn = update) and the
throughput it logs as Perf/total_fps = T * N * world_size / (collection + learn) (:179, :209) is also
returned by learn() through `self.last_iteration_stats` for benchmarking.
"""

from __future__ import annotations

import os
import sys
import statistics
import time
import warnings
from collections import deque

import torch

import rsl_rl_amd
from rsl_rl_amd.algorithms import PPO  # noqa: F401  (resolved by class_name)
from rsl_rl_amd.env import VecEnv
from rsl_rl_amd.networks import fused_mlp
from rsl_rl_amd.modules import ActorCritic, resolve_rnd_config, resolve_symmetry_config  # noqa: F401
from rsl_rl_amd.utils import resolve_obs_groups, store_code_state

_CLASSES = {"ActorCritic": ActorCritic, "PPO": PPO}


def _resolve_class(name):
    if not isinstance(name, str):
        return name
    if name in _CLASSES:
        return _CLASSES[name]
    raise ValueError(f"Unknown class_name '{name}' (available in rsl_rl_amd: {sorted(_CLASSES)})")


class OnPolicyRunner:
    """On-policy runner for training and evaluation of actor-critic methods."""

    def __init__(self, env: VecEnv, train_cfg: dict, log_dir: str | None = None, device="cpu"):
        self.cfg = train_cfg
        self.alg_cfg = train_cfg["algorithm"]
        self.policy_cfg = train_cfg["policy"]
        self.device = device
        self.env = env
        self._configure_multi_gpu()
        self.num_steps_per_env = self.cfg["num_steps_per_env"]
        self.save_interval = self.cfg["save_interval"]

        obs = self.env.get_observations()
        default_sets = ["critic"]
        if self.alg_cfg.get("rnd_cfg") is not None:
            default_sets.append("rnd_state")
        self.cfg["obs_groups"] = resolve_obs_groups(obs, self.cfg["obs_groups"], default_sets)
        self.alg = self._construct_algorithm(obs)

        self.disable_logs = self.is_distributed and self.gpu_global_rank != 0
        self.log_dir = log_dir
        self.writer = None
        self.logger_type = self.cfg.get("logger", "tensorboard").lower()
        self.tot_timesteps = 0
        self.tot_time = 0
        self.current_learning_iteration = 0
        self.git_status_repos = [rsl_rl_amd.__file__]
        self.last_iteration_stats: dict = {}
        # (collection_time, learn_time) of the latest iterations (benchmarking; bounded for long training runs)
        self.iteration_stats_history: deque = deque(maxlen=1024)

    # ------------------------------------------------------------------ training loop (:61-175)
    def learn(self, num_learning_iterations: int, init_at_random_ep_len: bool = False):  # noqa: C901
        self._prepare_logging_writer()
        if init_at_random_ep_len:
            self.env.episode_length_buf = torch.randint_like(
                self.env.episode_length_buf, high=int(self.env.max_episode_length)
            )
        obs = self.env.get_observations().to(self.device)
        self.train_mode()

        ep_infos = []
        rewbuffer, lenbuffer = deque(maxlen=100), deque(maxlen=100)
        n_env = self.env.num_envs
        cur_reward_sum = torch.zeros(n_env, dtype=torch.float, device=self.device)
        cur_episode_length = torch.zeros(n_env, dtype=torch.float, device=self.device)
        if self.alg.rnd:
            erewbuffer, irewbuffer = deque(maxlen=100), deque(maxlen=100)
            cur_ereward_sum = torch.zeros(n_env, dtype=torch.float, device=self.device)
            cur_ireward_sum = torch.zeros(n_env, dtype=torch.float, device=self.device)

        if self.is_distributed:
            print(f"Synchronizing parameters for rank {self.gpu_global_rank}...")
            self.alg.broadcast_parameters()

        start_iter = self.current_learning_iteration
        tot_iter = start_iter + num_learning_iterations
        for it in range(start_iter, tot_iter):
            start = time.time()
            with torch.inference_mode(), fused_mlp.frozen_weights():
                for _ in range(self.num_steps_per_env):
                    actions = self.alg.act(obs)
                    obs, rewards, dones, extras = self.env.step(actions.to(self.env.device))
                    obs, rewards, dones = obs.to(self.device), rewards.to(self.device), dones.to(self.device)
                    self.alg.process_env_step(obs, rewards, dones, extras)
                    intrinsic_rewards = self.alg.intrinsic_rewards if self.alg.rnd else None
                    if self.log_dir is not None:
                        if "episode" in extras:
                            ep_infos.append(extras["episode"])
                        elif "log" in extras:
                            ep_infos.append(extras["log"])
                        if self.alg.rnd:
                            cur_ereward_sum += rewards
                            cur_ireward_sum += intrinsic_rewards
                            cur_reward_sum += rewards + intrinsic_rewards
                        else:
                            cur_reward_sum += rewards
                        cur_episode_length += 1
                        new_ids = (dones > 0).nonzero(as_tuple=False)
                        rewbuffer.extend(cur_reward_sum[new_ids][:, 0].cpu().numpy().tolist())
                        lenbuffer.extend(cur_episode_length[new_ids][:, 0].cpu().numpy().tolist())
                        cur_reward_sum[new_ids] = 0
                        cur_episode_length[new_ids] = 0
                        if self.alg.rnd:
                            erewbuffer.extend(cur_ereward_sum[new_ids][:, 0].cpu().numpy().tolist())
                            irewbuffer.extend(cur_ireward_sum[new_ids][:, 0].cpu().numpy().tolist())
                            cur_ereward_sum[new_ids] = 0
                            cur_ireward_sum[new_ids] = 0
                stop = time.time()
                collection_time = stop - start
                start = stop
                self.alg.compute_returns(obs)

            loss_dict = self.alg.update()
            stop = time.time()
            learn_time = stop - start
            self.current_learning_iteration = it
            steps = self.num_steps_per_env * n_env * self.gpu_world_size
            self.last_iteration_stats = {
                "collection_time": collection_time,
                "learn_time": learn_time,
                "total_fps": steps / (collection_time + learn_time),
                "loss_dict": loss_dict,
            }
            self.iteration_stats_history.append((collection_time, learn_time))
            if self.log_dir is not None and not self.disable_logs:
                self.log(locals())
                if it % self.save_interval == 0:
                    self.save(os.path.join(self.log_dir, f"model_{it}.pt"))
            ep_infos.clear()
            if it == start_iter and not self.disable_logs and self.log_dir is not None:
                paths = store_code_state(self.log_dir, self.git_status_repos)
                if self.logger_type in ["wandb", "neptune"] and paths:
                    for path in paths:
                        self.writer.save_file(path)

        if self.log_dir is not None and not self.disable_logs:
            self.save(os.path.join(self.log_dir, f"model_{self.current_learning_iteration}.pt"))

    # ------------------------------------------------------------------ logging (:177-287)
    def log(self, locs: dict, width: int = 80, pad: int = 35):
        collection_size = self.num_steps_per_env * self.env.num_envs * self.gpu_world_size
        iteration_time = locs["collection_time"] + locs["learn_time"]
        self.tot_timesteps += collection_size
        self.tot_time += iteration_time
        it = locs["it"]

        ep_string = ""
        if locs["ep_infos"]:
            for key in locs["ep_infos"][0]:
                parts = []
                for ep_info in locs["ep_infos"]:
                    if key not in ep_info:
                        continue
                    v = ep_info[key]
                    if not isinstance(v, torch.Tensor):
                        v = torch.Tensor([v])
                    if v.dim() == 0:
                        v = v.unsqueeze(0)
                    parts.append(v.to(self.device))
                value = torch.mean(torch.cat(parts)) if parts else torch.tensor(float("nan"))
                if "/" in key:
                    self.writer.add_scalar(key, value, it)
                    ep_string += f"{f'{key}:':>{pad}} {value:.4f}\n"
                else:
                    self.writer.add_scalar("Episode/" + key, value, it)
                    ep_string += f"{f'Mean episode {key}:':>{pad}} {value:.4f}\n"

        mean_std = self.alg.policy.action_std.mean()
        fps = int(collection_size / iteration_time)
        for key, value in locs["loss_dict"].items():
            self.writer.add_scalar(f"Loss/{key}", value, it)
        self.writer.add_scalar("Loss/learning_rate", self.alg.learning_rate, it)
        self.writer.add_scalar("Policy/mean_noise_std", mean_std.item(), it)
        self.writer.add_scalar("Perf/total_fps", fps, it)
        self.writer.add_scalar("Perf/collection time", locs["collection_time"], it)
        self.writer.add_scalar("Perf/learning_time", locs["learn_time"], it)
        rew, ln = locs["rewbuffer"], locs["lenbuffer"]
        if len(rew) > 0:
            if self.alg.rnd:
                self.writer.add_scalar("Rnd/mean_extrinsic_reward", statistics.mean(locs["erewbuffer"]), it)
                self.writer.add_scalar("Rnd/mean_intrinsic_reward", statistics.mean(locs["irewbuffer"]), it)
                self.writer.add_scalar("Rnd/weight", self.alg.rnd.weight, it)
            self.writer.add_scalar("Train/mean_reward", statistics.mean(rew), it)
            self.writer.add_scalar("Train/mean_episode_length", statistics.mean(ln), it)
            if self.logger_type != "wandb":
                self.writer.add_scalar("Train/mean_reward/time", statistics.mean(rew), self.tot_time)
                self.writer.add_scalar("Train/mean_episode_length/time", statistics.mean(ln), self.tot_time)

        title = f" \033[1m Learning iteration {it}/{locs['tot_iter']} \033[0m "
        lines = [
            "#" * width,
            title.center(width, " "),
            "",
            f"{'Computation:':>{pad}} {fps:.0f} steps/s (collection: {locs['collection_time']:.3f}s, "
            f"learning {locs['learn_time']:.3f}s)",
            f"{'Mean action noise std:':>{pad}} {mean_std.item():.2f}",
        ]
        if len(rew) > 0:
            lines += [f"{f'Mean {k} loss:':>{pad}} {v:.4f}" for k, v in locs["loss_dict"].items()]
            if self.alg.rnd:
                lines.append(f"{'Mean extrinsic reward:':>{pad}} {statistics.mean(locs['erewbuffer']):.2f}")
                lines.append(f"{'Mean intrinsic reward:':>{pad}} {statistics.mean(locs['irewbuffer']):.2f}")
            lines.append(f"{'Mean reward:':>{pad}} {statistics.mean(rew):.2f}")
            lines.append(f"{'Mean episode length:':>{pad}} {statistics.mean(ln):.2f}")
        else:
            lines += [f"{f'{k}:':>{pad}} {v:.4f}" for k, v in locs["loss_dict"].items()]
        done_iters = it - locs["start_iter"] + 1
        eta = self.tot_time / done_iters * (locs["start_iter"] + locs["num_learning_iterations"] - it)
        text = "\n".join(lines) + "\n" + ep_string
        text += (
            f"{'-' * width}\n"
            f"{'Total timesteps:':>{pad}} {self.tot_timesteps}\n"
            f"{'Iteration time:':>{pad}} {iteration_time:.2f}s\n"
            f"{'Time elapsed:':>{pad}} {time.strftime('%H:%M:%S', time.gmtime(self.tot_time))}\n"
            f"{'ETA:':>{pad}} {time.strftime('%H:%M:%S', time.gmtime(eta))}\n"
        )
        print(text)

    # ------------------------------------------------------------------ checkpoints (:289-324)
    def save(self, path: str, infos=None):
        saved = {
            "model_state_dict": self.alg.policy.state_dict(),
            "optimizer_state_dict": self.alg.optimizer.state_dict(),
            "iter": self.current_learning_iteration,
            "infos": infos,
        }
        if self.alg.rnd:
            saved["rnd_state_dict"] = self.alg.rnd.state_dict()
            saved["rnd_optimizer_state_dict"] = self.alg.rnd_optimizer.state_dict()
        torch.save(saved, path)
        if self.logger_type in ["neptune", "wandb"] and not self.disable_logs and self.writer is not None:
            self.writer.save_model(path, self.current_learning_iteration)

    def load(self, path: str, load_optimizer: bool = True, map_location: str | None = None):
        # the reference loads with weights_only=False; these checkpoints hold only tensors, dicts and
        # numbers, so the safe loader reads them (and rejects anything that would execute code)
        loaded = torch.load(path, weights_only=True, map_location=map_location)
        resumed = self.alg.policy.load_state_dict(loaded["model_state_dict"])
        if self.alg.rnd:
            self.alg.rnd.load_state_dict(loaded["rnd_state_dict"])
        if load_optimizer and resumed:
            self.alg.optimizer.load_state_dict(loaded["optimizer_state_dict"])
            if self.alg.rnd:
                self.alg.rnd_optimizer.load_state_dict(loaded["rnd_optimizer_state_dict"])
        if resumed:
            self.current_learning_iteration = loaded["iter"]
        return loaded["infos"]

    def get_inference_policy(self, device=None):
        self.eval_mode()
        if device is not None:
            self.alg.policy.to(device)
        return self.alg.policy.act_inference

    def train_mode(self):
        self.alg.policy.train()
        if self.alg.rnd:
            self.alg.rnd.train()

    def eval_mode(self):
        self.alg.policy.eval()
        if self.alg.rnd:
            self.alg.rnd.eval()

    def add_git_repo_to_log(self, repo_file_path):
        self.git_status_repos.append(repo_file_path)

    # ------------------------------------------------------------------ helpers (:353-460)
    def _configure_multi_gpu(self):
        """One process per GPU: read WORLD_SIZE / LOCAL_RANK / RANK, validate, init RCCL ("nccl")
        (on_policy_runner.py:353-395, same checks and error messages).

        Test-only override: RSLRL_TEST_ONE_DEVICE=1 puts every rank on cuda:0 over a gloo group (RCCL refuses two
        ranks on one device), so the world > 1 path -- this method, broadcast_parameters, the per-mini-batch
        all-reduce, bench.py's max-over-ranks timing -- runs end to end on a one-GPU box (tests/test_bench_launch.py)."""
        self.gpu_world_size = int(os.getenv("WORLD_SIZE", "1"))
        self.is_distributed = self.gpu_world_size > 1
        if not self.is_distributed:
            self.gpu_local_rank = 0
            self.gpu_global_rank = 0
            self.multi_gpu_cfg = None
            return
        self.gpu_local_rank = int(os.getenv("LOCAL_RANK", "0"))
        self.gpu_global_rank = int(os.getenv("RANK", "0"))
        self.multi_gpu_cfg = {
            "global_rank": self.gpu_global_rank,
            "local_rank": self.gpu_local_rank,
            "world_size": self.gpu_world_size,
        }
        one_device = os.getenv("RSLRL_TEST_ONE_DEVICE") == "1"
        if one_device:
            # never meant for a real job: say so on every rank, loudly
            warnings.warn(
                f"RSLRL_TEST_ONE_DEVICE=1: rank {self.gpu_global_rank} of {self.gpu_world_size} runs on cuda:0 over a "
                "gloo group (a test-only override: every rank shares one GPU and RCCL is not used). Unset it for a "
                "multi-GPU run.", RuntimeWarning, stacklevel=2)
            print(f"[rsl_rl_amd] WARNING: RSLRL_TEST_ONE_DEVICE=1 -- rank {self.gpu_global_rank} on cuda:0 over gloo "
                  "(test-only override)", file=sys.stderr, flush=True)
        if self.device != ("cuda:0" if one_device else f"cuda:{self.gpu_local_rank}"):
            raise ValueError(
                f"Device '{self.device}' does not match expected device for local rank '{self.gpu_local_rank}'."
            )
        if self.gpu_local_rank >= self.gpu_world_size:
            raise ValueError(
                f"Local rank '{self.gpu_local_rank}' is greater than or equal to world size '{self.gpu_world_size}'."
            )
        if self.gpu_global_rank >= self.gpu_world_size:
            raise ValueError(
                f"Global rank '{self.gpu_global_rank}' is greater than or equal to world size '{self.gpu_world_size}'."
            )
        if not torch.distributed.is_initialized():
            torch.distributed.init_process_group(backend="gloo" if one_device else "nccl", rank=self.gpu_global_rank,
                                                 world_size=self.gpu_world_size)
        torch.cuda.set_device(0 if one_device else self.gpu_local_rank)

    def _construct_algorithm(self, obs) -> PPO:
        self.alg_cfg = resolve_rnd_config(self.alg_cfg, obs, self.cfg["obs_groups"], self.env)
        self.alg_cfg = resolve_symmetry_config(self.alg_cfg, self.env)
        if self.cfg.get("empirical_normalization") is not None:
            warnings.warn(
                "The `empirical_normalization` parameter is deprecated. Please set `actor_obs_normalization` and "
                "`critic_obs_normalization` as part of the `policy` configuration instead.",
                DeprecationWarning,
            )
            if self.policy_cfg.get("actor_obs_normalization") is None:
                self.policy_cfg["actor_obs_normalization"] = self.cfg["empirical_normalization"]
            if self.policy_cfg.get("critic_obs_normalization") is None:
                self.policy_cfg["critic_obs_normalization"] = self.cfg["empirical_normalization"]
        policy_class = _resolve_class(self.policy_cfg.pop("class_name"))
        policy = policy_class(obs, self.cfg["obs_groups"], self.env.num_actions, **self.policy_cfg).to(self.device)
        alg_class = _resolve_class(self.alg_cfg.pop("class_name"))
        alg: PPO = alg_class(policy, device=self.device, **self.alg_cfg, multi_gpu_cfg=self.multi_gpu_cfg)
        alg.init_storage("rl", self.env.num_envs, self.num_steps_per_env, obs, [self.env.num_actions])
        return alg

    def _prepare_logging_writer(self):
        if self.log_dir is None or self.writer is not None or self.disable_logs:
            return
        if self.logger_type in ("neptune", "wandb"):
            raise NotImplementedError(
                f"the {self.logger_type} writer (rsl_rl/utils/{self.logger_type}_utils.py) is observability outside "
                "the MI355X PPO hot-path scope (SURVEY.md §2); use logger='tensorboard'"
            )
        if self.logger_type != "tensorboard":
            raise ValueError("Logger type not found. Please choose 'neptune', 'wandb' or 'tensorboard'.")
        from torch.utils.tensorboard import SummaryWriter

        self.writer = SummaryWriter(log_dir=self.log_dir, flush_secs=10)
