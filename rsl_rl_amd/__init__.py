"""rsl_rl_amd -- MI355X-native PPO hot path behind the rsl_rl API.

Drop-in modules mirroring the reference package layout:
    rsl_rl_amd.runners.OnPolicyRunner, rsl_rl_amd.algorithms.PPO, rsl_rl_amd.storage.RolloutStorage,
    rsl_rl_amd.modules.ActorCritic, rsl_rl_amd.env.VecEnv, rsl_rl_amd.networks, rsl_rl_amd.utils
The hot path (GAE, permutation/mini-batch assembly, fused PPO loss) runs in librslrl_amd.so (HIP,
gfx950) through the C ABI of include/rslrl_amd.h; see DESIGN.md.
"""

__version__ = "0.1.0"
