"""Host-side synchronisation points of one C3 learning iteration: torch's sync debug mode (warn) with the Python stack
of each synchronising call, plus the host time of PPO.update's prologue (until the first mini-batch is yielded)."""
import collections
import os
import sys
import time
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd.env import SyntheticVecEnv  # noqa: E402
from rsl_rl_amd.runners import OnPolicyRunner  # noqa: E402
import bench  # noqa: E402


def main():
    class A:  # bench.py's C3 arguments
        hidden, layers, num_steps_per_env, num_obs, num_actions = 256, 3, 24, 48, 12
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    env = SyntheticVecEnv(65536, 48, 12, device=dev, seed=0)
    runner = OnPolicyRunner(env, bench.train_cfg(A), log_dir=None, device=dev)
    runner.learn(2)
    torch.cuda.synchronize()
    hits = collections.Counter()

    def show(message, category, filename, lineno, file=None, line=None):
        st = [f"{os.path.relpath(f.filename)}:{f.lineno} {f.name}" for f in traceback.extract_stack()[:-2]
              if "rsl_rl_amd" in f.filename or "bench" in f.filename]
        hits[(str(message)[:80], " <- ".join(reversed(st[-4:])))] += 1

    warnings.showwarning = show
    warnings.simplefilter("always")
    storage = runner.alg.storage
    orig = storage.mini_batch_generator
    marks = {}

    def mbg(*a, **k):
        marks["mbg_called"] = time.perf_counter()
        g = orig(*a, **k)
        first = next(g)
        marks["first_yield"] = time.perf_counter()
        yield first
        yield from g

    storage.mini_batch_generator = mbg
    upd = runner.alg.update

    def update():
        marks["update_start"] = time.perf_counter()
        r = upd()
        marks["update_end"] = time.perf_counter()
        return r

    runner.alg.update = update
    torch.cuda.set_sync_debug_mode(1)
    runner.learn(1)
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    for (m, st), c in hits.most_common():
        print(f"{c:4d}  {m} | {st}")
    print({k: round((v - marks["update_start"]) * 1e6, 1) for k, v in marks.items()}, "us from update start")


if __name__ == "__main__":
    main()
