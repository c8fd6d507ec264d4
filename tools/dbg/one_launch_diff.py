"""Debug: where the one-launch rollout's rows differ from the step loop's (first rollout)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]
import torch
from gsamd.config import load_config
from gsamd.ppo_agent import DevicePPOAgent
out = []
for one in (False, True):
    torch.manual_seed(42)
    cfg = load_config("LunarLander-v3", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=72, n_steps=96, batch_size=64, n_epochs=2))
    agent = DevicePPOAgent(cfg, device="cuda:0", use_graph=False, track_stats=True, one_launch=one)
    coll = agent.get_rollout_collector("train")
    coll.collect()
    b = coll.buffer
    out.append([t.clone() for t in (b.obs, b.actions, b.logprobs, b.values, b.rewards, b.dones)])
for j, (x, y) in enumerate(zip(*out)):
    d = (x != y).reshape(x.shape[0], x.shape[1], -1).any(-1) if x.dim() > 2 else (x != y)
    idx = torch.nonzero(d)
    print(j, "mismatches", idx.shape[0], "first", idx[:6].tolist())
    if idx.shape[0]:
        t, e = idx[0].tolist()
        print("   step", t, "env", e, x[t, e].tolist() if x.dim() > 2 else x[t, e].item(),
              y[t, e].tolist() if y.dim() > 2 else y[t, e].item())
