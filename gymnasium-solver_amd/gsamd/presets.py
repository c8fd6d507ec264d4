"""Resolved configs of the BASELINE.json workloads and the model presets.

PRESETS holds what the reference's load_config(...) resolves for each id (values taken
from config/environments/{CartPole-v1,LunarLander-v3,ALE-Pong-v5,ALE-Breakout-v5}.yaml
through utils/config.py; tests/golden/configs.json is the machine-generated record
tests/test_config.py compares against).  MODEL_REGISTRY mirrors
utils/model_registry.py:17-76.
"""

MODEL_REGISTRY = {
    "mlp_tiny": {"policy": "mlp_actorcritic", "hidden_dims": (64,)},
    "mlp_small": {"policy": "mlp_actorcritic", "hidden_dims": (128, 128)},
    "mlp_medium": {"policy": "mlp_actorcritic", "hidden_dims": (256, 256)},
    "mlp_large": {"policy": "mlp_actorcritic", "hidden_dims": (512, 512)},
    "cnn_nature": {"policy": "cnn_actorcritic", "hidden_dims": (512,),
                   "channels": (32, 64, 64), "kernel_sizes": (8, 4, 3), "strides": (4, 2, 1)},
    "cnn_impala": {"policy": "cnn_actorcritic", "hidden_dims": (256,),
                   "channels": (16, 32, 32), "kernel_sizes": (8, 4, 3), "strides": (4, 2, 1)},
    "cnn_large": {"policy": "cnn_actorcritic", "hidden_dims": (1024,),
                  "channels": (32, 64, 128), "kernel_sizes": (8, 4, 3), "strides": (4, 2, 1)},
}

_COMMON = dict(algo_id="ppo", clip_range_vf=0.2, vf_coef=0.5, max_grad_norm=0.5, normalize_advantages="batch",
               seed=42, target_kl=None, optimizer="adam")

PRESETS = {
    "CartPole-v1:ppo": dict(
        _COMMON, env_id="CartPole-v1", project_id="CartPole-v1", n_envs=8, n_steps=32, batch_size=256, n_epochs=20,
        gamma=0.98, gae_lambda=0.8, clip_range=0.1, ent_coef=0.0, policy_lr=0.001, model_id="mlp_medium",
        max_env_steps=100000.0, obs_type="vector", accelerator="cpu",
        spec={"action_space": {"discrete": 2}, "observation_space": {"default": "state",
                                                                     "variants": {"state": {"shape": [4]}}}}),
    "LunarLander-v3:ppo": dict(
        _COMMON, env_id="LunarLander-v3", project_id="LunarLander-v3", n_envs=8, n_steps=2048, batch_size=64,
        n_epochs=10, gamma=0.99, gae_lambda=0.95, clip_range=0.2, ent_coef=0.0, policy_lr=0.0003,
        model_id="mlp_small", max_env_steps=5000000.0, obs_type="vector",
        spec={"action_space": {"discrete": 4}, "observation_space": {"default": "state",
                                                                     "variants": {"state": {"shape": [8]}}}}),
    "ALE-Pong-v5:rgb_ppo": dict(
        _COMMON, env_id="ALE/Pong-v5", project_id="ALE-Pong-v5_rgb", n_envs=32, n_steps=256, batch_size=1024,
        n_epochs=15, gamma=0.99, gae_lambda=0.95, clip_range=0.2, ent_coef=0.01, policy_lr=0.0003,
        model_id="cnn_nature", max_env_steps=5000000.0, obs_type="rgb", frame_stack=4,
        spec={"action_space": {"discrete": 18, "valid": [0, 3, 4]}}),
    "ALE-Breakout-v5:rgb_ppo": dict(
        _COMMON, env_id="ALE/Breakout-v5", project_id="ALE-Breakout-v5_rgb", n_envs=32, n_steps=128,
        batch_size=1024, n_epochs=4, gamma=0.99, gae_lambda=0.95, clip_range=0.1, ent_coef=0.01,
        policy_lr=0.0003, model_id="cnn_nature", max_env_steps=None, obs_type="rgb", frame_stack=4,
        spec={"action_space": {"discrete": 18, "valid": [0, 1, 3, 4]}}),
}
