"""CPU: hyper-parameter schedules against the reference's own scheduler
callback and position resolver (tests/golden/schedules.npz, made by make_golden.py from
trainer_callbacks/hyperparameter_scheduler.py and utils/schedule_resolver.py).  Bar: 1e-12
relative (the same double-precision formulas)."""
import numpy as np
import pytest


def test_scheduler_values_match_reference(golden):
    from gsamd.schedules import Scheduler
    z = golden("schedules.npz")
    for case, row in zip(z["cases"], z["values"]):
        kind, warm, sv, ev, s0, s1 = str(case).split("|")
        s = Scheduler("p", kind, float(sv), float(ev), float(s0), float(s1), float(warm))
        got = np.array([s.value(t) for t in z["steps"]])
        np.testing.assert_allclose(got, row, rtol=1e-12, atol=1e-15, err_msg=str(case))


def test_schedule_positions_match_reference(golden):
    from gsamd.schedules import schedule_pos_to_vec_steps
    z = golden("schedules.npz")
    args = ((None, False, 1e6, 8), (None, True, 1e6, 8), (0.5, False, 1e6, 8), (1.0, True, 2e5, 16),
            (4096.0, False, None, 8), (123456.0, True, 1e6, 32))
    for (raw, dmax, mx, n), want in zip(args, z["pos"][:, 0]):
        assert schedule_pos_to_vec_steps(raw, param="p", default_to_max=dmax, max_env_steps=mx, n_envs=n) == want
    with pytest.raises(ValueError):
        schedule_pos_to_vec_steps(None, param="p", default_to_max=True, max_env_steps=None, n_envs=8)
    with pytest.raises(ValueError):
        schedule_pos_to_vec_steps(0.5, param="p", default_to_max=False, max_env_steps=None, n_envs=8)


def test_config_schedule_forms():
    """Dict syntax (utils/config.py:626-655) and the resolved attribute form a reference Config
    object carries (utils/config.py:188-196) give the same schedulers."""
    from types import SimpleNamespace

    from gsamd.config import PPOConfig, from_reference_config
    from gsamd.schedules import build_schedulers
    c = PPOConfig(env_id="x", n_envs=8, max_env_steps=80_000,
                  policy_lr={"start": 1e-3, "end": 1e-4, "schedule": "cosine", "warmup": 0.1}, ent_coef=0.01)
    assert c.policy_lr == 1e-3 and set(c.schedules) == {"policy_lr"}
    ref = SimpleNamespace(env_id="x", n_envs=8, max_env_steps=80_000, policy_lr=1e-3, ent_coef=0.01,
                          policy_lr_schedule="cosine", policy_lr_schedule_start_value=1e-3,
                          policy_lr_schedule_end_value=1e-4, policy_lr_schedule_start=0.0,
                          policy_lr_schedule_end=1.0, policy_lr_schedule_warmup=0.1, ent_coef_schedule=None)
    c2 = from_reference_config(ref)
    a, b = build_schedulers(c.schedules, c.max_env_steps, 8), build_schedulers(c2.schedules, c2.max_env_steps, 8)
    assert len(a) == len(b) == 1
    for t in (0, 500, 1000, 5000, 9999, 10000, 20000):
        assert a[0].value(t) == b[0].value(t)
    assert a[0].end_step == 10_000.0
    with pytest.raises(ValueError):
        build_schedulers({"n_envs": c.schedules["policy_lr"]}, 1e5, 8)


def test_scheduled_lr_matches_reference_hp_log():
    """trajectory_stats.npz's hp/policy_lr per epoch (the reference's HyperparameterSchedulerCallback
    applied at each epoch end through _change_optimizers_lr, logged by _log_hyperparameters at the
    next epoch start) equals gsamd.schedules on the same spec, bit for bit."""
    import os
    import numpy as np
    from gsamd.schedules import build_schedulers
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "trajectory_stats.npz"))
    N, T = (int(x) for x in z["dims"][:2])
    sv, ev, s0, s1 = (float(x) for x in z["lr_schedule"])
    sch = build_schedulers({"policy_lr": {"schedule": "linear", "start_value": sv, "end_value": ev, "start": None,
                                          "end": s1 * N, "warmup": 0.0}}, None, N)[0]
    names = [str(x) for x in z["hp_names"]]
    lr = [float(row[names.index("hp/policy_lr")]) for row in z["hp_values"]]
    assert lr[0] == sv
    assert [sch.value(T * (e + 1)) for e in range(len(lr) - 1)] == lr[1:]
