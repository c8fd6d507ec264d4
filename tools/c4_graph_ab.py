"""C4 update timing, eager launches vs one captured graph of the same gs_cnn_ppo_update call
(same box, same state, alternated): Pong rgb_ppo, 256 envs x T steps (T = 32: 8 minibatches of
B = 1024 per epoch), fp32 or --bf16.  Prints us per minibatch for each form.
Usage: python tools/c4_graph_ab.py [--bf16] [--reps 3]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]

import torch  # noqa: E402

from gsamd._lib import GS_HP_BF16, check, lib, ptr  # noqa: E402
from gsamd.config import load_config  # noqa: E402
from gsamd.ppo_agent import DevicePPOAgent  # noqa: E402


def main():
    bf = "--bf16" in sys.argv
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
    torch.manual_seed(42)
    over = dict(env_dynamics="synthetic", n_envs=256, n_steps=32, n_epochs=4)
    if bf:
        over["precision"] = "bf16"
    cfg = load_config("ALE-Pong-v5", "rgb_ppo", overrides=over)
    agent = DevicePPOAgent(cfg, device=torch.device("cuda:0"), use_graph=False, track_stats=False)
    coll = agent.get_rollout_collector("train")
    coll.collect()
    idx = agent.prefetcher.upload(0)
    pm = agent.policy_model
    hp = agent.hparams()
    assert bool(hp.flags & GS_HP_BF16) == bf
    K, B = agent.n_minibatches, agent.batch_size
    state = [t.clone() for t in (pm.params, agent.adam_m, agent.adam_v)]
    s = torch.cuda.Stream()

    def restore():
        for t, s0 in zip((pm.params, agent.adam_m, agent.adam_v), state):
            t.copy_(s0)
        torch.cuda.synchronize()

    def run():
        check(lib.gs_cnn_ppo_update(ptr(pm.params), ptr(agent.grads), ptr(agent.adam_m), ptr(agent.adam_v), pm.dims,
                                    hp, coll.buffer.view(), ptr(idx), B, K, 0, ptr(agent.metrics_buf),
                                    ptr(agent.stop_flag), ptr(agent.workspace), None, s.cuda_stream),
              "gs_cnn_ppo_update")

    with torch.cuda.stream(s):
        run()                       # warm: kernel attributes, code objects
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    restore()
    with torch.cuda.graph(g, stream=s):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(reps):
        for form in ("eager", "graph"):
            restore()
            with torch.cuda.stream(s):
                e0.record(s)
                if form == "eager":
                    run()
                else:
                    g.replay()
                e1.record(s)
            e1.synchronize()
            print(f"{'bf16' if bf else 'fp32'} {form} rep {r}: {e0.elapsed_time(e1) * 1e3 / K:.1f} us per minibatch "
                  f"({K} minibatches of {B})", flush=True)


if __name__ == "__main__":
    main()
