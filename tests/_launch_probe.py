"""Rank body for tests/test_bench_launcher_cpu.py: started by bench.launch_ranks with the
same argv bench.py would get; joins a gloo group from the launcher's environment, checks
rank/world against a sum over ranks, and (rank 0) prints one JSON line like bench.py."""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--fail-rank", type=int, default=-1)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if rank == args.fail_rank:
        sys.exit(3)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    line = {"rank": rank, "world": world, "gpus": args.gpus, "local_rank": int(os.environ["LOCAL_RANK"]),
            "master": f"{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}", "sum": float(t.item()),
            "steps": args.steps}
    if rank == 0:
        print(json.dumps(line), flush=True)
    else:
        os.write(2, (json.dumps(line) + "\n").encode())   # one write: ranks share stderr
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
