"""One rank of a multi-process search on a real HIP engine (started by
test_distributed_search_real_engine_two_ranks as a fresh child process per rank).

    python dist_rank_worker.py RANK WORLD PORT WORKLOAD OUT.json [BATCH] [SEED_UNITS]

The ranks share cuda:0 and talk over gloo (CPU tensors only: units are staged through host
memory by distributed_search); rank 0 writes the result.  This is the code path of
`bench.py --gpus N`: quorum_intersection_amd.distributed.distributed_search over
DeviceSearch (C-ABI qi_search_*).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def workload_text(name):
    from quorum_intersection_amd import fbas_gen
    if name.startswith("two_tier_"):
        _, _, k, n = name.split("_")
        return fbas_gen.two_tier(int(k), int(n))
    if name.startswith("planted_deep_"):
        _, _, k, n = name.split("_")
        return fbas_gen.planted_deep(int(k), int(n))
    if name.startswith("tiered_"):
        return fbas_gen.tiered(int(name.split("_")[1]))
    raise SystemExit(f"unknown workload {name}")


def main():
    rank, world, port, name, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    batch = int(sys.argv[6]) if len(sys.argv) > 6 else 64
    seed_units = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import quorum_intersection_amd as qa
    from quorum_intersection_amd.distributed import DeviceSearch, SharedBest, distributed_search

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    fb = qa.FBAS(workload_text(name), device=0)
    be = DeviceSearch(fb, jit=2, batch=batch)
    shared = SharedBest.for_group(tag=port)  # the ranks' shared best key, as bench.py --gpus N sets it up
    be.share_best(shared)
    print(f"rank {rank}: engine ready, {name}", flush=True)
    r = distributed_search(be, device=torch.device("cpu"), seed_units=seed_units, shared=shared)
    print(f"rank {rank}: shared best word {shared.value:#x}", flush=True)
    be.share_best(None)
    print(f"rank {rank}: nodes {r.nodes} moved {r.moved_units}", flush=True)
    if rank == 0:
        with open(out, "w") as fh:
            json.dump({"verdict": r.verdict, "nodes": r.nodes, "evals": r.evals, "minq": r.minq, "q1": r.q1, "q2": r.q2,
                       "launches": r.launches, "moved_units": r.moved_units, "world": world}, fh)
    dist.barrier()
    shared.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
