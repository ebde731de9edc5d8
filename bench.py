"""bench.py -- events ordered/sec of Babble's hashgraph consensus path on MI355X.

A step = one pass of the hot path over the resident DAG: coordinates
(initEventCoordinates), DivideRounds, DecideFame, DecideRoundReceived,
ProcessDecidedRounds (frame sort + blocks), all in libbabble_hip on one GPU.
The DAG (generation, hashing, signing, H2D copy) is prepared before the timed
region.  Workload: BASELINE.json's headline config C3 (128 participants,
10M-event random-gossip DAG).  Multi-GPU: one process per GPU, each orders
its own DAG (replicas, weak scaling; the reference has no sharded path and
the engine's passes need no exchange between independent DAGs).

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--cfg 3] [--events N]
       torchrun ... bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "events ordered/sec (rounds+fame+order), 128 peers 10M events, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def max_over_ranks(x, dist=None):
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, dist=None):
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(cfg, sample_events, log):
    """CPU restatement of the reference Go path (oracle/, 1 thread) on the
    first `sample_events` events of the same DAG (a valid DAG prefix)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import Oracle
    from babble_amd.dag import Dag
    d = Dag.config(cfg, N=sample_events, sig_mode=0)
    o = Oracle(d.n, d.participant_ids, capacity=sample_events)
    try:
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    except (AttributeError, OSError):
        pass
    t0 = time.perf_counter()
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    dt = time.perf_counter() - t0
    ordered = len(o.consensus_order())
    o.close()
    log(f"cpu baseline: {ordered} events ordered in {dt:.2f}s")
    return dict(value=ordered / dt, unit="events/s", cores=1, kind="port",
                sample=f"first {sample_events} events of the cfg{cfg} DAG (prefix), batch schedule "
                       f"(coordinates+DivideRounds+DecideFame+DecideRoundReceived+ProcessDecidedRounds), "
                       f"C restatement of hashgraph.go, 1 thread, {ordered} events ordered in {dt:.2f}s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--events", type=int, default=0, help="override DAG size")
    ap.add_argument("--sig", type=int, default=0, help="1 = deterministic ECDSA signatures")
    ap.add_argument("--cpu-sample", type=int, default=-1, help="events for the CPU baseline (0 = skip)")
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    def log(*a):
        if not args.quiet and rank == 0:
            print(*a, file=sys.stderr, flush=True)

    from babble_amd import Hashgraph
    from babble_amd.dag import CONFIGS, Dag
    c = CONFIGS[args.cfg]
    N = args.events or c["N"]
    t0 = time.perf_counter()
    dag = Dag.config(args.cfg, N=N, sig_mode=args.sig, rank=rank)
    log(f"generated cfg{args.cfg} n={c['n']} N={N} in {time.perf_counter() - t0:.1f}s")
    t0 = time.perf_counter()
    hg = Hashgraph(dag.participant_ids, N, device=local)
    st = hg.insert_dag(dag)
    assert not st.any(), "generator produced a rejected event"
    hg.synchronize()
    log(f"inserted (H2D) in {time.perf_counter() - t0:.1f}s")

    def barrier():
        if dist is not None:
            dist.barrier()

    def sync():
        hg.synchronize()
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        except ImportError:
            pass

    for w in range(args.warmup):
        hg.run_consensus()
        log(f"warmup {w}: stages_ms={['%.2f' % x for x in hg.stage_ms()]}")
    sweep_ms, stage_tot = [], np.zeros(5)
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hg.run_consensus()
        sweep_ms.append(hg.profile()[1])
        stage_tot += np.array(hg.stage_ms())
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, dist)
    stats = hg.stats()
    ordered = stats.consensus_events
    total_ordered = sum_over_ranks(ordered * args.steps, dist)
    iters, _ = hg.profile()
    value = total_ordered / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # roofline of the coordinate kernel (k_flow / k_la_sweep):
    # algorithmic bytes per event = 8*n (two parent LA rows) + 4*n (own row)
    # + 12 (LT of both parents + own); per launch x N events
    n = c["n"]
    sweep_avg_ms = float(np.mean(sweep_ms))
    alg_bytes = N * (12 * n + 12)
    achieved = alg_bytes / (sweep_avg_ms * 1e-3) / 1e9
    # HBM traffic of that kernel per launch, from the committed PMC passes
    # (tools/pmc.sh -> tools/pmc_summary.py -> profiles/pmc_traffic.json;
    # FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction)
    traffic = None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            tr = json.load(f).get(hg.profile_kernel(), {})
        if tr.get("participants") == n and tr.get("events") == N:
            traffic = tr["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
    # roofline of the round loop (the dominant kernel by total time at every
    # config: one launch per round).  Algorithmic bytes per launch: each of
    # the n workgroups streams every candidate's FD row (n x npad int32),
    # its chain's 32-row LA window and 32-row FD window (32 x npad int32
    # each), from L2/MALL; average launch duration = the rounds stage (HIP
    # events, graph replay) / iterations, launch gaps included
    npad = (n + 3) & ~3
    round_kernel = "k_round2" if npad <= 128 else "k_round"
    round_alg = n * (n * npad * 4 + 2 * 32 * npad * 4)
    rounds_ms = float(stage_tot[1] / args.steps)
    round_avg_ms = rounds_ms / max(iters, 1)
    round_achieved = round_alg / (round_avg_ms * 1e-3) / 1e9
    round_traffic = None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            tr = json.load(f).get(round_kernel, {})
        if tr.get("participants") == n and tr.get("events") == N:
            round_traffic = tr["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": f"cfg{args.cfg}: {n} participants, {N}-event random-gossip DAG "
                               f"(seed 0xBABB1E00+{args.cfg}), batch consensus: coordinates + "
                               f"DivideRounds + DecideFame + DecideRoundReceived + ProcessDecidedRounds",
                   "participants": n, "events": N, "events_ordered_per_step": ordered,
                   "rounds": stats.last_round + 1, "blocks": stats.blocks,
                   "parallelism": f"replicas x{world}" if world > 1 else "1 GPU"},
        "roofline": {"kernel": round_kernel, "bound": "hbm", "achieved": round_achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round_achieved / HBM_PEAK_GBS,
                     "traffic": round_traffic, "alg_bytes_per_launch": round_alg,
                     "avg_launch_ms": round_avg_ms, "launches": iters,
                     "note": "latency-bound per round (a serial chain of rounds); bytes come from L2/MALL"},
        "roofline_coordinates": {"kernel": hg.profile_kernel(), "bound": "hbm", "achieved": achieved,
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                                 "traffic": traffic, "alg_bytes_per_launch": alg_bytes,
                                 "avg_launch_ms": sweep_avg_ms,
                                 "note": "bound by the DAG's critical path x per-step issue, not bandwidth"},
        "stages_ms": dict(zip(["coordinates", "rounds", "fame", "round_received", "order"],
                              (stage_tot / args.steps).round(3).tolist())),
        "round_loop_iterations": iters,
    }
    cpu_sample = args.cpu_sample
    if cpu_sample < 0:
        cpu_sample = min(N, {1: 10_000, 2: 1_000_000, 3: 500_000, 4: 100_000, 5: 500_000}[args.cfg])
    if rank == 0 and world == 1 and cpu_sample > 0:
        out["cpu_baseline"] = cpu_baseline(args.cfg, cpu_sample, log)
        cv = out["cpu_baseline"]["value"]
        out["speedup_vs_cpu"] = value / cv if cv > 0 else None
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    hg.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
