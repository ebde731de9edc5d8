"""bench.py -- events ordered/sec of Babble's hashgraph consensus path on MI355X.

A step = one pass of the hot path over the resident DAG: coordinates
(initEventCoordinates), DivideRounds, DecideFame, DecideRoundReceived,
ProcessDecidedRounds (frame sort + blocks), all in libbabble_hip on one GPU.
The DAG (generation, hashing, signing, H2D copy) is prepared before the timed
region.  Workload: BASELINE.json's headline config C3 (128 participants,
10M-event random-gossip DAG).

Multi-GPU (one process per GPU):
  --mode shards (the default): the ranks order ONE DAG together (strong
      scaling; value = the DAG's events ordered per step / the slowest
      rank's time).  At n <= 128 (C3) from 3 ranks, ranks 1..N-1 run the coordinate
      dataflow over LA column ranges and all-gather every pipeline
      segment's columns (ncclBroadcast per coordinate rank over xGMI,
      16-bit packed); every rank runs the round loop on them, and the fame
      rounds and frame sorts are split between all ranks (bh_shard_range)
      and exchanged.  At 128 < n <= 512 (C4) from 4 ranks the coordinate
      ranks send their columns to rank 0, which runs the loop, fame and
      order.  Below that (C3 at 2 ranks: one link would carry the step's
      2.7 GB of columns in ~42 ms, longer than the step) every rank computes
      the coordinates and the loop, and the fame rounds and frame sorts are
      split.  One hashgraph's rounds
      are a serial chain (the round loop is ~95 % of a C3 step), so the
      expected curve is flat (DESIGN.md section 7's table);
  --mode replicas: every rank orders a DAG of its own (weak scaling, no
      data-path collective) -- N copies of the 1-GPU number, labelled so.

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--cfg 3] [--events N] [--mode replicas|shards]
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


def _pmc_table(n, N):
    """Per-kernel PMC HBM bytes of this config (tools/pmc.sh ->
    tools/pmc_summary.py -> profiles/pmc_traffic.json) and the commit they
    were measured at, or ({}, None).  bench.py cannot read PMC counters
    itself (rocprofv3 --pmc runs the program under the profiler), so the
    line names the table it quotes."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return {}, None
    cfg = tab.get(f"n{n}_N{N}", {})
    meta = (tab.get("_meta") or {}).get(f"n{n}_N{N}")
    ok = all(isinstance(v, dict) and "hbm_bytes_per_step" in v for v in cfg.values())
    return (cfg if ok else {}), meta


def _per_launch(pmc, kernel, launches):
    """a kernel's PMC HBM bytes per launch of THIS run: the table's bytes per
    step over this run's launches per step (BH_SEGMENTS changes the launch
    count, not the step's bytes)"""
    v = pmc.get(kernel)
    return v["hbm_bytes_per_step"] / launches if v and launches else None


def _shard_mode(n, world):
    """the engine's shard mode (BH_SHARD_COORDS; api.cpp shard_mode)"""
    e = os.environ.get("BH_SHARD_COORDS")
    if e in ("columns", "replicate", "split"):
        return e
    return "split" if (n <= 128 and world >= 3) or (n <= 512 and world >= 4) else "replicate"


def _parallelism(world, n, one_dev=False):
    mode = _shard_mode(n, world)
    xp = "host transport over gloo, all ranks on device 0" if one_dev else None
    if mode == "split" and n <= 128:
        return (f"{world} shards ({xp or 'RCCL broadcast over xGMI'}): ranks 1..{world - 1} run the coordinate "
                f"dataflow over LA column ranges and all-gather every segment's columns (16-bit packed); every "
                f"rank runs the round loop; fame rounds and frame sorts split over all {world} ranks")
    if mode == "split":
        return (f"{world} shards ({xp or 'RCCL send/recv over xGMI'}): rank 0 runs the round loop, fame and "
                f"order; ranks 1..{world - 1} run the coordinate dataflow over LA column ranges and ship every "
                f"segment's columns to rank 0 (16-bit packed)")
    if mode == "columns":
        return (f"{world} shards ({xp or 'RCCL broadcast'}): LA columns, fame rounds and frame sorts split, "
                f"round loop replicated")
    return (f"{world} shards ({xp or 'RCCL broadcast'}): fame rounds + frame sorts split, coordinates and "
            f"round loop replicated")


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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
    out = dict(value=ordered / dt, unit="events/s", cores=1, kind="port", cpu_model=_cpu_model(),
               nproc=os.cpu_count(), threads_used=1, host="this bench box (rank 0's host cores)",
               sample=f"first {sample_events} events of the cfg{cfg} DAG (prefix), batch schedule "
                      f"(coordinates+DivideRounds+DecideFame+DecideRoundReceived+ProcessDecidedRounds), "
                      f"C restatement of hashgraph.go, 1 thread, {ordered} events ordered in {dt:.2f}s")
    # the same oracle over the WHOLE DAG, from the run that made the committed
    # digests (tests/golden/make_whole_digests.py) -- not timed here (minutes
    # to an hour); its per-event cost grows with the DAG, so the prefix rate
    # above flatters the CPU
    try:
        with open(os.path.join(ROOT, "tests", "golden", f"whole_c{cfg}.json")) as f:
            w = json.load(f)
        o = w["oracle"]
        sec = o["insert_s"] + o["consensus_s"]
        out["whole_dag"] = dict(
            value=w["n_ordered"] / sec, unit="events/s", threads=o.get("threads", 1), events=w["events"],
            ordered=w["n_ordered"], seconds=sec,
            host="the build container (Intel Xeon Processor, 8 vCPU), not the bench box",
            source=f"tests/golden/whole_c{cfg}.json: oracle ({o['lib']}), insert {o['insert_s']} s + "
                   f"consensus {o['consensus_s']} s")
        out["prefix_over_whole"] = out["value"] / out["whole_dag"]["value"]
    except (OSError, ValueError, KeyError):
        pass
    return out


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
    ap.add_argument("--mode", choices=("shards", "replicas"), default="shards",
                    help="N>1: shard one DAG over the ranks (strong, the default) or order one DAG per rank (weak)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # BH_BENCH_ONE_DEVICE=1: every rank on device 0, the barrier (and the
    # shards' exchange) over gloo -- rehearses the multi-process paths on a
    # one-GPU box
    one_dev = os.environ.get("BH_BENCH_ONE_DEVICE") == "1"
    if one_dev:
        local = 0
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if one_dev else "nccl")

    def log(*a):
        if not args.quiet and rank == 0:
            print(*a, file=sys.stderr, flush=True)

    from babble_amd import Hashgraph, comm_unique_id
    from babble_amd.dag import CONFIGS, Dag
    c = CONFIGS[args.cfg]
    N = args.events or c["N"]
    sharded = world > 1 and args.mode == "shards"
    t0 = time.perf_counter()
    dag = Dag.config(args.cfg, N=N, sig_mode=args.sig, rank=0 if sharded else rank)
    log(f"generated cfg{args.cfg} n={c['n']} N={N} in {time.perf_counter() - t0:.1f}s")
    t0 = time.perf_counter()
    hg = Hashgraph(dag.participant_ids, N, device=local)
    if sharded and one_dev:
        # RCCL refuses two ranks on one device: the engine's host transport
        # over the gloo group carries the same exchanges (bh_comm_init_transport)
        import torch

        def tb(b):
            return torch.frombuffer(b, dtype=torch.uint8)
        hg.comm_init_transport(rank, world, lambda b, p: dist.send(tb(b), dst=p),
                               lambda b, p: dist.recv(tb(b), src=p), lambda b, r: dist.broadcast(tb(b), src=r))
    elif sharded:  # one RCCL communicator of the engine's own, id from rank 0
        obj = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        hg.comm_init(rank, world, obj[0])
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

    # a step = one consensus pass over the whole resident DAG: the engine keeps
    # its results between calls (a call only processes what was inserted
    # since), so every step starts from reset_consensus -- the state of a
    # Hashgraph that has just had the DAG inserted (BenchmarkConsensus)
    for w in range(args.warmup):
        hg.reset_consensus()
        hg.run_consensus()
        log(f"warmup {w}: stages_ms={['%.2f' % x for x in hg.stage_ms()]}")
    persist0 = hg.loop_stats()[0]
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hg.reset_consensus()
        hg.run_consensus()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, dist)
    persist_per_step = (hg.loop_stats()[0] - persist0) / args.steps  # persistent loop launches (one per segment)
    if sharded and rank > 0 and _shard_mode(c["n"], world) == "split" and c["n"] > 128:
        # a coordinate rank of the wide split holds no consensus results (the
        # engine refuses the query); rank 0 reports the step
        hg.close()
        dist.destroy_process_group()
        return
    # the device timings of the last step's stages and kernels (HIP events
    # recorded inside the timed region, read after it: reading them between
    # steps would hold the device idle)
    stage_last = np.array(hg.stage_ms())
    coord_ms = float(hg.profile()[1])
    stats = hg.stats()
    ordered = stats.consensus_events
    # whole-job events ordered: one DAG per step when sharded, one per rank per step as replicas
    total_ordered = ordered * args.steps if (sharded or world == 1) else sum_over_ranks(ordered * args.steps, dist)
    iters, _ = hg.profile()
    value = total_ordered / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    n = c["n"]
    npad = (n + 3) & ~3
    stages = dict(zip(["coordinates", "rounds", "fame", "round_received", "order", "exchange"],
                      stage_last.round(3).tolist()))
    pmc, pmc_meta = _pmc_table(n, N)
    # the table holds THIS build's kernels only if it names the coordinate
    # kernel this run timed (a table of an older build reads as no table)
    if pmc and hg.profile_kernel() not in pmc:
        pmc, pmc_meta = {}, None
    # roofline: the path is integer and
    # HBM-bound; algorithmic bytes per ordered event B(n) = 12n + 96 (two
    # parent LA rows read, own row written, per-event scalars, sort key and
    # value, signature tie-break) against the 8 TB/s HBM peak
    B = 12 * n + 96
    achieved = value * B / 1e9
    traffic_step = sum(v["hbm_bytes_per_step"] for v in pmc.values()) if pmc else None
    traffic_source = ("profiles/pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (FETCH_SIZE x 2 + "
                      f"WRITE_SIZE) of this config, measured at commit {pmc_meta.get('commit') if pmc_meta else '?'}"
                      if pmc else "none: profiles/pmc_traffic.json holds no table of this build's kernels for "
                                  "this config")
    # the round loop, timed live by HIP events around each launch on the
    # loop's stream (stage 7).  Persistent (the default): n <= 128
    # k_round_lean (k_round2p with BH_ROUND_F32=0), one launch per pipeline
    # segment running all of that segment's rounds; n <= 512
    # k_round_wide<..., true>, one launch per call.  Otherwise one k_round2 /
    # k_round_wide launch per round
    persistent = persist_per_step > 0
    if npad <= 128:
        lean = os.environ.get("BH_ROUND_F32", "1") != "0"
        round_kernel = ("k_round_lean" if lean else "k_round2p") if persistent else "k_round2"
    else:
        round_kernel = "k_round_wide"
    segments = hg.pipeline()[0]
    loop_ms = float(stage_last[7]) if len(stage_last) > 7 else 0.0
    if loop_ms <= 0:  # (BH_LOOP_TIMING=0: the rounds stage instead)
        loop_ms = float(stage_last[1])
    iter_us = 1000.0 * loop_ms / max(iters, 1)
    loop_launches = persist_per_step if persistent else iters
    # B(n) split between the two kernels, so that their fractions add up to
    # the whole step's: the coordinate kernel is charged 12n + 12 B per
    # inserted event (two parent LA rows read, its own row and LT written),
    # the loop the remainder of the step's B(n) x ordered events -- the
    # per-event scalars, sort key and value, signature tie-break (84 B per
    # event at any n), which the loop's rounds decide.  What the loop READS
    # (window rows, candidates' rows, from L2 / MALL) is not algorithmic: its
    # PMC traffic is quoted beside it
    coord_alg = N * (12 * n + 12)
    loop_alg = max(ordered * B - coord_alg, 0)
    loop_obj = {"kernel": round_kernel, "launches_per_step": loop_launches, "device_ms_per_step": loop_ms,
                "avg_launch_ms": loop_ms / max(loop_launches, 1e-9),
                "alg_bytes_per_launch": loop_alg / max(loop_launches, 1e-9),
                "achieved": loop_alg / (loop_ms * 1e-3) / 1e9, "frac": loop_alg / (loop_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "alg_bytes_per_event": (loop_alg / ordered) if ordered else None,
                "round_iterations": iters, "us_per_iteration": iter_us,
                "traffic_per_launch": _per_launch(pmc, round_kernel, loop_launches),
                "note": "latency-bound: the rounds are a serial chain; one persistent launch per pipeline "
                        "segment (k_round_lean: workgroups hand each other the candidates' rows as data-tagged "
                        "dwords) or per call (k_round_wide: a grid barrier per round)"}
    # the coordinate kernel: the sum of its launches per step (one per
    # segment; k_flow32x2 carries LT inside them), HIP events on the
    # coordinate stream around each launch
    coord_launches = segments if hg.profile_kernel() in ("k_flow32x2", "k_flow32", "k_floww2", "k_floww") else 1
    coord_obj = {"kernel": hg.profile_kernel(), "launches_per_step": coord_launches, "device_ms_per_step": coord_ms,
                 "avg_launch_ms": coord_ms / max(coord_launches, 1),
                 "alg_bytes_per_launch": coord_alg / max(coord_launches, 1),
                 "alg_bytes_per_event": 12 * n + 12,
                 # (shards: rank 0 runs no dataflow -- its coordinate time is the exchange)
                 "achieved": coord_alg / (coord_ms * 1e-3) / 1e9 if coord_ms > 0 else None,
                 "frac": coord_alg / (coord_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if coord_ms > 0 else None,
                 "traffic_per_launch": _per_launch(pmc, hg.profile_kernel(), coord_launches),
                 "note": "LA columns and Lamport timestamps (12n + 12 B per event); bound by the DAG's critical "
                         "path x per-step issue, not bandwidth"}
    # the dominant kernel: the larger device-time share of the step
    dom = loop_obj if loop_ms >= coord_ms else coord_obj
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.mode == "shards" else "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": f"cfg{args.cfg}: {n} participants, {N}-event random-gossip DAG "
                               f"(seed 0xBABB1E00+{args.cfg}), batch consensus: coordinates + "
                               f"DivideRounds + DecideFame + DecideRoundReceived + ProcessDecidedRounds",
                   "participants": n, "events": N, "events_ordered_per_step": ordered,
                   "rounds": stats.last_round + 1, "blocks": stats.blocks,
                   "parallelism": _parallelism(world, n, one_dev) if sharded else
                                  (f"replicas x{world}" + (" on device 0" if one_dev else "") if world > 1
                                   else "1 GPU")},
        # the dominant kernel's roofline (per launch), then the whole step's
        "roofline": {"bound": "hbm", "kernel": dom["kernel"], "achieved": dom["achieved"], "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": dom["frac"], "traffic": dom["traffic_per_launch"],
                     "alg_bytes_per_launch": dom["alg_bytes_per_launch"], "avg_launch_ms": dom["avg_launch_ms"],
                     "chosen_by": f"device time per step: loop {loop_ms:.2f} ms, coordinates {coord_ms:.2f} ms",
                     "traffic_source": traffic_source,
                     "whole_step": {"achieved": achieved, "frac": achieved / HBM_PEAK_GBS,
                                    "alg_bytes_per_event": B, "alg_bytes_per_step": ordered * B,
                                    "traffic": traffic_step,
                                    "scope": "events ordered/s x B(n), SURVEY 8(d)"},
                     "loop": loop_obj, "coordinates": coord_obj},
        "stages_ms": stages,
        "round_loop_iterations": iters,
        "pipeline": {"segments": segments, "incremental_calls": hg.pipeline()[1]},
    }
    cpu_sample = args.cpu_sample
    if cpu_sample < 0:
        cpu_sample = min(N, {1: 10_000, 2: 1_000_000, 3: 500_000, 4: 100_000, 5: 500_000}[args.cfg])
    if rank == 0 and world == 1 and cpu_sample > 0:
        out["cpu_baseline"] = cpu_baseline(args.cfg, cpu_sample, log)
        cv = out["cpu_baseline"]["value"]
        out["speedup_vs_cpu"] = value / cv if cv > 0 else None  # (against the prefix rate)
        wd = out["cpu_baseline"].get("whole_dag")
        if wd:
            out["speedup_vs_cpu_whole_dag"] = value / wd["value"]
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    hg.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
