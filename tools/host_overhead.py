"""Host time around bench.py's steps (C3 by default): how long the Python
side of a step and bh_reset_consensus hold the device idle between two
run_consensus calls.

usage: python tools/host_overhead.py [--cfg 3] [--steps 5]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from babble_amd import Hashgraph  # noqa: E402
from babble_amd.dag import CONFIGS, Dag  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    c = CONFIGS[a.cfg]
    dag = Dag.config(a.cfg, N=c["N"])
    hg = Hashgraph(dag.participant_ids, c["N"], device=0)
    hg.insert_dag(dag)
    hg.synchronize()
    hg.reset_consensus()
    hg.run_consensus()
    t_py, t_reset, t_run = [], [], []
    stage_tot = np.zeros(8)
    for _ in range(a.steps):
        t0 = time.perf_counter_ns()
        hg.reset_consensus()
        t1 = time.perf_counter_ns()
        hg.run_consensus()
        t2 = time.perf_counter_ns()
        hg.profile()
        stage_tot += np.array(hg.stage_ms())
        t3 = time.perf_counter_ns()
        t_reset.append(t1 - t0)
        t_run.append(t2 - t1)
        t_py.append(t3 - t2)
    us = lambda v: f"{np.median(v) / 1e3:.1f} us"  # noqa: E731
    print(f"reset_consensus {us(t_reset)}, run_consensus {np.median(t_run) / 1e6:.3f} ms, "
          f"bench bookkeeping {us(t_py)}")


if __name__ == "__main__":
    main()
