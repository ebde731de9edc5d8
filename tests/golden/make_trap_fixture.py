"""Writes tests/golden/trap_schedule.json: a seeded lagging-peer gossip DAG
(the repo's own deterministic generator, babble_amd/csrc/dag_gen.c) on which
the live node's schedule -- RunConsensus after every `step` inserted events
(node.go:583-603) -- diverges from one batch run through the RoundInfo.queued
trap (hashgraph.go:809-815, roundInfo.go:35).

The expected values come from the CPU oracle (oracle/hg_oracle.c), which
restates DivideRounds' queueing, updatePendingRounds' sticky flags and
DecideRoundReceived's WitnessesDecided break literally.  The reference holds
no fixture for this case (its tests run one schedule per DAG), so the
values are pinned by that restatement.  Run from the repo root:
    python tests/golden/make_trap_fixture.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle_py import UNSET, Oracle  # noqa: E402
from babble_amd.dag import Dag  # noqa: E402

P = dict(n=7, N=3000, seed=1028, lagging=2, lag_div=60, step=5)


def main():
    d = Dag(P["n"], P["N"], P["seed"], lagging=P["lagging"], lag_div=P["lag_div"], sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    b = Oracle(P["n"], d.participant_ids, capacity=P["N"])
    b.insert_dag(*args)
    b.run_consensus()
    o = Oracle(P["n"], d.participant_ids, capacity=P["N"])
    for lo in range(0, P["N"], P["step"]):
        o.insert_dag(*(a[lo:lo + P["step"]] for a in args))
        o.run_consensus()
    rb, ro = b.results(), o.results()
    fame_diff = np.nonzero(rb["fame"] != ro["fame"])[0]
    rr_diff = np.nonzero(rb["round_received"] != ro["round_received"])[0]
    assert len(fame_diff) == 1 and ro["fame"][fame_diff[0]] == 0, "no trapped witness"

    def rr(v):
        return None if v == UNSET else int(v)
    fx = dict(P)
    fx["trapped_witness"] = int(fame_diff[0])
    fx["per_sync"] = dict(fame={str(e): int(ro["fame"][e]) for e in fame_diff},
                          round_received={str(e): rr(ro["round_received"][e]) for e in rr_diff},
                          consensus_events=int(len(o.consensus_order())))
    fx["batch"] = dict(fame={str(e): int(rb["fame"][e]) for e in fame_diff},
                       round_received={str(e): rr(rb["round_received"][e]) for e in rr_diff},
                       consensus_events=int(len(b.consensus_order())))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "trap_schedule.json")
    with open(out, "w") as f:
        json.dump(fx, f, indent=1)
    print(json.dumps(fx))


if __name__ == "__main__":
    main()
