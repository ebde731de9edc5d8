"""Summarise tools/pmc.sh's SQ pass (p2) into profiles/pmc_sq.json.

Per kernel (summed over its dispatches of one bench step): the raw SQ
counters, and the ratios the north star asks for as evidence:
  lds_conflict_per_inst = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS  (cycles a
      wave's LDS instruction waited on bank conflicts, per LDS instruction)
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (waves parked on waitcnt / barrier)
  active_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (waves issuing)
  valu_per_wave = SQ_INSTS_VALU / SQ_WAVES
Entries are keyed by config ("n<participants>_N<events>").
usage: python tools/pmc_sq_summary.py gpurun_out/pmc_c3 <participants> <events>
"""
import collections
import csv
import json
import os
import sys


def main():
    d, n, N = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(d, "p2", "run_counter_collection.csv"))):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bh::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    tab = {}
    for k in sorted(acc):
        c = dict(acc[k])
        e = {"dispatches": len(disp[k]), **c}
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if c.get("SQ_INSTS_LDS"):
            e["lds_conflict_per_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_INSTS_LDS"]
        if wc:
            e["wait_frac"] = c.get("SQ_WAIT_ANY", 0.0) / wc
            e["active_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
        if c.get("SQ_WAVES"):
            e["valu_per_wave"] = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_WAVES"]
        tab[k] = e
        print(k, {x: round(y, 3) for x, y in e.items() if isinstance(y, float) and x.endswith(("inst", "frac", "wave"))})
    out_path = os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_sq.json")
    try:
        out = json.load(open(out_path))
    except (OSError, ValueError):
        out = {}
    out[f"n{n}_N{N}"] = {"source": f"rocprofv3 --pmc (tools/pmc.sh pass 2), {os.path.basename(d.rstrip('/'))}",
                         "kernels": tab}
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
