"""Where a bench step's time goes on the round loop's queue.

usage: python tools/gaps.py <rocprofv3 output dir> [loop kernel substring]

Reads run_kernel_trace.csv (+ run_memory_copy_trace.csv if present) of a
`rocprofv3 --kernel-trace [--memory-copy-trace]` run of bench.py, takes the
last step (from the last `k_round_init`-free window: the last group of
persistent-loop launches between two fame launches), and prints every
operation between the first and the last loop launch of that step on the
loop's queue, with the idle gaps between consecutive loop launches and what
the device ran in them.
"""
import csv
import os
import sys


def load(d):
    ops = []
    with open(os.path.join(d, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                        int(r["Queue_Id"])))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        with open(p) as f:
            for r in csv.DictReader(f):
                ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "memcpy " + r["Direction"][12:], -1))
    ops.sort()
    return ops


def main(d, loopk="k_round_lean"):
    ops = load(d)
    fame = [o for o in ops if "k_fame_masks" in o[2]]
    loops = [o for o in ops if loopk in o[2]]
    # the last step: loop launches after the second-to-last fame launch
    t_lo = fame[-2][1] if len(fame) >= 2 else 0
    step_loops = [o for o in loops if o[0] > t_lo]
    t0, t1 = step_loops[0][0], fame[-1][1]
    print(f"step window {(t1 - t0) / 1e6:.3f} ms from the first loop launch to the end of fame; "
          f"{len(step_loops)} loop launches, {sum(o[1] - o[0] for o in step_loops) / 1e6:.3f} ms of loop")
    gap_tot = 0
    for a, b in zip(step_loops, step_loops[1:]):
        g = b[0] - a[1]
        gap_tot += g
        inside = [o for o in ops if o[0] >= a[1] and o[1] <= b[0]]
        names = {}
        for o in inside:
            names[o[2]] = names.get(o[2], 0) + (o[1] - o[0])
        desc = ", ".join(f"{k} {v / 1e3:.0f}us" for k, v in sorted(names.items(), key=lambda x: -x[1])[:6])
        print(f"  loop {(a[1] - a[0]) / 1e6:7.3f} ms | gap {g / 1e3:7.1f} us: {desc}")
    print(f"gaps between loop launches: {gap_tot / 1e6:.3f} ms")
    tail = [o for o in ops if o[0] >= step_loops[-1][1] and o[1] <= t1]
    print(f"after the last loop launch: {(t1 - step_loops[-1][1]) / 1e6:.3f} ms")
    for o in tail:
        print(f"  {o[2]:40s} {(o[0] - step_loops[-1][1]) / 1e3:8.1f} us +{(o[1] - o[0]) / 1e3:7.1f} us")
    head = [o for o in ops if t_lo < o[0] < t0]
    print(f"before the first loop launch (after the previous step's fame): {(t0 - t_lo) / 1e6:.3f} ms")
    for o in head[-25:]:
        print(f"  {o[2]:40s} {(o[0] - t_lo) / 1e3:8.1f} us +{(o[1] - o[0]) / 1e3:7.1f} us q{o[3]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
