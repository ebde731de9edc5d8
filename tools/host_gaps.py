"""Device idle time between a bench step's last round loop and the next
step's first, with the host's HIP calls beside the device operations.

usage: python tools/host_gaps.py <rocprofv3 dir> [step]
(the dir of `rocprofv3 --kernel-trace --hip-runtime-trace
--memory-copy-trace --output-format csv -d DIR -o run -- python3 bench.py
--cfg 3 --steps 3 --warmup 1 --cpu-sample 0`; step 2 by default: the
loop launches of the timed steps are 16 per step, the warmup's first)
"""
import csv
import os
import sys


def rows(path, f):
    p = os.path.join(path, f)
    return list(csv.DictReader(open(p))) if os.path.exists(p) else []


def main(d, step=2, per_step=16):
    dev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"].split("(")[0][-30:])
           for r in rows(d, "run_kernel_trace.csv")]
    dev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M " + r["Direction"])
            for r in rows(d, "run_memory_copy_trace.csv")]
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "    " + r["Function"])
           for r in rows(d, "run_hip_api_trace.csv")]
    dev.sort()
    loops = [o for o in dev if "round_lean" in o[2] or "round2p" in o[2]]
    a, b = loops[(step + 1) * per_step - 1], loops[(step + 1) * per_step]
    lo = a[1]
    busy, idle = lo, 0
    for o in dev:
        if lo <= o[0] <= b[0]:
            idle += max(0, o[0] - busy)
            busy = max(busy, o[1])
    print(f"from the last loop's end to the next step's first loop: {(b[0] - lo) / 1e3:.1f} us, "
          f"device idle {idle / 1e3:.1f} us")
    for e in sorted(o for o in dev + api if lo <= o[0] <= b[0]):
        print(f"{(e[0] - lo) / 1e3:9.1f} +{(e[1] - e[0]) / 1e3:7.1f} {e[2]}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
