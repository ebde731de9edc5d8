"""Summarise tools/pmc.sh counter passes into profiles/pmc_traffic.json.

HBM bytes of each kernel = FETCH_SIZE x 2 (gfx950 reports half the bytes of
wide coalesced reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, both in
KiB per dispatch as rocprofv3 reports them (summed over XCDs).  The profiled
command runs exactly one bench step (--steps 1 --warmup 0), so the sum over
a kernel's dispatches is its bytes per step.  Entries are keyed by config
("n<participants>_N<events>").
usage: python tools/pmc_summary.py gpurun_out/pmc_c3 <participants> <events>
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    by_kernel = collections.defaultdict(list)
    for dsp, v in acc.items():
        by_kernel[names[dsp].split("(")[0].split("<")[0].replace("void ", "").replace("bh::", "")].append(v)
    return by_kernel


def main():
    d, n, N = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    fetch = per_kernel(os.path.join(d, "p0", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "p1", "run_counter_collection.csv"), "WRITE_SIZE")
    out_path = os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    try:
        out = json.load(open(out_path))
    except (OSError, ValueError):
        out = {}
    key = f"n{n}_N{N}"
    tab = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        launches = max(len(f), len(w))
        fb, wb = sum(f) * 1024 * 2, sum(w) * 1024
        tab[k] = {"launches": launches, "fetch_bytes_corrected": fb, "write_bytes": wb,
                  "hbm_bytes_per_step": fb + wb, "hbm_bytes_per_launch": (fb + wb) / max(launches, 1),
                  "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, {os.path.basename(d.rstrip('/'))}"}
        print(k, tab[k])
    out[key] = tab
    # the build the counters were collected on (bench.py quotes it)
    import subprocess
    try:
        rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                             cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip()
    except OSError:
        rev = "?"
    out.setdefault("_meta", {})[key] = {"commit": rev, "dir": os.path.basename(d.rstrip("/")),
                                        "kernels": sorted(tab)}
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
