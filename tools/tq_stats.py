"""Spread of k_round_wide's per-candidate answers (BH_DIAG=1 BH_TIMELINE=file, chains 0..7,
rounds TL_R0 .. TL_R0 + 63): T_q = the first row of the chain's final window that strongly sees
candidate q.  Prints, per (round, chain), the spread of T_q over candidates, and over rounds the
change of a candidate's T_q offset from the previous round -- what a search started from a
prediction would have to cover -- and, per wave of 16 candidates (8 lane groups x 2 interleaved),
the largest error, since a wave executes its slowest lane group's probes."""
import sys

import numpy as np

TL_NR, NC = 64, 128


def main(path):
    a = np.fromfile(path, dtype=np.uint64)
    off = 32 + TL_NR * NC * 4 + 2 * TL_NR * 512 * 4 - 32  # DG_TQ - DG_TL
    blk = a[off: off + TL_NR * 8 * 66]
    if blk.size < TL_NR * 8 * 66:
        print("no T_q block")
        return
    w = blk.view(np.uint32).reshape(TL_NR, 8, 132)
    tq = w[:, :, :128].copy().view(np.uint8).reshape(TL_NR, 8, 512)
    hdr = w[:, :, 128:]
    n = int(hdr[:, :, 3].max())
    spreads, iqr, dprev, wave_err = [], [], [], []
    for c in range(8):
        prev = None
        for r in range(TL_NR):
            if hdr[r, c, 2] == 0:
                prev = None
                continue
            t = tq[r, c, :n].astype(np.int32)
            ok = t < 32
            if ok.sum() < 8:
                prev = None
                continue
            tt = t[ok]
            spreads.append(tt.max() - tt.min())
            iqr.append(np.percentile(tt, 75) - np.percentile(tt, 25))
            # absolute row offset from the chain's boundary
            absr = t + int(hdr[r, c, 0])
            if prev is not None:
                both = ok & prev[1]
                dd = absr[both] - prev[0][both]
                dprev.extend(dd.tolist())
                # per wave: 16 consecutive candidates (pass pairs of 32 per workgroup: candidates k*32 + t/8)
                med = int(np.median(dd)) if len(dd) else 0
                e = np.abs(absr - prev[0] - med)
                for w0 in range(0, n, 16):
                    m = both[w0:w0 + 16]
                    if m.any():
                        wave_err.append(int(e[w0:w0 + 16][m].max()))
            prev = (absr, ok)
    sp, iq = np.array(spreads), np.array(iqr)
    print(f"rounds x chains: {len(sp)}; T_q spread over candidates: median {np.median(sp):.0f} rows, IQR median {np.median(iq):.1f}")
    if dprev:
        d = np.array(dprev)
        print(f"T_q offset change from the previous round: median {np.median(d):.0f}, |dev from median| p50/p90 "
              f"{np.percentile(np.abs(d - np.median(d)), 50):.0f}/{np.percentile(np.abs(d - np.median(d)), 90):.0f} rows")
        we = np.array(wave_err)
        print(f"per 16-candidate wave, largest |error| of the previous-round prediction: p50 {np.median(we):.0f}, "
              f"p90 {np.percentile(we, 90):.0f} rows")


if __name__ == "__main__":
    main(sys.argv[1])
