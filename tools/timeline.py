"""Summarise the round loop's realtime stamps (BH_DIAG=1 BH_TIMELINE=file).

Per round r (TL_R0 .. TL_R0 + TL_NR) and chain c the kernel stores four
s_memrealtime stamps (100 MHz): workgroup start (low 52 bits), search end,
hand-off barrier, workgroup end.  Prints medians over rounds of
  launch spread  (last start - first start of the round's workgroups),
  loads          (first barrier - start, per workgroup),
  search         (search end - first barrier),
  hand-off       (end - search end),
  round span     (last end - first start),
  boundary       (first start of round r+1 - last end of round r).
"""
import sys

import numpy as np

TL_NR, NC = 64, 128


def main(path):
    a = np.fromfile(path, dtype=np.uint64)[: TL_NR * NC * 4].reshape(TL_NR, NC, 4)
    start = (a[:, :, 0] & ((1 << 52) - 1)).astype(np.int64)
    srch, end = a[:, :, 1].astype(np.int64), a[:, :, 3].astype(np.int64)
    ld = a[:, :, 2].astype(np.int64)
    live = (start > 0) & (end > 0)
    rows = []
    for r in range(TL_NR):
        m = live[r]
        if m.sum() < 2:
            continue
        s, e, q = start[r, m], end[r, m], srch[r, m]
        nxt = None
        if r + 1 < TL_NR and live[r + 1].sum() > 1:
            nxt = start[r + 1, live[r + 1]].min() - e.max()
        l = ld[r, m]
        rows.append((s.max() - s.min(), np.median(l - s), np.median(q - l), np.median(e - q), e.max() - s.min(), nxt))
    if not rows:
        print("no stamps")
        return
    ns = 10.0  # s_memrealtime ticks at 100 MHz
    cols = ["launch spread", "loads", "search", "hand-off", "round span", "boundary"]
    for i, name in enumerate(cols):
        v = [x[i] for x in rows if x[i] is not None]
        print(f"{name:14s} median {np.median(v) * ns / 1000:6.2f} us  p90 {np.percentile(v, 90) * ns / 1000:6.2f} us")
    per_round = np.diff(np.array([start[r, live[r]].min() for r in range(TL_NR) if live[r].sum() > 1]))
    print(f"{'round period':14s} median {np.median(per_round) * ns / 1000:6.2f} us")
    barrier(path)


def tagged(path):
    """k_round2p's data-tagged hand-over (round 5; BH_DIAG=1 BH_TIMELINE=file):
    per round r and chain c, the second block holds (waiting starts, inputs
    current, polls, rows stored).  Prints medians over rounds of: the hop
    (the last producer's store of round r - 1 -> each consumer's inputs
    current: first, median, last), the wait per workgroup, the work
    (current -> stored), the store spread, polls per workgroup and the round
    period (first current to first current)."""
    b = np.fromfile(path, dtype=np.uint64)
    off = TL_NR * NC * 4
    b = b[off: off + TL_NR * 512 * 4].reshape(TL_NR, 512, 4).astype(np.int64)[:, :NC]
    flags = (b[:, :, 0] >> 60) & 0xF  # (k_round_lean: a wave took the bounded hand-off count)
    b[:, :, 0] &= (1 << 60) - 1
    live = (b[:, :, 1] > 0) & (b[:, :, 3] > 0)
    rows, lastc = [], []
    for r in range(1, TL_NR):
        m, mp = live[r], live[r - 1]
        if m.sum() < 2 or mp.sum() < 2:
            continue
        last_store = b[r - 1, mp, 3].max()
        cur = b[r, m, 1]
        rows.append((cur.min() - last_store, np.median(cur - last_store), cur.max() - last_store,
                     np.median(b[r, m, 1] - b[r, m, 0]), np.median(b[r, m, 3] - b[r, m, 1]),
                     b[r, m, 3].max() - b[r, m, 3].min(), np.median(b[r, m, 2] & 0xFFFFFFFF),
                     cur.min() - b[r - 1, mp, 1].min()))
        # k_round_lean: the last consumer's own path -- its store of round r - 1
        # -> its iteration start -> own stores acknowledged -> inputs current
        ack = b[r, :, 2] >> 32
        w = int(np.flatnonzero(m)[np.argmax(cur)])
        if ack[w] > 0 and mp[w]:
            lastc.append((b[r, w, 0] - b[r - 1, w, 3], ack[w], b[r, w, 1] - b[r, w, 0] - ack[w],
                          int(w == int(np.flatnonzero(mp)[np.argmax(b[r - 1, mp, 3])]))))
    if not rows:
        print("no tagged stamps")
        return
    ns = 10.0
    names = ["hop first", "hop median", "hop last", "wait", "work", "store spread", "polls", "round period"]
    for i, name in enumerate(names):
        v = [x[i] for x in rows]
        scale = 1.0 if name == "polls" else ns / 1000
        unit = "" if name == "polls" else " us"
        print(f"{name:14s} median {np.median(v) * scale:6.2f}{unit}  p90 {np.percentile(v, 90) * scale:6.2f}{unit}")
    if lastc:
        for i, name in enumerate(["last: store->it", "last: own ack", "last: ack->cur"]):
            v = [x[i] for x in lastc]
            print(f"{name:14s} median {np.median(v) * ns / 1000:6.2f} us  p90 {np.percentile(v, 90) * ns / 1000:6.2f} us")
        print(f"{'last = last st':14s} {np.mean([x[3] for x in lastc]):6.2f}  (share of rounds whose last consumer stored last)")
    if flags.any():
        print(f"{'bounded count':14s} {np.mean(flags[live] & 1):6.3f}  (share of workgroup-rounds)")
        print(f"{'hand-off miss':14s} {np.mean((flags[live] >> 1) & 1):6.3f}  (share of workgroup-rounds: an entry past the 64 loaded rows)")
        for r in range(1, TL_NR):
            pass
        # rounds whose latest row had a miss / bounded count
        lat = [(flags[r, live[r]][np.argmax(b[r, live[r], 3])]) for r in range(TL_NR) if live[r].sum() > 1]
        print(f"{'latest row flg':14s} miss {np.mean([(x >> 1) & 1 for x in lat]):6.3f}  bounded {np.mean([x & 1 for x in lat]):6.3f}  (the round's last-completed row)")
    # the work's two phases from the first block (k_round2p: inputs current,
    # search done, window staged, rows stored): search, then the hand-off
    # (the new candidate's FD entries counted, its rows stored)
    a = np.fromfile(path, dtype=np.uint64)[: TL_NR * NC * 4].reshape(TL_NR, NC, 4).astype(np.int64)
    ok = (a > 0).all(axis=2)
    for name, v in (("search", (a[:, :, 1] - a[:, :, 0])[ok]), ("hand-off", (a[:, :, 3] - a[:, :, 1])[ok])):
        print(f"{name:14s} median {np.median(v) * ns / 1000:6.2f} us  p90 {np.percentile(v, 90) * ns / 1000:6.2f} us")
    # the search's phases (third block): wave 0's probes, the other waves'
    # (to the histogram barrier), the scan (to the search's end), probe count
    raw = np.fromfile(path, dtype=np.uint64)
    off3 = TL_NR * NC * 4 + TL_NR * 512 * 4
    if raw.size >= off3 + TL_NR * 512 * 4:
        g = raw[off3: off3 + TL_NR * 512 * 4].reshape(TL_NR, 512, 4).astype(np.int64)[:, :NC]
        m = ok & (g[:, :, 0] > 0) & (g[:, :, 1] > 0)
        if m.any():
            for name, v in (("probes (w0)", (g[:, :, 0] - a[:, :, 0])[m]), ("other waves", (g[:, :, 1] - g[:, :, 0])[m]),
                            ("scan", (g[:, :, 3] - g[:, :, 1])[m])):
                print(f"{name:14s} median {np.median(v) * ns / 1000:6.2f} us  p90 {np.percentile(v, 90) * ns / 1000:6.2f} us")
            pc = g[:, :, 2][m] & 0xFFFFFFFF
            spread = (g[:, :, 2][m] >> 32).astype(np.int64)
            if (pc & 0x80000000).all():  # k_round_lean: the last wave's probes done (from wave 0's inputs current)
                v = pc & 0x7FFFFFFF
                print(f"{'last probes':14s} median {np.median(v) * ns / 1000:6.2f} us  p90 {np.percentile(v, 90) * ns / 1000:6.2f} us  (last wave's probes done - wave 0's inputs current)")
                # (ts[3]: the last wave's hand-off start; tl[3]: every wave stored)
                hs = (g[:, :, 3] - a[:, :, 0])[m]
                hst = (a[:, :, 3] - g[:, :, 3])[m]
                print(f"{'last hand st':14s} median {np.median(hs) * ns / 1000:6.2f} us  p90 {np.percentile(hs, 90) * ns / 1000:6.2f} us  (last wave's hand-off start - wave 0's inputs current)")
                print(f"{'hand st->row':14s} median {np.median(hst) * ns / 1000:6.2f} us  p90 {np.percentile(hst, 90) * ns / 1000:6.2f} us  (-> every wave stored)")
            else:
                print(f"{'probe count':14s} median {np.median(pc):6.1f}     p90 {np.percentile(pc, 90):6.1f}")
            if spread.any():
                print(f"{'waves current':14s} median {np.median(spread) * ns / 1000:6.2f} us  p90 {np.percentile(spread, 90) * ns / 1000:6.2f} us  (last wave's inputs current - wave 0's)")


def barrier(path):
    """The persistent loops' barrier phases (second block, every chain): per
    round, drain (arrived - end), stage (staged - arrived; k_round2p: its
    loads issued), end spread, last arrival -> first release (the barrier's
    own latency), release spread, and last staged - first release (> 0: the
    next round waits on staging, not on the barrier)."""
    b = np.fromfile(path, dtype=np.uint64)
    off = TL_NR * NC * 4
    if b.size < off + TL_NR * 512 * 4:
        return
    b = b[off: off + TL_NR * 512 * 4].reshape(TL_NR, 512, 4).astype(np.int64)
    live = (b > 0).all(axis=2)
    rows = []
    for r in range(TL_NR):
        m = live[r]
        if m.sum() < 2:
            continue
        e, a, s, rl = (b[r, m, k] for k in range(4))
        rows.append((np.median(a - e), np.median(s - a), e.max() - e.min(), rl.min() - a.max(), rl.max() - rl.min(),
                     s.max() - rl.min(), int(m.sum())))
    if not rows:
        return
    ns = 10.0
    names = ["drain", "stage", "end spread", "last arr->rel", "release spread", "last staged-rel"]
    for i, name in enumerate(names):
        v = [x[i] for x in rows]
        print(f"{name:15s} median {np.median(v) * ns / 1000:6.2f} us  p90 {np.percentile(v, 90) * ns / 1000:6.2f} us")
    print(f"{'workgroups':15s} {rows[0][6]}")
    # k_round_wide's staging phases (third block): arrived -> fit check start -> fit decided -> window staged
    off3 = off + TL_NR * 512 * 4
    full = np.fromfile(path, dtype=np.uint64)
    if full.size < off3 + TL_NR * 512 * 4:
        return
    g = full[off3: off3 + TL_NR * 512 * 4].reshape(TL_NR, 512, 4).astype(np.int64)
    ok = live & (g[:, :, :3] > 0).all(axis=2)
    if ok.sum() < 2:
        return
    a1 = b[:, :, 1][ok]
    f0, f1, f2 = g[:, :, 0][ok], g[:, :, 1][ok], g[:, :, 2][ok]
    for name, v in (("stage entry", f0 - a1), ("fit check", f1 - f0), ("window", f2 - f1)):
        print(f"{name:15s} median {np.median(v) * ns / 1000:6.2f} us  p90 {np.percentile(v, 90) * ns / 1000:6.2f} us")
    # the workgroup that arrived last, per round
    lastw = [int(np.argmax(np.where(live[r], b[r, :, 1], 0))) for r in range(TL_NR) if live[r].sum() > 1]
    rr = [r for r in range(TL_NR) if live[r].sum() > 1]
    v = np.array([[g[r, w, 0] - b[r, w, 1], g[r, w, 1] - g[r, w, 0], g[r, w, 2] - g[r, w, 1]] for r, w in zip(rr, lastw)
                  if (g[r, w, :3] > 0).all()])
    if len(v):
        print("last arriver: stage entry / fit check / window: " + " / ".join(f"{np.median(v[:, k]) * ns / 1000:.2f}" for k in range(3)) + " us")


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[1] == "--tagged":
    tagged(sys.argv[2])
    sys.exit(0)
if __name__ == "__main__":
    main(sys.argv[1])
