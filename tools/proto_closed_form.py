"""Dev prototype (not shipped, not a test oracle): the engine's closed-form
batch algorithm in numpy, checked against the CPU oracle on random DAGs.
It exists to validate the math of the HIP design (round boundaries per
chain, candidate resolution, bitset fame, closed-form round-received)
before it is written as kernels.  usage: python tools/proto_closed_form.py n N [lag]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from babble_amd.dag import Dag  # noqa: E402
from oracle_py import UNSET, Oracle  # noqa: E402

MAXI = 2 ** 31 - 1


def engine(n, creator, index, sp, op, hashes, sig_r, ntx):
    N = len(creator)
    SM = 2 * n // 3 + 1
    # --- coordinates + LT (the sweep) ---
    LA = np.full((N, n), -1, np.int32)
    LT = np.zeros(N, np.int32)
    for e in range(N):
        a = LA[sp[e]] if sp[e] >= 0 else np.full(n, -1, np.int32)
        b = LA[op[e]] if op[e] >= 0 else np.full(n, -1, np.int32)
        LA[e] = np.maximum(a, b)
        LA[e, creator[e]] = index[e]
        LT[e] = max(LT[sp[e]] if sp[e] >= 0 else -1, LT[op[e]] if op[e] >= 0 else -1) + 1
    chain = [np.nonzero(creator == c)[0] for c in range(n)]
    clen = np.array([len(ch) for ch in chain])

    def ss_la(x, w):  # SS via LA only: x's last ancestors on >= SM chains see w
        cnt = 0
        for i in range(n):
            k = LA[x, i]
            if k >= 0 and LA[chain[i][k], creator[w]] >= index[w]:
                cnt += 1
        return cnt >= SM

    def fd_row(w):
        row = np.full(n, MAXI, np.int32)
        for i in range(n):
            col = LA[chain[i], creator[w]]
            k = np.searchsorted(col, index[w], side="left")
            if k < len(col):
                row[i] = k
        return row

    def resolve(B):
        cand = {c: chain[c][B[c]] for c in range(n) if B[c] < clen[c]}
        if not cand:
            return []
        wit = []
        flagged = []
        for c, x in cand.items():
            anc = sum(1 for c2 in cand if c2 != c and LA[x, c2] >= B[c2])
            (flagged if anc >= SM else wit).append(x)
        for x in sorted(flagged):
            cnt = sum(1 for w in wit if w < x and LA[x, creator[w]] >= index[w] and ss_la(x, w))
            if cnt < SM:
                wit.append(x)
        return sorted(wit)

    Bs = [np.zeros(n, np.int64)]
    Ws = [resolve(Bs[0])]
    FDW = [np.stack([fd_row(w) for w in Ws[0]])]
    ALLC = os.environ.get("ALLC") == "1"
    while True:
        r = len(Bs) - 1
        W, F = Ws[r], FDW[r]
        if ALLC:  # scan against every candidate of round r
            cands = [chain[c][Bs[r][c]] for c in range(n) if Bs[r][c] < clen[c]]
            F = np.stack([fd_row(w) for w in cands])
        Bn = Bs[r].copy()
        for c in range(n):
            k = Bs[r][c]
            while k < clen[c]:
                x = chain[c][k]
                cnt = int(np.sum(np.all(LA[x][None, :] >= F, axis=1) * 0 + (np.sum(LA[x][None, :] >= F, axis=1) >= SM)))
                if cnt >= SM:
                    break
                k += 1
            Bn[c] = k
        Wn = resolve(Bn)
        if not Wn:
            break
        Bs.append(Bn)
        Ws.append(Wn)
        FDW.append(np.stack([fd_row(w) for w in Wn]))
    R = len(Ws)
    rnd = np.empty(N, np.int32)
    for c in range(n):
        for k, x in enumerate(chain[c]):
            rnd[x] = max(r for r in range(R) if Bs[r][c] <= k)
    wit = np.zeros(N, np.int8)
    for W in Ws:
        wit[W] = 1
    # --- fame ---
    fame = np.full(N, -1, np.int8)
    decided = np.zeros(R, bool)

    def ssf(y, wi, j):  # SS(y, W(j)[wi]) via FD rows
        return np.sum(LA[y] >= FDW[j][wi]) >= SM

    for r in range(R):
        for x in Ws[r]:
            fame[x] = 0
            prev = None
            for j in range(r + 1, R):
                diff = j - r
                cur = np.zeros(len(Ws[j]), bool)
                dec = False
                for yi, y in enumerate(Ws[j]):
                    if diff == 1:
                        cur[yi] = LA[y, creator[x]] >= index[x]
                        continue
                    S = np.array([ssf(y, wi, j - 1) for wi in range(len(Ws[j - 1]))], bool)
                    yays = int(np.sum(S & prev))
                    nays = int(np.sum(S)) - yays
                    v = yays >= nays
                    t = yays if v else nays
                    if diff % n:
                        if t >= SM:
                            fame[x] = 1 if v else 2
                            dec = True
                            break
                        cur[yi] = v
                    else:
                        cur[yi] = v if t >= SM else hashes[y][16] != 0
                if dec:
                    break
                prev = cur
        decided[r] = all(fame[x] != 0 for x in Ws[r])
    # --- round received ---
    rr = np.full(N, UNSET, np.int32)
    for x in range(N):
        for i in range(rnd[x] + 1, R):
            if not decided[i]:
                break
            FW = [w for w in Ws[i] if fame[w] == 1]
            if FW and all(LA[w, creator[x]] >= index[x] for w in FW):
                rr[x] = i
                break
    P = 0
    while P < R and decided[P]:
        P += 1
    sel = np.nonzero((rr != UNSET) & (rr < P))[0]
    keys = sorted(sel, key=lambda e: (rr[e], LT[e], bytes(sig_r[e])))
    return dict(round=rnd, witness=wit, lamport=LT, round_received=rr, fame=fame,
                order=np.array(keys, np.int32), R=R, P=P)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    lag = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    for seed in range(3):
        d = Dag(n, N, 1234 + seed, lagging=lag, sig_mode=0)
        o = Oracle(n, d.participant_ids, capacity=N)
        o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
        o.run_consensus()
        ref = o.results()
        got = engine(n, d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
        ok = True
        for k in ("round", "witness", "lamport", "round_received", "fame"):
            a, b = ref[k], got[k]
            if k == "fame":
                a = np.where(ref["witness"] == 1, a, -1)
            if not np.array_equal(a, b):
                bad = np.nonzero(a != b)[0]
                print(f"seed {seed} MISMATCH {k}: {len(bad)} e.g. {bad[:5]} ref={a[bad[:5]]} got={b[bad[:5]]}")
                ok = False
        oo = o.consensus_order()
        if not np.array_equal(oo, got["order"]):
            print(f"seed {seed} MISMATCH order len {len(oo)} vs {len(got['order'])}")
            ok = False
        print(f"seed {seed}: n={n} N={N} rounds={got['R']} processed={got['P']} "
              f"ordered={len(oo)} {'OK' if ok else 'FAIL'}")


if __name__ == "__main__":
    main()
