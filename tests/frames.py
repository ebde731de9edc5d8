"""Frame / block byte helpers for the parity tests (test infrastructure).

Independent restatements, in Python's json module, of the Go encodings the
block projection hashes:
  * EventBody.Marshal (event.go:32-39) of a synthetic event, and its
    Signature string crypto.EncodeSignature (crypto/utils.go:39-41);
  * Frame.Marshal (frame.go:17-26) of a frame given its roots and events;
  * Block.Marshal / BlockBody.Marshal (block.go:13-29, 178-185).
Go's encoding/json writes struct fields in declaration order, map keys
sorted, []byte as padded base64, no spaces, and a trailing newline from
Encoder.Encode; json.dumps(separators=(",", ":")) over insertion-ordered
dicts is byte-identical for these ASCII payloads."""
import base64
import hashlib
import json

import numpy as np


def _dumps(x):
    return json.dumps(x, separators=(",", ":"))


def hexup(h):
    return "0x" + bytes(h).hex().upper()


def base36(b):
    v = int.from_bytes(bytes(b), "big")
    if v == 0:
        return "0"
    out = []
    while v:
        v, r = divmod(v, 36)
        out.append("0123456789abcdefghijklmnopqrstuvwxyz"[r])
    return "".join(reversed(out))


def kat_event_bytes(d, e):
    """A Go-JSON body and signature string for KAT event e (synthetic keys:
    the reference's tests use random ones)."""
    pid = int(d.participant_ids[d.creator[e]])
    txs = [t.encode() for t in d.txs[e]]
    sp, op = int(d.sp[e]), int(d.op[e])
    body = {
        "Transactions": [base64.b64encode(t).decode() for t in txs] if txs else None,
        "Parents": ["Root%d" % pid if sp < 0 else hexup(d.hashes[sp]),
                    "" if op < 0 else hexup(d.hashes[op])],
        "Creator": base64.b64encode(hashlib.sha256(b"key%d" % pid).digest() * 2 + b"\x04").decode(),
        "Index": int(d.index[e]),
        "BlockSignatures": None,
    }
    s = hashlib.sha256(b"s" + d.names[e].encode()).digest()
    return (_dumps(body) + "\n").encode(), (base36(d.sig_r[e]) + "|" + base36(s)).encode()


def root_event(ev, slot, ids, hashes, index, lt, rnd):
    """RootEvent (root.go:65-71); ev < 0 = the base root event of `slot`"""
    if ev < 0:
        return {"Hash": "Root%d" % ids[slot], "CreatorID": int(ids[slot]), "Index": -1,
                "LamportTimestamp": -1, "Round": -1}
    return {"Hash": hexup(hashes[ev]), "CreatorID": int(ids[slot]), "Index": int(index[ev]),
            "LamportTimestamp": int(lt[ev]), "Round": int(rnd[ev])}


def frame_json(rr, roots, events, creator, ids, hashes, index, lt, rnd, bodies, sigs):
    """Frame.Marshal; roots as Oracle.frame_roots returns them, events in
    frame order, bodies / sigs by event id (bodies with their newline)"""
    out_roots = []
    for p, (nr, sp, others) in enumerate(roots):
        oth = {}
        for k, v in sorted(others, key=lambda kv: bytes(hashes[kv[0]])):
            oth[hexup(hashes[k])] = root_event(v, creator[v], ids, hashes, index, lt, rnd)
        out_roots.append({"NextRound": nr,
                          "SelfParent": root_event(sp, p if sp < 0 else creator[sp], ids, hashes,
                                                   index, lt, rnd),
                          "Others": oth})
    evs = [{"Body": json.loads(bodies[e]), "Signature": sigs[e].decode()} for e in events]
    return (_dumps({"Round": rr, "Roots": out_roots, "Events": evs}) + "\n").encode()


def block_json(index, rr, frame_hash, events, bodies, body_only=False):
    txs = []
    for e in events:
        txs += json.loads(bodies[e])["Transactions"] or []
    body = {"Index": index, "RoundReceived": rr, "StateHash": None,
            "FrameHash": base64.b64encode(frame_hash).decode(), "Transactions": txs}
    if body_only:
        return (_dumps(body) + "\n").encode()
    return (_dumps({"Body": body, "Signatures": {}}) + "\n").encode()


def roots_by_name(roots, d, lt, rnd):
    """Oracle/engine roots in the fixtures' by-name form (make_kat_fixtures.root)"""
    def re(ev, slot):
        if ev < 0:
            return ["Root", slot, -1, -1, -1]
        return [d.names[ev], int(d.creator[ev]), int(d.index[ev]), int(lt[ev]), int(rnd[ev])]
    out = []
    for p, (nr, sp, others) in enumerate(roots):
        out.append({"next_round": nr, "self_parent": re(sp, p),
                    "others": {d.names[k]: re(v, int(d.creator[v])) for k, v in others}})
    return out


def matches_fixture(got, want):
    """want's next_round None = not asserted by the Go test"""
    if len(got) != len(want):
        return False
    for g, w in zip(got, want):
        if w["next_round"] is not None and g["next_round"] != w["next_round"]:
            return False
        if g["self_parent"] != w["self_parent"] or g["others"] != w["others"]:
            return False
    return True


def sha(b):
    return hashlib.sha256(b).digest()


__all__ = ["kat_event_bytes", "frame_json", "block_json", "roots_by_name", "matches_fixture", "sha",
           "hexup", "base36", "np"]
