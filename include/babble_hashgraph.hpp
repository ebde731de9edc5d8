// babble_hashgraph.hpp -- C++ host mirror of the reference's Go `Hashgraph`
// (src/hashgraph/hashgraph.go), over the C ABI in babble_hip.h.
//
// Go is not available to host the engine behind the reference's own type, so
// this header restates that type's interface in C++: the same method names,
// the same argument meaning and the same error behaviour (a Go `error`
// becomes a thrown babble::HashgraphError carrying the BH_ERR_* kind).  It
// is header-only and holds no state besides the engine handle; every call
// goes to libbabble_hip (there is no CPU path).
//
//   Go (reference)                                 C++ (this header)
//   NewHashgraph(participants, store, ...) :43     Hashgraph(ids, max_events, device)
//   (*Hashgraph).InsertEvent(ev, wire) :714        InsertEvent(WireEvent) / InsertEvents(batch)
//   (*Hashgraph).DivideRounds() :767               DivideRounds()
//   (*Hashgraph).DecideFame() :852                 DecideFame()
//   (*Hashgraph).DecideRoundReceived() :951        DecideRoundReceived()
//   (*Hashgraph).ProcessDecidedRounds() :1041      ProcessDecidedRounds()
//   Core.RunConsensus (node/core.go:337-369)       RunConsensus()
//   .LastConsensusRound *int                       LastConsensusRound() -> std::optional<int>
//   .ConsensusTransactions / .PendingLoadedEvents  ConsensusTransactions() / PendingLoadedEvents()
//   .UndeterminedEvents / .PendingRounds           UndeterminedEvents() / PendingRounds()
//   Store.ConsensusEvents / LastBlockIndex         ConsensusEvents() / Blocks()
//   Event.round / lamportTimestamp / ...           EventMeta(id) / Coordinates(id)
#pragma once
#include <algorithm>
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "babble_hip.h"

namespace babble {

// A Go `error` from the hashgraph methods; kind() is the BH_ERR_* code
// (checkSelfParent, checkOtherParent, UnknownParticipant, SkippedIndex, ...).
class HashgraphError : public std::runtime_error {
 public:
  HashgraphError(int kind, const std::string &msg) : std::runtime_error(msg), kind_(kind) {}
  int kind() const { return kind_; }

 private:
  int kind_;
};

// WireEvent body (event.go:353-363) plus the hash / signature r the engine
// needs; parents are (creator ID, index) pairs, -1 = Root / none.
struct WireEvent {
  int64_t creator_id = 0;
  int32_t index = 0;
  int32_t self_parent_index = -1;
  int64_t other_parent_creator_id = -1;
  int32_t other_parent_index = -1;
  uint8_t hash[32] = {};
  uint8_t sig_r[32] = {};
  int32_t n_transactions = 0;
};

// Event private fields after the passes (event.go:107-116).
struct EventMeta {
  std::optional<int32_t> round, lamport_timestamp, round_received;
  bool witness = false;
  int8_t famous = -1;  // -1 not a witness, 0 Undefined, 1 True, 2 False (roundInfo.go:10-16)
  int64_t consensus_position = -1;
};

struct PendingRound {
  int32_t index;
  bool decided;
};

// RoundInfo (roundInfo.go:33-128) as Store.GetRound returns it
struct RoundInfo {
  int32_t round = 0;
  int32_t n_events = 0, n_consensus = 0;
  bool queued = false, witnesses_decided = false, pending = false, pending_decided = false;
  std::vector<int32_t> witnesses;  // event ids, participant order
  std::vector<int8_t> fame;        // Trilean: 0 Undefined, 1 True, 2 False
};

struct Block {  // block.go:100-123 (bodies are reassembled by the caller)
  int64_t index;
  int32_t round_received;
  int64_t first_event;  // position in ConsensusEvents()
  int64_t n_events;
  int64_t n_transactions;
};

class Hashgraph {
 public:
  // NewHashgraph (hashgraph.go:43-73); ids are the peers' IDs in ascending
  // order (peers.go:63-73), max_events the store capacity.
  Hashgraph(const std::vector<int64_t> &participant_ids, int64_t max_events, int device = 0) {
    bh_config cfg{(int32_t)participant_ids.size(), participant_ids.data(), max_events, device, 0, nullptr};
    const int rc = bh_create(&cfg, &h_);
    if (rc != BH_OK) {
      std::string msg = h_ ? bh_last_error(h_) : "bh_create failed";
      if (h_) bh_destroy(h_);
      h_ = nullptr;
      throw HashgraphError(rc, msg);
    }
  }
  ~Hashgraph() {
    if (h_) bh_destroy(h_);
  }
  Hashgraph(const Hashgraph &) = delete;
  Hashgraph &operator=(const Hashgraph &) = delete;
  Hashgraph(Hashgraph &&o) noexcept : h_(std::exchange(o.h_, nullptr)) {}

  // InsertEvent (hashgraph.go:714-761): throws on checkSelfParent /
  // checkOtherParent / participant errors; the event is then not inserted.
  void InsertEvent(const WireEvent &ev) {
    std::vector<int32_t> st = InsertEvents(std::vector<WireEvent>{ev});
    if (st[0] != BH_OK) throw HashgraphError(st[0], bh_last_error(h_));
  }

  // A batch in topological order; rejected events are skipped (as
  // createHashgraph does in hashgraph_test.go:134-138).  Returns the status
  // of each event (BH_OK or the error kind).
  std::vector<int32_t> InsertEvents(const std::vector<WireEvent> &evs) {
    const size_t m = evs.size();
    std::vector<int64_t> cr(m), opc(m);
    std::vector<int32_t> idx(m), spi(m), opi(m), ntx(m), st(m, BH_OK);
    std::vector<uint8_t> hash(m * 32), sig(m * 32);
    for (size_t i = 0; i < m; ++i) {
      cr[i] = evs[i].creator_id;
      idx[i] = evs[i].index;
      spi[i] = evs[i].self_parent_index;
      opc[i] = evs[i].other_parent_creator_id;
      opi[i] = evs[i].other_parent_index;
      ntx[i] = evs[i].n_transactions;
      std::copy(evs[i].hash, evs[i].hash + 32, hash.begin() + 32 * i);
      std::copy(evs[i].sig_r, evs[i].sig_r + 32, sig.begin() + 32 * i);
    }
    bh_events b{(int64_t)m, cr.data(), idx.data(), spi.data(), opc.data(),
                opi.data(), hash.data(), sig.data(), ntx.data()};
    int64_t accepted = 0;
    const int rc = bh_insert_events(h_, &b, st.data(), &accepted);
    if (rc == BH_ERR_DEVICE || rc == BH_ERR_INVALID) throw HashgraphError(rc, bh_last_error(h_));
    return st;
  }

  // Reset(block, frame) (hashgraph.go:1324-1369) on a fresh Hashgraph,
  // before frame.Events are inserted: the frame's roots in participant order
  // and their Others flattened (bh_roots, include/babble_hip.h)
  struct RootOther {
    int32_t root;         // position of the Root holding the entry
    uint8_t key[32];      // hash of the event keying it (Others[ev.Hex()])
    int64_t creator_id;   // RootEvent.CreatorID
    int32_t index, lamport_timestamp, round;
    uint8_t hash[32];     // RootEvent.Hash
  };
  // self_parent_hash: each Root.SelfParent.Hash, 32 bytes per root (needed
  // with frames on; empty otherwise)
  void Reset(int32_t round_received, int64_t block_index, const std::vector<int32_t> &next_round,
             const std::vector<int32_t> &self_parent_index, const std::vector<int32_t> &self_parent_lamport,
             const std::vector<int32_t> &self_parent_round, const std::vector<RootOther> &others,
             const std::vector<uint8_t> &self_parent_hash = {}) {
    const size_t k = others.size();
    std::vector<int32_t> root(k), idx(k), lt(k), rnd(k);
    std::vector<int64_t> cre(k);
    std::vector<uint8_t> key(k * 32), hash(k * 32);
    for (size_t i = 0; i < k; ++i) {
      root[i] = others[i].root;
      cre[i] = others[i].creator_id;
      idx[i] = others[i].index;
      lt[i] = others[i].lamport_timestamp;
      rnd[i] = others[i].round;
      std::copy(others[i].key, others[i].key + 32, key.begin() + 32 * i);
      std::copy(others[i].hash, others[i].hash + 32, hash.begin() + 32 * i);
    }
    bh_roots rt{round_received, block_index, next_round.data(), self_parent_index.data(),
                self_parent_lamport.data(), self_parent_round.data(), (int32_t)k, root.data(), key.data(),
                cre.data(), idx.data(), lt.data(), rnd.data(), hash.data(),
                self_parent_hash.empty() ? nullptr : self_parent_hash.data()};
    check(bh_reset(h_, &rt));
  }

  void DivideRounds() { check(bh_divide_rounds(h_)); }
  void DecideFame() { check(bh_decide_fame(h_)); }
  void DecideRoundReceived() { check(bh_decide_round_received(h_)); }
  void ProcessDecidedRounds() { check(bh_process_decided_rounds(h_)); }
  // Core.RunConsensus (node/core.go:337-369): the four passes in order
  void RunConsensus() { check(bh_run_consensus(h_)); }

  std::optional<int> LastConsensusRound() const {
    const bh_stats s = stats();
    if (s.last_consensus_round < 0) return std::nullopt;
    return s.last_consensus_round;
  }
  int64_t ConsensusTransactions() const { return stats().consensus_transactions; }
  int64_t PendingLoadedEvents() const { return stats().pending_loaded_events; }
  int32_t LastRound() const { return stats().last_round; }

  std::vector<int32_t> UndeterminedEvents() const {
    const int64_t cnt = bh_get_undetermined(h_, nullptr, 0);
    if (cnt < 0) check((int)-cnt);  // a negated BH_ERR_* code
    std::vector<int32_t> ids((size_t)std::max<int64_t>(cnt, 0));
    if (cnt > 0) bh_get_undetermined(h_, ids.data(), cnt);
    return ids;
  }

  std::vector<PendingRound> PendingRounds() const {
    const int32_t cnt = bh_get_pending_rounds(h_, nullptr, nullptr, 0);
    if (cnt < 0) check(-cnt);  // a negated BH_ERR_* code
    std::vector<int32_t> idx((size_t)std::max(cnt, 0));
    std::vector<int8_t> dec((size_t)std::max(cnt, 0));
    if (cnt > 0) bh_get_pending_rounds(h_, idx.data(), dec.data(), cnt);
    std::vector<PendingRound> out;
    for (int32_t i = 0; i < cnt; ++i) out.push_back({idx[i], dec[i] != 0});
    return out;
  }

  // Store.ConsensusEvents as event ids (the full sequence, not the Go
  // store's rolling window, inmem_store.go:165-172)
  std::vector<int32_t> ConsensusEvents() const {
    const int64_t cnt = stats().consensus_events;
    std::vector<int32_t> ids((size_t)cnt);
    if (cnt > 0) check(bh_get_consensus_order(h_, 0, cnt, ids.data()));
    return ids;
  }

  std::vector<Block> Blocks() const {
    const int64_t cnt = stats().blocks;
    std::vector<int32_t> rr((size_t)cnt);
    std::vector<int64_t> first((size_t)cnt), ne((size_t)cnt), nt((size_t)cnt);
    if (cnt > 0) check(bh_get_blocks(h_, 0, cnt, rr.data(), first.data(), ne.data(), nt.data()));
    std::vector<Block> out;
    for (int64_t i = 0; i < cnt; ++i) out.push_back({i, rr[i], first[i], ne[i], nt[i]});
    return out;
  }

  EventMeta GetEventMeta(int64_t id) const {
    int32_t round, lamport, rr;
    int8_t wit, fame;
    int64_t pos;
    check(bh_get_event_meta(h_, id, 1, &round, &wit, &lamport, &rr, &fame, &pos));
    EventMeta m;
    if (round != INT32_MIN) m.round = round;
    if (lamport != INT32_MIN) m.lamport_timestamp = lamport;
    if (rr != INT32_MIN) m.round_received = rr;
    m.witness = wit != 0;
    m.famous = fame;
    m.consensus_position = pos;
    return m;
  }

  // Store.GetRound (inmem_store.go:185-191): throws KeyNotFound for a round
  // that does not exist
  RoundInfo GetRound(int32_t r) const {
    bh_round_info info{};
    const int cap = 4096;
    std::vector<int32_t> w(cap);
    std::vector<int8_t> f(cap);
    check(bh_get_round_info(h_, r, &info, w.data(), f.data(), cap));
    RoundInfo out;
    out.round = info.round;
    out.n_events = info.n_events;
    out.n_consensus = info.n_consensus;
    out.queued = info.queued != 0;
    out.witnesses_decided = info.witnesses_decided != 0;
    out.pending = info.pending != 0;
    out.pending_decided = info.pending_decided != 0;
    const int k = std::min(info.n_witnesses, cap);
    out.witnesses.assign(w.begin(), w.begin() + k);
    out.fame.assign(f.begin(), f.begin() + k);
    return out;
  }
  // Store.RoundWitnesses (inmem_store.go:205-211): [] for a missing round
  std::vector<int32_t> RoundWitnesses(int32_t r) const {
    if (r < 0 || r > LastRound()) return {};
    return GetRound(r).witnesses;
  }

  // lastAncestors / firstDescendants indexes of one event (event.go:115-116),
  // in participant order; -1 / INT32_MAX as in the reference
  std::pair<std::vector<int32_t>, std::vector<int32_t>> Coordinates(int64_t id, int n) const {
    std::vector<int32_t> la((size_t)n), fd((size_t)n);
    check(bh_get_coordinates(h_, id, la.data(), fd.data()));
    return {la, fd};
  }

  bh_stats stats() const {
    bh_stats s{};
    check(bh_get_stats(h_, &s));
    return s;
  }
  bh_handle *handle() const { return h_; }

 private:
  void check(int rc) const {
    if (rc != BH_OK) throw HashgraphError(rc, bh_last_error(h_));
  }
  bh_handle *h_ = nullptr;
};

}  // namespace babble
