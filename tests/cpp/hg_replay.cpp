// hg_replay -- drives the engine through the C++ mirror (babble_hashgraph.hpp)
// from a text play list, the way hashgraph_test.go drives *Hashgraph, and
// prints the results for tests/test_cpp_mirror.py to compare with the oracle.
//
// usage: hg_replay <playlist>      (hg_replay --link-check: no device calls)
// play list lines:
//   ids <id0> <id1> ...            participant IDs, ascending (NewHashgraph)
//   cap <max_events>
//   ev <creator_id> <index> <sp_index> <op_creator_id> <op_index> <hash hex> <sig_r hex> <ntx>
//   insert                          InsertEvent for every pending `ev` line, in order
//   divide | fame | received | process | run
//   dump                            print the state (format in print_state)
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "babble_hashgraph.hpp"

static void hex32(const std::string &s, uint8_t *out) {
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)std::stoi(s.substr(2 * i, 2), nullptr, 16);
}

static void print_state(const babble::Hashgraph &hg, int64_t n_events) {
  const auto lcr = hg.LastConsensusRound();
  std::printf("stats %d %lld %lld %d\n", lcr ? *lcr : -1, (long long)hg.ConsensusTransactions(),
              (long long)hg.PendingLoadedEvents(), hg.LastRound());
  for (int64_t id = 0; id < n_events; ++id) {
    const babble::EventMeta m = hg.GetEventMeta(id);
    std::printf("meta %lld %d %d %d %d %d %lld\n", (long long)id, m.round ? *m.round : INT32_MIN,
                m.witness ? 1 : 0, m.lamport_timestamp ? *m.lamport_timestamp : INT32_MIN,
                m.round_received ? *m.round_received : INT32_MIN, (int)m.famous,
                (long long)m.consensus_position);
  }
  std::printf("order");
  for (int32_t id : hg.ConsensusEvents()) std::printf(" %d", id);
  std::printf("\npending");
  for (const auto &p : hg.PendingRounds()) std::printf(" %d:%d", p.index, p.decided ? 1 : 0);
  std::printf("\nundetermined");
  for (int32_t id : hg.UndeterminedEvents()) std::printf(" %d", id);
  std::printf("\n");
  for (const auto &b : hg.Blocks())
    std::printf("block %lld %d %lld %lld %lld\n", (long long)b.index, b.round_received,
                (long long)b.first_event, (long long)b.n_events, (long long)b.n_transactions);
  std::printf("end\n");
}

int main(int argc, char **argv) {
  if (argc > 1 && !std::strcmp(argv[1], "--link-check")) {
    // resolve every entry point without touching a device
    const void *fns[] = {(void *)&bh_create, (void *)&bh_destroy, (void *)&bh_insert_events,
                         (void *)&bh_run_consensus, (void *)&bh_get_event_meta, (void *)&bh_get_blocks};
    for (const void *f : fns)
      if (!f) return 1;
    std::printf("link ok\n");
    return 0;
  }
  if (argc < 2) {
    std::fprintf(stderr, "usage: hg_replay <playlist>\n");
    return 2;
  }
  std::ifstream in(argv[1]);
  std::vector<int64_t> ids;
  int64_t cap = 0, inserted = 0;
  std::vector<babble::WireEvent> pending;
  babble::Hashgraph *hg = nullptr;
  std::string line;
  try {
    while (std::getline(in, line)) {
      std::istringstream ls(line);
      std::string cmd;
      ls >> cmd;
      if (cmd == "ids") {
        int64_t v;
        while (ls >> v) ids.push_back(v);
      } else if (cmd == "cap") {
        ls >> cap;
      } else if (cmd == "ev") {
        babble::WireEvent e;
        std::string h, s;
        ls >> e.creator_id >> e.index >> e.self_parent_index >> e.other_parent_creator_id >>
            e.other_parent_index >> h >> s >> e.n_transactions;
        hex32(h, e.hash);
        hex32(s, e.sig_r);
        pending.push_back(e);
      } else {
        if (!hg) hg = new babble::Hashgraph(ids, cap);
        if (cmd == "insert") {
          // one InsertEvent per event, as Core does (hashgraph.go:714)
          for (size_t i = 0; i < pending.size(); ++i) {
            try {
              hg->InsertEvent(pending[i]);
              ++inserted;
            } catch (const babble::HashgraphError &err) {
              std::printf("reject %lld %d\n", (long long)i, err.kind());
            }
          }
          pending.clear();
        } else if (cmd == "divide") hg->DivideRounds();
        else if (cmd == "fame") hg->DecideFame();
        else if (cmd == "received") hg->DecideRoundReceived();
        else if (cmd == "process") hg->ProcessDecidedRounds();
        else if (cmd == "run") hg->RunConsensus();
        else if (cmd == "dump") print_state(*hg, inserted);
      }
    }
  } catch (const babble::HashgraphError &err) {
    std::printf("error %d %s\n", err.kind(), err.what());
    delete hg;
    return 1;
  }
  delete hg;
  return 0;
}
