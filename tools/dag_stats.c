/* dag_stats: generate a synthetic DAG, run the CPU oracle, print shape stats.
 * Dev tool (not shipped).  usage: dag_stats n N [lagging] [sig_mode] */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "../babble_amd/csrc/dag_gen.h"
#include "../oracle/hg_oracle.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char **argv) {
  bg_params p = {0};
  p.n = argc > 1 ? atoi(argv[1]) : 32;
  p.N = argc > 2 ? atoll(argv[2]) : 100000;
  p.lagging = argc > 3 ? atoi(argv[3]) : 0;
  p.sig_mode = argc > 4 ? atoi(argv[4]) : 0;
  p.lag_div = 50;
  p.seed = 0xBABB1E00ull + 2;
  p.tx_prob = 0.5;
  bg_dag d;
  double t0 = now();
  if (bg_generate(&p, &d)) { fprintf(stderr, "gen failed\n"); return 1; }
  double t1 = now();
  hgo *h = hgo_create(d.n, d.participant_ids, d.N);
  for (int64_t e = 0; e < d.N; e++)
    if (hgo_insert(h, d.creator[e], d.index[e], d.self_parent[e], d.other_parent[e],
                   d.hash + e * 32, d.sig_r + e * 32, d.ntx[e])) { fprintf(stderr, "ins %lld\n", (long long)e); return 1; }
  double t2 = now();
  hgo_divide_rounds(h);
  double t3 = now();
  hgo_decide_fame(h);
  double t4 = now();
  hgo_decide_round_received(h);
  double t5 = now();
  hgo_process_decided_rounds(h);
  double t6 = now();
  int32_t *round = malloc(d.N * 4), *lt = malloc(d.N * 4), *rr = malloc(d.N * 4);
  int8_t *wit = malloc(d.N), *fame = malloc(d.N);
  int64_t *cp = malloc(d.N * 8);
  hgo_event_results(h, round, wit, lt, rr, fame, cp);
  int32_t maxlt = 0;
  int64_t nw = 0, nfam = 0, nnf = 0;
  for (int64_t e = 0; e < d.N; e++) {
    if (lt[e] > maxlt) maxlt = lt[e];
    if (wit[e]) { nw++; if (fame[e] == 1) nfam++; else if (fame[e] == 2) nnf++; }
  }
  int32_t lr = hgo_last_round(h);
  int64_t nb = hgo_num_blocks(h);
  int64_t *cnt = malloc((nb + 1) * 8);
  hgo_blocks(h, NULL, NULL, cnt, NULL);
  int64_t maxf = 0;
  for (int64_t b = 0; b < nb; b++) if (cnt[b] > maxf) maxf = cnt[b];
  printf("n=%d N=%lld gen=%.2fs insert=%.2fs divide=%.2fs fame=%.2fs rr=%.2fs proc=%.2fs\n", d.n,
         (long long)d.N, t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5);
  printf("levels=%d (N/n=%.1f ratio=%.2f) rounds=%d ev/round=%.1f witnesses=%lld (%.1f/round) famous=%lld notfamous=%lld\n",
         maxlt + 1, (double)d.N / d.n, (maxlt + 1) / ((double)d.N / d.n), lr + 1,
         (double)d.N / (lr + 1), (long long)nw, (double)nw / (lr + 1), (long long)nfam, (long long)nnf);
  printf("consensus=%lld blocks=%lld maxframe=%lld undetermined=%lld lcr=%d txs=%lld\n",
         (long long)hgo_num_consensus_events(h), (long long)nb, (long long)maxf,
         (long long)hgo_num_undetermined(h), hgo_last_consensus_round(h),
         (long long)hgo_consensus_transactions(h));
  return 0;
}
