// engine.h -- internal device-state layout and kernel launchers of libbabble_hip.
//
// HBM layout (structure of arrays, event id = insertion order):
//   creator/index/sp/op/ntx  int32[N]       event bodies (sp/op: global ids, -1 = Root/none)
//   coin                     uint8[N]       hash[16] != 0  (middleBit, hashgraph.go:1526-1535)
//   sigw                     uint32[N][8]   ECDSA r as 8 big-endian words (tie-break key)
//   chain_ids                int32[N]       ids grouped by creator, ordered by index
//   epos                     int32[N]       row of event e = chain_start[creator] + index
//   la                       int32[N][npad] lastAncestors indexes (-1 = none), chain-major rows
//   la_ev                    int32[n][N] the sweep's output (one column per slab, event
//                                           order), permuted into `la` afterwards
//   lt                       int32[N]       Lamport timestamp
//   B                        int32[R_cap+1][n] first index on chain c with round >= r
//   wids / wofs / wcnt       witnesses of each round (chain order)
//   fd                       int32[N][npad] firstDescendants, chain-major rows (kernels_fd.hip)
//   fdt                      int32[npad][N] the FD walk's column-major output (aliases la_ev)
//   round/witness/fame/rr    per-event results
// See DESIGN.md for the algorithm and the roofline of each kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace bh {

constexpr int32_t UNSET = INT32_MIN;    // Go nil
constexpr int32_t FD_NONE = INT32_MAX;  // math.MaxInt32 (hashgraph.go:447)
// k_round_lean's hand-off encoding of a firstDescendants entry x (a chain
// row < 2^22 - 1, or FD_NONE as 2^22 - 1) with the 1-bit tag b: the f32
// 2^22 + x + b / 2, bits 0x4A800000 + 2x + b (the binade [2^22, 2^23) has
// spacing 1/2), so a received entry is used as it arrives
constexpr uint32_t FE_BASE = 0x4A800000u;
constexpr int32_t FE_NONE_X = (1 << 22) - 1;
__host__ __device__ inline uint32_t fe_encode(int32_t x, uint32_t b) {
  const uint32_t v = x == FD_NONE || x >= FE_NONE_X ? (uint32_t)FE_NONE_X : (uint32_t)x;
  return FE_BASE + 2u * v + b;
}
__host__ __device__ inline int32_t fe_decode(uint32_t bits) {
  const int32_t x = (int32_t)((bits - FE_BASE) >> 1);
  return x >= FE_NONE_X ? FD_NONE : x;
}
constexpr int32_t P16_MAXLEN = 65000;  // longest chain the 16-bit round loop takes
constexpr int P8G_DELTA = 20;  // k_round_wide's shared 8-bit base: B[r-1][i] - 20
constexpr int P8_XMAX = 126;  // largest window-relative LA of k_round_wide's 8-bit rows (bit 7 is the compare's)
constexpr int SCAN_WIN = 32;            // rows per round-boundary scan window
constexpr int FRAME_LDS_MAX = 8192;     // frames sorted in LDS up to this size (96 KiB)
constexpr int FL_MAXN = 128;            // participants the dataflow sweep (k_flow) handles
constexpr int FW_MAXN = 512;            // participants the wide dataflow (k_floww2) handles

enum StateSlot {
  ST_CUR0 = 0,     // round r of the iteration with parity 0 (ST_CUR0 + 1: parity 1)
  ST_DONE = 2,     // round loop finished
  ST_ROUNDS = 3,   // number of rounds R (LastRound + 1)
  ST_ERR = 4,      // capacity overflow / inconsistency
  ST_P = 5,        // processed prefix: rounds [0, P) are decided and ordered
  ST_NCONS = 6,    // consensus events (int32 ok: < 2^31)
  ST_ITERS = 7,    // round-loop iterations executed
  ST_PFAIL = 8,    // sticky within a DivideRounds call: a segment's loop failed (1 capacity, 3 barrier gave up)
  ST_NBLOCKS = 9,
  ST_FLOWOVF = 10,  // k_flow32: a Lamport timestamp reached 2^21 (LT recomputed by k_flow)
  ST_RESUME = 11,   // k_resume_point: the last round whose boundaries B[r][*] a prefix run fixed
  ST_FIATMAX = 12,  // k_fiat: the highest round of an event below the closed form's first round (-1: none)
  ST_FIATDONE = 13, ST_FIATEV = 14, ST_FIATCH = 15,  // k_fiat: chains done, events visited, chunks scanned
  // k_round2p's entry gate: ST_FLOWOVF == 2 as the kernel before the loop on
  // the loop stream saw it (k_cand_rows / k_seg_resume).  ST_FLOWOVF itself
  // may change while a loop's workgroups are being dispatched (the split's
  // unpack of a LATER segment runs on the coordinate stream), so every
  // workgroup of one loop decides on this copy
  ST_GATE = 16,
  ST_COUNT = 18  // (even: the pinned staging words after ST_COUNT hold an 8-byte value at ST_COUNT + 6)
};

// FDT: firstDescendants by column, tiled by 64 chain-major rows --
// [row / 64][column i][row % 64].  Runs of consecutive rows of one column
// (what the walks write and the round loop's windows read) are contiguous,
// and a window's 128 column segments share one or two 32 KiB tiles (a
// [column][row] layout would put each in its own page).
__host__ __device__ inline int64_t fdt_pos(int64_t row, int i, int npad) {
  return (((row >> 6) * npad + i) << 6) + (row & 63);
}

struct Dev {
  int32_t n, npad, sm;
  int64_t N;
  int32_t R_cap;
  int64_t la_rows;  // capacity rows of la / lt; 64 scratch rows follow
  int64_t W_cap;
  // event bodies
  int32_t *creator, *index, *sp, *op, *ntx;
  uint8_t *coin;
  uint32_t *sigw;
  // chains
  int32_t *chain_start, *chain_len, *chain_ids, *epos;
  // coordinates
  int32_t *la, *lt;
  int32_t *la_ev;  // [n][la_rows+64] sweep output: column-major, event order
  int32_t ring_log2;  // the sweep's LDS value ring holds 1 << ring_log2 events
  // chain dataflow (kernels_flow.hip)
  int32_t *opdesc;  // [N] chain-major other-parent (creator << 22 | index), -1 = none
  int32_t *la_col;  // [n][la_rows+64] column-major LA, chain-major rows (aliases la_ev)
  int32_t *lt_row;  // [la_rows+64] LT by chain-major row
  int32_t col0, ncol;  // k_flow / k_flow32: this shard's LA columns [col0, col0 + ncol) (+ the LT workgroup)
  // Segments (insertion-order prefixes of the DAG):
  // the coordinate kernels compute chain c's events [seg_lo[c], chain_len[c])
  // (chain_len = the prefix's lengths); rows of the chain-major layout
  // (chain_start) are those of all `rows` events; descriptors are built for
  // event ids [e0, N).  One segment = seg_lo all 0, e0 0, rows N.
  int32_t *seg_lo;
  int64_t e0, rows;
  const int32_t *tile_list;  // k_flow_transpose: the segment's 64-row tiles (null: every tile)
  int64_t ntiles;
  int32_t *hdone;  // mapped pinned host word: set when the round loop is done
  int32_t flow_ltclamp;  // k_flow32 LT limit (2^21 - 256; BH_FLOW_LTCLAMP lowers it to test the fallback)
  int32_t flow_lt;       // k_flow32 runs the LT workgroup beside its columns (0: a coordinate shard without it)
  int32_t flow_wd;       // k_floww / k_floww2 watchdog: stalled headers before it gives up (BH_FLOWW_WATCHDOG; -1 fires at once)
  uint8_t *depth, *chunk_maxd;
  int4 *desc;  // [N] packed sweep descriptors (kernels_coords.hip)
  // rounds
  int32_t *B, *wofs, *wcnt, *wids;
  int32_t *wrow;   // [W] chain-major row of each witness (its LA row)
  int32_t *Bp;     // [2][n] B[r] / B[r+1] by round parity
  // firstDescendants of every event (updateAncestorFirstDescendant)
  int32_t *fd;      // [la_rows + 64][npad] chain-major rows
  uint32_t *cand16;  // [2][n][(npad + 7) / 8 * 4] k_round_wide<*, true>: the candidates' FD rows as 16-bit FD + 1
                     // (0xFFFF: none), two per dword, by round parity -- gathered from FDT by the workgroup that
                     // finds the candidate (the hand-off); aliases candfd (n > 128 only)
  int32_t *fdt;     // walk output, tiled by 64 chain-major rows (fdt_pos; shares la_ev's allocation)
  // fd_cols (npad <= 128): FDT is complete (the walks write MaxInt32 where
  // no event of a chain sees a row) and is the only per-event FD table; the
  // round loop reads windows of it and hands fame its stronglySee results
  // as ballots (ssm); no fd
  int32_t fd_cols;
  // fd_rows (npad > 128): k_fd_transpose writes the 32-bit fd rows; 0 when
  // the 16-bit loop runs on a complete FDT (k_flow_transpose walked it), and
  // FD readers then read FDT
  int32_t fd_rows;
  // [n][rspan][16 waves] k_round2 ballots: lane (q * LPC) % 64 of wave
  // q * LPC / 64 = candidate (c, B[r][c]) strongly sees (q, B[r-1][q]);
  // row ballot_row(d, c, r).  The ballot tables hold rounds [rbase, rbase +
  // rspan): the round loop only writes rounds above the first one it
  // starts from (0, or a Reset hashgraph's r0), so a Reset at a high round
  // does not pay for the rounds below it
  unsigned long long *ssm;
  // k_round2 path: the LA row of each candidate (c, B[r][c]) at row
  // ballot_row(d, c, r), npad wide, stored by the workgroup that finds it
  // (from its LDS window) -- fame's first votes and minLA read witnesses'
  // rows here, whole and coalesced, instead of n scattered column reads
  int32_t *cla;
  int32_t cla_span;  // rounds cla holds: a ring over rounds (cla_row), rounds > R - cla_span intact
  int32_t use_cla;  // the loop that ran wrote cla (k_round2; not the resident k_round_solo)
  int32_t wide_cols;  // the 16-bit wide loop reads la_col (k_round_wide<*, true, true>; no FDT)
  int32_t round_persist;  // k_round2p: the whole n <= 128 loop in one launch (default; BH_ROUND_PERSIST=0: one launch per iteration)
  int32_t round_f32;      // k_round2p's search compares in packed f32 (BH_ROUND_F32=0: the int32 sign-bit count)
  int32_t cand_fe;        // candfd rows in k_round_lean's float encoding (set by the launchers, cand_fe())
  int32_t *pbar;          // the persistent wide loop's grid barrier (k_round2p hands off through tagged Bp / candfd dwords instead)
  int32_t pbar_spin;      // polls before a persistent loop gives up waiting (barrier or tagged hand-off; BH_PBAR_SPIN lowers it to test the fallback)
  int32_t pbar_mode;      // the wide persistent loop's barrier: 0 one counter, 1 XCD-hierarchical (n > 64; BH_PBAR=xcd|flat)
  int32_t prestage;       // the wide persistent loop stages its next window while the barrier completes (BH_PRESTAGE=0: off)
  int32_t xpose_fd;       // k_flow_transpose also walks firstDescendants into FDT (0: LA rows only)
  int32_t win_reuse;      // persistent k_round_wide: the next window reuses the rows it shares with the last
  int32_t wide_prio;      // persistent k_round_wide: 1 hand-off / barrier / staging at priority 2, 2 also alternate the search
  int32_t *psnap;         // the loop's inputs (Bp and candfd of parity 0, the state block) kept for that fallback
  int32_t round_src_rows;  // k_round2r: windows from the row-major LA, hand-off from FDT (BH_ROUND_SRC=rows, A/B)
  int32_t rbase, rspan;
  int32_t round_lpc;  // lanes per candidate of k_round2 (8), the layout of its ssm ballots
  int32_t round_p8;   // k_round_wide<*, true>: 8-bit window-relative rows where the window's LA spread is at most this
                      // (P8_XMAX; BH_ROUND_P8=<x> lowers it to force the 16-bit fallback, 0: off)
  // round-based 8-bit candidate rows (k_round_wide<*, true>):
  // iteration r's byte columns are relative to base_i = max(B[r-1][i] -
  // round_p8g, 0), a base every workgroup of the iteration shares, so the
  // workgroup that hands a candidate over converts its row once (cand8)
  // instead of every workgroup converting every candidate.  c8tag[p][c] = r
  // when cand8[p][c] was written for iteration r (-1: convert from cand16)
  uint8_t *cand8;     // [2][n][(npad + 15) / 16 * 16] bytes
  int32_t *c8tag;     // [2][n]
  int32_t *Bq;        // [2][npad] k_round2 bytes: B[r - 1] for the iteration of parity p (written by iteration r - 1)
  int32_t round_p8g;  // base offset below B[r-1] (P8G_DELTA; BH_ROUND_P8G=0 turns the shared base off)
  int32_t round_ilp2;  // k_round_wide byte rows: two candidates' searches interleaved per lane group (BH_ROUND_ILP2=0: one)
  // [n][rspan][8] k_round_wide's stronglySee masks (n <= 512, !fd_cols):
  // word w bit b = candidate (64 w + b, B[r-1]) is strongly seen by (c, B[r][c])
  unsigned long long *ssw;
  int32_t *last_la; // [n][npad] LA row of each chain's last event
  int32_t *rq;      // [n] k_resume_point: each chain's first round whose boundary left the prefix
  int32_t max_chain_len;
  // round-loop hand-off (k_round2, npad <= 128), by round parity
  int32_t *candfd;   // [2][n][npad] FD row of each chain's candidate (c, B[r][c])
  int32_t *state;
  int32_t *round;
  int8_t *witness, *fame;
  // fame / received
  int8_t *decided;
  int8_t *wfame;   // [W] fame of witness wofs[r] + i (chain order), as the fame pass decides it
  int32_t *nfam, *minla;
  int32_t *rr;
  // per-sync schedule (hashgraph.go:809-815, roundInfo.go:35):
  // a witness whose round was already processed when it arrived (or was
  // still undecided when its round was processed) is never decided again --
  // its fame stays Undefined and its round never again reports
  // WitnessesDecided.  trapped[e] marks such witnesses, blocked[r] counts
  // them per round.
  int8_t *trapped;
  int32_t *blocked;
  // frames
  int32_t *frame_cnt, *frame_ofs, *frame_cur, *blk_of_frame;
  int32_t *order;
  int64_t *cons_pos;
  int64_t *frame_ntx;
  int32_t *frame_loaded;  // [R] loaded events per frame (IsLoaded, event.go:169-178)
  int64_t *counters;  // [0] consensus txs, [1] loaded consensus events, [2] unused, [3] undetermined
  // diagnostic phase counters (BH_DIAG=1 builds the buffer; null otherwise).
  // Only a separate diagnostic run reads them; no result depends on them.
  unsigned long long *diag;
  // Reset / FastSync roots (bh_reset; hashgraph.go:1324-1369, root.go,
  // docs/fastsync.rst:140-175); all null / 0 for a fresh hashgraph.  Event
  // indexes on the device are chain positions; chain c's first event has
  // Index chain_base[c] (its Root's SelfParent.Index + 1).
  int32_t *chain_base;     // [n]
  int32_t *lt_seed;        // [n] Root.SelfParent.LamportTimestamp
  int32_t *root_next;      // [n] Root.NextRound
  int32_t *root_sp_round;  // [n] Root.SelfParent.Round
  int8_t *rflag;           // [C] bit 0: the other-parent is the one Root.Others[event] names
  int32_t *ext_lt;         // [C] LamportTimestamp of that Root.Others entry (INT32_MIN: none)
  // The closed form of the round loop holds from round r0 = F + 1 on, F the
  // highest NextRound / SelfParent.Round of a root;
  // k_fiat computes rounds below it event by event.  fw[(r - rlo) * n + c]:
  // chain c's witness of fiat round r (-1: none; its FD row is read from
  // FDT, so the table costs one word per (round, chain) whatever n);
  // rexists[r]: round r < r0 has an event (RoundInfo exists,
  // inmem_store.go:185-191).
  int32_t r0, rlo;
  int32_t *fw;
  int8_t *rexists;
  int32_t frame_lo;  // frames below it are never emitted (Reset: LastConsensusRound's, hashgraph.go:1063-1065)
  int32_t blk_base;  // Block.Index of the first block this handle makes (LastBlockIndex()+1: after a Reset block.Index()+1)
};

__host__ __device__ inline int64_t la_col_stride(const Dev &d) { return d.la_rows + 64; }

// LA[row][col] of chain-major row `row`.  n <= 128 (fd_cols): the dataflow's
// column-major copy, which every coordinate path writes; the pipelined path
// builds the row-major `la` (and FDT) only when a query asks for them.
// Wider: the row-major table (la_col may share FDT's memory there).
__device__ __forceinline__ int32_t la_at(const Dev &d, int64_t row, int col) {
  return d.fd_cols || d.wide_cols ? d.la_col[(int64_t)col * la_col_stride(d) + row] : d.la[row * d.npad + col];
}
// row of (chain c, round r) in the ballot tables ssm / ssw
__host__ __device__ inline int64_t ballot_row(const Dev &d, int c, int r) {
  return (int64_t)c * d.rspan + (r - d.rbase);
}
// row of (chain c, round r) in cla: a ring of cla_span rounds (at most
// CLA_BYTES; C4's 512 x 512 rows would take 61 GB over R_cap = C / SM rounds)
constexpr size_t CLA_BYTES = (size_t)8 << 30;
__host__ __device__ inline int64_t cla_row(const Dev &d, int c, int r) {
  return (int64_t)c * d.cla_span + (r - d.rbase) % d.cla_span;
}
constexpr int32_t RR_DROP = INT32_MIN + 1;  // left UndeterminedEvents with no round received (hashgraph.go:970-977)

// Block projection (kernels_frames.hip, frames.cpp): the
// roots GetFrame gives each frame (hashgraph.go:1125-1231, createRoot
// :546-640), Frame.Marshal -> FrameHash (frame.go:17-41) and Block.Marshal
// -> the block's hash (block.go:100-123, 178-205).  Allocated when
// bh_config.frames is set.  Frames are indexed by round received f; a
// root is (f, p) = f * n + p.
struct Frames {
  uint8_t *hash;                 // [C][32] event hashes (Event.Hex keys, RootEvent.Hash)
  int64_t *pids;                 // [n] participant IDs (RootEvent.CreatorID)
  uint8_t *arena;                // event bytes: Go-JSON bodies (no newline) and Signature strings
  int64_t *body_off, *sig_off;   // [C] offsets into arena
  int32_t *body_len, *sig_len;   // [C], -1 = not given
  int32_t *root_src;             // [R1][n] the event createRoot made root (f, p) from; -1 = base Root
  int32_t *last_pos;             // [n] consensus position of each creator's last consensus event, -1 none
  int32_t *first_pos, *last_in;  // [R1][n] scratch: first / last position of creator p in frame f
  int64_t *oofs;                 // [R1 * n + 1] Others of root g: okey / oval [oofs[g], oofs[g + 1])
  int32_t *okey, *oval;          // Others: key event -> RootEvent of value event, sorted by key hash
  int32_t *ocur;                 // [R1][n] scratch fill cursors
  int64_t *sz, *sz2;             // [max(R1 * n, C) + 1] scratch sizes -> exclusive scans
  int64_t *part;                 // scan partials
  int8_t *missing;               // [R1] scratch: some event of the frame has no bytes
  int64_t *jofs, *bofs;          // [R1 + 1] frame / block JSON offsets (scratch)
  int32_t *jlen, *blen;          // [R1] their lengths
  uint8_t *fhash, *bhash;        // [R1][32] FrameHash / block hash of frame f's block
  int8_t *fvalid;                // [R1] fhash / bhash computed
  uint8_t *dig;                  // [R1][32] scratch digests
  uint8_t *json, *bjson;         // materialized Frame / Block JSON of the last projection
  // A Reset hashgraph's installed Roots (bh_reset with frames; null
  // otherwise): a participant with no consensus event since the Reset keeps
  // its Root whole in every frame (inmem_store.go:136-150 -> GetRoot), a
  // first event's SelfParent RootEvent is its Root's, and an other-parent its
  // creator's Root names (Others[ev] with the same Hash) is that entry
  // (createOtherParentRootEvent, hashgraph.go:568-578).  Others keys / values
  // (okey / oval) >= 0 are events; -2 - k is installed entry k.
  uint8_t *rsp_hash;             // [n][32] Root.SelfParent.Hash (its Index, LT, Round: chain_base - 1, lt_seed, root_sp_round)
  uint8_t *ro_key, *ro_hash;     // [K][32] entry k: the key event's hash, RootEvent.Hash
  int32_t *ro_creator, *ro_index, *ro_lt, *ro_round;  // [K] RootEvent (creator slot, Index, LamportTimestamp, Round)
  int32_t *ro_ofs, *ro_list;     // [n + 1], [K]: Root p's entries, unique keys sorted by key hash
  int32_t *oth_of;               // [C] the entry of the event's creator Root naming its other-parent, -1 none
};
constexpr int32_t NO_FIRST = 0x7f7f7f7f;  // first_pos of a creator absent from the frame (memset 0x7f)

// frames [f0, f0 + F), whose consensus positions are [i0, i1) (frames.cpp)
void launch_frame_roots(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                        int64_t obase, hipStream_t s);
void launch_frame_json_size(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                            hipStream_t s);  // -> jofs[F] = bytes
void launch_frame_json_write(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                             bool store, hipStream_t s);  // -> json, fhash (store)
void launch_block_json_size(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                            hipStream_t s);  // -> bofs[F]
void launch_block_json_write(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                             bool store, hipStream_t s);  // -> bjson, bhash (store)
// FrameHash / block hash of frames [f0, f0 + F) from digests `dig` ([F][32],
// device memory) computed elsewhere (frames.cpp: the host's SHA-256 for a
// call that emits few frames)
void launch_frame_store(const Dev &d, const Frames &fr, int32_t f0, int32_t F, const uint8_t *dig, hipStream_t s);
void launch_block_store(const Dev &d, const Frames &fr, int32_t f0, int32_t F, const uint8_t *dig, hipStream_t s);
// root (f, p) for every p: out[3p] NextRound, out[3p+1] SelfParent event (-1 base), out[3p+2] #Others
void launch_root_query(const Dev &d, const Frames &fr, int32_t f, int32_t *out, hipStream_t s);

enum DiagSlot {
  DG_SW_TOTAL = 0, DG_SW_WAIT_DESC, DG_SW_WAIT_RING, DG_SW_SUBSTEPS, DG_SW_FAR, DG_SW_CHUNKS,
  DG_SW_MEM_PREF, DG_SW_MEM_STORE, DG_SW_MEM_IDLE,
  DG_RD_B = 10, DG_RD_LOAD, DG_RD_COMP, DG_RD_TOTAL, DG_RD_CALLS,
  DG_FL_STEPS = 16, DG_FL_CYC, DG_FL_ADV, DG_FL_FAR, DG_FL_WAITD,
  DG_RD_HMISS = 21, DG_RD_WMISS,  // k_round2: waves whose hand-off searched past its 64 rows; windows without SM
  DG_TL = 32,  // k_round2 timeline: rounds TL_R0 .. TL_R0+TL_NR, [r][c][4] realtime stamps
  DG_TLB = 32 + 64 * 128 * 4,  // persistent loops' barrier phases: [r][c < 512][4] (end, arrived, staged, released)
  DG_TLS = DG_TLB + 64 * 512 * 4,  // k_round_wide's staging of the next window: [r][c][4] (fit loads, fit decided, staged)
  DG_TQ = DG_TLS + 64 * 512 * 4,  // k_round_wide chains < 8: [r][c][66] (T_q bytes of 512 candidates, offsets)
  DG_COUNT = DG_TQ + 64 * 8 * 66
};
constexpr int TL_R0 = 1000, TL_NR = 64;
#ifdef __HIPCC__  // (kernel-side helper; the host files also build with g++ for the host-ASan library)
__device__ __forceinline__ unsigned long long stamp() { return __builtin_amdgcn_s_memtime(); }
#endif

// launchers (kernels_*.hip)
void configure_round_kernels();
void configure_fame_kernels();
void configure_order_kernels();
void configure_coord_kernels();
void configure_flow_kernels();
bool flow_eligible(const Dev &d);
void launch_flow_coordinates(const Dev &d, hipStream_t s);  // LA + LT, chain dataflow
void launch_flow_desc(const Dev &d, hipStream_t s);
void launch_flow(const Dev &d, hipStream_t s);
bool flow32_eligible(const Dev &d);
bool flow32x2_eligible(const Dev &d);  // k_flow32x2: two values per workgroup
const char *flow_kernel(const Dev &d);  // k_flow32x2, k_flow32 or k_flow
void launch_flow_lt_fallback(const Dev &d, hipStream_t s);
void launch_sha256(const uint8_t *data, const int64_t *off, const int32_t *len, int64_t count, uint8_t *out,
                   hipStream_t s);  // kernels_sha.hip
void launch_ecdsa_verify(const uint8_t *hash, const uint8_t *r, const uint8_t *s, const int32_t *key,
                         const uint8_t *pub, int64_t count, uint8_t *ok, hipStream_t st);  // kernels_ecdsa.hip
void launch_flow_transpose(const Dev &d, hipStream_t s);
// the chain dataflow for 128 < n <= 512 (kernels_flow_wide.hip): column-major
// LA + LT rows; LA rows come from launch_flow_transpose, FD from kernels_fd
bool floww_eligible(const Dev &d);
void launch_floww(const Dev &d, hipStream_t s);
const char *floww_kernel(const Dev &d);  // k_floww2 (two values per workgroup) or k_floww
void launch_prep(const Dev &d, hipStream_t s);  // every event: chain table (gap rows -1), loop state
void launch_chain_scatter(const Dev &d, int64_t e_begin, hipStream_t s);  // events [e_begin, N)
void launch_coordinates(const Dev &d, hipStream_t s);  // = chunk_depth + la_sweep
void launch_chunk_depth(const Dev &d, hipStream_t s);
void launch_la_sweep(const Dev &d, hipStream_t s);
void launch_permute(const Dev &d, hipStream_t s);  // sweep slabs -> chain-major LA rows
void launch_round_init(const Dev &d, hipStream_t s);  // hand-off buffers for round 0
// resume the round loop at round ST_RESUME (boundaries B[r0] kept from a
// prefix run): hand-off buffers and loop state for iteration r0
void launch_round_resume(const Dev &d, hipStream_t s);
// ST_RESUME = the last round r whose B[r][q] lie inside the prefix
// (chain_len) for every chain q that grows in the next prefix (next_len;
// null: every chain), so they hold for that prefix; rq[q] = chain q's
// first r with B[r][q] >= len_q (kernels_rounds.hip)
void launch_resume_point(const Dev &d, int32_t R, const int32_t *next_len, hipStream_t s);
// the n <= 128 persistent pipeline's next segment in one launch: the previous
// loop's resume point (d.seg_lo = the previous prefix's lengths, d.chain_len
// this one's), k_round_resume's loop state and k_cand_rows' first candidates
void launch_seg_resume(const Dev &d, hipStream_t s);
// FD entries of a segment's new rows for chains with no event in the segment
void launch_fd_idle(const Dev &d, hipStream_t s);
// the coordinate split's packed blocks (kernels_split.hip): one per
// coordinate shard and segment
constexpr int SPLIT_OV_CAP = 64;  // raw 64-row chunks per block (columns whose chunk spans > 65535)
struct SplitBlock {
  int64_t S = 0, NQ = 0;  // the segment's events; its 64-row chunks per column
  int32_t c0 = 0, ncol = 0;
  int32_t range = 65535;  // largest 16-bit offset (BH_SPLIT_RANGE lowers it to test the overflow slots)
  bool lt_on = false;     // the block carries the segment's LT rows (the LT shard)
  int32_t *hdr = nullptr;
  uint16_t *pay = nullptr;
  int32_t *ovf_count = nullptr, *err = nullptr;  // err[0]: overflow slots exhausted, err[1]: LT clamp (k_flow32)
  int32_t *ovf = nullptr, *lt = nullptr;
};
// byte size of a block (and its pointers from `base` when b is given)
size_t split_layout(int ncol, int64_t S, int64_t NQ, bool lt, SplitBlock *b, uint8_t *base);
// pack (coordinate shard) / unpack (shard 0) the segment view v's rows; pq =
// the segment's [P, Q][n + 1] tables on the device
void launch_split_pack(const Dev &v, const int32_t *pq, const SplitBlock &b, hipStream_t s);
void launch_split_unpack(const Dev &v, const int32_t *pq, const SplitBlock &b, hipStream_t s);
// Lamport timestamps of the segment's events [e0, N) from the chain-major
// LT rows (what the transpose does beside LA / FDT, for a segment whose
// row-major LA and FDT are left unbuilt: n <= 128)
void launch_lt_rows(const Dev &d, hipStream_t s);
void launch_round_iteration(const Dev &d, int parity, hipStream_t s);  // k_round
// n <= 32 on the chain dataflow: the whole loop in one resident workgroup
// (k_round_solo; opt-in with BH_ROUND_SOLO=1, measured A/B)
bool round_solo_eligible(const Dev &d);
bool round2_eligible(const Dev &d);
bool round_persist_eligible(const Dev &d);
bool round_lean_eligible(const Dev &d);  // k_round_lean (float-encoded hand-off, chains < 2^22 - 2) over k_round2p
// the loop that runs on this Dev is k_round_lean: candfd rows in its float
// encoding (fe_encode; the launchers of k_cand_rows / k_seg_resume set it)
bool cand_fe(const Dev &d);
void launch_cand_defe(const Dev &d, hipStream_t s);  // parity-0 candfd rows: fe_encode -> plain
void launch_round_persist(const Dev &d, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
bool round_wide_persist_eligible(const Dev &d);
void launch_round_wide_persist(const Dev &d, hipStream_t s);
void launch_round_solo(const Dev &d, hipStream_t s);
// Reset hashgraphs: coordinates of events [0, d.N) one event at a time (the
// batch whose other-parents only Root.Others knows), and the rounds below r0
// in insertion order with B[r0] for the loop (kernels_reset.hip)
void launch_reset_coords(const Dev &d, hipStream_t s);
void launch_fiat(const Dev &d, hipStream_t s);
void launch_witness_tables(const Dev &d, int R, hipStream_t s);  // wids/wofs/wcnt/wrow
// per-event round / witness; events >= n_prev (inserted since the last
// division) also get their initial fame / rr / consensus position, and are
// marked trapped when they are witnesses of a round < P (already processed)
void launch_assign_rounds(const Dev &d, int64_t e_begin, int64_t n_prev, int32_t P, hipStream_t s);
// DecideFame of rounds [r0, r1) into wfame / decided / nfam / minla
void launch_fame(const Dev &d, int32_t R, int32_t r0, int32_t r1, hipStream_t s);
// wfame -> per-event fame (trapped witnesses stay Undefined); W witnesses
void launch_fame_scatter(const Dev &d, int32_t W, hipStream_t s);
// DecideFame of the rounds [r0, r1): wfame entries [wofs[r0], wofs[r1]) to fame
void launch_fame_scatter_range(const Dev &d, int32_t w0, int32_t w1, hipStream_t s);
void launch_fame_scatter_rounds(const Dev &d, int32_t P, int32_t R, hipStream_t s);  // bounds from wofs on the device
// rr of events still undetermined (rr already set is kept); rounds < P are
// live-decided iff no trapped witness; counters[3] = undetermined after it;
// frame_cnt[r] = events received in r (every r < R)
// (lcr: LastConsensusRound, for the rounds a Reset hashgraph lacks)
void launch_round_received(const Dev &d, int32_t R, int32_t P, int32_t lcr, hipStream_t s);
// frames / order / blocks of rounds [0, P): ST_P holds P (set by the host).
// launch_order_buckets: frame offsets and unsorted frame buckets of every
// frame; launch_order_sort: sort frames [f0, f1), their tx / loaded counts
// and consensus positions
// (frames < P0 were processed by earlier calls: their order stays)
void launch_order_buckets(const Dev &d, int32_t R, int32_t P0, hipStream_t s);
void launch_order_sort(const Dev &d, int32_t f0, int32_t f1, hipStream_t s);
// cons_pos[order[i]] = i for i in [i0, i1) (after frames sorted elsewhere arrive)
void launch_cons_pos(const Dev &d, int64_t i0, int64_t i1, hipStream_t s);
// witnesses of rounds [P0, P1) still Undefined when those rounds were processed
void launch_trap_processed(const Dev &d, int32_t P0, int32_t P1, hipStream_t s);
// k_pack_frames' layout: int32 words, the int64 transaction counts from word pack_ntx_at(k)
__host__ __device__ inline int32_t pack_ntx_at(int32_t k) { return (ST_COUNT + 3 * k + 1) & ~1; }
inline size_t pack_words(int32_t k) { return (size_t)pack_ntx_at(k) + 2 * (size_t)k; }
void launch_pack_frames(const Dev &d, int32_t P0, int32_t k, int32_t *out, hipStream_t s);
// pair predicates for bh_query_events (kernels_query.hip): kind 0 ancestor,
// 1 selfAncestor, 2 see, 3 stronglySee, 4 roundDiff
void launch_query(const Dev &d, int32_t kind, int64_t count, const int64_t *x, const int64_t *y, int32_t *out,
                  hipStream_t s);
void configure_fd_kernels();
void launch_first_descendants(const Dev &d, hipStream_t s, bool walked);
// the 16-bit wide round loop applies (cand16 rows, chains <= P16_MAXLEN)
bool round_p16(const Dev &d);  // fd from la (FDT already written by k_flow_transpose when walked)

}  // namespace bh
