// frames.cpp -- host side of the block projection: the
// device state of bh_config.frames, the event-bytes arena, the projection
// ProcessDecidedRounds runs on the frames it emits, and the C ABI queries
// (bh_set_event_bytes, bh_get_frame_roots / _json, bh_get_block_hashes /
// _json).  The kernels are in kernels_frames.hip; the algorithm and its
// reference lines are described there.
#include <hip/hip_runtime.h>
#include <openssl/sha.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "babble_hip.h"
#include "engine.h"
#include "handle.h"

namespace {

std::vector<bh_handle *> shards_of(bh_handle *h) {
  return h->group.empty() ? std::vector<bh_handle *>{h} : h->group;
}

// device buffer of at least `need` bytes (+128 B of read slack for the
// SHA-256 block loads), grown geometrically; contents are not kept
int ensure_buf(bh_handle *h, uint8_t **p, size_t *cap, size_t need) {
  need += 128;
  if (need <= *cap && *p) return BH_OK;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const size_t c = std::max(need, *cap * 2);
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIPCHK(h, hipMalloc((void **)p, c));
  *cap = c;
  return BH_OK;
}

int read_i64(bh_handle *h, const int64_t *src, int64_t *out) {
  HIPCHK(h, hipMemcpyAsync(out, src, 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return BH_OK;
}

// Where the SHA-256 digests of the JSON a call just built are computed
// (FrameHash, frame.go:35-41; the block hash, block.go:196-205).  SHA-256 of
// one message is a serial chain of 64-byte compressions: on the device one
// lane hashes one frame at ~20 MB/s (a lone wave issues a dependent VALU op
// every 8 cycles), every frame of the call in parallel; the host's SHA
// extensions (OpenSSL) hash ~2.5 GB/s per thread.  So a call that emits few
// frames -- the live node's schedule, one or two per RunConsensus -- copies
// the device-built JSON to the host and hashes it there, and a call that
// emits thousands (a batch run over a whole DAG) hashes on the device.  The
// choice is by estimated time: device = the longest message / 20 MB/s;
// host = the bytes / (2.5 GB/s x threads) + the copy at 20 GB/s.
// BH_FRAME_HASH=device | host forces one (the tests run both against the
// oracle).  The bytes hashed are the device's either way.
constexpr double DEV_SHA_BPS = 20e6, HOST_SHA_BPS = 2.5e9, D2H_BPS = 20e9;
constexpr int HOST_SHA_THREADS = 8;

bool hash_on_host(const std::vector<int64_t> &ofs, int32_t F) {
  const char *e = getenv("BH_FRAME_HASH");
  if (e && !strcmp(e, "device")) return false;
  if (e && !strcmp(e, "host")) return true;
  int64_t mx = 0;
  for (int32_t j = 0; j < F; ++j) mx = std::max(mx, ofs[(size_t)j + 1] - ofs[(size_t)j]);
  const double total = (double)ofs[(size_t)F];
  const int th = std::max(1, std::min<int>(HOST_SHA_THREADS, F));
  return total / (HOST_SHA_BPS * th) + total / D2H_BPS < (double)mx / DEV_SHA_BPS;
}

// digests of the F messages buf[ofs[j], ofs[j + 1]) (device memory) into
// the device buffer dig ([F][32]), on the host
int host_digests(bh_handle *h, const uint8_t *buf, const std::vector<int64_t> &ofs, int32_t F, uint8_t *dig) {
  const size_t total = (size_t)ofs[(size_t)F];
  if (total > h->host_json_cap) {
    if (h->host_json) (void)hipHostFree(h->host_json);
    h->host_json = nullptr;
    h->host_json_cap = 0;
    HIPCHK(h, hipHostMalloc((void **)&h->host_json, std::max<size_t>(total, 1 << 20), hipHostMallocDefault));
    h->host_json_cap = std::max<size_t>(total, 1 << 20);
  }
  if (total) HIPCHK(h, hipMemcpyAsync(h->host_json, buf, total, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  std::vector<uint8_t> out((size_t)F * 32);
  auto work = [&](int32_t a, int32_t b) {
    for (int32_t j = a; j < b; ++j)
      SHA256(h->host_json + ofs[(size_t)j], (size_t)(ofs[(size_t)j + 1] - ofs[(size_t)j]), out.data() + (size_t)j * 32);
  };
  const int th = std::max(1, std::min<int>(HOST_SHA_THREADS, F));
  if (th == 1) {
    work(0, F);
  } else {
    std::vector<std::thread> ts;
    for (int t = 0; t < th; ++t) ts.emplace_back(work, (int32_t)((int64_t)F * t / th), (int32_t)((int64_t)F * (t + 1) / th));
    for (auto &t : ts) t.join();
  }
  HIPCHK(h, hipMemcpyAsync(dig, out.data(), out.size(), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return BH_OK;
}

int read_offsets(bh_handle *h, const int64_t *src, int32_t F, std::vector<int64_t> *ofs) {
  ofs->resize((size_t)F + 1);
  HIPCHK(h, hipMemcpyAsync(ofs->data(), src, ((size_t)F + 1) * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return BH_OK;
}

// Frame JSON of frames [f0, f0 + F) into fr.json (+ FrameHash when store),
// then, with blocks, the Block JSON into fr.bjson (+ block hash when store)
int project_json(bh_handle *h, int32_t f0, int32_t F, int64_t i0, int64_t i1, bool store, bool blocks) {
  bh::Frames &fr = h->fr;
  const Dev &d = h->d;
  hipStream_t s = h->stream;
  std::vector<int64_t> ofs;
  bh::launch_frame_json_size(d, fr, f0, F, i0, i1, s);
  HIPCHK(h, hipGetLastError());
  if (int rc = read_offsets(h, fr.jofs, F, &ofs)) return rc;
  if (int rc = ensure_buf(h, &fr.json, &h->json_cap, (size_t)ofs[(size_t)F])) return rc;
  const bool fhost = store && hash_on_host(ofs, F);
  bh::launch_frame_json_write(d, fr, f0, F, i0, i1, store && !fhost, s);
  HIPCHK(h, hipGetLastError());
  if (fhost) {
    if (int rc = host_digests(h, fr.json, ofs, F, fr.dig)) return rc;
    bh::launch_frame_store(d, fr, f0, F, fr.dig, s);
  }
  h->hash_host_frames += fhost ? F : 0;
  if (!blocks) {
    HIPCHK(h, hipStreamSynchronize(s));
    return BH_OK;
  }
  bh::launch_block_json_size(d, fr, f0, F, i0, i1, s);
  HIPCHK(h, hipGetLastError());
  if (int rc = read_offsets(h, fr.bofs, F, &ofs)) return rc;
  if (int rc = ensure_buf(h, &fr.bjson, &h->bjson_cap, (size_t)ofs[(size_t)F])) return rc;
  const bool bhost = store && hash_on_host(ofs, F);
  bh::launch_block_json_write(d, fr, f0, F, i0, i1, store && !bhost, s);
  HIPCHK(h, hipGetLastError());
  if (bhost) {
    if (int rc = host_digests(h, fr.bjson, ofs, F, fr.dig)) return rc;
    bh::launch_block_store(d, fr, f0, F, fr.dig, s);
  }
  HIPCHK(h, hipStreamSynchronize(s));
  return BH_OK;
}

// consensus positions of processed frame f
int frame_span(bh_handle *h, int32_t f, int64_t *i0, int64_t *i1) {
  int32_t ofs = 0, cnt = 0;
  HIPCHK(h, hipMemcpyAsync(&ofs, h->d.frame_ofs + f, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipMemcpyAsync(&cnt, h->d.frame_cnt + f, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  *i0 = ofs;
  *i1 = (int64_t)ofs + cnt;
  return BH_OK;
}

}  // namespace

// the device tables of the projection for R1 rounds (and, with a Reset's
// roots, K installed Others entries) into fr; on failure nothing stays
// allocated.  Contents are initialized by frames_init.
int frames_alloc_tables(bh_handle *h, bh::Frames &fr, int64_t R1, int64_t K, bool reset) {
  const int64_t n = h->d.n, C = std::max<int64_t>(h->cap, 1), G = R1 * n;
  const int64_t S = std::max(G, C) + 1;
  int rc = BH_OK;
  auto A = [&](auto **p, int64_t cnt) {
    if (rc == BH_OK) rc = dalloc(h, p, (size_t)cnt);
  };
  A(&fr.hash, C * 32); A(&fr.pids, n);
  A(&fr.body_off, C); A(&fr.sig_off, C); A(&fr.body_len, C); A(&fr.sig_len, C);
  A(&fr.root_src, G); A(&fr.last_pos, n); A(&fr.first_pos, G); A(&fr.last_in, G);
  // Others: at most one per consensus event plus one per root made from a
  // last consensus event, plus a Reset's installed entries in every frame
  // until their participant's first consensus event
  A(&fr.oofs, G + 1); A(&fr.okey, C + G + (reset ? K * R1 : 0)); A(&fr.oval, C + G + (reset ? K * R1 : 0));
  A(&fr.ocur, std::max(G, 3 * n));
  A(&fr.sz, S); A(&fr.sz2, S); A(&fr.part, S / 4096 + 2);
  A(&fr.missing, R1); A(&fr.jofs, R1 + 1); A(&fr.bofs, R1 + 1); A(&fr.jlen, R1); A(&fr.blen, R1);
  A(&fr.fhash, R1 * 32); A(&fr.bhash, R1 * 32); A(&fr.fvalid, R1); A(&fr.dig, R1 * 32);
  if (reset) {
    A(&fr.rsp_hash, n * 32); A(&fr.ro_key, K * 32); A(&fr.ro_hash, K * 32); A(&fr.ro_creator, K);
    A(&fr.ro_index, K); A(&fr.ro_lt, K); A(&fr.ro_round, K); A(&fr.ro_ofs, n + 1); A(&fr.ro_list, K);
    A(&fr.oth_of, C);
  }
  if (rc != BH_OK) frames_free_tables(fr);
  return rc;
}

void frames_free_tables(bh::Frames &fr) {
  void *ptrs[] = {fr.hash, fr.pids, fr.arena, fr.body_off, fr.sig_off, fr.body_len, fr.sig_len, fr.root_src,
                  fr.last_pos, fr.first_pos, fr.last_in, fr.oofs, fr.okey, fr.oval, fr.ocur, fr.sz, fr.sz2,
                  fr.part, fr.missing, fr.jofs, fr.bofs, fr.jlen, fr.blen, fr.fhash, fr.bhash, fr.fvalid,
                  fr.dig, fr.json, fr.bjson, fr.rsp_hash, fr.ro_key, fr.ro_hash, fr.ro_creator, fr.ro_index,
                  fr.ro_lt, fr.ro_round, fr.ro_ofs, fr.ro_list, fr.oth_of};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  fr = bh::Frames{};
}

// the initial contents of a table set for R1 rounds (no event bytes,
// nothing projected) and its 1 MiB JSON buffers: every step that can fail,
// so that bh_reset can prepare a new set before it commits to it
int frames_prepare(bh_handle *h, bh::Frames &fr, int64_t R1, size_t *json_cap, size_t *bjson_cap) {
  const int64_t n = h->d.n, C = std::max<int64_t>(h->cap, 1);
  HIPCHK(h, hipMemcpy(fr.pids, h->pids.data(), (size_t)n * 8, hipMemcpyHostToDevice));
  HIPCHK(h, hipMemset(fr.body_len, 0xff, (size_t)C * 4));
  HIPCHK(h, hipMemset(fr.sig_len, 0xff, (size_t)C * 4));
  if (fr.oth_of) HIPCHK(h, hipMemset(fr.oth_of, 0xff, (size_t)C * 4));
  HIPCHK(h, hipMemset(fr.last_pos, 0xff, (size_t)n * 4));
  HIPCHK(h, hipMemset(fr.oofs, 0, 8));
  HIPCHK(h, hipMemset(fr.fvalid, 0, (size_t)R1));
  HIPCHK(h, hipMemset(fr.fhash, 0, (size_t)R1 * 32));
  HIPCHK(h, hipMemset(fr.bhash, 0, (size_t)R1 * 32));
  const size_t cap = (1 << 20) + 128;
  *json_cap = *bjson_cap = 0;
  int rc;
  if (!fr.json && (rc = dalloc(h, &fr.json, cap))) return rc;
  if (!fr.bjson && (rc = dalloc(h, &fr.bjson, cap))) return rc;
  *json_cap = *bjson_cap = cap;
  return BH_OK;
}

// the handle's tables' initial contents
int frames_init(bh_handle *h) {
  h->arena_cap = h->arena_len = 0;
  h->others_total = 0;
  return frames_prepare(h, h->fr, (int64_t)h->d.R_cap + 1, &h->json_cap, &h->bjson_cap);
}

int frames_alloc(bh_handle *h) {
  int rc;
  if ((rc = frames_alloc_tables(h, h->fr, (int64_t)h->d.R_cap + 1, 0, false))) return rc;
  HIPCHK(h, hipEventCreate(&h->ev_fr[0]));
  HIPCHK(h, hipEventCreate(&h->ev_fr[1]));
  return frames_init(h);
}

void frames_free(bh_handle *h) {
  frames_free_tables(h->fr);
  for (auto &e : h->ev_fr)
    if (e) (void)hipEventDestroy(e);
  if (h->host_json) (void)hipHostFree(h->host_json);
  h->host_json = nullptr;
  h->host_json_cap = 0;
}

// RunConsensus from scratch (bh_reset_consensus): no frame processed yet;
// the event bytes stay (they belong to the events)
void frames_reset(bh_handle *h) {
  bh::Frames &fr = h->fr;
  const int64_t R1 = (int64_t)h->d.R_cap + 1;
  (void)hipMemset(fr.last_pos, 0xff, (size_t)h->d.n * 4);
  (void)hipMemset(fr.oofs, 0, 8);
  (void)hipMemset(fr.fvalid, 0, (size_t)R1);
  (void)hipMemset(fr.fhash, 0, (size_t)R1 * 32);
  (void)hipMemset(fr.bhash, 0, (size_t)R1 * 32);
  h->others_total = 0;
}

int frames_project(bh_handle *h, int32_t P0, int32_t P1, int64_t i0, int64_t i1) {
  const int32_t F = P1 - P0;
  HIPCHK(h, hipEventRecord(h->ev_fr[0], h->stream));
  bh::launch_frame_roots(h->d, h->fr, P0, F, i0, i1, h->others_total, h->stream);
  HIPCHK(h, hipGetLastError());
  if (int rc = read_i64(h, h->fr.oofs + (int64_t)P1 * h->d.n, &h->others_total)) return rc;
  if (int rc = project_json(h, P0, F, i0, i1, true, true)) return rc;
  HIPCHK(h, hipEventRecord(h->ev_fr[1], h->stream));
  HIPCHK(h, hipEventSynchronize(h->ev_fr[1]));
  HIPCHK(h, hipEventElapsedTime(&h->frames_ms, h->ev_fr[0], h->ev_fr[1]));
  return BH_OK;
}

extern "C" {

int bh_set_event_bytes(bh_handle *h, int64_t first, int64_t count, const uint8_t *bodies,
                       const int64_t *body_offsets, const uint8_t *sigs, const int64_t *sig_offsets) {
  if (!h) return BH_ERR_INVALID;
  if (!h->frames_on) return h->fail(BH_ERR_STATE, "bh_set_event_bytes: the handle was created without frames");
  if (count < 0 || first < 0 || (count > 0 && (!bodies || !body_offsets || !sigs || !sig_offsets)))
    return h->fail(BH_ERR_INVALID, "bh_set_event_bytes: null buffer or negative range");
  if (first + count > (int64_t)h->h_creator.size())
    return h->fail(BH_ERR_INVALID, "bh_set_event_bytes: events [%lld, %lld) not inserted", (long long)first,
                   (long long)(first + count));
  if (count == 0) return BH_OK;
  const int64_t b0 = body_offsets[0], s0 = sig_offsets[0];
  const int64_t btot = body_offsets[count] - b0, stot = sig_offsets[count] - s0;
  std::vector<int64_t> boff((size_t)count), soff((size_t)count);
  std::vector<int32_t> blen((size_t)count), slen((size_t)count);
  for (int64_t i = 0; i < count; ++i) {
    const int64_t bl = body_offsets[i + 1] - body_offsets[i], sl = sig_offsets[i + 1] - sig_offsets[i];
    if (bl < 0 || sl < 0 || bl > INT32_MAX / 4 || sl > INT32_MAX / 4)
      return h->fail(BH_ERR_INVALID, "bh_set_event_bytes: offsets not ascending");
    boff[(size_t)i] = body_offsets[i] - b0;
    // the Encoder's newline ends the body's bytes but not the Event's JSON
    blen[(size_t)i] = (int32_t)(bl > 0 && bodies[body_offsets[i + 1] - 1] == '\n' ? bl - 1 : bl);
    soff[(size_t)i] = btot + sig_offsets[i] - s0;
    slen[(size_t)i] = (int32_t)sl;
  }
  for (bh_handle *x : shards_of(h)) {
    HIPCHK(h, hipSetDevice(x->device));
    bh::Frames &fr = x->fr;
    const int64_t need = x->arena_len + btot + stot;
    if (need > x->arena_cap) {  // grow, keeping what is stored
      const int64_t c = std::max<int64_t>({need, 2 * x->arena_cap, 1 << 20});
      uint8_t *na = nullptr;
      HIPCHK(h, hipStreamSynchronize(x->stream));
      HIPCHK(h, hipMalloc((void **)&na, (size_t)c));
      if (x->arena_len) HIPCHK(h, hipMemcpy(na, fr.arena, (size_t)x->arena_len, hipMemcpyDeviceToDevice));
      if (fr.arena) (void)hipFree(fr.arena);
      fr.arena = na;
      x->arena_cap = c;
    }
    const int64_t at = x->arena_len;
    std::vector<int64_t> bo(boff), so(soff);
    for (auto &v : bo) v += at;
    for (auto &v : so) v += at;
    hipStream_t s = x->stream;
    HIPCHK(h, hipMemcpyAsync(fr.arena + at, bodies + b0, (size_t)btot, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipMemcpyAsync(fr.arena + at + btot, sigs + s0, (size_t)stot, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipMemcpyAsync(fr.body_off + first, bo.data(), (size_t)count * 8, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipMemcpyAsync(fr.sig_off + first, so.data(), (size_t)count * 8, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipMemcpyAsync(fr.body_len + first, blen.data(), (size_t)count * 4, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipMemcpyAsync(fr.sig_len + first, slen.data(), (size_t)count * 4, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipStreamSynchronize(s));
    x->arena_len = at + btot + stot;
  }
  HIPCHK(h, hipSetDevice(h->device));
  return BH_OK;
}

int32_t bh_get_frame_roots(bh_handle *h, int32_t rr, int32_t *next_round, int32_t *self_parent, int32_t *n_others,
                           int32_t *other_key, int32_t *other_value, int32_t cap) {
  if (!h) return -BH_ERR_INVALID;
  if (h->no_results()) return -h->fail(BH_ERR_STATE, "results live on rank 0 of a split group");
  if (!h->frames_on) return -h->fail(BH_ERR_STATE, "bh_get_frame_roots: the handle was created without frames");
  if (rr < 0 || rr >= h->P) return -h->fail(BH_ERR_KEY_NOT_FOUND, "GetFrame(%d): not a processed round", rr);
  const int n = h->d.n;
  (void)hipSetDevice(h->device);
  bh::launch_root_query(h->d, h->fr, rr, h->fr.ocur, h->stream);
  std::vector<int32_t> q((size_t)3 * n);
  int64_t o[2];
  if (hipMemcpyAsync(q.data(), h->fr.ocur, q.size() * 4, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
      hipMemcpyAsync(o, h->fr.oofs + (int64_t)rr * n, 8, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
      hipMemcpyAsync(o + 1, h->fr.oofs + (int64_t)(rr + 1) * n, 8, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
      hipStreamSynchronize(h->stream) != hipSuccess)
    return -h->fail(BH_ERR_DEVICE, "bh_get_frame_roots: device copy failed");
  for (int p = 0; p < n; ++p) {
    if (next_round) next_round[p] = q[(size_t)3 * p];
    if (self_parent) self_parent[p] = q[(size_t)3 * p + 1];
    if (n_others) n_others[p] = q[(size_t)3 * p + 2];
  }
  const int64_t tot = o[1] - o[0];
  const int64_t k = std::min<int64_t>(tot, std::max(cap, 0));
  if (k > 0 && other_key && hipMemcpy(other_key, h->fr.okey + o[0], (size_t)k * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return -h->fail(BH_ERR_DEVICE, "bh_get_frame_roots: device copy failed");
  if (k > 0 && other_value && hipMemcpy(other_value, h->fr.oval + o[0], (size_t)k * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return -h->fail(BH_ERR_DEVICE, "bh_get_frame_roots: device copy failed");
  return (int32_t)tot;
}

int64_t bh_get_frame_json(bh_handle *h, int32_t rr, uint8_t *buf, int64_t cap) {
  if (!h) return -BH_ERR_INVALID;
  if (h->no_results()) return -h->fail(BH_ERR_STATE, "results live on rank 0 of a split group");
  if (!h->frames_on) return -h->fail(BH_ERR_STATE, "bh_get_frame_json: the handle was created without frames");
  if (rr < 0 || rr >= h->P) return -h->fail(BH_ERR_KEY_NOT_FOUND, "GetFrame(%d): not a processed round", rr);
  (void)hipSetDevice(h->device);
  int64_t i0, i1;
  if (int rc = frame_span(h, rr, &i0, &i1)) return -rc;
  if (int rc = project_json(h, rr, 1, i0, i1, false, false)) return -rc;
  int64_t o[2];
  int8_t miss = 0;
  if (hipMemcpy(o, h->fr.jofs, 16, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&miss, h->fr.missing, 1, hipMemcpyDeviceToHost) != hipSuccess)
    return -h->fail(BH_ERR_DEVICE, "bh_get_frame_json: device copy failed");
  if (miss) return -h->fail(BH_ERR_STATE, "GetFrame(%d): some event's bytes were not given", rr);
  const int64_t len = o[1] - o[0];
  if (buf && cap > 0 && hipMemcpy(buf, h->fr.json + o[0], (size_t)std::min(len, cap), hipMemcpyDeviceToHost) != hipSuccess)
    return -h->fail(BH_ERR_DEVICE, "bh_get_frame_json: device copy failed");
  return len;
}

int bh_get_block_hashes(bh_handle *h, int64_t first, int64_t count, uint8_t *frame_hash, uint8_t *block_hash,
                        int8_t *valid) {
  if (!h) return BH_ERR_INVALID;
  if (h->no_results()) return h->fail(BH_ERR_STATE, "results live on rank 0 of a split group");
  if (!h->frames_on) return h->fail(BH_ERR_STATE, "bh_get_block_hashes: the handle was created without frames");
  if (first < 0 || count < 0 || first + count > (int64_t)h->blocks.size())
    return h->fail(BH_ERR_INVALID, "bh_get_block_hashes: blocks [%lld, %lld) out of range", (long long)first,
                   (long long)(first + count));
  if (count == 0) return BH_OK;
  (void)hipSetDevice(h->device);
  HIPCHK(h, hipStreamSynchronize(h->stream));
  // blocks are in round-received order: one copy of each per-frame array
  const int32_t r0 = h->blocks[(size_t)first].rr, r1 = h->blocks[(size_t)(first + count - 1)].rr + 1;
  std::vector<int8_t> ok((size_t)(r1 - r0));
  std::vector<uint8_t> fh((size_t)(r1 - r0) * 32), bk((size_t)(r1 - r0) * 32);
  HIPCHK(h, hipMemcpy(ok.data(), h->fr.fvalid + r0, ok.size(), hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemcpy(fh.data(), h->fr.fhash + (int64_t)r0 * 32, fh.size(), hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemcpy(bk.data(), h->fr.bhash + (int64_t)r0 * 32, bk.size(), hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < count; ++i) {
    const size_t f = (size_t)(h->blocks[(size_t)(first + i)].rr - r0);
    if (valid) valid[i] = ok[f];
    if (frame_hash) {
      if (ok[f]) memcpy(frame_hash + 32 * i, fh.data() + 32 * f, 32);
      else memset(frame_hash + 32 * i, 0, 32);
    }
    if (block_hash) {
      if (ok[f]) memcpy(block_hash + 32 * i, bk.data() + 32 * f, 32);
      else memset(block_hash + 32 * i, 0, 32);
    }
  }
  return BH_OK;
}

int64_t bh_get_block_json(bh_handle *h, int64_t b, int32_t body_only, uint8_t *buf, int64_t cap) {
  if (!h) return -BH_ERR_INVALID;
  if (h->no_results()) return -h->fail(BH_ERR_STATE, "results live on rank 0 of a split group");
  if (!h->frames_on) return -h->fail(BH_ERR_STATE, "bh_get_block_json: the handle was created without frames");
  if (b < 0 || b >= (int64_t)h->blocks.size())
    return -h->fail(BH_ERR_KEY_NOT_FOUND, "GetBlock(%lld): no such block", (long long)b);
  (void)hipSetDevice(h->device);
  const Block &bk = h->blocks[(size_t)b];
  int8_t ok = 0;
  if (hipMemcpy(&ok, h->fr.fvalid + bk.rr, 1, hipMemcpyDeviceToHost) != hipSuccess)
    return -h->fail(BH_ERR_DEVICE, "bh_get_block_json: device copy failed");
  if (!ok) return -h->fail(BH_ERR_STATE, "block %lld: some event's bytes were not given", (long long)b);
  if (int rc = project_json(h, bk.rr, 1, bk.first, bk.first + bk.count, false, true)) return -rc;
  int64_t o[2];
  if (hipMemcpy(o, h->fr.bofs, 16, hipMemcpyDeviceToHost) != hipSuccess)
    return -h->fail(BH_ERR_DEVICE, "bh_get_block_json: device copy failed");
  // Block.Marshal = {"Body":<BlockBody JSON>,"Signatures":{}}\n
  static const char HEAD[] = "{\"Body\":", TAIL[] = ",\"Signatures\":{}}\n";
  int64_t at = o[0], len = o[1] - o[0];
  if (body_only) {
    at += sizeof(HEAD) - 1;
    len -= (int64_t)(sizeof(HEAD) - 1 + sizeof(TAIL) - 1);
  }
  const int64_t out = len + (body_only ? 1 : 0);
  if (buf && cap > 0) {
    if (hipMemcpy(buf, h->fr.bjson + at, (size_t)std::min(len, cap), hipMemcpyDeviceToHost) != hipSuccess)
      return -h->fail(BH_ERR_DEVICE, "bh_get_block_json: device copy failed");
    if (body_only && cap > len) buf[len] = '\n';
  }
  return out;
}

}  // extern "C"
