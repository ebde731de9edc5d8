// comm.cpp -- the exchange of a multi-process shard group (DESIGN.md
// section 7): one interface, two transports.  The passes call it at the
// same places in the same order on every rank -- rank 0's base broadcast,
// the replicated exchanges' broadcasts per owner, the split's per-segment
// send (coordinate ranks) and receives (rank 0):
//   * RCCL (bh_comm_init): stream-ordered ncclSend / ncclRecv /
//     ncclBroadcast over xGMI on the shard's own communicator, grouped where
//     a rank receives from several peers at once;
//   * a host transport (bh_comm_init_transport): the caller's blocking
//     host-memory send / recv / broadcast, every message staged through
//     pinned memory (the stream is synchronised before a send and after a
//     receive).  It carries the same bytes in the same order, which is what
//     lets a one-GPU box run a multi-process group (RCCL refuses two ranks
//     on one device) and a Go node use links of its own.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "babble_hip.h"
#include "engine.h"
#include "handle.h"

namespace bh {

namespace {

struct RcclComm final : Comm {
  ncclComm_t c = nullptr;
  ~RcclComm() override {
    if (c) (void)ncclCommDestroy(c);
  }
  int bcast(bh_handle *h, void *buf, size_t bytes, int32_t root, hipStream_t s) override {
    if (ncclBroadcast(buf, buf, bytes, ncclChar, root, c, s) != ncclSuccess)
      return h->fail(BH_ERR_DEVICE, "ncclBroadcast (%zu bytes from rank %d)", bytes, root);
    return BH_OK;
  }
  int send(bh_handle *h, const void *buf, size_t bytes, int32_t peer, hipStream_t s) override {
    if (ncclSend(buf, bytes, ncclChar, peer, c, s) != ncclSuccess)
      return h->fail(BH_ERR_DEVICE, "ncclSend (%zu bytes to rank %d)", bytes, peer);
    return BH_OK;
  }
  int recv(bh_handle *h, void *buf, size_t bytes, int32_t peer, hipStream_t s) override {
    if (ncclRecv(buf, bytes, ncclChar, peer, c, s) != ncclSuccess)
      return h->fail(BH_ERR_DEVICE, "ncclRecv (%zu bytes from rank %d)", bytes, peer);
    return BH_OK;
  }
  int group_start(bh_handle *h) override {
    return ncclGroupStart() == ncclSuccess ? BH_OK : h->fail(BH_ERR_DEVICE, "ncclGroupStart");
  }
  int group_end(bh_handle *h) override {
    return ncclGroupEnd() == ncclSuccess ? BH_OK : h->fail(BH_ERR_DEVICE, "ncclGroupEnd");
  }
};

struct HostComm final : Comm {
  bool blocking() const override { return true; }
  bh_transport t{};
  int32_t rank = 0;
  uint8_t *stage = nullptr;  // pinned
  size_t cap = 0;
  ~HostComm() override {
    if (stage) (void)hipHostFree(stage);
  }
  int room(bh_handle *h, size_t bytes) {
    if (bytes <= cap) return BH_OK;
    if (stage) (void)hipHostFree(stage);
    stage = nullptr;
    cap = 0;
    const size_t c = bytes + bytes / 4;
    if (hipHostMalloc((void **)&stage, c, hipHostMallocDefault) != hipSuccess)
      return h->fail(BH_ERR_DEVICE, "host transport: pinned staging of %zu bytes", c);
    cap = c;
    return BH_OK;
  }
  int down(bh_handle *h, const void *buf, size_t bytes, hipStream_t s) {  // device -> staging
    if (hipMemcpyAsync(stage, buf, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return h->fail(BH_ERR_DEVICE, "host transport: staging copy");
    return BH_OK;
  }
  int up(bh_handle *h, void *buf, size_t bytes, hipStream_t s) {  // staging -> device
    if (hipMemcpyAsync(buf, stage, bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return h->fail(BH_ERR_DEVICE, "host transport: staging copy");
    return BH_OK;
  }
  int bcast(bh_handle *h, void *buf, size_t bytes, int32_t root, hipStream_t s) override {
    if (!bytes) return BH_OK;
    int rc;
    if ((rc = room(h, bytes))) return rc;
    if (rank == root && (rc = down(h, buf, bytes, s))) return rc;
    if (t.broadcast(t.ctx, stage, bytes, root) != 0)
      return h->fail(BH_ERR_DEVICE, "host transport: broadcast of %zu bytes from rank %d failed", bytes, root);
    return rank == root ? BH_OK : up(h, buf, bytes, s);
  }
  int send(bh_handle *h, const void *buf, size_t bytes, int32_t peer, hipStream_t s) override {
    if (!bytes) return BH_OK;
    int rc;
    if ((rc = room(h, bytes)) || (rc = down(h, buf, bytes, s))) return rc;
    if (t.send(t.ctx, stage, bytes, peer) != 0)
      return h->fail(BH_ERR_DEVICE, "host transport: send of %zu bytes to rank %d failed", bytes, peer);
    return BH_OK;
  }
  int recv(bh_handle *h, void *buf, size_t bytes, int32_t peer, hipStream_t s) override {
    if (!bytes) return BH_OK;
    int rc;
    if ((rc = room(h, bytes))) return rc;
    // (the stream's earlier work may still read the destination's old
    // bytes: it completes before the copy, which is ordered behind it)
    if (t.recv(t.ctx, stage, bytes, peer) != 0)
      return h->fail(BH_ERR_DEVICE, "host transport: receive of %zu bytes from rank %d failed", bytes, peer);
    return up(h, buf, bytes, s);
  }
};

}  // namespace

Comm *make_rccl_comm(bh_handle *h, int32_t rank, int32_t world, const uint8_t *id) {
  RcclComm *c = new RcclComm;
  ncclUniqueId u;
  memcpy(u.internal, id, sizeof u.internal);
  const ncclResult_t nr = ncclCommInitRank(&c->c, world, u, rank);
  if (nr != ncclSuccess) {
    c->c = nullptr;
    delete c;
    (void)h->fail(BH_ERR_DEVICE, "ncclCommInitRank(%d of %d): %s", rank, world, ncclGetErrorString(nr));
    return nullptr;
  }
  return c;
}

Comm *make_host_comm(const bh_transport &t, int32_t rank) {
  HostComm *c = new HostComm;
  c->t = t;
  c->rank = rank;
  return c;
}

}  // namespace bh
