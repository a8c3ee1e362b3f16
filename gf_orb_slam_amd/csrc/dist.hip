// Multi-GPU start-up exchange: one process per
// GPU, an RCCL communicator over xGMI, and broadcasts from rank 0 of the
// state every sequence shares — the ORB vocabulary (DBoW2 tree, device
// arrays; TemplatedVocabulary.h:1469-1536 is the layout it replaces on disk)
// and the local map of each stream. Sequences are independent afterwards:
// nothing is exchanged per frame. The reference has no distributed layer
// (single process, main.cc:92-157); this is the one exchange step the batched
// path adds.
#include <rccl/rccl.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "common.h"

// Transports behind the same entry points:
// - RCCL (gf_dist_init): one process per GPU, the product path of config 5;
// - loopback (gf_dist_init_loopback): the ranks are host threads of one
//   process sharing a gf_dist_channel; a broadcast is a rendezvous of all
//   ranks and a device-to-device copy from the root's buffer. It runs the
//   receiving side of every exchange (vocabulary header decode and
//   allocation, the map's reset) on one GPU;
// - host-staged (gf_dist_init_host): device -> host, a caller-supplied
//   collective on host memory (e.g. a torch.distributed gloo group), host ->
//   device; several processes may share one GPU.
struct gf_dist_channel {
    std::mutex m;
    std::condition_variable cv;
    int world = 1, arrived = 0;
    unsigned gen = 0;
    bool broken = false;
    std::vector<void*> ptr;
    std::vector<size_t> bytes;
};

struct gf_dist {
    gf_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    int transport = GF_DIST_RCCL;
    gf_dist_channel* ch = nullptr;
    gf_dist_host_fn fn = nullptr;
    void* user = nullptr;
    std::vector<uint8_t> host;
};

namespace {
constexpr int LOOPBACK_TIMEOUT_S = 120;

// all ranks of the channel arrive before any leaves; false on a timeout (a
// rank that never came), which breaks the channel for every later call
bool lb_barrier(gf_dist_channel* ch) {
    std::unique_lock<std::mutex> lk(ch->m);
    if (ch->broken) return false;
    const unsigned g = ch->gen;
    if (++ch->arrived == ch->world) {
        ch->arrived = 0;
        ch->gen++;
        ch->cv.notify_all();
        return true;
    }
    if (!ch->cv.wait_for(lk, std::chrono::seconds(LOOPBACK_TIMEOUT_S), [&] { return ch->gen != g || ch->broken; }) ||
        ch->broken) {
        ch->broken = true;
        ch->cv.notify_all();
        return false;
    }
    return true;
}

int lb_post(gf_dist* d, void* buf, size_t bytes) {
    // the buffer's producers on this rank's stream finish first (RCCL orders
    // the broadcast after them on the stream)
    const hipError_t e = hipStreamSynchronize(d->ctx->stream);
    {
        std::lock_guard<std::mutex> lk(d->ch->m);
        d->ch->ptr[d->rank] = buf;
        d->ch->bytes[d->rank] = bytes;
        if (e != hipSuccess) {  // the other ranks are released at once instead of timing out
            d->ch->broken = true;
            d->ch->cv.notify_all();
        }
    }
    if (e != hipSuccess) return gf::fail(GF_ERR_HIP, std::string("loopback transport: ") + hipGetErrorString(e));
    if (!lb_barrier(d->ch)) return gf::fail(GF_ERR_HIP, "loopback transport: a rank did not arrive");
    return GF_OK;
}

int lb_bcast(gf_dist* d, void* buf, size_t bytes, int root) {
    int rc = lb_post(d, buf, bytes);
    if (rc) return rc;
    gf_dist_channel* ch = d->ch;
    if (ch->bytes[root] != bytes) {
        (void)lb_barrier(ch);
        return gf::fail(GF_ERR_ARG, "loopback broadcast: byte counts differ between ranks");
    }
    hipError_t e = hipSuccess;
    if (d->rank != root && bytes) {
        e = hipMemcpyAsync(buf, ch->ptr[root], bytes, hipMemcpyDeviceToDevice, d->ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(d->ctx->stream);
    }
    // the root's buffer stays untouched until every receiver has copied it
    if (!lb_barrier(ch)) return gf::fail(GF_ERR_HIP, "loopback transport: a rank did not arrive");
    GF_HIP(e);
    return GF_OK;
}

void reduce_host(double* acc, const double* x, size_t n, int op) {
    for (size_t i = 0; i < n; i++)
        acc[i] = op == 0 ? acc[i] + x[i] : op == 1 ? (x[i] > acc[i] ? x[i] : acc[i]) : (x[i] < acc[i] ? x[i] : acc[i]);
}

int lb_allreduce(gf_dist* d, double* buf, size_t n, int op) {
    int rc = lb_post(d, buf, 8 * n);
    if (rc) return rc;
    gf_dist_channel* ch = d->ch;
    bool ok = true;
    for (int r = 0; r < ch->world; r++) ok = ok && ch->bytes[r] == 8 * n;
    // every rank reduces the same rank-ordered sequence, then writes its own buffer
    std::vector<double> acc(n), x(n);
    hipError_t e = hipSuccess;
    for (int r = 0; ok && r < ch->world && e == hipSuccess; r++) {
        e = hipMemcpy(r ? x.data() : acc.data(), ch->ptr[r], 8 * n, hipMemcpyDeviceToHost);
        if (r) reduce_host(acc.data(), x.data(), n, op);
    }
    if (!lb_barrier(ch)) return gf::fail(GF_ERR_HIP, "loopback transport: a rank did not arrive");
    if (!ok) return gf::fail(GF_ERR_ARG, "loopback all-reduce: lengths differ between ranks");
    GF_HIP(e);
    GF_HIP(hipMemcpy(buf, acc.data(), 8 * n, hipMemcpyHostToDevice));
    return GF_OK;
}

int host_call(gf_dist* d, int op, void* buf, size_t bytes, int root, bool send, bool recv) {
    // a local HIP failure still joins the collective (the peers would
    // otherwise wait for the callback's own timeout); the error is returned after it
    hipError_t e = hipStreamSynchronize(d->ctx->stream);
    if (d->host.size() < bytes) d->host.resize(bytes);
    if (e == hipSuccess && send && bytes) e = hipMemcpy(d->host.data(), buf, bytes, hipMemcpyDeviceToHost);
    const int r = d->fn(d->user, op, d->host.data(), bytes, root);
    if (e != hipSuccess) return gf::fail(GF_ERR_HIP, std::string("host-staged transport: ") + hipGetErrorString(e));
    if (r) return gf::fail(GF_ERR_HIP, "host-staged transport: the collective callback returned " + std::to_string(r));
    if (recv && bytes) GF_HIP(hipMemcpy(buf, d->host.data(), bytes, hipMemcpyHostToDevice));
    return GF_OK;
}
}  // namespace

namespace gf {
int dist_bcast(gf_dist* d, void* buf, size_t bytes, int root) {
    if (d->transport == GF_DIST_LOOPBACK) return lb_bcast(d, buf, bytes, root);
    if (!bytes) return GF_OK;
    if (d->transport == GF_DIST_HOST)
        return host_call(d, GF_DIST_OP_BCAST, buf, bytes, root, d->rank == root, d->rank != root);
    ncclResult_t r = ncclBroadcast(buf, buf, bytes, ncclUint8, root, d->comm, d->ctx->stream);
    if (r != ncclSuccess) return fail(GF_ERR_HIP, std::string("ncclBroadcast: ") + ncclGetErrorString(r));
    return GF_OK;
}
int dist_rank(gf_dist* d) { return d->rank; }
gf_ctx* dist_ctx(gf_dist* d) { return d->ctx; }
}  // namespace gf

extern "C" {

int gf_dist_unique_id(uint8_t* id) {
    GF_CHECK(id, GF_ERR_ARG, "null id");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return gf::fail(GF_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return GF_OK;
}

int gf_dist_init(gf_ctx* ctx, int rank, int world, const uint8_t* id, gf_dist** out) {
    GF_CHECK(ctx && id && out, GF_ERR_ARG, "null arg");
    GF_CHECK(world >= 1 && rank >= 0 && rank < world, GF_ERR_ARG, "bad rank / world");
    GF_HIP(hipSetDevice(ctx->device));
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    gf_dist* d = new gf_dist();
    d->ctx = ctx;
    d->rank = rank;
    d->world = world;
    ncclResult_t r = ncclCommInitRank(&d->comm, world, u, rank);
    if (r != ncclSuccess) {
        delete d;
        return gf::fail(GF_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    *out = d;
    return GF_OK;
}

int gf_dist_destroy(gf_dist* d) {
    if (!d) return GF_OK;
    (void)hipSetDevice(d->ctx->device);
    (void)hipStreamSynchronize(d->ctx->stream);
    if (d->comm) ncclCommDestroy(d->comm);
    delete d;
    return GF_OK;
}

int gf_dist_channel_create(int world, gf_dist_channel** out) {
    GF_CHECK(out && world >= 1, GF_ERR_ARG, "bad arg");
    gf_dist_channel* ch = new gf_dist_channel();
    ch->world = world;
    ch->ptr.assign(world, nullptr);
    ch->bytes.assign(world, 0);
    *out = ch;
    return GF_OK;
}

int gf_dist_channel_destroy(gf_dist_channel* ch) {
    delete ch;
    return GF_OK;
}

int gf_dist_init_loopback(gf_ctx* ctx, int rank, gf_dist_channel* ch, gf_dist** out) {
    GF_CHECK(ctx && ch && out, GF_ERR_ARG, "null arg");
    GF_CHECK(rank >= 0 && rank < ch->world, GF_ERR_ARG, "bad rank");
    gf_dist* d = new gf_dist();
    d->ctx = ctx;
    d->rank = rank;
    d->world = ch->world;
    d->transport = GF_DIST_LOOPBACK;
    d->ch = ch;
    *out = d;
    return GF_OK;
}

int gf_dist_init_host(gf_ctx* ctx, int rank, int world, gf_dist_host_fn fn, void* user, gf_dist** out) {
    GF_CHECK(ctx && fn && out, GF_ERR_ARG, "null arg");
    GF_CHECK(world >= 1 && rank >= 0 && rank < world, GF_ERR_ARG, "bad rank / world");
    gf_dist* d = new gf_dist();
    d->ctx = ctx;
    d->rank = rank;
    d->world = world;
    d->transport = GF_DIST_HOST;
    d->fn = fn;
    d->user = user;
    *out = d;
    return GF_OK;
}

int gf_dist_transport(gf_dist* d, int* transport) {
    GF_CHECK(d && transport, GF_ERR_ARG, "null arg");
    *transport = d->transport;
    return GF_OK;
}

int gf_dist_bcast(gf_dist* d, void* d_buf, size_t bytes, int root) {
    GF_CHECK(d && (d_buf || !bytes), GF_ERR_ARG, "null arg");
    GF_CHECK(root >= 0 && root < d->world, GF_ERR_ARG, "bad root");
    GF_HIP(hipSetDevice(d->ctx->device));
    int rc = gf::dist_bcast(d, d_buf, bytes, root);
    if (rc) return rc;
    GF_HIP(hipStreamSynchronize(d->ctx->stream));
    return GF_OK;
}

int gf_dist_allreduce(gf_dist* d, double* d_buf, size_t n, int op) {
    GF_CHECK(d && (d_buf || !n), GF_ERR_ARG, "null arg");
    GF_CHECK(op >= 0 && op <= 2, GF_ERR_ARG, "op: 0 sum, 1 max, 2 min");
    GF_HIP(hipSetDevice(d->ctx->device));
    if (d->transport == GF_DIST_LOOPBACK) return lb_allreduce(d, d_buf, n, op);
    if (d->transport == GF_DIST_HOST) return n ? host_call(d, GF_DIST_OP_SUM + op, d_buf, 8 * n, -1, true, true) : GF_OK;
    const ncclRedOp_t o = op == 0 ? ncclSum : op == 1 ? ncclMax : ncclMin;
    ncclResult_t r = ncclAllReduce(d_buf, d_buf, n, ncclFloat64, o, d->comm, d->ctx->stream);
    if (r != ncclSuccess) return gf::fail(GF_ERR_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    GF_HIP(hipStreamSynchronize(d->ctx->stream));
    return GF_OK;
}

int gf_dist_info(gf_dist* d, int* rank, int* world) {
    GF_CHECK(d, GF_ERR_ARG, "null dist");
    if (rank) *rank = d->rank;
    if (world) *world = d->world;
    return GF_OK;
}

}  // extern "C"
