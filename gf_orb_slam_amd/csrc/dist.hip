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

#include "common.h"

struct gf_dist {
    gf_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
};

namespace gf {
int dist_bcast(gf_dist* d, void* buf, size_t bytes, int root) {
    if (!bytes) return GF_OK;
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
