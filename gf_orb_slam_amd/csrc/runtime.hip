// libgfslam runtime: error reporting and per-thread contexts (one HIP stream each).
#include <string.h>

#include <algorithm>
#include <string>

#include "common.h"

namespace gf {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int ws_get(gf_ctx* ctx, int slot, size_t bytes, void** out) {
    GF_CHECK(slot >= 0 && slot < gf_ctx::kSlots, GF_ERR_ARG, "bad scratch slot");
    if (bytes == 0) bytes = 16;
    if (ctx->ws_size[slot] < bytes) {
        GF_CHECK(ctx->ws_pinned == 0, GF_ERR_ARG,
                 "scratch slot " + std::to_string(slot) +
                     " would grow while a captured front-end graph holds it: use another context for this call");
        if (ctx->ws[slot]) GF_HIP(hipFree(ctx->ws[slot]));
        ctx->ws[slot] = nullptr;
        ctx->ws_size[slot] = 0;
        size_t sz = bytes + bytes / 2;
        GF_HIP(hipMalloc(&ctx->ws[slot], sz));
        ctx->ws_size[slot] = sz;
    }
    *out = ctx->ws[slot];
    return GF_OK;
}

static hipEvent_t pool_event(gf_ctx* ctx) {
    hipEvent_t e = nullptr;
    if (!ctx->event_pool.empty()) {
        e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
        e = nullptr;
    }
    return e;
}

static thread_local ProfScope* tl_scope = nullptr;

ProfScope::ProfScope(gf_ctx* c, hipStream_t st, const char* name) : ctx(c), s(st) {
    if (!ctx || !ctx->prof) return;
    for (size_t i = 0; i < ctx->prof_entries.size(); i++)
        if (ctx->prof_entries[i].name == name) idx = (int)i;
    if (idx < 0) {
        ctx->prof_entries.push_back(ProfEntry{name, {}, {}});
        idx = (int)ctx->prof_entries.size() - 1;
    }
    prev = tl_scope;
    tl_scope = this;
}

ProfScope::~ProfScope() {
    if (idx < 0) return;
    tl_scope = prev;
    if (first && last) {
        ctx->prof_entries[idx].start.push_back(first);
        ctx->prof_entries[idx].stop.push_back(last);
    }
}

bool prof_launch_events(hipEvent_t* start, hipEvent_t* stop) {
    ProfScope* sc = tl_scope;
    if (!sc || sc->idx < 0) return false;
    hipEvent_t e = pool_event(sc->ctx);
    if (!e) return false;
    if (!sc->first) {
        hipEvent_t e0 = pool_event(sc->ctx);
        if (!e0) {
            sc->ctx->event_pool.push_back(e);
            return false;
        }
        sc->first = e0;
        *start = e0;
    } else {
        *start = nullptr;
        sc->ctx->prof_spent.push_back(sc->last);  // only the scope's last stop is read; pooled at reset
    }
    sc->last = e;
    *stop = e;
    return true;
}

int ws_upload(gf_ctx* ctx, int slot, const void* host, size_t bytes, void** out) {
    int rc = ws_get(ctx, slot, bytes, out);
    if (rc) return rc;
    if (host && bytes) GF_HIP(hipMemcpyAsync(*out, host, bytes, hipMemcpyHostToDevice, ctx->stream));
    return GF_OK;
}
}  // namespace gf

extern "C" {

int gf_version(void) { return 1; }

const char* gf_last_error(void) { return gf::g_err.c_str(); }

int gf_device_count(int* n) {
    GF_CHECK(n, GF_ERR_ARG, "null n");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = (e == hipSuccess) ? c : 0;
    return GF_OK;
}

int gf_ctx_create(int hip_device, gf_ctx** out) {
    GF_CHECK(out, GF_ERR_ARG, "null out");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return gf::fail(GF_ERR_NODEV, "no HIP device");
    GF_CHECK(hip_device >= 0 && hip_device < n, GF_ERR_ARG, "bad device index");
    GF_HIP(hipSetDevice(hip_device));
    gf_ctx* c = new gf_ctx();
    c->device = hip_device;
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, hip_device) == hipSuccess && ncu > 0)
            c->num_cus = ncu;
    }
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return gf::fail(GF_ERR_HIP, hipGetErrorString(e));
    }
    *out = c;
    return GF_OK;
}

int gf_ctx_destroy(gf_ctx* ctx) {
    if (!ctx) return GF_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (int i = 0; i < gf_ctx::kSlots; i++)
        if (ctx->ws[i]) (void)hipFree(ctx->ws[i]);
    for (auto& e : ctx->prof_entries) {
        for (auto ev : e.start) (void)hipEventDestroy(ev);
        for (auto ev : e.stop) (void)hipEventDestroy(ev);
    }
    for (auto ev : ctx->event_pool) (void)hipEventDestroy(ev);
    for (auto ev : ctx->prof_spent) (void)hipEventDestroy(ev);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return GF_OK;
}

int gf_ctx_stream(gf_ctx* ctx, void** stream) {
    GF_CHECK(ctx && stream, GF_ERR_ARG, "null arg");
    *stream = (void*)ctx->stream;
    return GF_OK;
}

int gf_prof_enable(gf_ctx* ctx, int on) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    ctx->prof = on != 0;
    return GF_OK;
}

int gf_prof_reset(gf_ctx* ctx) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    GF_HIP(hipSetDevice(ctx->device));
    GF_HIP(hipDeviceSynchronize());
    for (auto& e : ctx->prof_entries) {
        for (auto ev : e.start) ctx->event_pool.push_back(ev);
        for (auto ev : e.stop) ctx->event_pool.push_back(ev);
    }
    for (auto ev : ctx->prof_spent) ctx->event_pool.push_back(ev);
    ctx->prof_spent.clear();
    ctx->prof_entries.clear();
    return GF_OK;
}

int gf_prof_report(gf_ctx* ctx, int idx, char* name, int name_cap, double* total_ms, int* launches) {
    GF_CHECK(ctx && total_ms && launches, GF_ERR_ARG, "null arg");
    GF_CHECK(idx >= 0 && idx < (int)ctx->prof_entries.size(), GF_ERR_ARG, "no such profile entry");
    GF_HIP(hipSetDevice(ctx->device));
    const gf::ProfEntry& e = ctx->prof_entries[idx];
    double tot = 0;
    size_t n = std::min(e.start.size(), e.stop.size());
    for (size_t i = 0; i < n; i++) {
        GF_HIP(hipEventSynchronize(e.stop[i]));
        float ms = 0;
        GF_HIP(hipEventElapsedTime(&ms, e.start[i], e.stop[i]));
        tot += ms;
    }
    *total_ms = tot;
    *launches = (int)n;
    if (name && name_cap > 0) {
        size_t k = std::min((size_t)name_cap - 1, e.name.size());
        memcpy(name, e.name.data(), k);
        name[k] = 0;
    }
    return GF_OK;
}

int gf_ctx_sync(gf_ctx* ctx) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    GF_HIP(hipSetDevice(ctx->device));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

}  // extern "C"
