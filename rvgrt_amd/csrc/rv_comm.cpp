// rv_comm.cpp -- host side of librvgrt_hip.so, part 3 of the C ABI (include/rvgrt.h): the communicator of
// the multi-GPU loops -- RCCL resolved at run time from the library the process already uses, or the
// in-process loopback group -- and its entry points (rv_comm_*, rv_loopback_group_*).
#include <dlfcn.h>

#include "rv_host.h"

// ===================================================================== render loop
// RCCL, resolved at run time from the library the process already uses
// (torch's bundled librccl when called from Python: pass its path), so no
// second RCCL/HIP runtime is loaded next to it.
namespace {
struct RcclApi {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;   // optional
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;                   // optional
};
RcclApi g_rccl;

bool rccl_load(const char* path, std::string& err) {
    if (g_rccl.h) return true;
    const char* names[] = {path, "librccl.so.1", "librccl.so"};
    for (const char* n : names) {
        if (!n || !*n) continue;
        g_rccl.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
        if (g_rccl.h) break;
    }
    if (!g_rccl.h) { err = std::string("dlopen librccl: ") + dlerror(); return false; }
    auto sym = [&](const char* n) { return dlsym(g_rccl.h, n); };
    g_rccl.get_unique_id = (decltype(g_rccl.get_unique_id))sym("ncclGetUniqueId");
    g_rccl.comm_init_rank = (decltype(g_rccl.comm_init_rank))sym("ncclCommInitRank");
    g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))sym("ncclCommDestroy");
    g_rccl.send = (decltype(g_rccl.send))sym("ncclSend");
    g_rccl.recv = (decltype(g_rccl.recv))sym("ncclRecv");
    g_rccl.all_gather = (decltype(g_rccl.all_gather))sym("ncclAllGather");
    g_rccl.group_start = (decltype(g_rccl.group_start))sym("ncclGroupStart");
    g_rccl.group_end = (decltype(g_rccl.group_end))sym("ncclGroupEnd");
    g_rccl.error_string = (decltype(g_rccl.error_string))sym("ncclGetErrorString");
    g_rccl.async_error = (decltype(g_rccl.async_error))sym("ncclCommGetAsyncError");
    g_rccl.comm_abort = (decltype(g_rccl.comm_abort))sym("ncclCommAbort");
    if (!g_rccl.get_unique_id || !g_rccl.comm_init_rank || !g_rccl.comm_destroy || !g_rccl.send || !g_rccl.recv ||
        !g_rccl.all_gather || !g_rccl.group_start || !g_rccl.group_end || !g_rccl.error_string) {
        err = "librccl lacks a required symbol";
        g_rccl = RcclApi{};
        return false;
    }
    return true;
}
}  // namespace

RV_HIDDEN double comm_timeout_s() {
    if (const char* e = getenv("RV_COMM_TIMEOUT_S")) {
        char* end = nullptr;
        const double v = strtod(e, &end);
        if (end && *end == '\0' && v > 0) return v;
    }
    return 120.0;
}

RV_HIDDEN void comm_detach(rv_comm* m) { m->ctx = nullptr; }   // its context is being destroyed

#define NCCL_TRY(ctx, expr)                                                                  \
    do {                                                                                     \
        ncclResult_t r_ = (expr);                                                            \
        if (r_ != ncclSuccess)                                                               \
            return fail((ctx), RV_ERR_HIP, std::string(#expr) + ": " + g_rccl.error_string(r_)); \
    } while (0)

static rv_status loop_round(rv_ctx* c, rv_comm* m, hipStream_t s);

// Waits (host) until every stream of the context has drained, polling the
// communicator's asynchronous error; on an error or after timeout_s the
// communicator is aborted and RV_ERR_HIP returned (per-GPU
// timeouts in the multi-GPU driver) -- a dead peer never hangs the caller.
RV_HIDDEN rv_status comm_wait_bounded(rv_ctx* c, rv_comm* m, double timeout_s) {
    std::vector<hipStream_t> ss = {c->stream, c->comm_stream, c->gi_stream};
    for (hipStream_t f : c->fstreams) ss.push_back(f);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        bool busy = false;
        for (hipStream_t s : ss) {
            if (!s && s != c->stream) continue;   // an unused side stream (the caller's may be the NULL stream)
            const hipError_t e = hipStreamQuery(s);
            if (e == hipErrorNotReady) { busy = true; continue; }
            if (e != hipSuccess) return fail(c, RV_ERR_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(e));
        }
        if (!busy) return RV_OK;
        if (m && m->comm && g_rccl.async_error) {
            ncclResult_t ae = ncclSuccess;
            if (g_rccl.async_error(m->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                m->aborted = true;
                if (g_rccl.comm_abort) g_rccl.comm_abort(m->comm);
                return fail(c, RV_ERR_HIP, std::string("RCCL asynchronous error: ") + g_rccl.error_string(ae));
            }
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
            if (m) {
                m->aborted = true;
                if (m->comm && g_rccl.comm_abort) g_rccl.comm_abort(m->comm);
                if (m->loop) m->loop->abort();
            }
            return fail(c, RV_ERR_HIP, "timed out waiting for the frame loop (a peer rank stalled or died)");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

RV_HIDDEN rv_status comm_all_gather(rv_ctx* c, rv_comm* m, const void* send, void* recv, size_t bytes, hipStream_t s) {
    if (m->aborted) return fail(c, RV_ERR_HIP, "communicator aborted");
    if (m->comm) {
        NCCL_TRY(c, g_rccl.all_gather(send, recv, bytes, ncclUint8, m->comm, s));
        return RV_OK;
    }
    m->pending = LoopGroup::Post{};
    m->pending.kind = 1; m->pending.send = send; m->pending.recv = recv; m->pending.bytes = bytes;
    return loop_round(c, m, s);
}

RV_HIDDEN rv_status comm_group_start(rv_ctx* c, rv_comm* m) {
    if (m->aborted) return fail(c, RV_ERR_HIP, "communicator aborted");
    if (m->comm) NCCL_TRY(c, g_rccl.group_start());
    m->in_group = true;
    m->pending = LoopGroup::Post{};
    m->pending.kind = 2;
    return RV_OK;
}

RV_HIDDEN rv_status comm_send(rv_ctx* c, rv_comm* m, const void* buf, size_t bytes, int peer, hipStream_t s) {
    if (m->comm) { NCCL_TRY(c, g_rccl.send(buf, bytes, ncclUint8, peer, m->comm, s)); return RV_OK; }
    m->pending.p2p.emplace_back(1, peer, buf, nullptr, bytes);
    return RV_OK;
}

RV_HIDDEN rv_status comm_recv(rv_ctx* c, rv_comm* m, void* buf, size_t bytes, int peer, hipStream_t s) {
    if (m->comm) { NCCL_TRY(c, g_rccl.recv(buf, bytes, ncclUint8, peer, m->comm, s)); return RV_OK; }
    m->pending.p2p.emplace_back(0, peer, nullptr, buf, bytes);
    return RV_OK;
}

RV_HIDDEN rv_status comm_group_end(rv_ctx* c, rv_comm* m, hipStream_t s) {
    m->in_group = false;
    if (m->comm) { NCCL_TRY(c, g_rccl.group_end()); return RV_OK; }
    return loop_round(c, m, s);
}

// One loopback round (see LoopGroup): post, meet, fetch, meet, release.
static rv_status loop_round(rv_ctx* c, rv_comm* m, hipStream_t s) {
    LoopGroup* g = m->loop;
    if (!m->ready) HIP_TRY(c, hipEventCreateWithFlags(&m->ready, hipEventDisableTiming));
    if (!m->done) HIP_TRY(c, hipEventCreateWithFlags(&m->done, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(m->ready, s));
    m->pending.ready = m->ready; m->pending.done = m->done;
    {
        std::lock_guard<std::mutex> lk(g->m);
        g->post[(size_t)m->rank] = m->pending;
    }
    if (!g->barrier()) { m->aborted = true; return fail(c, RV_ERR_HIP, "loopback: a peer did not arrive (timeout)"); }
    // snapshot of the round: a peer posts its next round only after the second barrier
    std::vector<LoopGroup::Post> post;
    {
        std::lock_guard<std::mutex> lk(g->m);
        post = g->post;
    }
    const LoopGroup::Post& me = post[(size_t)m->rank];
    for (int q = 0; q < g->n; q++) {
        const LoopGroup::Post& o = post[(size_t)q];
        if (o.kind != me.kind) { m->aborted = true; g->abort(); return fail(c, RV_ERR_HIP, "loopback: ranks diverged"); }
    }
    if (me.kind == 1) {   // all-gather: fetch every rank's block
        for (int q = 0; q < g->n; q++) {
            const LoopGroup::Post& o = post[(size_t)q];
            if (o.bytes != me.bytes) { m->aborted = true; g->abort(); return fail(c, RV_ERR_HIP, "loopback: all-gather sizes differ"); }
            if (q != m->rank) HIP_TRY(c, hipStreamWaitEvent(s, o.ready, 0));
            HIP_TRY(c, hipMemcpyAsync(static_cast<char*>(me.recv) + (size_t)q * me.bytes, o.send, me.bytes,
                                      hipMemcpyDeviceToDevice, s));
        }
    } else {              // grouped p2p: every recv fetches the matching send of its peer (k-th with k-th)
        std::vector<int> used((size_t)g->n, 0);
        for (const auto& op : me.p2p) {
            if (std::get<0>(op)) continue;
            const int q = std::get<1>(op);
            if (q < 0 || q >= g->n) { m->aborted = true; g->abort(); return fail(c, RV_ERR_HIP, "loopback: bad peer"); }
            const LoopGroup::Post& o = post[(size_t)q];
            int seen = 0;
            const std::tuple<int, int, const void*, void*, size_t>* match = nullptr;
            for (const auto& so : o.p2p)
                if (std::get<0>(so) && std::get<1>(so) == m->rank && seen++ == used[(size_t)q]) { match = &so; break; }
            if (!match || std::get<4>(*match) != std::get<4>(op)) {
                m->aborted = true; g->abort();
                return fail(c, RV_ERR_HIP, "loopback: send/recv mismatch");
            }
            used[(size_t)q]++;
            if (q != m->rank) HIP_TRY(c, hipStreamWaitEvent(s, o.ready, 0));
            HIP_TRY(c, hipMemcpyAsync(std::get<3>(op), std::get<2>(*match), std::get<4>(op), hipMemcpyDeviceToDevice, s));
        }
    }
    HIP_TRY(c, hipEventRecord(m->done, s));
    if (!g->barrier()) { m->aborted = true; return fail(c, RV_ERR_HIP, "loopback: a peer did not arrive (timeout)"); }
    for (int q = 0; q < g->n; q++)   // my buffers are reusable once every reader's copies ran
        if (q != m->rank) HIP_TRY(c, hipStreamWaitEvent(s, post[(size_t)q].done, 0));
    return RV_OK;
}

extern "C" {

rv_status rv_comm_unique_id(const char* rccl_path, void* id, size_t bytes) {
    if (!id || bytes < sizeof(ncclUniqueId)) return RV_ERR_INVALID;
    std::string err;
    if (!rccl_load(rccl_path, err)) return RV_ERR_HIP;
    ncclUniqueId u;
    if (g_rccl.get_unique_id(&u) != ncclSuccess) return RV_ERR_HIP;
    memcpy(id, &u, sizeof(u));
    return RV_OK;
}

rv_status rv_comm_create(rv_ctx* c, const char* rccl_path, const void* id, size_t bytes, int32_t nranks, int32_t rank,
                         rv_comm** out) {
    if (!c || !id || !out || bytes < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks)
        return RV_ERR_INVALID;
    *out = nullptr;
    std::string err;
    if (!rccl_load(rccl_path, err)) return fail(c, RV_ERR_HIP, err);
    HIP_TRY(c, hipSetDevice(c->device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    rv_comm* m = new rv_comm();
    m->rank = rank; m->nranks = nranks; m->device = c->device; m->ctx = c;
    ncclResult_t r = g_rccl.comm_init_rank(&m->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        delete m;
        return fail(c, RV_ERR_HIP, std::string("ncclCommInitRank: ") + g_rccl.error_string(r));
    }
    *out = m;
    return RV_OK;
}

rv_status rv_loopback_group_create(int32_t nranks, int32_t timeout_ms, void** out) {
    if (nranks < 1 || !out) return RV_ERR_INVALID;
    LoopGroup* g = new LoopGroup();
    g->n = nranks;
    g->post.resize((size_t)nranks);
    if (timeout_ms > 0) g->timeout_s = timeout_ms * 1e-3;
    *out = g;
    return RV_OK;
}

void rv_loopback_group_destroy(void* group) { delete static_cast<LoopGroup*>(group); }

rv_status rv_comm_create_loopback(rv_ctx* c, void* group, int32_t nranks, int32_t rank, rv_comm** out) {
    LoopGroup* g = static_cast<LoopGroup*>(group);
    if (!c || !g || !out || nranks != g->n || rank < 0 || rank >= nranks) return RV_ERR_INVALID;
    rv_comm* m = new rv_comm();
    m->loop = g; m->rank = rank; m->nranks = nranks; m->device = c->device; m->ctx = c;
    *out = m;
    return RV_OK;
}

rv_status rv_comm_wait(rv_comm* m, int32_t timeout_ms) {
    if (!m || !m->ctx) return RV_ERR_INVALID;
    return comm_wait_bounded(m->ctx, m, timeout_ms > 0 ? timeout_ms * 1e-3 : comm_timeout_s());
}

void rv_comm_destroy(rv_comm* m) {
    if (!m) return;
    rv_ctx* c = m->ctx;
    const bool ok = !c || comm_wait_bounded(c, m, comm_timeout_s()) == RV_OK;
    if (c && c->comm_attached == m) c->comm_attached = nullptr;
    if (m->comm) {
        hipSetDevice(m->device);
        if (ok && !m->aborted && g_rccl.comm_destroy) g_rccl.comm_destroy(m->comm);
        else if (g_rccl.comm_abort) g_rccl.comm_abort(m->comm);   // a peer is gone: do not wait for it
    }
    if (m->ready) hipEventDestroy(m->ready);
    if (m->done) hipEventDestroy(m->done);
    if (m->vdev) hipFree(m->vdev);
    if (m->vhost) hipHostFree(m->vhost);
    delete m;
}

}  // extern "C"
