// Multi-GPU collectives of the correction loop over RCCL (include/prgpu.h pr_comm_*),
// linked into libprgpu so a GPU process needs no second runtime (torch is not loaded
// in the product's GPU processes).  One process per GPU; the communicator works on the
// context's stream.
//
// What crosses GPUs: the per-iteration masked-fraction statistic
// {bpt, bpN} (bin/proovread:1702-1720 -> mask_shortcut_frac 2026-2047) as an all-reduce,
// and in the exact-parity layout the seed-extension tasks (all-to-all to the long-read
// owners) and the corrected / masked reads (all-gather for the next iteration's index).
// Host-buffer calls stage through one device buffer and synchronise; device-buffer calls
// are asynchronous on the context stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/prgpu.h"

hipStream_t ctx_stream(pr_ctx *c);
int ctx_device(pr_ctx *c);
int pr_set_error(int code, const char *msg);

static_assert(PR_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
constexpr int64_t P2P_PIECE = (int64_t)1 << 28;   // bytes per ncclSend / ncclRecv

// An in-process group: the ranks are threads of one process, each with its own context (on
// one GPU or several).  The collectives meet at a barrier, publish their buffers and copy
// from each other's (device to device); they are synchronous.  The multi-rank code above the
// communicator (pr_aln_exchange, pr_lrset_commit, the loop) runs unchanged on it, so a
// single-GPU box exercises the world > 1 paths that RCCL runs across GPUs.
struct pr_comm_group {
    int world = 1;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    struct Slot {
        const void *send = nullptr;
        const int64_t *counts = nullptr;
        int64_t n = 0;
        std::vector<uint8_t> host;
    };
    std::vector<Slot> slot;
    bool aborted = false;   // pr_comm_group_abort: a rank left the collective sequence
    // false once the group is aborted (the waiters are woken; later barriers fail at once)
    bool barrier() {
        std::unique_lock<std::mutex> l(m);
        if (aborted) return false;
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        cv.wait(l, [&] { return gen != g || aborted; });
        return gen != g;
    }
    void abort() {
        std::lock_guard<std::mutex> l(m);
        aborted = true;
        cv.notify_all();
    }
};

static int group_aborted() { return pr_set_error(PR_ERR_ARG, "in-process group aborted (another rank failed)"); }

struct pr_comm {
    pr_ctx *ctx = nullptr;
    ncclComm_t nc = nullptr;
    pr_comm_group *grp = nullptr;   // in-process group (pr_comm_init_local) instead of RCCL
    int rank = 0, world = 1;
    void *stage = nullptr;   // device staging buffer for host-buffer collectives
    size_t stage_cap = 0;
};

#define HIPCHK(x)                                                                 \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::string m_ = std::string(#x) + " failed: " + hipGetErrorString(e_); \
            return pr_set_error(PR_ERR_HIP, m_.c_str());                          \
        }                                                                         \
    } while (0)
#define NCCLCHK(x)                                                                  \
    do {                                                                            \
        ncclResult_t r_ = (x);                                                      \
        if (r_ != ncclSuccess) {                                                    \
            std::string m_ = std::string(#x) + " failed: " + ncclGetErrorString(r_); \
            return pr_set_error(PR_ERR_HIP, m_.c_str());                            \
        }                                                                           \
    } while (0)

// (the staging buffer lives on the context's device, whatever the calling thread's current one)
static int stage(pr_comm *c, size_t bytes) {
    HIPCHK(hipSetDevice(ctx_device(c->ctx)));
    if (c->stage && c->stage_cap >= bytes) return 0;
    if (c->stage) (void)hipFree(c->stage);
    c->stage = nullptr;
    c->stage_cap = 0;
    const size_t want = bytes < 4096 ? 4096 : bytes;
    HIPCHK(hipMalloc(&c->stage, want));
    c->stage_cap = want;
    return 0;
}

static ncclDataType_t dtype_of(int dt, size_t *sz) {
    switch (dt) {
        case PR_DT_I64: *sz = 8; return ncclInt64;
        case PR_DT_F64: *sz = 8; return ncclFloat64;
        case PR_DT_I32: *sz = 4; return ncclInt32;
        default: *sz = 1; return ncclUint8;
    }
}

extern "C" int pr_comm_unique_id(uint8_t *id) {
    if (!id) return pr_set_error(PR_ERR_ARG, "null id");
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

extern "C" int pr_comm_init(pr_ctx *ctx, int world, int rank, const uint8_t *id, pr_comm **out) {
    if (!ctx || !out || !id) return pr_set_error(PR_ERR_ARG, "null arg");
    if (world < 1 || rank < 0 || rank >= world) return pr_set_error(PR_ERR_ARG, "bad rank / world size");
    HIPCHK(hipSetDevice(ctx_device(ctx)));
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    pr_comm *c = new pr_comm();
    c->ctx = ctx;
    c->rank = rank;
    c->world = world;
    const ncclResult_t r = ncclCommInitRank(&c->nc, world, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return pr_set_error(PR_ERR_HIP, (std::string("ncclCommInitRank failed: ") + ncclGetErrorString(r)).c_str());
    }
    *out = c;
    return 0;
}

extern "C" int pr_comm_group_create(int world, pr_comm_group **out) {
    if (!out || world < 1) return pr_set_error(PR_ERR_ARG, "bad arg");
    pr_comm_group *g = new pr_comm_group();
    g->world = world;
    g->slot.resize((size_t)world);
    *out = g;
    return 0;
}

extern "C" void pr_comm_group_destroy(pr_comm_group *g) { delete g; }

extern "C" void pr_comm_group_abort(pr_comm_group *g) {
    if (g) g->abort();
}

extern "C" int pr_comm_init_local(pr_ctx *ctx, pr_comm_group *g, int rank, pr_comm **out) {
    if (!ctx || !g || !out) return pr_set_error(PR_ERR_ARG, "null arg");
    if (rank < 0 || rank >= g->world) return pr_set_error(PR_ERR_ARG, "bad rank");
    pr_comm *c = new pr_comm();
    c->ctx = ctx;
    c->grp = g;
    c->rank = rank;
    c->world = g->world;
    *out = c;
    return 0;
}

// the in-process group's collectives (synchronous: each rank's stream is drained first)
static int local_sync(pr_comm *c) {
    HIPCHK(hipSetDevice(ctx_device(c->ctx)));
    HIPCHK(hipStreamSynchronize(ctx_stream(c->ctx)));
    return 0;
}

template <class T> static void reduce_into(T *acc, const T *v, int64_t n, int op) {
    for (int64_t i = 0; i < n; ++i)
        acc[i] = op == PR_RED_MAX ? std::max(acc[i], v[i]) : (op == PR_RED_MIN ? std::min(acc[i], v[i]) : acc[i] + v[i]);
}

static int local_allreduce_host(pr_comm *c, void *buf, int64_t n, int dtype, int op) {
    size_t sz;
    (void)dtype_of(dtype, &sz);
    pr_comm_group *g = c->grp;
    g->slot[(size_t)c->rank].send = buf;
    if (!g->barrier()) return group_aborted();
    std::vector<uint8_t> acc((size_t)n * sz);
    if (n) std::memcpy(acc.data(), g->slot[0].send, acc.size());
    for (int r = 1; r < c->world; ++r) {
        const void *v = g->slot[(size_t)r].send;
        if (dtype == PR_DT_I64) reduce_into((int64_t *)acc.data(), (const int64_t *)v, n, op);
        else if (dtype == PR_DT_F64) reduce_into((double *)acc.data(), (const double *)v, n, op);
        else if (dtype == PR_DT_I32) reduce_into((int32_t *)acc.data(), (const int32_t *)v, n, op);
        else reduce_into(acc.data(), (const uint8_t *)v, n, op);
    }
    if (!g->barrier()) return group_aborted();   // every rank has read every buffer
    if (n) std::memcpy(buf, acc.data(), acc.size());
    return 0;
}

static int local_allreduce_dev(pr_comm *c, const void *dev_in, void *dev_out, int64_t n, int dtype, int op) {
    size_t sz;
    (void)dtype_of(dtype, &sz);
    int rc = local_sync(c);
    if (rc) return rc;
    std::vector<uint8_t> h((size_t)n * sz + 1);
    if (n) HIPCHK(hipMemcpy(h.data(), dev_in, (size_t)n * sz, hipMemcpyDeviceToHost));
    if ((rc = local_allreduce_host(c, h.data(), n, dtype, op))) return rc;
    if (n) HIPCHK(hipMemcpy(dev_out, h.data(), (size_t)n * sz, hipMemcpyHostToDevice));
    return 0;
}

// rank me pulls block `me` of every rank's send buffer (alltoallv: the rank's counts say where
// it sits) or the whole send buffer (allgatherv: counts = nullptr)
static int local_pull(pr_comm *c, const void *send, const int64_t *send_counts, int64_t my_bytes, void *recv,
                      const int64_t *recv_counts) {
    // every rank reaches both barriers, a local failure included (it is reported after them)
    int rc = local_sync(c);
    pr_comm_group *g = c->grp;
    auto &me = g->slot[(size_t)c->rank];
    me.send = rc ? nullptr : send;
    me.counts = send_counts;
    me.n = rc ? -1 : my_bytes;   // -1: this rank failed, its block is not there
    if (!g->barrier()) return group_aborted();
    int64_t o = 0;
    for (int r = 0; r < c->world && !rc; ++r) {
        const auto &p = g->slot[(size_t)r];
        if (p.n < 0) {
            rc = pr_set_error(PR_ERR_ARG, "in-process collective: another rank failed before it");
            break;
        }
        int64_t off = 0, n = p.n;
        if (p.counts) {
            for (int k = 0; k < c->rank; ++k) off += p.counts[k];
            n = p.counts[c->rank];
        }
        if (n != recv_counts[r]) {
            rc = pr_set_error(PR_ERR_ARG, "all-to-all: block size differs from the receive count");
            break;
        }
        if (n && hipMemcpyAsync((uint8_t *)recv + o, (const uint8_t *)p.send + off, (size_t)n, hipMemcpyDefault,
                                ctx_stream(c->ctx)) != hipSuccess)
            rc = pr_set_error(PR_ERR_HIP, "in-process all-to-all copy failed");
        o += n;
    }
    if (!rc && hipStreamSynchronize(ctx_stream(c->ctx)) != hipSuccess) rc = pr_set_error(PR_ERR_HIP, "stream sync");
    if (!g->barrier()) return rc ? rc : group_aborted();   // every rank has finished reading the send buffers
    return rc;
}

extern "C" void pr_comm_destroy(pr_comm *c) {
    if (!c) return;
    (void)hipSetDevice(ctx_device(c->ctx));
    (void)hipStreamSynchronize(ctx_stream(c->ctx));
    if (c->nc) (void)ncclCommDestroy(c->nc);   // (an in-process group is the caller's: pr_comm_group_destroy)
    if (c->stage) (void)hipFree(c->stage);
    delete c;
}

extern "C" int pr_comm_allreduce_dev(pr_comm *c, const void *dev_in, void *dev_out, int64_t n, int dtype, int op) {
    if (!c || (n && (!dev_in || !dev_out)) || n < 0) return pr_set_error(PR_ERR_ARG, "bad arg");
    size_t sz;
    const ncclDataType_t t = dtype_of(dtype, &sz);
    const ncclRedOp_t o = op == PR_RED_MAX ? ncclMax : (op == PR_RED_MIN ? ncclMin : ncclSum);
    if (c->grp) return local_allreduce_dev(c, dev_in, dev_out, n, dtype, op);
    HIPCHK(hipSetDevice(ctx_device(c->ctx)));
    NCCLCHK(ncclAllReduce(dev_in, dev_out, (size_t)n, t, o, c->nc, ctx_stream(c->ctx)));
    return 0;
}

extern "C" int pr_comm_allreduce_host(pr_comm *c, void *buf, int64_t n, int dtype, int op) {
    if (!c || (n && !buf) || n < 0) return pr_set_error(PR_ERR_ARG, "bad arg");
    size_t sz;
    (void)dtype_of(dtype, &sz);
    const size_t bytes = (size_t)n * sz;
    if (c->grp) return local_allreduce_host(c, buf, n, dtype, op);
    int rc = stage(c, bytes);
    if (rc) return rc;
    hipStream_t s = ctx_stream(c->ctx);
    HIPCHK(hipSetDevice(ctx_device(c->ctx)));
    HIPCHK(hipMemcpyAsync(c->stage, buf, bytes, hipMemcpyHostToDevice, s));
    if ((rc = pr_comm_allreduce_dev(c, c->stage, c->stage, n, dtype, op))) return rc;
    HIPCHK(hipMemcpyAsync(buf, c->stage, bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

extern "C" int pr_comm_barrier(pr_comm *c) {
    int64_t one = 1;
    return pr_comm_allreduce_host(c, &one, 1, PR_DT_I64, PR_RED_SUM);
}

// variable-size all-gather: every rank's `nbytes` (all-gathered first), then one padded
// ncclAllGather; recv gets the ranks' blocks back to back, counts[r] their sizes
extern "C" int pr_comm_allgatherv_host(pr_comm *c, const uint8_t *send, int64_t nbytes, uint8_t *recv,
                                       int64_t recv_cap, int64_t *counts) {
    if (!c || nbytes < 0 || (nbytes && !send) || !counts) return pr_set_error(PR_ERR_ARG, "bad arg");
    const int W = c->world;
    std::vector<int64_t> sz((size_t)W, 0);
    sz[(size_t)c->rank] = nbytes;
    int rc = pr_comm_allreduce_host(c, sz.data(), W, PR_DT_I64, PR_RED_SUM);
    if (rc) return rc;
    int64_t cap = 1, tot = 0;
    for (int r = 0; r < W; ++r) {
        counts[r] = sz[(size_t)r];
        cap = sz[(size_t)r] > cap ? sz[(size_t)r] : cap;
        tot += sz[(size_t)r];
    }
    if (!recv) return 0;   // size query
    if (tot > recv_cap) return pr_set_error(PR_ERR_CAPACITY, "all-gather receive buffer too small");
    if (c->grp) {   // in-process: host blocks read directly
        pr_comm_group *g = c->grp;
        g->slot[(size_t)c->rank].send = send;
        if (!g->barrier()) return group_aborted();
        int64_t o = 0;
        for (int r = 0; r < W; o += sz[(size_t)r], ++r)
            if (sz[(size_t)r]) std::memcpy(recv + o, g->slot[(size_t)r].send, (size_t)sz[(size_t)r]);
        if (!g->barrier()) return group_aborted();
        return 0;
    }
    // in pieces of at most P2P_PIECE bytes per rank (one staging area of world + 1 pieces)
    const int64_t piece = std::min<int64_t>((cap + 255) & ~(int64_t)255, P2P_PIECE);
    if ((rc = stage(c, (size_t)piece * (size_t)(W + 1)))) return rc;
    hipStream_t s = ctx_stream(c->ctx);
    uint8_t *mine = (uint8_t *)c->stage + (size_t)piece * (size_t)W;
    uint8_t *all = (uint8_t *)c->stage;
    HIPCHK(hipSetDevice(ctx_device(c->ctx)));
    std::vector<int64_t> o((size_t)W + 1, 0);
    for (int r = 0; r < W; ++r) o[(size_t)r + 1] = o[(size_t)r] + sz[(size_t)r];
    for (int64_t k = 0; k < cap; k += piece) {
        const int64_t mk = std::min<int64_t>(piece, nbytes - k);
        if (mk > 0) HIPCHK(hipMemcpyAsync(mine, send + k, (size_t)mk, hipMemcpyHostToDevice, s));
        NCCLCHK(ncclAllGather(mine, all, (size_t)piece, ncclUint8, c->nc, s));
        for (int r = 0; r < W; ++r) {
            const int64_t n = std::min<int64_t>(piece, sz[(size_t)r] - k);
            if (n > 0) HIPCHK(hipMemcpyAsync(recv + o[(size_t)r] + k, all + (size_t)piece * r, (size_t)n,
                                             hipMemcpyDeviceToHost, s));
        }
        HIPCHK(hipStreamSynchronize(s));   // `mine` / `all` are reused by the next piece
    }
    return 0;
}

// all-to-all of byte blocks: send_counts[r] bytes go to rank r (blocks back to back in
// rank order); recv_counts[r] must equal what rank r sends here (exchange the counts
// first with pr_comm_alltoall_counts).  Point-to-point send/recv pairs in one group.
extern "C" int pr_comm_alltoallv_host(pr_comm *c, const uint8_t *send, const int64_t *send_counts, uint8_t *recv,
                                      const int64_t *recv_counts) {
    if (!c || !send_counts || !recv_counts) return pr_set_error(PR_ERR_ARG, "null arg");
    const int W = c->world;
    int64_t st = 0, rt = 0;
    for (int r = 0; r < W; ++r) {
        if (send_counts[r] < 0 || recv_counts[r] < 0) return pr_set_error(PR_ERR_ARG, "negative count");
        st += send_counts[r];
        rt += recv_counts[r];
    }
    if ((st && !send) || (rt && !recv)) return pr_set_error(PR_ERR_ARG, "null buffer");
    const size_t sa = ((size_t)st + 255) & ~(size_t)255;
    int rc = stage(c, sa + (size_t)rt + 256);
    if (rc) return rc;
    hipStream_t s = ctx_stream(c->ctx);
    uint8_t *ds = (uint8_t *)c->stage, *dr = (uint8_t *)c->stage + sa;
    HIPCHK(hipSetDevice(ctx_device(c->ctx)));
    if (st) HIPCHK(hipMemcpyAsync(ds, send, (size_t)st, hipMemcpyHostToDevice, s));
    if ((rc = pr_comm_alltoallv_dev(c, ds, send_counts, dr, recv_counts))) return rc;
    if (rt) HIPCHK(hipMemcpyAsync(recv, dr, (size_t)rt, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

// all-to-all of device byte blocks (the exact-parity layout's alignment exchange,
// pr_aln_exchange): asynchronous on the context stream, point-to-point pairs in one group
// (xGMI is point to point: every pair of GPUs has its own link)
extern "C" int pr_comm_alltoallv_dev(pr_comm *c, const void *send, const int64_t *send_counts, void *recv,
                                     const int64_t *recv_counts) {
    if (!c || !send_counts || !recv_counts) return pr_set_error(PR_ERR_ARG, "null arg");
    const int W = c->world;
    int64_t st = 0, rt = 0;
    for (int r = 0; r < W; ++r) {
        if (send_counts[r] < 0 || recv_counts[r] < 0) return pr_set_error(PR_ERR_ARG, "negative count");
        st += send_counts[r];
        rt += recv_counts[r];
    }
    if ((st && !send) || (rt && !recv)) return pr_set_error(PR_ERR_ARG, "null buffer");
    if (c->grp) return local_pull(c, send, send_counts, 0, recv, recv_counts);
    hipStream_t s = ctx_stream(c->ctx);
    HIPCHK(hipSetDevice(ctx_device(c->ctx)));
    const uint8_t *ds = (const uint8_t *)send;
    uint8_t *dr = (uint8_t *)recv;
    std::vector<int64_t> so((size_t)W + 1, 0), ro((size_t)W + 1, 0);
    for (int r = 0; r < W; ++r) {
        so[(size_t)r + 1] = so[(size_t)r] + send_counts[r];
        ro[(size_t)r + 1] = ro[(size_t)r] + recv_counts[r];
    }
    // this rank's own block: a device copy (no link involved)
    if (send_counts[c->rank] != recv_counts[c->rank]) return pr_set_error(PR_ERR_ARG, "self block sizes differ");
    if (send_counts[c->rank])
        HIPCHK(hipMemcpyAsync(dr + ro[(size_t)c->rank], ds + so[(size_t)c->rank], (size_t)send_counts[c->rank],
                              hipMemcpyDeviceToDevice, s));
    // the other ranks: send/recv pairs in pieces of at most P2P_PIECE bytes (multi-GB blocks in one
    // ncclSend/ncclRecv came back corrupted at configs[1] size; both sides cut a block the same way)
    NCCLCHK(ncclGroupStart());
    for (int r = 0; r < W; ++r) {
        if (r == c->rank) continue;
        for (int64_t k = 0; k < send_counts[r]; k += P2P_PIECE)
            NCCLCHK(ncclSend(ds + so[(size_t)r] + k, (size_t)std::min<int64_t>(P2P_PIECE, send_counts[r] - k), ncclUint8,
                             r, c->nc, s));
        for (int64_t k = 0; k < recv_counts[r]; k += P2P_PIECE)
            NCCLCHK(ncclRecv(dr + ro[(size_t)r] + k, (size_t)std::min<int64_t>(P2P_PIECE, recv_counts[r] - k), ncclUint8,
                             r, c->nc, s));
    }
    NCCLCHK(ncclGroupEnd());
    return 0;
}

// all-gather of device byte blocks of different sizes (counts[r] = rank r's bytes, known to every
// rank): rank r's block lands at the sum of the earlier counts; point-to-point pairs in pieces
extern "C" int pr_comm_allgatherv_dev(pr_comm *c, const void *send, const int64_t *counts, void *recv) {
    if (!c || !counts) return pr_set_error(PR_ERR_ARG, "null arg");
    const int W = c->world, me = c->rank;
    std::vector<int64_t> o((size_t)W + 1, 0);
    for (int r = 0; r < W; ++r) {
        if (counts[r] < 0) return pr_set_error(PR_ERR_ARG, "negative count");
        o[(size_t)r + 1] = o[(size_t)r] + counts[r];
    }
    if ((counts[me] && !send) || (o[(size_t)W] && !recv)) return pr_set_error(PR_ERR_ARG, "null buffer");
    if (c->grp) return local_pull(c, send, nullptr, counts[me], recv, counts);
    hipStream_t s = ctx_stream(c->ctx);
    HIPCHK(hipSetDevice(ctx_device(c->ctx)));
    uint8_t *dr = (uint8_t *)recv;
    const uint8_t *ds = (const uint8_t *)send;
    if (counts[me] && ds != dr + o[(size_t)me])
        HIPCHK(hipMemcpyAsync(dr + o[(size_t)me], ds, (size_t)counts[me], hipMemcpyDeviceToDevice, s));
    NCCLCHK(ncclGroupStart());
    for (int r = 0; r < W; ++r) {
        if (r == me) continue;
        for (int64_t k = 0; k < counts[me]; k += P2P_PIECE)
            NCCLCHK(ncclSend(ds + k, (size_t)std::min<int64_t>(P2P_PIECE, counts[me] - k), ncclUint8, r, c->nc, s));
        for (int64_t k = 0; k < counts[r]; k += P2P_PIECE)
            NCCLCHK(ncclRecv(dr + o[(size_t)r] + k, (size_t)std::min<int64_t>(P2P_PIECE, counts[r] - k), ncclUint8, r,
                             c->nc, s));
    }
    NCCLCHK(ncclGroupEnd());
    return 0;
}

pr_ctx *comm_ctx(pr_comm *c) { return c ? c->ctx : nullptr; }

// the counts exchange of an all-to-all: recv_counts[r] = what rank r sends to this rank
extern "C" int pr_comm_alltoall_counts(pr_comm *c, const int64_t *send_counts, int64_t *recv_counts) {
    if (!c || !send_counts || !recv_counts) return pr_set_error(PR_ERR_ARG, "null arg");
    const int W = c->world;
    std::vector<int64_t> ones((size_t)W, 8);
    return pr_comm_alltoallv_host(c, (const uint8_t *)send_counts, ones.data(), (uint8_t *)recv_counts, ones.data());
}

// every rank passes its local status; all get 0 only if every rank had 0 (the call every
// multi-rank entry point makes before its first data collective, so that an error on one rank
// returns on all of them instead of leaving the others inside a collective)
extern "C" int pr_comm_agree(pr_comm *c, int local_rc) {
    if (!c) return local_rc;
    const std::string msg = local_rc ? pr_last_error() : "";
    int64_t bad = local_rc != 0;
    const int rc = pr_comm_allreduce_host(c, &bad, 1, PR_DT_I64, PR_RED_MAX);
    if (local_rc) return pr_set_error(local_rc, msg.c_str());
    if (rc) return rc;
    if (bad) return pr_set_error(PR_ERR_ARG, "another rank failed in this multi-rank call");
    return 0;
}

extern "C" int pr_comm_rank(const pr_comm *c, int *rank, int *world) {
    if (!c) return pr_set_error(PR_ERR_ARG, "null comm");
    if (rank) *rank = c->rank;
    if (world) *world = c->world;
    return 0;
}
