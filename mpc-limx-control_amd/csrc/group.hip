// group.hip -- the multi-GPU group of include/mpcqp.h: one context per device, an RCCL
// communicator over the ranks, and the per-step exchange of the selection records.
//
// Reference side: the per-tick loop of src/mpc_control_fake_state.cpp:108-149 calling
// MPC::run -> computeSupportFootForce (include/MPCController.h:183-196), here over a batch of
// (state, gait candidate) QPs sharded across the GPUs of one node (SURVEY.md 8b ownership, 8e).
//
// Per step and member (rank) r:
//   solve stream      mpcqp_batch_solve_select on the rank's shard -> record rec[p] = [key | U]
//                     (the fused selection of the solve kernels: no selection launch)
//   collective stream waits for the record, ONE ncclAllGather of the records (RCCL; xGMI between
//                     the GPUs of a node), then k_reduce_records -> best: the global minimum key's
//                     record, identical on every rank
// The collective of step s runs beside the solve of step s + 1.  Records alternate between two
// buffers (p = step parity): the solve of step s + 2 waits, on device, for the all-gather of step
// s that read the same buffer.  No host synchronisation inside a step.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/mpcqp.h"

// mpcqp_kernels.hip (library-internal): k_reduce_records on a given stream of the ctx's device
extern "C" int mpcqp_reduce_records_on(mpcqp_ctx *c, void *stream, int n, const int64_t *records,
                                       int64_t *best);

namespace {

struct Member {
    int device = -1;
    int rank = 0;
    mpcqp_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    hipStream_t ss = nullptr;  // solve stream (the context runs on it)
    hipStream_t cs = nullptr;  // collective stream
    int64_t *rec[2] = {nullptr, nullptr};   // [1 + nV] this rank's record, by step parity
    int64_t *gath[2] = {nullptr, nullptr};  // [nranks][1 + nV] the all-gathered records
    hipEvent_t ev_rec = nullptr;            // the step's record is written (solve stream)
    hipEvent_t ev_gath[2] = {nullptr, nullptr};  // the all-gather of parity p has read rec[p]
    bool gath_pending[2] = {false, false};
    hipEvent_t ev_coll = nullptr;  // mpcqp_group_wait
    hipEvent_t ev_in = nullptr;    // mpcqp_group_wait_stream: the caller's inputs are ready
    // host path: device staging [x0 | xref | lin | contact | U | cost | status | iters | best]
    // and its pinned mirror
    char *dbuf = nullptr;
    size_t dcap = 0;
    char *pin = nullptr;
    size_t pcap = 0;
};

int hip_rc(hipError_t e) { return e == hipSuccess ? MPCQP_OK : MPCQP_ERR_DEVICE; }
int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? MPCQP_OK : MPCQP_ERR_DEVICE; }

}  // namespace

struct mpcqp_group {
    mpcqp_model m{};
    int nranks = 0, first = 0, nV = 0, lin_w = 0;
    int par = 0;
    bool whole = false;   // single process: every rank is a local member
    bool failed = false;  // a step failed part-way: communicators aborted, every call refused
    // test transport (MPCQP_GROUP_LOOPBACK=1 at mpcqp_group_create): no RCCL communicator; the
    // all-gather is device copies between the members' buffers, and members may share a device,
    // so the multi-member orchestration (shards, per-member streams, record double-buffering,
    // the cross-rank reduction) runs on a one-GPU machine.  Never for production: RCCL is the
    // transport.
    bool loopback = false;
    long step = 0;        // steps issued
    long inject = -1;     // fault injection (tests): step MPCQP_GROUP_INJECT_FAIL fails part-way
    std::vector<Member> mem;
};

namespace {

// per-member resources after its context exists and its communicator is set up
int member_init(mpcqp_group *g, Member &mb) {
    if (hipSetDevice(mb.device) != hipSuccess) return MPCQP_ERR_DEVICE;
    const size_t rb = sizeof(int64_t) * (1 + (size_t)g->nV);
    if (hipStreamCreateWithFlags(&mb.ss, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&mb.cs, hipStreamNonBlocking) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    int rc = mpcqp_set_stream(mb.ctx, mb.ss);
    if (rc) return rc;
    for (int p = 0; p < 2; ++p)
        if (hipMalloc(&mb.rec[p], rb) != hipSuccess ||
            hipMalloc(&mb.gath[p], rb * g->nranks) != hipSuccess ||
            hipMemset(mb.rec[p], 0, rb) != hipSuccess ||
            hipEventCreateWithFlags(&mb.ev_gath[p], hipEventDisableTiming) != hipSuccess)
            return MPCQP_ERR_DEVICE;
    if (hipEventCreateWithFlags(&mb.ev_rec, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&mb.ev_coll, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&mb.ev_in, hipEventDisableTiming) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    return MPCQP_OK;
}

void member_free(Member &mb) {
    if (mb.device < 0) return;
    hipSetDevice(mb.device);
    if (mb.ss) hipStreamSynchronize(mb.ss);
    if (mb.cs) hipStreamSynchronize(mb.cs);
    if (mb.ctx) mpcqp_ctx_destroy(mb.ctx);  // (does not own ss: mpcqp_set_stream)
    if (mb.comm) ncclCommDestroy(mb.comm);
    for (int p = 0; p < 2; ++p) {
        hipFree(mb.rec[p]);
        hipFree(mb.gath[p]);
        if (mb.ev_gath[p]) hipEventDestroy(mb.ev_gath[p]);
    }
    if (mb.ev_rec) hipEventDestroy(mb.ev_rec);
    if (mb.ev_coll) hipEventDestroy(mb.ev_coll);
    if (mb.ev_in) hipEventDestroy(mb.ev_in);
    hipFree(mb.dbuf);
    if (mb.pin) hipHostFree(mb.pin);
    if (mb.ss) hipStreamDestroy(mb.ss);
    if (mb.cs) hipStreamDestroy(mb.cs);
    mb = Member();
}

// A step that fails after its first enqueue would leave peer ranks blocked in that step's
// all-gather: abort every local communicator (peers' collectives then fail instead of hanging)
// and refuse every later call.  The group must be destroyed on every rank.
int group_fail(mpcqp_group *g) {
    g->failed = true;
    for (auto &mb : g->mem) {
        if (!mb.comm) continue;
        hipSetDevice(mb.device);
        ncclCommAbort(mb.comm);
        mb.comm = nullptr;
    }
    return MPCQP_ERR_DEVICE;
}

mpcqp_group *group_new(const mpcqp_model *m, int nranks) {
    mpcqp_group *g = new (std::nothrow) mpcqp_group();
    if (!g) return nullptr;
    g->m = *m;
    g->m.Q = g->m.R = g->m.P = nullptr;  // host pointers are not kept (the contexts copied them)
    g->nranks = nranks;
    g->nV = m->nu * m->N;
    g->lin_w = m->model == MPCQP_MODEL_DENSE ? m->nx * (m->nx + m->nu) : 8;
    if (const char *e = getenv("MPCQP_GROUP_INJECT_FAIL")) g->inject = atol(e);
    return g;
}

}  // namespace

extern "C" {

int mpcqp_shard(int total_states, int nranks, int rank, int *first_state, int *states) {
    if (!first_state || !states || total_states < 0 || nranks <= 0 || rank < 0 || rank >= nranks)
        return MPCQP_ERR_BAD_ARG;
    const int base = total_states / nranks, rem = total_states % nranks;
    *first_state = rank * base + std::min(rank, rem);
    *states = base + (rank < rem ? 1 : 0);
    return MPCQP_OK;
}

int mpcqp_group_destroy(mpcqp_group *g) {
    if (!g) return MPCQP_ERR_BAD_ARG;
    for (auto &mb : g->mem) member_free(mb);
    delete g;
    return MPCQP_OK;
}

int mpcqp_group_create(const mpcqp_model *m, int ndev, const int *devices, mpcqp_group **out) {
    if (!m || !out || ndev <= 0 || !devices) return MPCQP_ERR_BAD_ARG;
    *out = nullptr;
    const char *lb = getenv("MPCQP_GROUP_LOOPBACK");
    const bool loopback = lb && atoi(lb) == 1;
    for (int i = 0; i < ndev; ++i)
        for (int j = 0; j < i; ++j)
            if (devices[i] == devices[j] && !loopback) return MPCQP_ERR_BAD_ARG;  // one rank per device
    mpcqp_group *g = group_new(m, ndev);
    if (!g) return MPCQP_ERR_DEVICE;
    g->whole = true;
    g->loopback = loopback;
    g->first = 0;
    g->mem.resize(ndev);
    for (int i = 0; i < ndev; ++i) {
        g->mem[i].device = devices[i];
        g->mem[i].rank = i;
        const int rc = mpcqp_ctx_create(m, devices[i], &g->mem[i].ctx);
        if (rc) {
            mpcqp_group_destroy(g);
            return rc;
        }
    }
    if (!loopback) {
        std::vector<ncclComm_t> comms(ndev, nullptr);
        if (ncclCommInitAll(comms.data(), ndev, devices) != ncclSuccess) {
            mpcqp_group_destroy(g);
            return MPCQP_ERR_DEVICE;
        }
        for (int i = 0; i < ndev; ++i) g->mem[i].comm = comms[i];
    }
    for (auto &mb : g->mem) {
        const int rc = member_init(g, mb);
        if (rc) {
            mpcqp_group_destroy(g);
            return rc;
        }
    }
    *out = g;
    return MPCQP_OK;
}

int mpcqp_group_unique_id(unsigned char *uid) {
    if (!uid) return MPCQP_ERR_BAD_ARG;
    static_assert(sizeof(ncclUniqueId) == MPCQP_GROUP_UID_BYTES, "uid size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MPCQP_ERR_DEVICE;
    memcpy(uid, &id, sizeof(id));
    return MPCQP_OK;
}

int mpcqp_group_create_rank(const mpcqp_model *m, int device, int nranks, int rank,
                            const unsigned char *uid, mpcqp_group **out) {
    if (!m || !out || !uid || nranks <= 0 || rank < 0 || rank >= nranks) return MPCQP_ERR_BAD_ARG;
    *out = nullptr;
    mpcqp_group *g = group_new(m, nranks);
    if (!g) return MPCQP_ERR_DEVICE;
    g->whole = nranks == 1;
    g->first = rank;
    g->mem.resize(1);
    Member &mb = g->mem[0];
    mb.device = device;
    mb.rank = rank;
    int rc = mpcqp_ctx_create(m, device, &mb.ctx);
    if (rc) {
        mpcqp_group_destroy(g);
        return rc;
    }
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    hipSetDevice(device);
    if (ncclCommInitRank(&mb.comm, nranks, id, rank) != ncclSuccess) {
        mb.comm = nullptr;
        mpcqp_group_destroy(g);
        return MPCQP_ERR_DEVICE;
    }
    rc = member_init(g, mb);
    if (rc) {
        mpcqp_group_destroy(g);
        return rc;
    }
    *out = g;
    return MPCQP_OK;
}

int mpcqp_group_info(const mpcqp_group *g, int *local, int *nranks, int *first_rank) {
    if (!g) return MPCQP_ERR_BAD_ARG;
    if (local) *local = (int)g->mem.size();
    if (nranks) *nranks = g->nranks;
    if (first_rank) *first_rank = g->first;
    return MPCQP_OK;
}

mpcqp_ctx *mpcqp_group_ctx(mpcqp_group *g, int i) {
    if (!g || i < 0 || i >= (int)g->mem.size()) return nullptr;
    return g->mem[i].ctx;
}

int mpcqp_group_solve_select(mpcqp_group *g, const int *B, const int64_t *base,
                             const double *const *x0, const double *const *xref,
                             const double *const *lin, const uint64_t *const *contact,
                             double *const *U, double *const *cost, int *const *status,
                             int *const *iters, int64_t *const *best) {
    if (!g || !B || !base || !x0 || !xref || !lin || !U || !cost || !status || !iters || !best)
        return MPCQP_ERR_BAD_ARG;
    if (g->failed) return MPCQP_ERR_DEVICE;
    const int n = (int)g->mem.size();
    for (int i = 0; i < n; ++i)
        if (B[i] < 0 || !best[i] || !x0[i] || !xref[i] || !lin[i] || !U[i] || !cost[i] ||
            !status[i] || !iters[i] ||
            (g->m.model == MPCQP_MODEL_SRBM && (!contact || !contact[i])))
            return MPCQP_ERR_BAD_ARG;
    const int p = g->par;
    // from here on a failure is part-way through the step (group_fail)
    // solves (each on its member's solve stream), each followed by "record written"
    for (int i = 0; i < n; ++i) {
        Member &mb = g->mem[i];
        if (hipSetDevice(mb.device) != hipSuccess) return group_fail(g);
        // rec[p] is free once the all-gather two steps back has read it (loopback: every
        // member's copies read it, each on its own collective stream)
        for (int j = 0; j < (g->loopback ? n : 1); ++j) {
            const Member &mj = g->loopback ? g->mem[j] : mb;
            if (mj.gath_pending[p] && hipStreamWaitEvent(mb.ss, mj.ev_gath[p], 0) != hipSuccess)
                return group_fail(g);
        }
        int rc = mpcqp_batch_solve_select(mb.ctx, B[i], x0[i], xref[i], lin[i],
                                          contact ? contact[i] : nullptr, U[i], cost[i],
                                          status[i], iters[i], base[i], mb.rec[p]);
        if (rc) return group_fail(g);
        if (hipEventRecord(mb.ev_rec, mb.ss) != hipSuccess ||
            hipStreamWaitEvent(mb.cs, mb.ev_rec, 0) != hipSuccess)
            return group_fail(g);
    }
    if (g->step++ == g->inject) return group_fail(g);  // (tests: a failure after the solves)
    // ONE all-gather of the records over all ranks (grouped over this process's members)
    const size_t cnt = 1 + (size_t)g->nV;
    int rc = MPCQP_OK;
    if (g->loopback) {
        // (test transport) member i gathers every member's record, after each one is written
        for (int i = 0; i < n && !rc; ++i) {
            Member &mb = g->mem[i];
            hipSetDevice(mb.device);
            for (int j = 0; j < n && !rc; ++j) {
                const Member &mj = g->mem[j];
                rc = hip_rc(hipStreamWaitEvent(mb.cs, mj.ev_rec, 0));
                if (!rc)
                    rc = hip_rc(hipMemcpyAsync(mb.gath[p] + (size_t)j * cnt, mj.rec[p],
                                               sizeof(int64_t) * cnt, hipMemcpyDeviceToDevice,
                                               mb.cs));
            }
        }
    } else {
        if (n > 1 && ncclGroupStart() != ncclSuccess) return group_fail(g);
        for (int i = 0; i < n && !rc; ++i) {
            Member &mb = g->mem[i];
            hipSetDevice(mb.device);
            rc = nccl_rc(ncclAllGather(mb.rec[p], mb.gath[p], cnt, ncclInt64, mb.comm, mb.cs));
        }
        if (n > 1 && ncclGroupEnd() != ncclSuccess) rc = MPCQP_ERR_DEVICE;
    }
    if (rc) return group_fail(g);
    for (int i = 0; i < n; ++i) {
        Member &mb = g->mem[i];
        hipSetDevice(mb.device);
        if (hipEventRecord(mb.ev_gath[p], mb.cs) != hipSuccess) return group_fail(g);
        mb.gath_pending[p] = true;
        rc = mpcqp_reduce_records_on(mb.ctx, mb.cs, g->nranks, mb.gath[p], best[i]);
        if (rc) return group_fail(g);
    }
    g->par ^= 1;
    return MPCQP_OK;
}

int mpcqp_group_wait_stream(mpcqp_group *g, void *const *streams) {
    if (!g || !streams) return MPCQP_ERR_BAD_ARG;
    if (g->failed) return MPCQP_ERR_DEVICE;
    for (size_t i = 0; i < g->mem.size(); ++i) {
        Member &mb = g->mem[i];
        if (hipSetDevice(mb.device) != hipSuccess ||
            hipEventRecord(mb.ev_in, (hipStream_t)streams[i]) != hipSuccess ||
            hipStreamWaitEvent(mb.ss, mb.ev_in, 0) != hipSuccess)
            return MPCQP_ERR_DEVICE;
    }
    return MPCQP_OK;
}

int mpcqp_group_failed(const mpcqp_group *g) { return g && g->failed ? 1 : 0; }

int mpcqp_group_wait(mpcqp_group *g) {
    if (!g) return MPCQP_ERR_BAD_ARG;
    if (g->failed) return MPCQP_ERR_DEVICE;
    for (auto &mb : g->mem) {
        if (hipSetDevice(mb.device) != hipSuccess ||
            hipEventRecord(mb.ev_coll, mb.cs) != hipSuccess ||
            hipStreamWaitEvent(mb.ss, mb.ev_coll, 0) != hipSuccess)
            return MPCQP_ERR_DEVICE;
    }
    return MPCQP_OK;
}

int mpcqp_group_sync(mpcqp_group *g) {
    if (!g) return MPCQP_ERR_BAD_ARG;
    int rc = g->failed ? MPCQP_ERR_DEVICE : MPCQP_OK;
    for (auto &mb : g->mem) {
        hipSetDevice(mb.device);
        if (hipStreamSynchronize(mb.ss) != hipSuccess) rc = MPCQP_ERR_DEVICE;
        if (hipStreamSynchronize(mb.cs) != hipSuccess) rc = MPCQP_ERR_DEVICE;
    }
    return rc;
}

// [p, p + bytes) inside page-locked host memory (mpcqp_host_register / mpcqp_host_alloc)?  The
// same test as the single-context host path's (mpcqp_kernels.hip)
static bool group_host_locked(const void *p, size_t bytes) {
    if (!p || !bytes) return false;
    hipPointerAttribute_t at, at2;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (at.type != hipMemoryTypeHost) return false;
    if (hipPointerGetAttributes(&at2, (const char *)p + bytes - 1) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at2.type == hipMemoryTypeHost;
}

int mpcqp_group_solve_select_host(mpcqp_group *g, int S, int C, const double *x0,
                                  const double *xref, const double *lin, const uint64_t *contact,
                                  double *U, double *cost, int *status, int *iters,
                                  int64_t *best_host) {
    if (!g || !x0 || !xref || !lin || !U || !cost || !status || !iters || !best_host || S < 0 ||
        C <= 0)
        return MPCQP_ERR_BAD_ARG;
    if (g->m.model == MPCQP_MODEL_SRBM && !contact) return MPCQP_ERR_BAD_ARG;
    if (!g->whole) return MPCQP_ERR_BAD_ARG;  // every rank's shard must be local
    if (g->failed) return MPCQP_ERR_DEVICE;
    if ((long long)S * C > 0x7fffffffll) return MPCQP_ERR_BAD_DIMS;
    const int n = (int)g->mem.size();
    const size_t nx = g->m.nx, N = g->m.N, nV = g->nV, lw = g->lin_w;
    // per-instance bytes of each array, in staging order
    const size_t e_x0 = 8 * nx, e_xr = 8 * nx * (N + 1), e_lin = 8 * lw, e_ct = 8;
    const size_t e_u = 8 * nV, e_c = 8, e_s = 4, e_i = 4;
    const size_t e_in = e_x0 + e_xr + e_lin + e_ct, rb = 8 * (1 + nV);
    std::vector<int> Bm(n), s0(n);
    std::vector<int64_t> bm(n);
    std::vector<const double *> px0(n), pxr(n), plin(n);
    std::vector<const uint64_t *> pct(n);
    std::vector<double *> pU(n), pc(n);
    std::vector<int *> ps(n), pi(n);
    std::vector<int64_t *> pb(n);
    std::vector<size_t> off_out(n);
    // the caller's arrays page-locked: each member's shard is DMA'd straight from and into them
    // (no host memcpy through the staging), as mpcqp_batch_solve_host's direct path
    const size_t B_all = (size_t)S * C;
    const bool direct = B_all > 0 && group_host_locked(x0, e_x0 * B_all) &&
                        group_host_locked(xref, e_xr * B_all) && group_host_locked(lin, e_lin * B_all) &&
                        (!contact || group_host_locked(contact, e_ct * B_all)) &&
                        group_host_locked(U, e_u * B_all) && group_host_locked(cost, e_c * B_all) &&
                        group_host_locked(status, e_s * B_all) && group_host_locked(iters, e_i * B_all);
    for (int i = 0; i < n; ++i) {
        Member &mb = g->mem[i];
        int f = 0, ns = 0;
        mpcqp_shard(S, g->nranks, mb.rank, &f, &ns);
        const size_t b = (size_t)ns * C;
        Bm[i] = (int)b;
        s0[i] = f;
        bm[i] = (int64_t)f * C;
        // [inputs | 16-B aligned outputs | record]
        const size_t oo = (e_in * b + 15) & ~(size_t)15;
        const size_t ob = (oo + (e_u + e_c + e_s + e_i) * b + 15) & ~(size_t)15;
        const size_t bytes = ob + rb;
        off_out[i] = oo;
        if (hipSetDevice(mb.device) != hipSuccess) return MPCQP_ERR_DEVICE;
        if (mb.dcap < bytes) {
            hipStreamSynchronize(mb.ss);
            hipStreamSynchronize(mb.cs);
            hipFree(mb.dbuf);
            mb.dbuf = nullptr;
            mb.dcap = 0;
            if (hipMalloc(&mb.dbuf, bytes) != hipSuccess) return MPCQP_ERR_DEVICE;
            mb.dcap = bytes;
        }
        if (mb.pcap < bytes) {
            if (mb.pin) hipHostFree(mb.pin);
            mb.pin = nullptr;
            mb.pcap = 0;
            if (hipHostMalloc(&mb.pin, bytes, hipHostMallocDefault) != hipSuccess)
                return MPCQP_ERR_DEVICE;
            mb.pcap = bytes;
        }
        const size_t i0 = (size_t)f * C;
        char *h = mb.pin, *d = mb.dbuf;
        if (direct) {
            const hipMemcpyKind h2d = hipMemcpyHostToDevice;
            if (b && (hipMemcpyAsync(d, x0 + i0 * nx, e_x0 * b, h2d, mb.ss) != hipSuccess ||
                      hipMemcpyAsync(d + e_x0 * b, xref + i0 * nx * (N + 1), e_xr * b, h2d,
                                     mb.ss) != hipSuccess ||
                      hipMemcpyAsync(d + (e_x0 + e_xr) * b, lin + i0 * lw, e_lin * b, h2d,
                                     mb.ss) != hipSuccess ||
                      (contact && hipMemcpyAsync(d + (e_x0 + e_xr + e_lin) * b, contact + i0,
                                                 e_ct * b, h2d, mb.ss) != hipSuccess)))
                return MPCQP_ERR_DEVICE;
        } else {
            memcpy(h, x0 + i0 * nx, e_x0 * b);
            memcpy(h + e_x0 * b, xref + i0 * nx * (N + 1), e_xr * b);
            memcpy(h + (e_x0 + e_xr) * b, lin + i0 * lw, e_lin * b);
            if (contact) memcpy(h + (e_x0 + e_xr + e_lin) * b, contact + i0, e_ct * b);
            else memset(h + (e_x0 + e_xr + e_lin) * b, 0, e_ct * b);
            if (b && hipMemcpyAsync(d, h, e_in * b, hipMemcpyHostToDevice, mb.ss) != hipSuccess)
                return MPCQP_ERR_DEVICE;
        }
        px0[i] = (const double *)d;
        pxr[i] = (const double *)(d + e_x0 * b);
        plin[i] = (const double *)(d + (e_x0 + e_xr) * b);
        pct[i] = contact ? (const uint64_t *)(d + (e_x0 + e_xr + e_lin) * b) : nullptr;
        pU[i] = (double *)(d + oo);
        pc[i] = (double *)(d + oo + e_u * b);
        ps[i] = (int *)(d + oo + (e_u + e_c) * b);
        pi[i] = (int *)(d + oo + (e_u + e_c + e_s) * b);
        pb[i] = (int64_t *)(d + ob);
    }
    int rc = mpcqp_group_solve_select(g, Bm.data(), bm.data(), px0.data(), pxr.data(),
                                      plin.data(), pct.data(), pU.data(), pc.data(), ps.data(),
                                      pi.data(), pb.data());
    if (rc) return rc;
    rc = mpcqp_group_wait(g);
    if (rc) return rc;
    for (int i = 0; i < n; ++i) {
        Member &mb = g->mem[i];
        hipSetDevice(mb.device);
        const size_t b = (size_t)Bm[i], oo = off_out[i];
        const size_t ob = (oo + (e_u + e_c + e_s + e_i) * b + 15) & ~(size_t)15;
        if (direct) {
            const size_t i0 = (size_t)s0[i] * C;
            const char *d = mb.dbuf + oo;
            const hipMemcpyKind d2h = hipMemcpyDeviceToHost;
            if (b && (hipMemcpyAsync(U + i0 * nV, d, e_u * b, d2h, mb.ss) != hipSuccess ||
                      hipMemcpyAsync(cost + i0, d + e_u * b, e_c * b, d2h, mb.ss) != hipSuccess ||
                      hipMemcpyAsync(status + i0, d + (e_u + e_c) * b, e_s * b, d2h, mb.ss) !=
                          hipSuccess ||
                      hipMemcpyAsync(iters + i0, d + (e_u + e_c + e_s) * b, e_i * b, d2h,
                                     mb.ss) != hipSuccess))
                return MPCQP_ERR_DEVICE;
        } else if (b && hipMemcpyAsync(mb.pin + oo, mb.dbuf + oo, (e_u + e_c + e_s + e_i) * b,
                                       hipMemcpyDeviceToHost, mb.ss) != hipSuccess) {
            return MPCQP_ERR_DEVICE;
        }
        if (i == 0 && hipMemcpyAsync(mb.pin + ob, mb.dbuf + ob, rb, hipMemcpyDeviceToHost,
                                     mb.ss) != hipSuccess)
            return MPCQP_ERR_DEVICE;
    }
    rc = mpcqp_group_sync(g);
    if (rc) return rc;
    for (int i = 0; i < n; ++i) {
        const Member &mb = g->mem[i];
        const size_t b = (size_t)Bm[i], oo = off_out[i], i0 = (size_t)s0[i] * C;
        const char *h = mb.pin + oo;
        if (!direct) {
            memcpy(U + i0 * nV, h, e_u * b);
            memcpy(cost + i0, h + e_u * b, e_c * b);
            memcpy(status + i0, h + (e_u + e_c) * b, e_s * b);
            memcpy(iters + i0, h + (e_u + e_c + e_s) * b, e_i * b);
        }
        if (i == 0) {
            const size_t ob = (oo + (e_u + e_c + e_s + e_i) * b + 15) & ~(size_t)15;
            memcpy(best_host, mb.pin + ob, rb);
        }
    }
    return MPCQP_OK;
}

}  // extern "C"
