// shard.hip -- the column-sharded BB iteration of one rank, enqueued from C++
// with its RCCL collectives in the same loop (include/bsls_hip.h
// bsls_bb_shard_iterate).  The schedule is distributed.ShardedBB's (python),
// the orchestration the gloo tests pin against the oracle (fuse 2, default):
//     stage 10  K2 (g_g, the four local BB sums) + this rank's 1/world slice
//               of ||r||^2 (r is the same all-reduced vector on every rank)
//     RCCL      all-reduce(sum) of scal[SUMDG..RR]        40 B
//     stage 15  K3: f and the stopping test of i - 1 (every workgroup alike),
//               then t, z_g <- clip01(PAVA(z_g - t g_g)), x_g = colv N_g z_g, and
//               (atomic K1) r set to target / 0 for the next stage
//     stage 14  K1: r_g = A_g x_g (+ target on the shard_role 1 rank)
//     RCCL      all-reduce(sum) of r                      8 m B
// and stage 9 (f / stop test) after the last iteration of a call; fuse 1
// reads all of r for ||r||^2 in K2 (stage 8: the f of i - 1 in its last
// workgroup, 14 us of an 8-way C5 rank's iteration for the 8 MB), fuse 0 runs
// stage 3 and a stage 9 per iteration.  A Python
// loop enqueued the same thing at ~4 ctypes calls + 2 torch.distributed calls
// per iteration (tens of us of host time against a ~100-us device iteration
// on 8 ranks); here an iteration costs 4 kernel launches + 2 RCCL calls of host
// time and nothing waits on the host.
//
// RCCL is resolved at run time (dlopen of librccl.so.1: in a torch process the
// copy torch already loaded, so torch.distributed and this driver share one
// RCCL), so the library has no link-time RCCL dependency and loads without it.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include "bsls_common.hpp"

extern "C" int bsls_bb_stage(const bsls_bb_problem *p, int stage, int64_t iter, void *stream);
extern "C" int bsls_bb_k2_part(const bsls_bb_problem *p, int64_t iter, int part, void *stream);
extern "C" int bsls_bb_k1_rows(const bsls_bb_problem *p, int64_t iter, int64_t rb0, int64_t rb1,
                               void *stream);
extern "C" int64_t bsls_bb_row_blocks(const bsls_bb_problem *p, int64_t *rows_per_block);

namespace bsls {

struct RcclApi {
    bool ok = false;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    decltype(&ncclCommCount) count = nullptr;
};

static const RcclApi &rccl() {
    static RcclApi api = [] {
        RcclApi a;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return a;
        a.get_id = (decltype(a.get_id))dlsym(h, "ncclGetUniqueId");
        a.init = (decltype(a.init))dlsym(h, "ncclCommInitRank");
        a.destroy = (decltype(a.destroy))dlsym(h, "ncclCommDestroy");
        a.all_reduce = (decltype(a.all_reduce))dlsym(h, "ncclAllReduce");
        a.err = (decltype(a.err))dlsym(h, "ncclGetErrorString");
        a.count = (decltype(a.count))dlsym(h, "ncclCommCount");
        a.ok = a.get_id && a.init && a.destroy && a.all_reduce;
        return a;
    }();
    return api;
}

}  // namespace bsls

using namespace bsls;

constexpr int MAX_PARTS = 16;

struct bsls_comm {
    ncclComm_t comm;
    int world, rank;
    // run the collectives at world 1 too (bsls_comm_force_collectives): a
    // one-rank RCCL sum is the identity, so the results stay those of the
    // skipped form while every RCCL call of the loop executes
    bool force;
    bsls_all_reduce_fn fn;   // set: the host callback replaces RCCL
    void *user;
    // a modelled exchange (bsls_comm_create_model): no data moves, a spin
    // kernel of fixed_us + us_per_mb per MB holds the stream instead
    bool model;
    double fixed_us, us_per_mb;
    // the part pipeline's events (created on first use)
    bool events;
    hipEvent_t ev_k1[MAX_PARTS], ev_ar[MAX_PARTS];
    // the last K2 image whose column groups were checked against the K1
    // row-block parts (bsls_bb_shard_iterate_parts: one device read per image)
    const int64_t *parts_gc;
    int64_t parts_rb[MAX_PARTS + 1];
};

namespace bsls {
// one wave sleeping until `ticks` of the constant wall clock have passed
__global__ void comm_model_spin(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
}  // namespace bsls

// RCCL failures map to BSLS_E_COMM - ncclResult (distinct from hip errors)
static int comm_rc(ncclResult_t r) { return r == ncclSuccess ? BSLS_OK : BSLS_E_COMM - (int)r; }

extern "C" size_t bsls_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

extern "C" int bsls_comm_unique_id(void *id_out) {
    if (!id_out) return BSLS_E_ARG;
    const RcclApi &R = rccl();
    if (!R.ok) return BSLS_E_COMM;
    ncclUniqueId id;
    const int rc = comm_rc(R.get_id(&id));
    if (rc == BSLS_OK) memcpy(id_out, &id, sizeof(id));
    return rc;
}

extern "C" int bsls_comm_create(const void *id, int world, int rank, bsls_comm **out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world) return BSLS_E_ARG;
    const RcclApi &R = rccl();
    if (!R.ok) return BSLS_E_COMM;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    bsls_comm *c = new bsls_comm{};
    c->world = world;
    c->rank = rank;
    const int rc = comm_rc(R.init(&c->comm, world, uid, rank));
    if (rc != BSLS_OK) {
        delete c;
        return rc;
    }
    *out = c;
    return BSLS_OK;
}

extern "C" int bsls_comm_create_callback(int world, int rank, bsls_all_reduce_fn fn, void *user,
                                         bsls_comm **out) {
    if (!fn || !out || world < 1 || rank < 0 || rank >= world) return BSLS_E_ARG;
    bsls_comm *c = new bsls_comm{};
    c->world = world;
    c->rank = rank;
    c->fn = fn;
    c->user = user;
    *out = c;
    return BSLS_OK;
}

extern "C" int bsls_comm_create_model(int world, int rank, double fixed_us, double us_per_mb,
                                      bsls_comm **out) {
    if (!out || world < 1 || rank < 0 || rank >= world || !(fixed_us >= 0.0) ||
        !(us_per_mb >= 0.0))
        return BSLS_E_ARG;
    bsls_comm *c = new bsls_comm{};
    c->world = world;
    c->rank = rank;
    c->model = true;
    c->fixed_us = fixed_us;
    c->us_per_mb = us_per_mb;
    *out = c;
    return BSLS_OK;
}

extern "C" int bsls_comm_destroy(bsls_comm *c) {
    if (!c) return BSLS_OK;
    const int rc = (c->fn || c->model) ? BSLS_OK : comm_rc(rccl().destroy(c->comm));
    if (c->events)
        for (int q = 0; q < MAX_PARTS; ++q) {
            (void)hipEventDestroy(c->ev_k1[q]);
            (void)hipEventDestroy(c->ev_ar[q]);
        }
    delete c;
    return rc;
}

// the one all-reduce of every transport: in place, sum, on `stream`; i64:
// the words are int64 (a fixed-point r, bsls_bb_problem.r_fx: summed exactly)
static int comm_sum(bsls_comm *c, double *buf, size_t count, hipStream_t st, bool i64 = false) {
    if (c->fn) return c->fn(buf, (int64_t)count, (void *)st, c->user) == 0 ? BSLS_OK : BSLS_E_COMM;
    if (c->model) {
        static const double ticks_per_us = [] {
            int dev = 0, khz = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
                khz <= 0)
                khz = 100000;
            return khz / 1000.0;
        }();
        const double us = c->fixed_us + c->us_per_mb * (double)count * 8.0 / 1e6;
        comm_model_spin<<<1, 64, 0, st>>>((uint64_t)(us * ticks_per_us));
        return hipGetLastError() == hipSuccess ? BSLS_OK : BSLS_E_COMM;
    }
    return comm_rc(rccl().all_reduce(buf, buf, count, i64 ? ncclInt64 : ncclFloat64, ncclSum,
                                     c->comm, st));
}

// the ranks the communicator spans: RCCL's own count (ncclCommCount) for an
// RCCL communicator -- what the library, not the caller, believes the job is
extern "C" int bsls_comm_count(const bsls_comm *c, int *count_out) {
    if (!c || !count_out) return BSLS_E_ARG;
    if (c->fn || c->model) {
        *count_out = c->world;
        return BSLS_OK;
    }
    const RcclApi &R = rccl();
    if (!R.count) return BSLS_E_COMM;
    return comm_rc(R.count(c->comm, count_out));
}

extern "C" int bsls_comm_force_collectives(bsls_comm *c, int on) {
    if (!c || (on != 0 && on != 1)) return BSLS_E_ARG;
    c->force = on != 0;
    return BSLS_OK;
}

extern "C" int bsls_comm_all_reduce(bsls_comm *c, double *buf, int64_t count, void *stream) {
    if (!c || !buf || count < 0) return BSLS_E_ARG;
    return comm_sum(c, buf, (size_t)count, (hipStream_t)stream);
}

extern "C" int bsls_bb_shard_iterate(const bsls_bb_problem *p, bsls_comm *c, int64_t first_iter,
                                     int64_t count, int fuse, void *stream) {
    if (!p || !c || first_iter < 1 || count < 0 || fuse < 0 || fuse > 2) return BSLS_E_ARG;
    if (p->shard_role != (c->rank == 0 ? 1 : 2)) return BSLS_E_ARG;   // target added once
    hipStream_t st = (hipStream_t)stream;
    // a sum over one rank is the identity: a one-rank communicator (the
    // rehearsal of one rank's share on one GPU) skips the collectives, whose
    // one-rank form is RCCL's own copies and flag fills (~17 us an iteration),
    // unless forced (bsls_comm_force_collectives)
    const bool comm = c->world > 1 || c->force;
    auto all_reduce = [&](double *buf, size_t cnt) -> int {
        return comm ? comm_sum(c, buf, cnt, st) : BSLS_OK;
    };
    int rc;
    for (int64_t i = first_iter; i < first_iter + count; ++i) {
        if (fuse == 2) {
            // K2 with this rank's slice of ||r||^2, the five sums over ranks,
            // then f and the stop test of i - 1
            // (stage 13: K3 with stage 12 -- f and the stop test of i - 1 --
            // folded in)
            // (stage 15: 13 with the next K1's r initialisation folded in when
            // K1 adds its group sums by atomics; stage 14 is then stage 1 without it)
            if ((rc = bsls_bb_stage(p, 10, i, stream)) != BSLS_OK) return rc;
            if ((rc = all_reduce(p->scal + BSLS_S_SUMDG, 5)) != BSLS_OK) return rc;
            if ((rc = bsls_bb_stage(p, 15, i, stream)) != BSLS_OK) return rc;
        } else {
            // K2 (+ the fused f / stop test of i - 1), then the BB sums over ranks
            if ((rc = bsls_bb_stage(p, fuse ? 8 : 3, i, stream)) != BSLS_OK) return rc;
            if ((rc = all_reduce(p->scal + BSLS_S_SUMDG, 4)) != BSLS_OK) return rc;
            if ((rc = bsls_bb_stage(p, 4, i, stream)) != BSLS_OK) return rc;
        }
        // the partial residual, then r = the sum over ranks (the one real exchange)
        if ((rc = bsls_bb_stage(p, fuse == 2 ? 14 : 1, i, stream)) != BSLS_OK) return rc;
        if (comm && (rc = comm_sum(c, p->r, (size_t)p->m, st, p->r_fx > 0.0)) != BSLS_OK)
            return rc;
        if (!fuse && (rc = bsls_bb_stage(p, 9, i, stream)) != BSLS_OK) return rc;
    }
    if (count > 0 && fuse) return bsls_bb_stage(p, 9, first_iter + count - 1, stream);
    return BSLS_OK;
}

// The link-part pipeline (include/bsls_hip.h): K1 by row-block parts, each
// part's rows of r all-reduced on `comm_stream` as soon as the part is done,
// the next iteration's K2 by the matching column groups, each waiting only
// for its own part's exchange -- so part q's exchange runs under K1's later
// parts and K2's earlier ones instead of after the whole walk.
extern "C" int bsls_bb_shard_iterate_parts(const bsls_bb_problem *p, bsls_comm *c,
                                           int64_t first_iter, int64_t count, int nparts,
                                           const int64_t *rb_bounds, void *comm_stream,
                                           void *stream) {
    if (!p || !c || !rb_bounds || first_iter < 1 || count < 0 || nparts < 2 ||
        nparts > MAX_PARTS || !comm_stream || comm_stream == stream)
        return BSLS_E_ARG;
    if (p->shard_role != (c->rank == 0 ? 1 : 2)) return BSLS_E_ARG;
    if (p->ATt.ngroups != nparts || !p->ATt.ent) return BSLS_E_ARG;
    int64_t R = 0;
    const int64_t nrb = bsls_bb_row_blocks(p, &R);
    if (nrb < 0) return (int)nrb;
    if (rb_bounds[0] != 0 || rb_bounds[nparts] != nrb) return BSLS_E_ARG;
    for (int q = 0; q < nparts; ++q)
        if (rb_bounds[q + 1] <= rb_bounds[q]) return BSLS_E_ARG;
    // K2 part q waits only for exchange q, so its column group must be exactly
    // the rows that exchange delivers: group_col[q] = min(rb_bounds[q] R, m).
    // Checked once per (image, bounds): a mismatch would read rows of r whose
    // all-reduce is still running on comm_stream.
    bool same = c->parts_gc == p->ATt.group_col;
    for (int q = 0; same && q <= nparts; ++q) same = c->parts_rb[q] == rb_bounds[q];
    if (!same) {
        int64_t gc[MAX_PARTS + 1];
        BSLS_CHECK(hipMemcpy(gc, p->ATt.group_col, sizeof(int64_t) * (nparts + 1),
                             hipMemcpyDeviceToHost));
        for (int q = 0; q <= nparts; ++q) {
            const int64_t want = rb_bounds[q] * R < p->m ? rb_bounds[q] * R : p->m;
            if (gc[q] != want) return BSLS_E_ARG;
        }
        c->parts_gc = p->ATt.group_col;
        for (int q = 0; q <= nparts; ++q) c->parts_rb[q] = rb_bounds[q];
    }
    if (!c->events) {
        for (int q = 0; q < MAX_PARTS; ++q) {
            BSLS_CHECK(hipEventCreateWithFlags(&c->ev_k1[q], hipEventDisableTiming));
            BSLS_CHECK(hipEventCreateWithFlags(&c->ev_ar[q], hipEventDisableTiming));
        }
        c->events = true;
    }
    hipStream_t st = (hipStream_t)stream, cs = (hipStream_t)comm_stream;
    const bool comm = c->world > 1 || c->force;
    int rc;
    for (int64_t i = first_iter; i < first_iter + count; ++i) {
        // K2 by link parts: part q needs only its rows of r
        for (int q = 0; q < nparts; ++q) {
            if (comm && i > first_iter) BSLS_CHECK(hipStreamWaitEvent(st, c->ev_ar[q], 0));
            if ((rc = bsls_bb_k2_part(p, i, q, stream)) != BSLS_OK) return rc;
        }
        if (comm && (rc = comm_sum(c, p->scal + BSLS_S_SUMDG, 5, st)) != BSLS_OK) return rc;
        if ((rc = bsls_bb_stage(p, 15, i, stream)) != BSLS_OK) return rc;
        // K1 by the same parts, each part's exchange started behind it
        for (int q = 0; q < nparts; ++q) {
            if ((rc = bsls_bb_k1_rows(p, i, rb_bounds[q], rb_bounds[q + 1], stream)) != BSLS_OK)
                return rc;
            if (!comm) continue;
            const int64_t r0 = rb_bounds[q] * R;
            const int64_t r1 = rb_bounds[q + 1] * R < p->m ? rb_bounds[q + 1] * R : p->m;
            BSLS_CHECK(hipEventRecord(c->ev_k1[q], st));
            BSLS_CHECK(hipStreamWaitEvent(cs, c->ev_k1[q], 0));
            if ((rc = comm_sum(c, p->r + r0, (size_t)(r1 - r0), cs, p->r_fx > 0.0)) != BSLS_OK)
                return rc;
            BSLS_CHECK(hipEventRecord(c->ev_ar[q], cs));
        }
    }
    if (count > 0) {
        if (comm)
            for (int q = 0; q < nparts; ++q) BSLS_CHECK(hipStreamWaitEvent(st, c->ev_ar[q], 0));
        return bsls_bb_stage(p, 9, first_iter + count - 1, stream);
    }
    return BSLS_OK;
}
