/*
 * libhpnn communication layer: RCCL over xGMI (see include/libhpnn/comm.h).
 *
 * Reference counterpart: every MPI_* call site of src/ann.c / src/snn.c and the
 * CUDA hub copies of src/cuda_ann.cu.  There the collectives were
 * written inline in each compute function; here they are one small layer that the
 * engines (csrc/gpu/gpu_engine.cpp) and the Python data-parallel driver
 * (hpnn_amd/parallel) share.
 *
 * MI355X notes
 *   - xGMI is point-to-point (7 links per GPU): RCCL's ring / tree all-reduce is
 *     bound per link, so callers pass few, large buffers (one flat gradient bucket)
 *     rather than one collective per tensor.
 *   - the side stream gets the highest priority, so the communication kernels are
 *     scheduled ahead of queued compute work they are meant to overlap with.
 */
#include <libhpnn.h>
#include <libhpnn/comm.h>
#include <libhpnn/xar.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclReduceScatter) reduce_scatter = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    decltype(&ncclCommGetAsyncError) async_err = nullptr;
    int state = 0; /* 0 not tried, 1 loaded, -1 unavailable */
    std::mutex mu;

    bool load() {
        std::lock_guard<std::mutex> g(mu);
        if (state) return state > 0;
        const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        void *h = nullptr;
        for (const char *n : names)
            if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            NN_ERROR(stderr, "RCCL not found (%s)\n", dlerror());
            state = -1;
            return false;
        }
#define HPNN_SYM(field, name) field = (decltype(field))dlsym(h, name)
        HPNN_SYM(get_id, "ncclGetUniqueId");
        HPNN_SYM(init_rank, "ncclCommInitRank");
        HPNN_SYM(init_all, "ncclCommInitAll");
        HPNN_SYM(destroy, "ncclCommDestroy");
        HPNN_SYM(abort, "ncclCommAbort");
        HPNN_SYM(all_reduce, "ncclAllReduce");
        HPNN_SYM(broadcast, "ncclBroadcast");
        HPNN_SYM(all_gather, "ncclAllGather");
        HPNN_SYM(reduce_scatter, "ncclReduceScatter");
        HPNN_SYM(group_start, "ncclGroupStart");
        HPNN_SYM(group_end, "ncclGroupEnd");
        HPNN_SYM(err, "ncclGetErrorString");
        HPNN_SYM(async_err, "ncclCommGetAsyncError");
#undef HPNN_SYM
        const bool ok = get_id && init_rank && init_all && destroy && abort && all_reduce && broadcast &&
                        all_gather && reduce_scatter && group_start && group_end && err && async_err;
        if (!ok) NN_ERROR(stderr, "RCCL: missing symbols\n");
        state = ok ? 1 : -1;
        return ok;
    }
};
Rccl R;

ncclDataType_t to_nccl(hpnn_comm_dtype d) {
    switch (d) {
        case HPNN_DT_F64: return ncclFloat64;
        case HPNN_DT_BF16: return ncclBfloat16;
        case HPNN_DT_I32: return ncclInt32;
        case HPNN_DT_U8: return ncclUint8;
        default: return ncclFloat32;
    }
}
ncclRedOp_t to_nccl(hpnn_comm_op o) {
    switch (o) {
        case HPNN_OP_MAX: return ncclMax;
        case HPNN_OP_MIN: return ncclMin;
        default: return ncclSum;
    }
}

/* ---- fault injection: HPNN_FAULT="site:n[,site:n...]" ---- */
std::mutex g_fault_mu;
std::map<std::string, long> g_fault_at, g_fault_count;
bool g_fault_parsed = false;

void parse_faults() {
    g_fault_parsed = true;
    const char *e = getenv("HPNN_FAULT");
    if (!e) return;
    std::string s(e);
    size_t p = 0;
    while (p < s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        std::string item = s.substr(p, q - p);
        size_t c = item.find(':');
        if (c != std::string::npos) g_fault_at[item.substr(0, c)] = atol(item.c_str() + c + 1);
        else if (!item.empty()) g_fault_at[item] = 1;
        p = q + 1;
    }
}

constexpr int EV_RING = 64;

}  // namespace

struct hpnn_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, size = 1, device = 0;
    hipStream_t side = nullptr;
    hipEvent_t ev_in[EV_RING] = {}, ev_out[EV_RING] = {};
    int next = 0;     /* ring index of the next async collective */
    int pending = -1; /* ring index of the last async collective not joined yet */
    int *d_flag = nullptr;
    bool failed = false;
    /* one-shot xGMI all-reduce for small float32 sum buckets (csrc/dist/xgmi_ar.hip) */
    hpnn_xar *xar = nullptr;
    size_t xar_max = 0;
};

extern "C" int hpnn_fault_hit(const char *site) {
    std::lock_guard<std::mutex> g(g_fault_mu);
    if (!g_fault_parsed) parse_faults();
    auto it = g_fault_at.find(site);
    if (it == g_fault_at.end()) return 0;
    const long n = ++g_fault_count[site];
    if (n == it->second) {
        NN_ERROR(stderr, "fault injection: %s #%ld\n", site, n);
        return 1;
    }
    return 0;
}

#define COMM_CHK(call, what)                                                  \
    do {                                                                      \
        ncclResult_t _r = (call);                                             \
        if (_r != ncclSuccess) {                                              \
            NN_ERROR(stderr, "RCCL %s failed: %s\n", what, R.err(_r));        \
            return -3;                                                        \
        }                                                                     \
    } while (0)

static int setup_side(hpnn_comm *c) {
    int lo = 0, hi = 0;
    if (hipSetDevice(c->device) != hipSuccess) return -1;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    if (hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi) != hipSuccess) return -1;
    for (int i = 0; i < EV_RING; i++) {
        if (hipEventCreateWithFlags(&c->ev_in[i], hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&c->ev_out[i], hipEventDisableTiming) != hipSuccess) return -1;
    }
    if (hipMalloc(&c->d_flag, sizeof(int)) != hipSuccess) return -1;
    return 0;
}

extern "C" int hpnn_comm_available(void) { return R.load() ? 1 : 0; }

extern "C" int hpnn_comm_unique_id(unsigned char *id) {
    if (!R.load()) return -1;
    ncclUniqueId u;
    COMM_CHK(R.get_id(&u), "ncclGetUniqueId");
    memcpy(id, u.internal, HPNN_COMM_ID_BYTES);
    return 0;
}

extern "C" hpnn_comm *hpnn_comm_init_rank(const unsigned char *id, int nranks, int rank, int device) {
    if (!R.load() || nranks < 1 || rank < 0 || rank >= nranks) return nullptr;
    hpnn_comm *c = new hpnn_comm();
    c->rank = rank;
    c->size = nranks;
    c->device = device;
    if (setup_side(c)) {
        hpnn_comm_destroy(c);
        return nullptr;
    }
    ncclUniqueId u;
    memcpy(u.internal, id, HPNN_COMM_ID_BYTES);
    ncclResult_t r = R.init_rank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        NN_ERROR(stderr, "ncclCommInitRank(rank %d of %d, device %d) failed: %s\n", rank, nranks, device, R.err(r));
        c->comm = nullptr;
        hpnn_comm_destroy(c);
        return nullptr;
    }
    return c;
}

extern "C" int hpnn_comm_init_all(hpnn_comm **comms, int G, const int *devs) {
    if (!R.load() || G < 1 || G > 64) return -1;
    ncclComm_t raw[64];
    for (int g = 0; g < G; g++) comms[g] = nullptr;
    ncclResult_t r = R.init_all(raw, G, devs);
    if (r != ncclSuccess) {
        NN_ERROR(stderr, "ncclCommInitAll(%d GPUs) failed: %s\n", G, R.err(r));
        return -3;
    }
    int rc = 0;
    for (int g = 0; g < G; g++) {
        hpnn_comm *c = new hpnn_comm();
        c->comm = raw[g];
        c->rank = g;
        c->size = G;
        c->device = devs[g];
        if (setup_side(c)) rc = -1;
        comms[g] = c;
    }
    if (rc)
        for (int g = 0; g < G; g++) {
            hpnn_comm_destroy(comms[g]);
            comms[g] = nullptr;
        }
    return rc;
}

extern "C" void hpnn_comm_destroy(hpnn_comm *c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->side) hipStreamSynchronize(c->side);
    if (c->comm) {
        if (c->failed) R.abort(c->comm);
        else R.destroy(c->comm);
    }
    for (int i = 0; i < EV_RING; i++) {
        if (c->ev_in[i]) hipEventDestroy(c->ev_in[i]);
        if (c->ev_out[i]) hipEventDestroy(c->ev_out[i]);
    }
    if (c->side) hipStreamDestroy(c->side);
    if (c->d_flag) hipFree(c->d_flag);
    delete c;
}

extern "C" int hpnn_comm_rank(const hpnn_comm *c) { return c ? c->rank : 0; }
extern "C" int hpnn_comm_size(const hpnn_comm *c) { return c ? c->size : 1; }

static int injected(hpnn_comm *c) {
    if (hpnn_fault_hit("comm")) {
        c->failed = true;
        return -7;
    }
    return 0;
}

extern "C" int hpnn_comm_all_reduce(hpnn_comm *c, const void *send, void *recv, long count, hpnn_comm_dtype dt,
                                    hpnn_comm_op op, hipStream_t stream) {
    if (!c || !c->comm || count < 0) return -1;
    if (int f = injected(c)) return f;
    COMM_CHK(R.all_reduce(send, recv, (size_t)count, to_nccl(dt), to_nccl(op), c->comm, stream), "all_reduce");
    return 0;
}

extern "C" int hpnn_comm_broadcast(hpnn_comm *c, const void *send, void *recv, long count, hpnn_comm_dtype dt,
                                   int root, hipStream_t stream) {
    if (!c || !c->comm || count < 0) return -1;
    if (int f = injected(c)) return f;
    COMM_CHK(R.broadcast(send, recv, (size_t)count, to_nccl(dt), root, c->comm, stream), "broadcast");
    return 0;
}

extern "C" int hpnn_comm_all_gather(hpnn_comm *c, const void *send, void *recv, long count, hpnn_comm_dtype dt,
                                    hipStream_t stream) {
    if (!c || !c->comm || count < 0) return -1;
    if (int f = injected(c)) return f;
    COMM_CHK(R.all_gather(send, recv, (size_t)count, to_nccl(dt), c->comm, stream), "all_gather");
    return 0;
}

extern "C" int hpnn_comm_reduce_scatter(hpnn_comm *c, const void *send, void *recv, long count, hpnn_comm_dtype dt,
                                        hpnn_comm_op op, hipStream_t stream) {
    if (!c || !c->comm || count < 0) return -1;
    if (int f = injected(c)) return f;
    COMM_CHK(R.reduce_scatter(send, recv, (size_t)count, to_nccl(dt), to_nccl(op), c->comm, stream),
             "reduce_scatter");
    return 0;
}

extern "C" int hpnn_comm_group_start(void) {
    if (!R.load()) return -1;
    COMM_CHK(R.group_start(), "group_start");
    return 0;
}
extern "C" int hpnn_comm_group_end(void) {
    if (!R.load()) return -1;
    COMM_CHK(R.group_end(), "group_end");
    return 0;
}

extern "C" int hpnn_comm_all_reduce_async(hpnn_comm *c, void *buf, long count, hpnn_comm_dtype dt,
                                          hipStream_t compute) {
    if (!c) return -1;
    const int i = c->next;
    c->next = (c->next + 1) % EV_RING;
    /* fork: the side stream starts after what the compute stream has enqueued so far */
    if (hipEventRecord(c->ev_in[i], compute) != hipSuccess) return -2;
    if (hipStreamWaitEvent(c->side, c->ev_in[i], 0) != hipSuccess) return -2;
    const bool one_shot = c->xar && dt == HPNN_DT_F32 && (count & 3) == 0 && (size_t)count * 4 <= c->xar_max &&
                          ((uintptr_t)buf & 15) == 0;
    const int rc = one_shot ? hpnn_xar_all_reduce_f32(c->xar, (const float *)buf, (float *)buf, count, c->side)
                            : hpnn_comm_all_reduce(c, buf, buf, count, dt, HPNN_OP_SUM, c->side);
    if (rc) return rc;
    if (hipEventRecord(c->ev_out[i], c->side) != hipSuccess) return -2;
    c->pending = i;
    return 0;
}

extern "C" hipStream_t hpnn_comm_fork(hpnn_comm *c, hipStream_t compute) {
    if (!c || !c->side) return nullptr;
    const int i = c->next;
    if (hipEventRecord(c->ev_in[i], compute) != hipSuccess) return nullptr;
    if (hipStreamWaitEvent(c->side, c->ev_in[i], 0) != hipSuccess) return nullptr;
    return c->side;
}

extern "C" int hpnn_comm_fork_done(hpnn_comm *c) {
    if (!c) return -1;
    const int i = c->next;
    c->next = (c->next + 1) % EV_RING;
    if (hipEventRecord(c->ev_out[i], c->side) != hipSuccess) return -2;
    c->pending = i;
    return 0;
}

extern "C" int hpnn_comm_join(hpnn_comm *c, hipStream_t compute) {
    if (!c) return -1;
    if (c->pending < 0) return 0;
    /* the side stream is in order: its last event covers every earlier collective */
    if (hipStreamWaitEvent(compute, c->ev_out[c->pending], 0) != hipSuccess) return -2;
    c->pending = -1;
    return 0;
}

extern "C" int hpnn_comm_set_xar(hpnn_comm *c, hpnn_xar *x, size_t max_bytes) {
    if (!c) return -1;
    c->xar = x;
    c->xar_max = x ? (max_bytes < hpnn_xar_max_bytes(x) ? max_bytes : hpnn_xar_max_bytes(x)) : 0;
    return 0;
}

extern "C" int hpnn_comm_check(hpnn_comm *c) {
    if (!c) return -1;
    if (c->xar && hpnn_xar_status(c->xar) != 0) {
        NN_ERROR(stderr, "xgmi all-reduce barrier timed out on rank %d (a peer never arrived)\n", c->rank);
        c->failed = true;
        return -8;
    }
    if (c->failed || !c->comm) return -7;
    ncclResult_t ar = ncclSuccess;
    if (R.async_err(c->comm, &ar) != ncclSuccess || ar != ncclSuccess) {
        NN_ERROR(stderr, "RCCL asynchronous error on rank %d: %s\n", c->rank, R.err(ar));
        c->failed = true;
        return -3;
    }
    return 0;
}

extern "C" void hpnn_comm_abort(hpnn_comm *c) {
    if (!c || !c->comm) return;
    R.abort(c->comm);
    c->comm = nullptr;
    c->failed = true;
}

extern "C" int hpnn_comm_all_ok(hpnn_comm *c, int ok, hipStream_t stream) {
    if (!c) return ok ? 1 : 0;
    int v = ok ? 1 : 0;
    if (hipMemcpyAsync(c->d_flag, &v, sizeof(int), hipMemcpyHostToDevice, stream) != hipSuccess) return 0;
    if (hpnn_comm_all_reduce(c, c->d_flag, c->d_flag, 1, HPNN_DT_I32, HPNN_OP_MIN, stream)) return 0;
    if (hipMemcpyAsync(&v, c->d_flag, sizeof(int), hipMemcpyDeviceToHost, stream) != hipSuccess) return 0;
    if (hipStreamSynchronize(stream) != hipSuccess) return 0;
    return v;
}
