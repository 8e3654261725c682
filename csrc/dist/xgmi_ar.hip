/*
 * xGMI all-reduce (include/libhpnn/xar.h): one-shot and two-shot, one launch per call.
 *
 * Each rank owns two fine-grained (uncached) device allocations that every peer maps
 * through hipIpc: a data buffer of two halves (max_bytes each, used alternately by
 * consecutive calls) and a signal block (barrier flags).  Workgroup b of every rank
 * owns the same element set on every rank.
 *
 * one-shot (every rank reads every peer's whole buffer; best for 2 ranks, where both
 * algorithms move the same bytes per link, and for tiny buffers):
 *   1. copy its elements of `in` into this rank's data half (local slab sums included);
 *   2. barrier A: write epoch e into A[b][rank] of every peer, wait for A[b][p] >= e;
 *   3. out = sum_{p = 0..W-1} data_p (fixed rank order: identical bits on every rank).
 * two-shot (reduce-scatter + all-gather through the same buffers; with W ranks each
 * link carries 2/W of the buffer instead of all of it: 4x fewer link bytes at W = 8):
 *   1. copy in as above (block b owns sub-slice b of EVERY rank's shard);
 *   2. barrier A;
 *   3. this rank's shard: s = sum_p data_p[shard] in rank order, written to out and
 *      back into this rank's data half (peers only read their own shards in step 3);
 *   4. barrier B: every shard is reduced;
 *   5. out[shard q] = data_q[shard q] for every peer q.
 * No closing barrier: call e+2 reuses the data half of call e only after passing its
 * barrier A of call e+1, which no peer signals before its call-e kernel (all its reads
 * of that half) has completed.
 * Epochs are per workgroup (every call runs the full fixed grid, so they stay equal),
 * kept in ordinary device memory of this rank and advanced by the kernel,
 * so launches captured in a HIP graph replay correctly; all ranks issue the same
 * sequence of all-reduces (same sizes, same mode), so the epochs and halves agree.  Every
 * wait is bounded by a wall-clock timeout: a missing peer sets the error word, never
 * hangs the GPU.
 *
 * Fine-grained uncached memory keeps peer reads coherent without cache maintenance:
 * waiting for the data stores' acknowledgements orders them before the flag stores (no
 * L2 writeback), and an acquire invalidate precedes the peer reads.
 * Replaces the reference's hub copies through GPU0 (cuda_ann.cu EXP model).
 */
#include <hip/hip_runtime.h>
#include <libhpnn.h>
#include <libhpnn/xar.h>
#include <stddef.h>

#include "../gpu/mfma_common.h"
#include "../gpu/kernels.h"

HPNN_CO_PROBE(xar)
#include <stdlib.h>
#include <string.h>

namespace {

struct Signal {
    unsigned int flag[2][HPNN_XAR_MAX_BLOCKS][HPNN_XAR_MAX_RANKS]; /* barriers A, B */
    unsigned int error;
};

static_assert(sizeof(unsigned int) * HPNN_XAR_ERROR_WORD == offsetof(Signal, error), "xar.h signal layout");

struct XarPeers {
    float4 *buf[HPNN_XAR_MAX_RANKS];
    Signal *sig[HPNN_XAR_MAX_RANKS];
};

__device__ __forceinline__ void flag_store(unsigned int *p, unsigned int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned int flag_load(unsigned int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* threads 0..world-1 signal peer t and wait for peer t; bounded spin */
__device__ __forceinline__ void xbarrier(const XarPeers &P, int rank, int world, int b, unsigned int e, int which,
                                         unsigned long long timeout, int light) {
    /* release: this thread's data stores complete before any flag store.  Everything a
     * peer reads lives in the uncached (MTYPE UC) buffer, which no L2 holds, so waiting
     * for the store acknowledgements is enough; __threadfence_system() would also write
     * back every dirty L2 line of the XCD (buffer_wbl2) -- measured 18.6 -> 8.5 us per
     * 437 KB call at world 1 and 36.6 -> 12.5 us at world 2 (scripts/xar_bench.py);
     * HPNN_XAR_FENCE=1 restores the full fence */
    if (light == 1)
        __builtin_amdgcn_s_waitcnt(0);
    else if (!light)
        __threadfence_system();
    /* light == 2: the data was stored by an earlier kernel (in-place call), nothing to order */
    __syncthreads();
    const int t = threadIdx.x;
    if (t < world) {
        flag_store(&P.sig[t]->flag[which][b][rank], e);
        Signal *me = P.sig[rank];
        unsigned int *f = &me->flag[which][b][t];
        const unsigned long long t0 = wall_clock64();
        while (flag_load(f) < e) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > timeout) {
                __hip_atomic_store(&me->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
    }
    __syncthreads();
    /* acquire: light modes read peer data with system-coherent loads (sc0 sc1, ld_peer*), which
     * no cache serves stale, so no invalidating fence (in the fused MNIST exchange that fence,
     * one per workgroup, cost ~10 us per step: profiles/r4/m_dp_exchange_ab.txt) */
    if (!light) __threadfence_system();
}

/* system-coherent float4 load of a peer buffer (load and its wait in one asm block, see
 * ld_sc1_x8) */
__device__ __forceinline__ float4 ld_peer(const float4 *p) {
    hpnn::f32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return make_float4(v[0], v[1], v[2], v[3]);
}

/* the input of a call: up to HPNN_XAR_MAX_SEGS segments laid end to end in the output;
 * segment j is the sum of S_j slabs (stride in float4) -- the local split-K / block-slab
 * reduction happens in the copy-in phase, so no separate reduction launch precedes the
 * exchange */
struct XarIn {
    const float4 *src[HPNN_XAR_MAX_SEGS];
    long stride4[HPNN_XAR_MAX_SEGS];
    long end4[HPNN_XAR_MAX_SEGS]; /* exclusive prefix ends in float4 */
    int S[HPNN_XAR_MAX_SEGS];
    int nseg;
};

__device__ __forceinline__ void add4(float4 &a, const float4 &b) {
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
}

/* local sum of element i of the input: slabs s = k (mod U) accumulate in acc[k], U = 8 loads
 * in flight per thread, combined in a fixed tree (2 in flight took 15.2 us per MNIST step,
 * 8 took 11.3).  More measured slower on the N > 1 step path timed on one GPU: 16 per batch
 * +0.7-1.1 us, a software-pipelined 16 + 16 variant +8 us (round-2 A/B script, since pruned;
 * profiles/r2/s5_xar_launch_shape.txt). */
template <int U>
__device__ __forceinline__ float4 xar_load_in_u(const float4 *p, long st, int S) {
    float4 acc[U];
    int s = 0;
    if (S >= U) {
#pragma unroll
        for (int k = 0; k < U; k++) acc[k] = p[(long)k * st];
        for (s = U; s + U <= S; s += U) {
            float4 v[U];
#pragma unroll
            for (int k = 0; k < U; k++) v[k] = p[(long)(s + k) * st];
#pragma unroll
            for (int k = 0; k < U; k++) add4(acc[k], v[k]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < U; k++) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < U; k++)
        if (s + k < S) add4(acc[k], p[(long)(s + k) * st]);
#pragma unroll
    for (int w = 1; w < U; w *= 2)
#pragma unroll
        for (int k = 0; k < U; k += 2 * w) add4(acc[k], acc[k + w]);
    return acc[0];
}

__device__ __forceinline__ float4 xar_load_in(const XarIn &in, long i) {
    int j = 0;
    while (j + 1 < in.nseg && i >= in.end4[j]) j++;
    const long li = i - (j ? in.end4[j - 1] : 0);
    const float4 *p = in.src[j] + li;
    const int S = in.S[j];
    if (S == 1) return p[0];
    return xar_load_in_u<8>(p, in.stride4[j], S);
}

/* sum of element i over the first `world` data halves, rank order.  The 8 loads go out in
 * one block; slots past `world` re-read this rank's OWN half (local memory) and are dropped --
 * re-reading rank 0's instead would put world - 1 .. 7 extra reads per element on the xGMI
 * link of every other rank (6 extra at world 2). */
static_assert(HPNN_XAR_MAX_RANKS == 8, "one ld_sc1_x8 per element");
__device__ __forceinline__ float4 sum_peers(const XarPeers &P, long half4, int world, int rank, long i) {
    const float *q[8];
#pragma unroll
    for (int p = 0; p < 8; p++) q[p] = (const float *)(P.buf[p < world ? p : rank] + half4 + i);
    hpnn::f32x4 v[8];
    hpnn::ld_sc1_x8<true>(v, q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]);
    hpnn::f32x4 s = v[0];
#pragma unroll
    for (int p = 1; p < 8; p++)
        if (p < world) s += v[p];
    return make_float4(s[0], s[1], s[2], s[3]);
}

/* optimizer step fused after the exchange (hpnn_xar_all_reduce_slabs_update_f32) */
struct XarUpd {
    float *W32[HPNN_XAR_MAX_LAYERS], *V32[HPNN_XAR_MAX_LAYERS];
    __bf16 *Wb[HPNN_XAR_MAX_LAYERS], *Wt[HPNN_XAR_MAX_LAYERS], *Wf[HPNN_XAR_MAX_LAYERS];
    int N[HPNN_XAR_MAX_LAYERS], K[HPNN_XAR_MAX_LAYERS];
    long end4[HPNN_XAR_MAX_LAYERS]; /* exclusive prefix ends in float4 */
    int nl;
    float lr, alpha, scale;
    int momentum;
};

/* float4 i of the reduced gradient = 4 consecutive k of one row n of one layer: the
 * step of sgd_tile (kernels_misc.hip) on those 4 weights.  The master weights and momenta
 * (local, independent of the peers) can be loaded before the barrier: XarPre */
struct XarPre {
    float4 w, v;
};
__device__ __forceinline__ int xar_layer(const XarUpd &u, long i, long &e) {
    int l = 0;
    while (l + 1 < u.nl && i >= u.end4[l]) l++;
    e = (i - (l ? u.end4[l - 1] : 0)) * 4;
    return l;
}
__device__ __forceinline__ XarPre xar_pre(const XarUpd &u, long i) {
    long e;
    const int l = xar_layer(u, i, e);
    XarPre p;
    p.w = *(const float4 *)(u.W32[l] + e);
    p.v = u.momentum ? *(const float4 *)(u.V32[l] + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    return p;
}
__device__ __forceinline__ void xar_update4(const XarUpd &u, long i, float4 g, const XarPre *pre = nullptr) {
    long e;
    const int l = xar_layer(u, i, e);
    const int K = u.K[l], N = u.N[l];
    const int n = (int)(e / K), k = (int)(e % K);
    float4 w = pre ? pre->w : *(const float4 *)(u.W32[l] + e);
    float gv[4] = {g.x, g.y, g.z, g.w}, wv[4] = {w.x, w.y, w.z, w.w};
    if (u.momentum) {
        float4 v = pre ? pre->v : *(const float4 *)(u.V32[l] + e);
        float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int r = 0; r < 4; r++) {
            vv[r] += u.lr * (gv[r] * u.scale);
            wv[r] += vv[r];
            vv[r] *= u.alpha;
        }
        *(float4 *)(u.V32[l] + e) = make_float4(vv[0], vv[1], vv[2], vv[3]);
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) wv[r] += u.lr * (gv[r] * u.scale);
    }
    *(float4 *)(u.W32[l] + e) = make_float4(wv[0], wv[1], wv[2], wv[3]);
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    bf16x4 wb;
#pragma unroll
    for (int r = 0; r < 4; r++) wb[r] = (__bf16)wv[r];
    *(bf16x4 *)(u.Wb[l] + e) = wb;
    if (u.Wf[l]) {
        const size_t fo = (((size_t)(n >> 4) * (K / 32) + (k >> 5)) * 64 + (n & 15) + 16 * ((k >> 3) & 3)) * 8 + (k & 7);
        *(bf16x4 *)(u.Wf[l] + fo) = wb;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) u.Wt[l][(size_t)(k + r) * N + n] = wb[r];
}

/* TWO = false: one-shot, element slice b of the whole buffer per workgroup.
 * TWO = true: shard s = [s * sh, min((s + 1) * sh, n4)), workgroup b owns
 * [s * sh + b * per, ...+ per) of every shard */
template <bool TWO, bool UPD>
__global__ __launch_bounds__(256) void xar_kernel(XarPeers P, int rank, int world, XarIn in, float4 *__restrict__ out,
                                                  long n4, long half_stride4, unsigned long long timeout, int light,
                                                  XarUpd upd, unsigned int *__restrict__ ep) {
    const int b = blockIdx.x;
    Signal *me = P.sig[rank];
    __shared__ unsigned int s_ep;
    if (threadIdx.x == 0) {
        /* the epochs live in ordinary device memory (only this workgroup of this rank ever
         * touches ep[b], and kernel boundaries order launches): one uncached round trip
         * less per call than keeping them in the signal block */
        const unsigned int e = ep[b] + 1;
        ep[b] = e;
        s_ep = e;
    }
    __syncthreads();
    const unsigned int e = s_ep;
    const long half4 = (e & 1) ? half_stride4 : 0;
    float4 *mine = P.buf[rank] + half4;
    if constexpr (!TWO) {
        const long per = (n4 + gridDim.x - 1) / gridDim.x;
        const long lo = (long)b * per, hi = lo + per < n4 ? lo + per : n4;
        if (in.nseg) /* else in place: an earlier kernel wrote this call's data half */
            for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = xar_load_in(in, i);
        const long i0 = lo + threadIdx.x;
        XarPre pre = {};
        if constexpr (UPD)
            if (i0 < hi) pre = xar_pre(upd, i0); /* in flight while the barrier waits */
        xbarrier(P, rank, world, b, e, 0, timeout, in.nseg ? light : (light ? 2 : 0));
        for (long i = i0; i < hi; i += blockDim.x) {
            const float4 v = sum_peers(P, half4, world, rank, i);
            out[i] = v;
            if constexpr (UPD) xar_update4(upd, i, v, i == i0 ? &pre : nullptr);
        }
    } else {
        const long sh = (n4 + world - 1) / world;
        const long per = (sh + gridDim.x - 1) / gridDim.x;
        auto range = [&](int s, long &lo, long &hi) {
            const long s_end = (long)(s + 1) * sh < n4 ? (long)(s + 1) * sh : n4;
            lo = (long)s * sh + (long)b * per;
            hi = lo + per < s_end ? lo + per : s_end;
        };
        long lo, hi;
        if (in.nseg)
            for (int s = 0; s < world; s++) {
                range(s, lo, hi);
                for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = xar_load_in(in, i);
            }
        xbarrier(P, rank, world, b, e, 0, timeout, in.nseg ? light : (light ? 2 : 0));
        range(rank, lo, hi);
        for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
            const float4 v = sum_peers(P, half4, world, rank, i);
            mine[i] = v;
            out[i] = v;
            if constexpr (UPD) xar_update4(upd, i, v);
        }
        xbarrier(P, rank, world, b, e, 1, timeout, light);
        for (int q = 1; q < world; q++) { /* start after this rank: spread the link load */
            const int s = (rank + q) % world;
            range(s, lo, hi);
            const float4 *src = P.buf[s] + half4;
            for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
                const float4 v = light ? ld_peer(src + i) : src[i];
                out[i] = v;
                if constexpr (UPD) xar_update4(upd, i, v);
            }
        }
    }
}

/* self-test pattern: rank r, element i -> (r + 1) * (i % 97 + 1) / 16; sums over <= 8
 * ranks are small multiples of 1/16, exact in FP32 in any order */
__global__ void xar_fill_kernel(float *__restrict__ v, long n, int rank) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        v[i] = (float)(rank + 1) * (float)(i % 97 + 1) * 0.0625f;
}
__global__ void xar_check_kernel(const float *__restrict__ v, long n, int world, unsigned int *__restrict__ bad) {
    const float tri = (float)(world * (world + 1) / 2);
    unsigned int nbad = 0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        nbad += v[i] != tri * (float)(i % 97 + 1) * 0.0625f;
    if (nbad) atomicAdd(bad, nbad);
}

struct IpcHandles {
    hipIpcMemHandle_t buf, sig;
};
static_assert(sizeof(IpcHandles) <= HPNN_XAR_HANDLE_BYTES, "handle size");

}  // namespace

struct hpnn_xar {
    int rank = 0, world = 1, device = 0;
    size_t max_bytes = 0;
    void *buf = nullptr;
    Signal *sig = nullptr;
    unsigned int *ep = nullptr; /* per-workgroup barrier epochs (this rank only) */
    XarPeers peers = {};
    bool opened[HPNN_XAR_MAX_RANKS] = {};
    unsigned long long timeout = 0;
    int mode = 0;     /* HPNN_XAR_MODE: 0 auto, 1 one-shot, 2 two-shot */
    int light = 1;    /* HPNN_XAR_FENCE=1 -> 0: full system fences, see xbarrier */
    int blocks = 128; /* HPNN_XAR_BLOCKS (same on every rank), <= HPNN_XAR_MAX_BLOCKS */
};

extern "C" hpnn_xar *hpnn_xar_create(int rank, int world, size_t max_bytes) {
    if (world < 1 || world > HPNN_XAR_MAX_RANKS || rank < 0 || rank >= world || max_bytes == 0) return nullptr;
    hpnn_xar *c = new hpnn_xar();
    c->rank = rank;
    c->world = world;
    c->max_bytes = (max_bytes + 255) / 256 * 256;
    if (hipGetDevice(&c->device) != hipSuccess ||
        hipExtMallocWithFlags(&c->buf, 2 * c->max_bytes, hipDeviceMallocUncached) != hipSuccess ||
        hipExtMallocWithFlags((void **)&c->sig, sizeof(Signal), hipDeviceMallocUncached) != hipSuccess ||
        hipMemset(c->sig, 0, sizeof(Signal)) != hipSuccess ||
        hipMalloc((void **)&c->ep, HPNN_XAR_MAX_BLOCKS * sizeof(unsigned int)) != hipSuccess ||
        hipMemset(c->ep, 0, HPNN_XAR_MAX_BLOCKS * sizeof(unsigned int)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        NN_ERROR(stderr, "xgmi all-reduce: device allocation failed\n");
        hpnn_xar_destroy(c);
        return nullptr;
    }
    int khz = 100000;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device);
    const char *e = getenv("HPNN_XAR_TIMEOUT_MS");
    const long ms = e ? atol(e) : 20000; /* generous: a late peer in the first step (lazy module loads) is not a failure */
    c->timeout = (unsigned long long)(ms > 0 ? ms : 20000) * (unsigned long long)(khz > 0 ? khz : 100000);
    const char *m = getenv("HPNN_XAR_MODE");
    c->mode = m ? atoi(m) : 0;
    const char *fe = getenv("HPNN_XAR_FENCE");
    c->light = !(fe && fe[0] == '1');
    const char *nb = getenv("HPNN_XAR_BLOCKS");
    if (nb && atoi(nb) > 0) c->blocks = atoi(nb) < HPNN_XAR_MAX_BLOCKS ? atoi(nb) : HPNN_XAR_MAX_BLOCKS;
    c->peers.buf[rank] = (float4 *)c->buf;
    c->peers.sig[rank] = c->sig;
    return c;
}

extern "C" int hpnn_xar_handles(hpnn_xar *c, void *out) {
    if (!c || !out) return -1;
    IpcHandles h;
    memset(&h, 0, sizeof h);
    if (hipIpcGetMemHandle(&h.buf, c->buf) != hipSuccess || hipIpcGetMemHandle(&h.sig, c->sig) != hipSuccess) {
        NN_ERROR(stderr, "xgmi all-reduce: hipIpcGetMemHandle failed\n");
        return -2;
    }
    memset(out, 0, HPNN_XAR_HANDLE_BYTES);
    memcpy(out, &h, sizeof h);
    return 0;
}

extern "C" int hpnn_xar_open(hpnn_xar *c, const void *all) {
    if (!c || !all) return -1;
    for (int p = 0; p < c->world; p++) {
        if (p == c->rank) continue;
        IpcHandles h;
        memcpy(&h, (const char *)all + (size_t)p * HPNN_XAR_HANDLE_BYTES, sizeof h);
        void *b = nullptr, *s = nullptr;
        if (hipIpcOpenMemHandle(&b, h.buf, hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
            hipIpcOpenMemHandle(&s, h.sig, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            NN_ERROR(stderr, "xgmi all-reduce: hipIpcOpenMemHandle of rank %d failed\n", p);
            return -2;
        }
        c->peers.buf[p] = (float4 *)b;
        c->peers.sig[p] = (Signal *)s;
        c->opened[p] = true;
    }
    return 0;
}

extern "C" size_t hpnn_xar_max_bytes(const hpnn_xar *c) { return c ? c->max_bytes : 0; }

static int xar_launch(hpnn_xar *c, const XarIn &in, float *out, long count, hipStream_t stream,
                      const XarUpd *upd = nullptr) {
    if (!c || count <= 0 || (count & 3) || (size_t)count * 4 > c->max_bytes) return -1;
    if ((uintptr_t)out & 15) return -1;
    for (int p = 0; p < c->world; p++)
        if (!c->peers.buf[p]) return -3; /* not opened */
    const long n4 = count / 4;
    /* two-shot from 4 ranks and 64 KiB up (each link then carries 2/W of the buffer
     * instead of all of it, for one extra barrier); the choice depends only on values
     * every rank shares, so all ranks run the same protocol */
    const bool two = c->mode == 2 || (c->mode == 0 && c->world >= 4 && count * 4 >= (64 << 10));
    /* the grid is the same for every call: every workgroup then takes part in every call,
     * so the per-workgroup epochs (and the data half they select) stay equal across the
     * grid -- with a size-dependent grid a workgroup skipping a call would flip halves
     * against the others and could refill elements a peer still reads.  128 workgroups:
     * half the CUs, so when several ranks share one GPU (the 1-GPU tests) a rank's
     * spinning workgroups never occupy every CU while a peer's full-CU kernel (the fused
     * MNIST front) still has to run before that peer reaches its all-reduce */
    const long blocks = c->blocks;
    const long half4 = (long)(c->max_bytes / 16);
    XarUpd none = {};
    const XarUpd &u = upd ? *upd : none;
#define HPNN_XARL(T_, U_)                                                                                          \
    hipLaunchKernelGGL((xar_kernel<T_, U_>), dim3((unsigned)blocks), dim3(256), 0, stream, c->peers, c->rank,       \
                       c->world, in, (float4 *)out, n4, half4, c->timeout, c->light, u, c->ep)
    if (two) {
        if (upd) HPNN_XARL(true, true);
        else HPNN_XARL(true, false);
    } else {
        if (upd) HPNN_XARL(false, true);
        else HPNN_XARL(false, false);
    }
#undef HPNN_XARL
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_xar_all_reduce_f32(hpnn_xar *c, const float *in, float *out, long count, hipStream_t stream) {
    if ((uintptr_t)in & 15) return -1;
    XarIn x = {};
    x.src[0] = (const float4 *)in;
    x.stride4[0] = 0;
    x.end4[0] = count / 4;
    x.S[0] = 1;
    x.nseg = 1;
    return xar_launch(c, x, out, count, stream);
}

extern "C" int hpnn_xar_all_reduce_slabs_f32(hpnn_xar *c, const hpnn_xar_seg *segs, int nseg, float *out,
                                             hipStream_t stream) {
    if (!segs || nseg < 1 || nseg > HPNN_XAR_MAX_SEGS) return -1;
    XarIn x = {};
    long tot = 0;
    for (int j = 0; j < nseg; j++) {
        const hpnn_xar_seg &g = segs[j];
        if (!g.src || g.S < 1 || g.count <= 0 || (g.count & 3) || (g.stride & 3) || ((uintptr_t)g.src & 15))
            return -1;
        x.src[j] = (const float4 *)g.src;
        x.stride4[j] = g.stride / 4;
        x.S[j] = g.S;
        tot += g.count;
        x.end4[j] = tot / 4;
    }
    x.nseg = nseg;
    return xar_launch(c, x, out, tot, stream);
}

static int xar_upd_args(const hpnn_xar_upd_layer *layers, int nl, float lr, float alpha, float scale, int momentum,
                        long tot, XarUpd &u) {
    if (!layers || nl < 1 || nl > HPNN_XAR_MAX_LAYERS) return -1;
    u = {};
    long lt = 0;
    for (int l = 0; l < nl; l++) {
        const hpnn_xar_upd_layer &L = layers[l];
        if (!L.W32 || !L.Wbf || !L.Wt || (momentum && !L.V32) || L.N <= 0 || L.K <= 0 || L.K % 4) return -1;
        /* float4 / bf16x4 accesses: misaligned tensors take the caller's fallback path */
        if (((uintptr_t)L.W32 | (uintptr_t)(momentum ? L.V32 : L.W32)) & 15 || ((uintptr_t)L.Wbf | (uintptr_t)L.Wt) & 7)
            return -1;
        if (L.Wf && (L.N % 16 || L.K % 32)) return -1;
        u.W32[l] = L.W32;
        u.V32[l] = L.V32;
        u.Wb[l] = (__bf16 *)L.Wbf;
        u.Wt[l] = (__bf16 *)L.Wt;
        u.Wf[l] = (__bf16 *)L.Wf;
        u.N[l] = L.N;
        u.K[l] = L.K;
        lt += (long)L.N * L.K;
        u.end4[l] = lt / 4;
    }
    if (lt != tot) return -2; /* the layers must tile the reduced vector exactly */
    u.nl = nl;
    u.lr = lr;
    u.alpha = alpha;
    u.scale = scale;
    u.momentum = momentum;
    return 0;
}

extern "C" int hpnn_xar_local(hpnn_xar *c, float **buf, long *half, const unsigned int **sel) {
    if (!c || !buf || !half || !sel) return -1;
    *buf = (float *)c->buf;
    *half = (long)(c->max_bytes / 4);
    *sel = c->ep; /* every workgroup's epoch is the same after each call: word 0 stands for all */
    return 0;
}

extern "C" int hpnn_xar_view_get(hpnn_xar *c, hpnn_xar_view *v) {
    if (!c || !v) return -1;
    memset(v, 0, sizeof *v);
    for (int p = 0; p < c->world; p++) {
        if (!c->peers.buf[p]) return -3; /* not opened */
        v->buf[p] = (float *)c->peers.buf[p];
        v->sig[p] = (unsigned int *)c->peers.sig[p];
    }
    v->half = (long)(c->max_bytes / 4);
    v->ep = c->ep;
    v->rank = c->rank;
    v->world = c->world;
    v->timeout = c->timeout;
    return 0;
}

extern "C" int hpnn_xar_reduce_local_update_f32(hpnn_xar *c, long count, float *out, const hpnn_xar_upd_layer *layers,
                                                int nl, float lr, float alpha, float scale, int momentum,
                                                hipStream_t stream) {
    XarUpd u;
    int r;
    if ((r = xar_upd_args(layers, nl, lr, alpha, scale, momentum, count, u))) return r;
    XarIn x = {}; /* nseg = 0: in place */
    return xar_launch(c, x, out, count, stream, &u);
}

extern "C" int hpnn_xar_all_reduce_slabs_update_f32(hpnn_xar *c, const hpnn_xar_seg *segs, int nseg, float *out,
                                                    const hpnn_xar_upd_layer *layers, int nl, float lr, float alpha,
                                                    float scale, int momentum, hipStream_t stream) {
    if (!segs || nseg < 1 || nseg > HPNN_XAR_MAX_SEGS || !layers || nl < 1 || nl > HPNN_XAR_MAX_LAYERS) return -1;
    XarIn x = {};
    long tot = 0;
    for (int j = 0; j < nseg; j++) {
        const hpnn_xar_seg &g = segs[j];
        if (!g.src || g.S < 1 || g.count <= 0 || (g.count & 3) || (g.stride & 3) || ((uintptr_t)g.src & 15))
            return -1;
        x.src[j] = (const float4 *)g.src;
        x.stride4[j] = g.stride / 4;
        x.S[j] = g.S;
        tot += g.count;
        x.end4[j] = tot / 4;
    }
    x.nseg = nseg;
    XarUpd u;
    int r;
    if ((r = xar_upd_args(layers, nl, lr, alpha, scale, momentum, tot, u))) return r;
    return xar_launch(c, x, out, tot, stream, &u);
}

extern "C" int hpnn_xar_status(hpnn_xar *c) {
    if (!c) return -1;
    unsigned int err = 0;
    if (hipMemcpy(&err, &c->sig->error, 4, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    return err ? -1 : 0;
}

extern "C" int hpnn_xar_status_enqueue(hpnn_xar *c, unsigned int *dst, hipStream_t stream) {
    if (!c) return -1;
    return hipMemcpyAsync(dst, &c->sig->error, 4, hipMemcpyDeviceToHost, stream) == hipSuccess ? 0 : -2;
}

extern "C" int hpnn_xar_self_test(hpnn_xar *c, hipStream_t stream) {
    if (!c) return -3;
    /* one-shot size (4 KiB) and the whole buffer (two-shot from 4 ranks), each twice:
     * consecutive calls use alternate halves */
    const long full = (long)(c->max_bytes / 4) & ~3L, small = full < 1024 ? full : 1024;
    float *v = nullptr;
    unsigned int *bad = nullptr;
    int rc = 0;
    if (hipMalloc((void **)&v, (size_t)full * 4) != hipSuccess || hipMalloc((void **)&bad, 4) != hipSuccess ||
        hipMemsetAsync(bad, 0, 4, stream) != hipSuccess)
        rc = -3;
    const long sizes[4] = {small, small, full, full};
    for (int t = 0; t < 4 && rc == 0; t++) {
        const long n = sizes[t];
        hipLaunchKernelGGL(xar_fill_kernel, dim3(256), dim3(256), 0, stream, v, n, c->rank);
        if (hpnn_xar_all_reduce_f32(c, v, v, n, stream) != 0) rc = -3;
        hipLaunchKernelGGL(xar_check_kernel, dim3(256), dim3(256), 0, stream, v, n, c->world, bad);
    }
    unsigned int nbad = 0;
    if (rc == 0 && (hipMemcpyAsync(&nbad, bad, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
                    hipStreamSynchronize(stream) != hipSuccess))
        rc = -3;
    if (rc == 0 && hpnn_xar_status(c) != 0) rc = -2;
    else if (rc == 0 && nbad) {
        NN_ERROR(stderr, "xgmi all-reduce self-test: %u wrong elements on rank %d\n", nbad, c->rank);
        rc = -1;
    }
    hipStreamSynchronize(stream);
    if (v) hipFree(v);
    if (bad) hipFree(bad);
    return rc;
}

extern "C" void hpnn_xar_destroy(hpnn_xar *c) {
    if (!c) return;
    hipDeviceSynchronize();
    for (int p = 0; p < HPNN_XAR_MAX_RANKS; p++) {
        if (!c->opened[p]) continue;
        hipIpcCloseMemHandle(c->peers.buf[p]);
        hipIpcCloseMemHandle(c->peers.sig[p]);
    }
    if (c->buf) hipFree(c->buf);
    if (c->sig) hipFree(c->sig);
    if (c->ep) hipFree(c->ep);
    delete c;
}
