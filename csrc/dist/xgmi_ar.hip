/*
 * One-shot xGMI all-reduce (include/libhpnn/xar.h).
 *
 * Each rank owns two fine-grained (uncached) device allocations that every peer maps
 * through hipIpc: a data buffer (max_bytes) and a signal block (barrier flags).  One
 * kernel launch per all-reduce; workgroup b owns float4 slice b of the buffer:
 *   1. copy its slice of `in` into this rank's data buffer;
 *   2. barrier "start": write epoch e into start[b][rank] of every peer's signal block,
 *      wait until start[b][p] >= e for every p in this rank's block;
 *   3. out[slice] = sum_{p = 0..world-1} data_p[slice] (fixed rank order: every rank
 *      computes the same bits);
 *   4. barrier "end" (same protocol): no rank refills its data slice while a peer may
 *      still read it.
 * Epochs are per workgroup, kept in this rank's signal block and advanced by the kernel,
 * so launches captured in a HIP graph replay correctly; all ranks issue the same
 * sequence of all-reduces, so the epochs agree.  Every wait is bounded by a wall-clock
 * timeout: a missing peer sets the error word, never hangs the GPU.
 *
 * Fine-grained memory keeps peer reads coherent without cache maintenance; the
 * system-scope fences order the data stores before the flag stores.
 * Replaces the reference's hub copies through GPU0 (cuda_ann.cu EXP model).
 */
#include <hip/hip_runtime.h>
#include <libhpnn.h>
#include <libhpnn/xar.h>
#include <stdlib.h>
#include <string.h>

namespace {

struct Signal {
    unsigned int start[HPNN_XAR_MAX_BLOCKS][HPNN_XAR_MAX_RANKS];
    unsigned int end[HPNN_XAR_MAX_BLOCKS][HPNN_XAR_MAX_RANKS];
    unsigned int epoch[HPNN_XAR_MAX_BLOCKS];
    unsigned int error;
};

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
__device__ __forceinline__ void xbarrier(const XarPeers &P, int rank, int world, int b, unsigned int e, bool end,
                                         unsigned long long timeout) {
    __threadfence_system(); /* this thread's data stores before any flag store */
    __syncthreads();
    const int t = threadIdx.x;
    if (t < world) {
        Signal *peer = P.sig[t];
        flag_store(end ? &peer->end[b][rank] : &peer->start[b][rank], e);
        Signal *me = P.sig[rank];
        unsigned int *f = end ? &me->end[b][t] : &me->start[b][t];
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
    __threadfence_system();
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

__device__ __forceinline__ float4 xar_load_in(const XarIn &in, long i) {
    int j = 0;
    while (j + 1 < in.nseg && i >= in.end4[j]) j++;
    const long li = i - (j ? in.end4[j - 1] : 0);
    const float4 *p = in.src[j] + li;
    const long st = in.stride4[j];
    float4 a = p[0];
    if (in.S[j] > 1) {
        float4 b = p[st];
        int s = 2;
        for (; s + 1 < in.S[j]; s += 2) {
            const float4 x = p[(long)s * st], y = p[(long)(s + 1) * st];
            a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
            b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
        }
        if (s < in.S[j]) {
            const float4 x = p[(long)s * st];
            a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
        }
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    return a;
}

__global__ __launch_bounds__(256) void xar_kernel(XarPeers P, int rank, int world, XarIn in,
                                                  float4 *__restrict__ out, long n4, unsigned long long timeout) {
    const int b = blockIdx.x;
    Signal *me = P.sig[rank];
    __shared__ unsigned int s_ep;
    if (threadIdx.x == 0) {
        const unsigned int e = me->epoch[b] + 1; /* only this workgroup writes epoch[b] */
        me->epoch[b] = e;
        s_ep = e;
    }
    __syncthreads();
    const unsigned int e = s_ep;
    const long per = (n4 + gridDim.x - 1) / gridDim.x;
    const long lo = (long)b * per, hi = lo + per < n4 ? lo + per : n4;
    float4 *mine = P.buf[rank];
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = xar_load_in(in, i);
    xbarrier(P, rank, world, b, e, false, timeout);
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        float4 v[HPNN_XAR_MAX_RANKS];
#pragma unroll
        for (int p = 0; p < HPNN_XAR_MAX_RANKS; p++)
            if (p < world) v[p] = P.buf[p][i];
        float4 s = v[0];
#pragma unroll
        for (int p = 1; p < HPNN_XAR_MAX_RANKS; p++)
            if (p < world) {
                s.x += v[p].x;
                s.y += v[p].y;
                s.z += v[p].z;
                s.w += v[p].w;
            }
        out[i] = s;
    }
    xbarrier(P, rank, world, b, e, true, timeout);
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
    XarPeers peers = {};
    bool opened[HPNN_XAR_MAX_RANKS] = {};
    unsigned long long timeout = 0;
};

extern "C" hpnn_xar *hpnn_xar_create(int rank, int world, size_t max_bytes) {
    if (world < 1 || world > HPNN_XAR_MAX_RANKS || rank < 0 || rank >= world || max_bytes == 0) return nullptr;
    hpnn_xar *c = new hpnn_xar();
    c->rank = rank;
    c->world = world;
    c->max_bytes = (max_bytes + 255) / 256 * 256;
    if (hipGetDevice(&c->device) != hipSuccess ||
        hipExtMallocWithFlags(&c->buf, c->max_bytes, hipDeviceMallocUncached) != hipSuccess ||
        hipExtMallocWithFlags((void **)&c->sig, sizeof(Signal), hipDeviceMallocUncached) != hipSuccess ||
        hipMemset(c->sig, 0, sizeof(Signal)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        NN_ERROR(stderr, "xgmi all-reduce: device allocation failed\n");
        hpnn_xar_destroy(c);
        return nullptr;
    }
    int khz = 100000;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device);
    const char *e = getenv("HPNN_XAR_TIMEOUT_MS");
    const long ms = e ? atol(e) : 5000;
    c->timeout = (unsigned long long)(ms > 0 ? ms : 5000) * (unsigned long long)(khz > 0 ? khz : 100000);
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

static int xar_launch(hpnn_xar *c, const XarIn &in, float *out, long count, hipStream_t stream) {
    if (!c || count <= 0 || (count & 3) || (size_t)count * 4 > c->max_bytes) return -1;
    if ((uintptr_t)out & 15) return -1;
    for (int p = 0; p < c->world; p++)
        if (!c->peers.buf[p]) return -3; /* not opened */
    const long n4 = count / 4;
    long blocks = (n4 + 127) / 128; /* ~half a float4 per thread: many CUs share the slab reads */
    if (blocks > HPNN_XAR_MAX_BLOCKS) blocks = HPNN_XAR_MAX_BLOCKS;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(xar_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, c->peers, c->rank, c->world, in,
                       (float4 *)out, n4, c->timeout);
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

extern "C" int hpnn_xar_status(hpnn_xar *c) {
    if (!c) return -1;
    unsigned int err = 0;
    if (hipMemcpy(&err, &c->sig->error, 4, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    return err ? -1 : 0;
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
    delete c;
}
