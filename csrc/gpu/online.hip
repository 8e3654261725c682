/*
 * libhpnn online (batch-1, iterate-to-convergence) FP64 engine for gfx950.
 *
 * Reference behaviour (ann.c:2281-2467, snn.c:1417-1595,
 * cuda_ann.cu:2098-2898): for one sample, repeat
 *     Ep = E(o); deltas with pre-update weights; update every layer (BP or
 *     BPM); re-forward; dEp = Ep - E(o')
 * until (dEp <= delta && argmax(o) == target && iter > MIN) or iter > MAX.
 * The reference launches >= 5 kernels per layer per iteration and reads the
 * output back to the host every iteration.  Here the entire loop runs in ONE
 * persistent workgroup (1024 threads = 16 wave64): vectors live in LDS,
 * weights stream through L2, the layer update and the re-forward of that
 * layer are fused (each weight is read and written once per iteration), and
 * the stop test is evaluated on the device.  The host sees one launch and
 * one 5-double result per sample.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include "kernels.h"

HPNN_CO_PROBE(online)

namespace {

constexpr int NTH = 1024;
constexpr int NWAVES = NTH / 64;
constexpr double TINY = 1e-14;

/* the vectors live in LDS (use_lds) or in global scratch, the weights in global memory;
 * all of them are reached through plain double* in the argument block, and generic
 * (flat) accesses make every load wait on both the VMEM and the LDS counter.  These
 * accessors cast to the real address space so the hot loops issue ds_read / global_load
 * and the two queues overlap (the per-iteration time of the MNIST online loop was set by
 * flat-access latency, not by bandwidth). */
typedef __attribute__((address_space(3))) double lds_d;
typedef __attribute__((address_space(1))) double glb_d;
template <bool LDS>
__device__ __forceinline__ double vld(const double *p, int i) {
    if constexpr (LDS) return ((const lds_d *)p)[i];
    else return ((const glb_d *)p)[i];
}
__device__ __forceinline__ double gld(const double *p, size_t i) { return ((const glb_d *)p)[i]; }
__device__ __forceinline__ void gst(double *p, size_t i, double v) { ((glb_d *)p)[i] = v; }

__device__ __forceinline__ double act(double x) { return 2.0 / (1.0 + exp(-1.0 * x)) - 1.0; }
__device__ __forceinline__ double dact(double y) { return -0.5 * (y * y - 1.0); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

/* block-wide sum; every thread receives the result */
__device__ double block_sum(double v, double *red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NWAVES; w++) s += red[w];
    return s;
}

struct Vecs {
    double *xin;
    double *h[2][16];
    double *d[16];
};

/* forward of layer l: out[j] = f(W_l[j,:] . in) ; wave per row */
template <bool LDS>
__device__ void layer_forward(const hpnn_online_args &a, int l, const double *in, double *out, bool use_act) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int N = a.N[l], M = a.M[l];
    const double *W = a.W[l];
    for (int j = wave; j < N; j += NWAVES) {
        const double *w = W + (size_t)j * M;
        double s = 0.0;
        for (int i = lane; i < M; i += 64) s += gld(w, i) * vld<LDS>(in, i);
        s = wave_sum(s);
        if (lane == 0) out[j] = use_act ? act(s) : s;
    }
}

/* SNN output: o = e^{z-1}/(TINY + sum e^{z-1}) (reference form, snn.c:296-335) */
__device__ void softmax_out(double *o, int N, double *red) {
    double part = 0.0;
    for (int j = threadIdx.x; j < N; j += NTH) {
        o[j] = exp(o[j] - 1.0);
        part += o[j];
    }
    const double dv = TINY + block_sum(part, red);
    for (int j = threadIdx.x; j < N; j += NTH) o[j] /= dv;
    __syncthreads();
}

__device__ double error_of(const hpnn_online_args &a, const double *o, double *red) {
    const int N = a.N[a.L - 1];
    double part = 0.0;
    for (int j = threadIdx.x; j < N; j += NTH) {
        const double t = a.t[j];
        if (a.type == 2) {
            if (o[j] > 0.) part += t * log(o[j] + TINY);
        } else {
            part += (t - o[j]) * (t - o[j]);
        }
    }
    const double s = block_sum(part, red);
    return a.type == 2 ? s * (-1.0 / (double)N) : 0.5 * s;
}

template <bool LDS>
__device__ void forward_all(const hpnn_online_args &a, const Vecs &v, int buf, double *red) {
    const double *in = v.xin;
    for (int l = 0; l < a.L; l++) {
        const bool last = (l == a.L - 1);
        layer_forward<LDS>(a, l, in, v.h[buf][l], !last || a.type == 0);
        __syncthreads();
        in = v.h[buf][l];
    }
    if (a.type == 2) softmax_out(v.h[buf][a.L - 1], a.N[a.L - 1], red);
}

/* reference argmax: probe=-1, strict '<' (first max), target = last t==1 */
__device__ void argmax_pair(const hpnn_online_args &a, const double *o, int *sidx, double *sval, int &max_p,
                            int &p_trg) {
    const int N = a.N[a.L - 1];
    double bv = -1.0;
    int bi = -1, ti = -1;
    for (int j = threadIdx.x; j < N; j += NTH) {
        if (o[j] > bv) {
            bv = o[j];
            bi = j;
        }
        if (a.t[j] == 1.0) ti = j;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        double ov = __shfl_xor(bv, off, 64);
        int oi = __shfl_xor(bi, off, 64);
        int ot = __shfl_xor(ti, off, 64);
        if (oi >= 0 && (bi < 0 || ov > bv || (ov == bv && oi < bi))) {
            bv = ov;
            bi = oi;
        }
        if (ot > ti) ti = ot;
    }
    __syncthreads();
    if (lane == 0) {
        sval[wave] = bv;
        sidx[wave] = bi;
        sidx[NWAVES + wave] = ti;
    }
    __syncthreads();
    double fv = -1.0;
    int fi = -1, ft = -1;
    for (int w = 0; w < NWAVES; w++) {
        if (sidx[w] >= 0 && (fi < 0 || sval[w] > fv || (sval[w] == fv && sidx[w] < fi))) {
            fv = sval[w];
            fi = sidx[w];
        }
        if (sidx[NWAVES + w] > ft) ft = sidx[NWAVES + w];
    }
    max_p = fi < 0 ? 0 : fi;
    p_trg = ft < 0 ? 0 : ft;
}

template <bool LDS>
__global__ __launch_bounds__(NTH) void online_kernel(hpnn_online_args a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    __shared__ double red[NWAVES];
    __shared__ double sval[NWAVES];
    __shared__ int sidx[2 * NWAVES];
    __shared__ int sflag;

    double *base = a.use_lds ? smem : a.scratch;
    Vecs v;
    size_t off = 0;
    v.xin = base;
    off += a.n_in;
    for (int l = 0; l < a.L; l++) {
        v.h[0][l] = base + off;
        off += a.N[l];
        v.h[1][l] = base + off;
        off += a.N[l];
        v.d[l] = base + off;
        off += a.N[l];
    }
    for (int i = threadIdx.x; i < a.n_in; i += NTH) v.xin[i] = a.x[i];
    __syncthreads();

    const int L = a.L;
    const int n_out = a.N[L - 1];
    int cur = 0;
    forward_all<LDS>(a, v, cur, red);
    double Ep = error_of(a, v.h[cur][L - 1], red);
    if (a.forward_only) {
        for (int j = threadIdx.x; j < n_out; j += NTH) a.out[j] = v.h[cur][L - 1][j];
        if (threadIdx.x == 0) a.result[1] = Ep;
        return;
    }
    const double init_err = Ep;
    int iter = 0, first_ok = 0, is_ok = 0;
    double dEp = 0.0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (;;) {
        iter++;
        /* ---- deltas with pre-update weights ---- */
        {
            const double *o = v.h[cur][L - 1];
            double *dl = v.d[L - 1];
            for (int j = threadIdx.x; j < n_out; j += NTH) {
                const double diff = a.t[j] - o[j];
                dl[j] = (a.type == 0) ? diff * dact(o[j]) : diff;
            }
            __syncthreads();
            for (int l = L - 2; l >= 0; l--) {
                const int N = a.N[l + 1], M = a.M[l + 1];
                const double *W = a.W[l + 1];
                const double *dn = v.d[l + 1];
                const double *h = v.h[cur][l];
                for (int m = threadIdx.x; m < M; m += NTH) {
                    double s = 0.0;
                    for (int n = 0; n < N; n++) s += gld(W, (size_t)n * M + m) * vld<LDS>(dn, n);
                    v.d[l][m] = s * dact(h[m]);
                }
                __syncthreads();
            }
        }
        /* ---- fused update + re-forward, layer by layer ---- */
        const int nxt = cur ^ 1;
        for (int l = 0; l < L; l++) {
            const int N = a.N[l], M = a.M[l];
            double *W = a.W[l];
            double *dW = a.dW[l];
            const double *hin_old = l ? v.h[cur][l - 1] : v.xin;
            const double *hin_new = l ? v.h[nxt][l - 1] : v.xin;
            const bool use_act = (l < L - 1) || a.type == 0;
            for (int j = wave; j < N; j += NWAVES) {
                const double coef = a.lr * v.d[l][j];
                double *w = W + (size_t)j * M;
                double s = 0.0;
                /* UNR row chunks per lane: all loads of a chunk are issued before its stores
                 * (the compiler cannot hoist a load above a store through generic pointers),
                 * so each wave keeps UNR x 2 x 512 B in flight instead of 1 KB -- the loop
                 * streams the weights through L2 and was latency-bound */
                constexpr int UNR = 16;
                if (a.momentum) {
                    double *vw = dW + (size_t)j * M;
                    for (int i0 = lane; i0 < M; i0 += 64 * UNR) {
                        double wv[UNR], vv[UNR];
#pragma unroll
                        for (int u = 0; u < UNR; u++) {
                            const int i = i0 + 64 * u;
                            wv[u] = i < M ? gld(w, i) : 0.0;
                            vv[u] = i < M ? gld(vw, i) : 0.0;
                        }
#pragma unroll
                        for (int u = 0; u < UNR; u++) {
                            const int i = i0 + 64 * u;
                            if (i < M) {
                                const double v2 = vv[u] + coef * vld<LDS>(hin_old, i);
                                const double ww = wv[u] + v2;
                                gst(vw, i, v2 * a.alpha);
                                gst(w, i, ww);
                                s += ww * vld<LDS>(hin_new, i);
                            }
                        }
                    }
                } else {
                    for (int i0 = lane; i0 < M; i0 += 64 * UNR) {
                        double wv[UNR];
#pragma unroll
                        for (int u = 0; u < UNR; u++) {
                            const int i = i0 + 64 * u;
                            wv[u] = i < M ? gld(w, i) : 0.0;
                        }
#pragma unroll
                        for (int u = 0; u < UNR; u++) {
                            const int i = i0 + 64 * u;
                            if (i < M) {
                                const double ww = wv[u] + coef * vld<LDS>(hin_old, i);
                                gst(w, i, ww);
                                s += ww * vld<LDS>(hin_new, i);
                            }
                        }
                    }
                }
                s = wave_sum(s);
                if (lane == 0) v.h[nxt][l][j] = use_act ? act(s) : s;
            }
            __syncthreads();
        }
        if (a.type == 2) softmax_out(v.h[nxt][L - 1], n_out, red);
        const double Epr = error_of(a, v.h[nxt][L - 1], red);
        dEp = Ep - Epr;
        Ep = Epr;
        cur = nxt;
        int max_p, p_trg;
        argmax_pair(a, v.h[cur][L - 1], sidx, sval, max_p, p_trg);
        if (threadIdx.x == 0) {
            int ok = (max_p == p_trg);
            if (iter == 1) first_ok = ok;
            int stop;
            if (iter > a.max_iter) {
                stop = 1;
            } else {
                ok = ok && (iter > a.min_iter);
                stop = !((dEp > a.delta) || !ok);
            }
            is_ok = ok;
            sflag = stop;
        }
        __syncthreads();
        const int stop = sflag;
        __syncthreads();
        if (stop) break;
    }
    for (int j = threadIdx.x; j < n_out; j += NTH) a.out[j] = v.h[cur][L - 1][j];
    if (threadIdx.x == 0) {
        a.result[0] = dEp;
        a.result[1] = init_err;
        a.result[2] = (double)iter;
        a.result[3] = (double)is_ok;
        a.result[4] = (double)first_ok;
    }
}

}  // namespace

extern "C" long hpnn_online_vec_bytes(const hpnn_online_args *a) {
    long n = a->n_in;
    for (int l = 0; l < a->L; l++) n += 3L * a->N[l];
    return n * (long)sizeof(double);
}

extern "C" int hpnn_online_launch(const hpnn_online_args *a, hipStream_t stream) {
    if (a->L < 1 || a->L > 16) return -1;
    const long bytes = a->use_lds ? hpnn_online_vec_bytes(a) : 0;
    if (bytes > 150 * 1024) return -2;
    if (a->use_lds) {
        if (bytes > 48 * 1024)
            (void)hipFuncSetAttribute((const void *)online_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)bytes);
        hipLaunchKernelGGL(online_kernel<true>, dim3(1), dim3(NTH), (unsigned)bytes, stream, *a);
    } else {
        hipLaunchKernelGGL(online_kernel<false>, dim3(1), dim3(NTH), 0, stream, *a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* ====================================================================== */
/* Cooperative online kernel: one sample, many workgroups                  */
/* ====================================================================== */
/* The single-workgroup kernel above streams every weight of the network through ONE CU
 * per iteration (784-300-10: ~80 us per iteration).  Here the rows of every layer are
 * dealt round-robin to G resident workgroups (row j of any layer -> workgroup j % G),
 * and each workgroup only ever reads and writes ITS OWN weight rows:
 *   - forward / fused update + re-forward: owner computes its rows' outputs;
 *   - hidden deltas delta_{l-1}[m] = f'(h[m]) sum_n W_l[n][m] delta_l[n]: each owner of
 *     layer-l rows publishes its partial sum over its rows for every m; the owner of
 *     row m of layer l-1 adds the partials in workgroup order (deterministic).
 * So weights never cross workgroups (no coherence traffic for 99% of the bytes); what
 * crosses are layer outputs and delta partials, stored write-through (agent-scope
 * relaxed atomics = sc1 stores), drained (vmcnt(0)), signalled by ONE counter add per
 * workgroup, and read back only with agent-scope atomic loads, so no acquire fence is
 * needed (cdna_hip_programming.md Guideline 16, R1).  2L-1 grid barriers per
 * iteration; softmax, error, argmax and the stop test are evaluated redundantly (and
 * bit-identically) by every workgroup, so all leave the loop together.  Every spin is
 * bounded: a barrier that times out sets ctl[1] and the host reports the failure. */
namespace {

constexpr int CNT = 256;           /* threads per workgroup */
constexpr int CNW = CNT / 64;      /* waves */
constexpr int COOP_MAX_GRID = 128; /* <= CUs: every workgroup resident */
constexpr unsigned long long COOP_TIMEOUT = 2000000000ULL; /* wall-clock ticks (~20 s at 100 MHz) */

typedef __attribute__((address_space(1))) double gdbl;
typedef __attribute__((address_space(1))) unsigned int gu32;

/* SYS: the grid spans several devices (exchange buffer and counters in fine-grained memory
 * every device maps): system-scope accesses, i.e. write-through to memory and reads that
 * bypass every cache on the way */
template <bool SYS>
__device__ __forceinline__ void xpub(double *p, size_t i, double v) {
    if constexpr (SYS) __hip_atomic_store((gdbl *)p + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_store((gdbl *)p + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool SYS>
__device__ __forceinline__ double xget(const double *p, size_t i) {
    if constexpr (SYS) return __hip_atomic_load((const gdbl *)p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else return __hip_atomic_load((const gdbl *)p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* counter barrier: every wave drains its write-through stores, one lane adds, one lane
 * polls until all G workgroups of this phase arrived.  Arrivals are spread over 8
 * counters on separate 64-byte lines (workgroup g adds to counter g % 8) so the adds do
 * not serialize on one address; the poller sums the 8.  Counters are never reset inside a
 * launch (zeroed by the launcher's memset); the timeout word is ctl[COOP_ERR]. */
constexpr int COOP_SUB = 8, COOP_LINE = 16, COOP_ERR = COOP_SUB * COOP_LINE;
template <bool SYS>
__device__ __forceinline__ void coop_barrier(unsigned int *ctl, unsigned int target, int g) {
    constexpr int SC = SYS ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        gu32 *c = (gu32 *)ctl;
        __hip_atomic_fetch_add(c + (g % COOP_SUB) * COOP_LINE, 1u, __ATOMIC_RELAXED, SC);
        const unsigned long long t0 = wall_clock64();
        for (;;) {
            unsigned int sum = 0;
#pragma unroll
            for (int k = 0; k < COOP_SUB; k++) sum += __hip_atomic_load(c + k * COOP_LINE, __ATOMIC_RELAXED, SC);
            if (sum >= target) break;
            /* another workgroup already timed out: every later barrier gives up at once */
            if (__hip_atomic_load(c + COOP_ERR, __ATOMIC_RELAXED, SC)) break;
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > COOP_TIMEOUT) {
                __hip_atomic_store(c + COOP_ERR, 1u, __ATOMIC_RELAXED, SC);
                break;
            }
        }
    }
    __syncthreads();
}

__device__ double cblock_sum(double v, double *red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < CNW; w++) s += red[w];
    return s;
}

/* same arithmetic as softmax_out / error_of / argmax_pair, on CNT threads */
template <class P>
__device__ void c_softmax(P o, int N, double *red) {
    double part = 0.0;
    for (int j = threadIdx.x; j < N; j += CNT) {
        o[j] = exp(o[j] - 1.0);
        part += o[j];
    }
    const double dv = TINY + cblock_sum(part, red);
    for (int j = threadIdx.x; j < N; j += CNT) o[j] /= dv;
    __syncthreads();
}

template <class P>
__device__ double c_error(const hpnn_online_args &a, P o, P t, double *red) {
    const int N = a.N[a.L - 1];
    double part = 0.0;
    for (int j = threadIdx.x; j < N; j += CNT) {
        if (a.type == 2) {
            if (o[j] > 0.) part += t[j] * log(o[j] + TINY);
        } else {
            part += (t[j] - o[j]) * (t[j] - o[j]);
        }
    }
    const double s = cblock_sum(part, red);
    return a.type == 2 ? s * (-1.0 / (double)N) : 0.5 * s;
}

template <class P>
__device__ void c_argmax(int N, P o, P t, int *sidx, double *sval, int &max_p, int &p_trg) {
    double bv = -1.0;
    int bi = -1, ti = -1;
    for (int j = threadIdx.x; j < N; j += CNT) {
        if (o[j] > bv) {
            bv = o[j];
            bi = j;
        }
        if (t[j] == 1.0) ti = j;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        double ov = __shfl_xor(bv, off, 64);
        int oi = __shfl_xor(bi, off, 64);
        int ot = __shfl_xor(ti, off, 64);
        if (oi >= 0 && (bi < 0 || ov > bv || (ov == bv && oi < bi))) {
            bv = ov;
            bi = oi;
        }
        if (ot > ti) ti = ot;
    }
    __syncthreads();
    if (lane == 0) {
        sval[wave] = bv;
        sidx[wave] = bi;
        sidx[CNW + wave] = ti;
    }
    __syncthreads();
    double fv = -1.0;
    int fi = -1, ft = -1;
    for (int w = 0; w < CNW; w++) {
        if (sidx[w] >= 0 && (fi < 0 || sval[w] > fv || (sval[w] == fv && sidx[w] < fi))) {
            fv = sval[w];
            fi = sidx[w];
        }
        if (sidx[CNW + w] > ft) ft = sidx[CNW + w];
    }
    max_p = fi < 0 ? 0 : fi;
    p_trg = ft < 0 ? 0 : ft;
}

struct CoopLayout {
    long hv[2][16]; /* exchange offsets (doubles) of layer outputs, two generations */
    long part[16];  /* delta partials of layer l: [G][M_l] */
    long total;
};

__host__ __device__ inline CoopLayout coop_layout(const hpnn_online_args &a, int G) {
    CoopLayout c;
    long off = 0;
    for (int g = 0; g < 2; g++)
        for (int l = 0; l < a.L; l++) {
            c.hv[g][l] = off;
            off += a.N[l];
        }
    for (int l = 0; l < a.L; l++) {
        c.part[l] = off;
        off += l ? (long)G * a.M[l] : 0;
    }
    c.total = off;
    return c;
}

template <bool SYS>
__global__ __launch_bounds__(CNT) void online_coop_kernel(hpnn_online_args a) {
    extern __shared__ __attribute__((aligned(16))) double cs[];
    __shared__ double red[CNW], sval[CNW];
    __shared__ int sidx[2 * CNW];
    const int slots = a.n_slots > 1 ? a.n_slots : 1;
    const int G = (int)gridDim.x * slots, g = (slots > 1 ? a.dev_slot : 0) * (int)gridDim.x + (int)blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int L = a.L, n_out = a.N[L - 1];
    const CoopLayout X = coop_layout(a, G);
    /* LDS: x | t | h[0][l] | h[1][l] | d[l] (full-length copies; d valid for own rows) */
    /* LDS-typed pointers: ds_read / ds_write instead of flat accesses */
    lds_d *const lb = (lds_d *)cs;
    lds_d *xin = lb, *tt = lb + a.n_in;
    lds_d *h[2][16], *d[16];
    {
        long off = a.n_in + n_out;
        for (int l = 0; l < L; l++) {
            h[0][l] = lb + off;
            off += a.N[l];
            h[1][l] = lb + off;
            off += a.N[l];
            d[l] = lb + off;
            off += a.N[l];
        }
    }
    for (int i = threadIdx.x; i < a.n_in; i += CNT) xin[i] = a.x[i];
    for (int i = threadIdx.x; i < n_out; i += CNT) tt[i] = a.t[i];
    __syncthreads();
    unsigned int phase = 0;
    int cur = 0;

    /* forward of the whole net into generation `gen`, rows by owner, exchanged per layer */
    auto forward = [&](int gen) {
        for (int l = 0; l < L; l++) {
            const int N = a.N[l], M = a.M[l];
            const lds_d *in = l ? h[gen][l - 1] : xin;
            const bool use_act = (l < L - 1) || a.type == 0;
            for (int r = wave; g + (long)G * r < N; r += CNW) {
                const int j = g + G * r;
                const double *w = a.W[l] + (size_t)j * M;
                double s = 0.0;
                for (int i = lane; i < M; i += 64) s += gld(w, i) * in[i];
                s = wave_sum(s);
                if (lane == 0) xpub<SYS>(a.xch, X.hv[gen][l] + j, use_act ? act(s) : s);
            }
            coop_barrier<SYS>(a.ctl, (++phase) * G, g);
            for (int i = threadIdx.x; i < N; i += CNT) h[gen][l][i] = xget<SYS>(a.xch, X.hv[gen][l] + i);
            __syncthreads();
        }
        if (a.type == 2) c_softmax(h[gen][L - 1], n_out, red);
    };

    forward(cur);
    double Ep = c_error(a, h[cur][L - 1], tt, red);
    if (a.forward_only) {
        if (g == 0) {
            for (int j = threadIdx.x; j < n_out; j += CNT) a.out[j] = h[cur][L - 1][j];
            if (threadIdx.x == 0) a.result[1] = Ep;
        }
        return;
    }
    const double init_err = Ep;
    int iter = 0, first_ok = 0, is_ok = 0;
    double dEp = 0.0;
    for (;;) {
        iter++;
        /* ---- deltas with the pre-update weights ---- */
        {
            const lds_d *o = h[cur][L - 1];
            for (int j = threadIdx.x; j < n_out; j += CNT) {
                const double diff = tt[j] - o[j];
                d[L - 1][j] = (a.type == 0) ? diff * dact(o[j]) : diff;
            }
            __syncthreads();
            for (int l = L - 1; l >= 1; l--) {
                const int N = a.N[l], M = a.M[l];
                /* partial over this workgroup's rows of layer l, for every column m */
                if (g < N) {
                    for (int m = threadIdx.x; m < M; m += CNT) {
                        double s = 0.0;
                        for (int j = g; j < N; j += G) s += gld(a.W[l], (size_t)j * M + m) * d[l][j];
                        xpub<SYS>(a.xch, X.part[l] + (long)g * M + m, s);
                    }
                }
                coop_barrier<SYS>(a.ctl, (++phase) * G, g);
                /* own rows m of layer l-1: sum the partials in workgroup order */
                const int Gp = G < N ? G : N;
                for (int r = wave; g + (long)G * r < M; r += CNW) {
                    const int m = g + G * r;
                    double s = 0.0;
                    for (int q = lane; q < Gp; q += 64) s += xget<SYS>(a.xch, X.part[l] + (long)q * M + m);
                    s = wave_sum(s);
                    if (lane == 0) d[l - 1][m] = s * dact(h[cur][l - 1][m]);
                }
                __syncthreads();
            }
        }
        /* ---- fused update + re-forward, layer by layer ---- */
        const int nxt = cur ^ 1;
        for (int l = 0; l < L; l++) {
            const int N = a.N[l], M = a.M[l];
            const lds_d *hin_old = l ? h[cur][l - 1] : xin;
            const lds_d *hin_new = l ? h[nxt][l - 1] : xin;
            const bool use_act = (l < L - 1) || a.type == 0;
            for (int r = wave; g + (long)G * r < N; r += CNW) {
                const int j = g + G * r;
                const double coef = a.lr * d[l][j];
                double *w = a.W[l] + (size_t)j * M;
                double s = 0.0;
                if (a.momentum) {
                    double *vw = a.dW[l] + (size_t)j * M;
                    for (int i = lane; i < M; i += 64) {
                        const double v2 = gld(vw, i) + coef * hin_old[i];
                        const double ww = gld(w, i) + v2;
                        gst(vw, i, v2 * a.alpha);
                        gst(w, i, ww);
                        s += ww * hin_new[i];
                    }
                } else {
                    for (int i = lane; i < M; i += 64) {
                        const double ww = gld(w, i) + coef * hin_old[i];
                        gst(w, i, ww);
                        s += ww * hin_new[i];
                    }
                }
                s = wave_sum(s);
                if (lane == 0) xpub<SYS>(a.xch, X.hv[nxt][l] + j, use_act ? act(s) : s);
            }
            coop_barrier<SYS>(a.ctl, (++phase) * G, g);
            for (int i = threadIdx.x; i < N; i += CNT) h[nxt][l][i] = xget<SYS>(a.xch, X.hv[nxt][l] + i);
            __syncthreads();
        }
        if (a.type == 2) c_softmax(h[nxt][L - 1], n_out, red);
        const double Epr = c_error(a, h[nxt][L - 1], tt, red);
        dEp = Ep - Epr;
        Ep = Epr;
        cur = nxt;
        int max_p, p_trg;
        c_argmax(n_out, h[cur][L - 1], tt, sidx, sval, max_p, p_trg);
        int ok = (max_p == p_trg);
        if (iter == 1) first_ok = ok;
        int stop;
        if (iter > a.max_iter) {
            stop = 1;
        } else {
            ok = ok && (iter > a.min_iter);
            stop = !((dEp > a.delta) || !ok);
        }
        is_ok = ok;
        /* every workgroup holds the same values: the same decision everywhere; a timed-out
         * barrier (ctl[1]) ends the loop on every workgroup that sees it */
        if (__hip_atomic_load((gu32 *)a.ctl + COOP_ERR, __ATOMIC_RELAXED,
                              SYS ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT))
            stop = 1;
        if (stop) break;
    }
    if (g == 0) {
        for (int j = threadIdx.x; j < n_out; j += CNT) a.out[j] = h[cur][L - 1][j];
        if (threadIdx.x == 0) {
            a.result[0] = dEp;
            a.result[1] = init_err;
            a.result[2] = (double)iter;
            a.result[3] = (double)is_ok;
            a.result[4] = (double)first_ok;
        }
    }
}

}  // namespace

extern "C" int hpnn_online_coop_grid(const hpnn_online_args *a) {
    static const int off = [] { const char *e = getenv("HPNN_ONLINE_COOP"); return e && e[0] == '0'; }();
    if (off || a->L < 1 || a->L > 16) return 0;
    int maxn = 0;
    long lds = a->n_in + a->N[a->L - 1];
    for (int l = 0; l < a->L; l++) {
        maxn = a->N[l] > maxn ? a->N[l] : maxn;
        lds += 3L * a->N[l];
    }
    if (lds * 8 > 150 * 1024) return 0;
    /* one row per wave per pass; tiny nets stay on the single-workgroup kernel */
    int G = (maxn + CNW - 1) / CNW;
    if (G > COOP_MAX_GRID) G = COOP_MAX_GRID;
    return G >= 8 ? G : 0;
}

extern "C" int hpnn_online_coop_grid_slots(const hpnn_online_args *a, int n_slots, int per_device_cap) {
    if (n_slots <= 1) return hpnn_online_coop_grid(a);
    if (a->L < 1 || a->L > 16) return 0;
    int maxn = 0;
    long lds = a->n_in + a->N[a->L - 1];
    for (int l = 0; l < a->L; l++) {
        maxn = a->N[l] > maxn ? a->N[l] : maxn;
        lds += 3L * a->N[l];
    }
    if (lds * 8 > 150 * 1024) return 0;
    /* one row per wave per pass over all slots' workgroups */
    int g = (maxn + CNW * n_slots - 1) / (CNW * n_slots);
    const int cap = per_device_cap < COOP_MAX_GRID ? per_device_cap : COOP_MAX_GRID;
    if (g > cap) g = cap;
    return g >= 1 ? g : 0;
}

/* grid: the TOTAL number of workgroups (n_slots x per-slot grid) */
extern "C" long hpnn_online_coop_xch_bytes(const hpnn_online_args *a, int grid) {
    return coop_layout(*a, grid).total * (long)sizeof(double);
}

/* n_slots > 1: the caller zeroes ctl once, before any slot is launched */
extern "C" int hpnn_online_coop_launch(const hpnn_online_args *a, int grid, hipStream_t stream) {
    if (grid < 1 || grid > COOP_MAX_GRID || !a->xch || !a->ctl) return -1;
    long lds = a->n_in + a->N[a->L - 1];
    for (int l = 0; l < a->L; l++) lds += 3L * a->N[l];
    const unsigned bytes = (unsigned)(lds * 8);
    const bool sys = a->n_slots > 1;
    const void *fn = sys ? (const void *)online_coop_kernel<true> : (const void *)online_coop_kernel<false>;
    if (bytes > 48 * 1024) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (!sys && hipMemsetAsync(a->ctl, 0, HPNN_ONLINE_CTL_BYTES, stream) != hipSuccess) return -5;
    if (sys)
        hipLaunchKernelGGL(online_coop_kernel<true>, dim3(grid), dim3(CNT), bytes, stream, *a);
    else
        hipLaunchKernelGGL(online_coop_kernel<false>, dim3(grid), dim3(CNT), bytes, stream, *a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_online_coop_status(const hpnn_online_args *a) {
    unsigned int v = 0;
    if (hipMemcpy(&v, a->ctl + COOP_ERR, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    return v ? -1 : 0;
}
