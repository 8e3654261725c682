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

#include "kernels.h"

namespace {

constexpr int NTH = 1024;
constexpr int NWAVES = NTH / 64;
constexpr double TINY = 1e-14;

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
__device__ void layer_forward(const hpnn_online_args &a, int l, const double *in, double *out, bool use_act) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int N = a.N[l], M = a.M[l];
    const double *W = a.W[l];
    for (int j = wave; j < N; j += NWAVES) {
        const double *w = W + (size_t)j * M;
        double s = 0.0;
        for (int i = lane; i < M; i += 64) s += w[i] * in[i];
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

__device__ void forward_all(const hpnn_online_args &a, const Vecs &v, int buf, double *red) {
    const double *in = v.xin;
    for (int l = 0; l < a.L; l++) {
        const bool last = (l == a.L - 1);
        layer_forward(a, l, in, v.h[buf][l], !last || a.type == 0);
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
    forward_all(a, v, cur, red);
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
                    for (int n = 0; n < N; n++) s += W[(size_t)n * M + m] * dn[n];
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
                if (a.momentum) {
                    double *vw = dW + (size_t)j * M;
                    for (int i = lane; i < M; i += 64) {
                        double vv = vw[i] + coef * hin_old[i];
                        double ww = w[i] + vv;
                        vw[i] = vv * a.alpha;
                        w[i] = ww;
                        s += ww * hin_new[i];
                    }
                } else {
                    for (int i = lane; i < M; i += 64) {
                        double ww = w[i] + coef * hin_old[i];
                        w[i] = ww;
                        s += ww * hin_new[i];
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
    if (bytes > 48 * 1024) {
        (void)hipFuncSetAttribute((const void *)online_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    }
    hipLaunchKernelGGL(online_kernel, dim3(1), dim3(NTH), (unsigned)bytes, stream, *a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
