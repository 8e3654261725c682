/*
 * FP64 / FP32 batched-engine kernels (gfx950): the reference-precision path of the GPU
 * batched engine ([dtype] f64 | f32).  The reference computes everything in double
 * (cuda_ann.cu:41-148 kernels, cublasDgemv / cublasDger at cuda_ann.cu:546-548 and
 * 2139-2142); here the dense products run on the matrix cores' exact FP64 / FP32 MFMA
 * (v_mfma_f64_16x16x4_f64, v_mfma_f32_16x16x4_f32: one rounding per product, the result
 * of a k-ordered fma chain), with the reference's epilogues fused:
 *
 *   gemm_fp   C[M x N] = sum_k A(m, k) B(n, k), A(m, k) = A[m][k] or A[k][m] (TA),
 *             B(n, k) = B[n][k] or B[k][n] (TB); epilogue none / bipolar f / * f'(aux);
 *             split-K over blockIdx.z into slabs (weight gradients: k = the batch).
 *   output_fp softmax / bipolar / linear output, loss, delta, argmax hits (one wave
 *             per sample row, any n_out).
 *   update_fp slab sum * scale, BP (W += lr g) or BPM (V += lr g; W += V; V *= alpha).
 *
 * Tiles: 256-thread workgroups, 64 x 64 output tile (4 waves x 2 x 2 MFMA tiles of
 * 16 x 16), K in steps of 16 staged k-major in LDS ([16][64 + 16]: the padding puts the
 * two k-rows a ds_read_b64 / b32 half-wave reads into disjoint banks), the next k-step's
 * operands loaded to registers while the current one is multiplied.  Any M, N, K (edges
 * zero-filled); operands need no padding.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kernels.h"

HPNN_CO_PROBE(fp)

namespace {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) double f64x4;

constexpr int BM = 64, BN = 64, BK = 16, LDT = BM + 16;
constexpr double TINY = 1e-14, LOG_TINY = -32.236191301916641; /* common.h TINY, ln(1e-14) */

template <typename T>
struct Acc;
template <>
struct Acc<double> {
    typedef f64x4 type;
    __device__ static f64x4 mma(double a, double b, f64x4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
    /* C/D of the f64 form: col = lane & 15, row = (lane >> 4) + 4 r */
    __device__ static int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <>
struct Acc<float> {
    typedef f32x4 type;
    __device__ static f32x4 mma(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
    /* standard C/D map: col = lane & 15, row = 4 (lane >> 4) + r */
    __device__ static int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

template <typename T>
__device__ __forceinline__ T act_fp(T x) {
    return (T)2 / ((T)1 + exp(-x)) - (T)1;
}
template <typename T>
__device__ __forceinline__ T dact_fp(T y) {
    return (T)(-0.5) * (y * y - (T)1);
}

/* one operand tile [BK][BM] (k-major) of a 64-row block: 4 elements per thread */
template <typename T, bool TRANS>
__device__ __forceinline__ void load_tile(const T *__restrict__ P, int ld, int r0, int k0, int R, int K, T (&v)[4]) {
    const int t = threadIdx.x;
    if (!TRANS) { /* P[r][k]: k contiguous -> thread reads 4 consecutive k of one row */
        const int r = r0 + (t >> 2), k = k0 + (t & 3) * 4;
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = (r < R && k + i < K) ? P[(size_t)r * ld + k + i] : (T)0;
    } else { /* P[k][r]: r contiguous -> 4 consecutive r of one k */
        const int k = k0 + (t >> 4), r = r0 + (t & 15) * 4;
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = (k < K && r + i < R) ? P[(size_t)k * ld + r + i] : (T)0;
    }
}
template <typename T, bool TRANS>
__device__ __forceinline__ void store_tile(T *s, const T (&v)[4]) {
    const int t = threadIdx.x;
    if (!TRANS) {
        const int r = t >> 2, k = (t & 3) * 4;
#pragma unroll
        for (int i = 0; i < 4; i++) s[(k + i) * LDT + r] = v[i];
    } else {
        const int k = t >> 4, r = (t & 15) * 4;
#pragma unroll
        for (int i = 0; i < 4; i++) s[k * LDT + r + i] = v[i];
    }
}

template <typename T, int EPI, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_fp_kernel(const T *__restrict__ A, int lda, const T *__restrict__ B, int ldb,
                                                      T *__restrict__ C, int ldc, const T *__restrict__ aux, int ldaux,
                                                      int M, int N, int K, int kchunk, long slab_stride) {
    typedef typename Acc<T>::type accT;
    __shared__ T As[BK * LDT], Bs[BK * LDT];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
    C += (size_t)blockIdx.z * slab_stride;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    accT acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = accT{0, 0, 0, 0};
    T va[4], vb[4];
    if (kb < ke) {
        load_tile<T, TA>(A, lda, m0, kb, M, ke, va);
        load_tile<T, TB>(B, ldb, n0, kb, N, ke, vb);
    }
    for (int k0 = kb; k0 < ke; k0 += BK) {
        __syncthreads();
        store_tile<T, TA>(As, va);
        store_tile<T, TB>(Bs, vb);
        __syncthreads();
        if (k0 + BK < ke) {
            load_tile<T, TA>(A, lda, m0, k0 + BK, M, ke, va);
            load_tile<T, TB>(B, ldb, n0, k0 + BK, N, ke, vb);
        }
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
            const int k = kk + (lane >> 4);
            T a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; i++) a[i] = As[k * LDT + wm + 16 * i + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 2; j++) b[j] = Bs[k * LDT + wn + 16 * j + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) acc[i][j] = Acc<T>::mma(a[i], b[j], acc[i][j]);
        }
    }
    /* epilogue: D[row][col] with A as the MFMA A operand (rows m) and B as B (cols n) */
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = m0 + wm + 16 * i + Acc<T>::row(lane, r), n = n0 + wn + 16 * j + (lane & 15);
                if (m >= M || n >= N) continue;
                T v = acc[i][j][r];
                if constexpr (EPI == HPNN_EPI_ACT) v = act_fp<T>(v);
                if constexpr (EPI == HPNN_EPI_DACT) v *= dact_fp<T>(aux[(size_t)m * ldaux + n]);
                C[(size_t)m * ldc + n] = v;
            }
}

/* ---- 128 x 128 tiles: the large-GEMM path -------------------------------------------
 * 256 threads = 4 waves in 2 x 2, wave tile 64 x 64 = 4 x 4 MFMA tiles (16 accumulators);
 * K in stages of 16 (4 MFMA k-steps), two LDS stages: the next stage's operands are loaded
 * with 16-byte global loads into registers while the current stage is multiplied, then
 * written to the other LDS buffer; one barrier per stage.  Both operands are staged k-major
 * ([16][BM + 16]): an MFMA fragment (16 consecutive rows x 4 k) is one ds_read_b64 / b32 per
 * lane, and the 16-element padding puts the two k-rows a half-wave reads into disjoint banks.
 * Column c of k-row k holds row c ^ swz(k) (swz permutes within 16-row groups, so fragment
 * reads stay conflict-free): with it the stores of row-major ([row][k]) operands, where the
 * lanes of a group write 8 (f64) / 4 (f32) different k-rows, hit distinct banks too.
 * Per stage and CU: f64 64 MFMAs x 64 cycles per SIMD against 32 KiB staged -- the
 * matrix-core rate of FP64 needs ~8 B/clock/CU from the L2. */
constexpr int BB = 128, LDB = BB + 16;

template <typename T>
struct FpBig {
    static constexpr int VW = 16 / sizeof(T); /* elements per 16-byte load */
    /* column swizzle of k-row k (see above) */
    __device__ static int swz(int k) { return sizeof(T) == 8 ? ((k >> 1) & 7) * 2 : ((k >> 2) & 3) * 8; }
};

/* one operand stage: rows [r0, r0 + 128) x k [k0, k0 + 16) of P (row-major [row][k] when
 * !TRANS, [k][row] when TRANS) into registers: NL chunks of VW elements per thread */
template <typename T, bool TRANS>
struct StageLoad {
    static constexpr int VW = FpBig<T>::VW;
    static constexpr int NL = BB * BK / VW / 256;
    T v[NL][VW];
    __device__ void load(const T *__restrict__ P, int ld, int r0, int k0, int R, int K, bool vec) {
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < NL; i++) {
            int r, k;
            if (!TRANS) { /* lanes along k first: BK / VW lanes cover a row's 16 k */
                constexpr int LPR = BK / VW;
                r = r0 + (t + 256 * i) / LPR;
                k = k0 + ((t + 256 * i) % LPR) * VW;
            } else { /* lanes along the rows: BB / VW lanes cover one k-row */
                constexpr int LPK = BB / VW;
                k = k0 + (t + 256 * i) / LPK;
                r = r0 + ((t + 256 * i) % LPK) * VW;
            }
            const T *src = !TRANS ? P + (size_t)r * ld + k : P + (size_t)k * ld + r;
            const bool whole = !TRANS ? (r < R && k + VW <= K) : (k < K && r + VW <= R);
            if (vec && whole) {
                typedef __attribute__((ext_vector_type(VW))) T vT;
                const vT x = *(const vT *)src;
#pragma unroll
                for (int e = 0; e < VW; e++) v[i][e] = x[e];
            } else {
#pragma unroll
                for (int e = 0; e < VW; e++) {
                    const bool in = !TRANS ? (r < R && k + e < K) : (k < K && r + e < R);
                    v[i][e] = in ? src[e] : (T)0;
                }
            }
        }
    }
    __device__ void store(T *s) const {
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < NL; i++) {
            if (!TRANS) {
                constexpr int LPR = BK / VW;
                const int r = (t + 256 * i) / LPR, k = ((t + 256 * i) % LPR) * VW;
#pragma unroll
                for (int e = 0; e < VW; e++) s[(k + e) * LDB + (r ^ FpBig<T>::swz(k + e))] = v[i][e];
            } else {
                constexpr int LPK = BB / VW;
                const int k = (t + 256 * i) / LPK, r = ((t + 256 * i) % LPK) * VW;
                typedef __attribute__((ext_vector_type(VW))) T vT;
                vT x;
#pragma unroll
                for (int e = 0; e < VW; e++) x[e] = v[i][e];
                *(vT *)(s + k * LDB + (r ^ FpBig<T>::swz(k))) = x; /* swz keeps VW-aligned runs contiguous */
            }
        }
    }
};

template <typename T, int EPI, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_fp_big_kernel(const T *__restrict__ A, int lda, const T *__restrict__ B,
                                                          int ldb, T *__restrict__ C, int ldc, const T *__restrict__ aux,
                                                          int ldaux, int M, int N, int K, int kchunk, long slab_stride,
                                                          int vec, int tiles_n) {
    typedef typename Acc<T>::type accT;
    __shared__ T As[2][BK * LDB], Bs[2][BK * LDB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    /* XCD-aware order: consecutive tiles of a row of C (sharing the A rows) on one XCD */
    const int nt = gridDim.x, b = blockIdx.x;
    const int per = nt / 8, rem = nt % 8, x = b & 7, j = b >> 3;
    const int tile = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + j;
    const int m0 = (tile / tiles_n) * BB, n0 = (tile % tiles_n) * BB;
    const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
    C += (size_t)blockIdx.z * slab_stride;
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    accT acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int jj = 0; jj < 4; jj++) acc[i][jj] = accT{0, 0, 0, 0};
    StageLoad<T, TA> la;
    StageLoad<T, TB> lb;
    const int nst = (ke - kb + BK - 1) / BK;
    if (nst > 0) {
        la.load(A, lda, m0, kb, M, ke, vec);
        lb.load(B, ldb, n0, kb, N, ke, vec);
        la.store(As[0]);
        lb.store(Bs[0]);
    }
    __syncthreads();
    const int fr = lane & 15, fk = lane >> 4;
    for (int st = 0; st < nst; st++) {
        const int cur = st & 1;
        if (st + 1 < nst) {
            la.load(A, lda, m0, kb + (st + 1) * BK, M, ke, vec);
            lb.load(B, ldb, n0, kb + (st + 1) * BK, N, ke, vec);
        }
        const T *as = As[cur], *bs = Bs[cur];
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
            const int k = kk + fk, sw = FpBig<T>::swz(k);
            T a[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; i++) a[i] = as[k * LDB + ((wm + 16 * i + fr) ^ sw)];
#pragma unroll
            for (int jj = 0; jj < 4; jj++) bv[jj] = bs[k * LDB + ((wn + 16 * jj + fr) ^ sw)];
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int jj = 0; jj < 4; jj++) acc[i][jj] = Acc<T>::mma(a[i], bv[jj], acc[i][jj]);
        }
        if (st + 1 < nst) {
            la.store(As[cur ^ 1]);
            lb.store(Bs[cur ^ 1]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int jj = 0; jj < 4; jj++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = m0 + wm + 16 * i + Acc<T>::row(lane, r), n = n0 + wn + 16 * jj + fr;
                if (m >= M || n >= N) continue;
                T v = acc[i][jj][r];
                if constexpr (EPI == HPNN_EPI_ACT) v = act_fp<T>(v);
                if constexpr (EPI == HPNN_EPI_DACT) v *= dact_fp<T>(aux[(size_t)m * ldaux + n]);
                C[(size_t)m * ldc + n] = v;
            }
}

template <typename T>
__device__ __forceinline__ T wave_max_fp(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_sum_fp(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

/* one wave per sample row; O (optional) receives the network output, guess (optional)
 * the argmax index of the output (the reference's evaluation rule: first maximum) */
template <typename T>
__global__ __launch_bounds__(256) void output_fp_kernel(const T *__restrict__ Z, int ldz, const T *__restrict__ Tg,
                                                        int ldt, T *__restrict__ D, int ldd, T *__restrict__ O, int ldo,
                                                        int *__restrict__ guess, float *__restrict__ loss_acc,
                                                        unsigned int *__restrict__ correct, int B, int n_valid,
                                                        int n_out, int type) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= B) return;
    const bool valid = row < n_valid;
    const T *z = Z + (size_t)row * ldz;
    T zmax = -INFINITY, den = 0;
    if (type == 2) {
        for (int c = lane; c < n_out; c += 64) zmax = fmax(zmax, z[c]);
        zmax = wave_max_fp(zmax);
        for (int c = lane; c < n_out; c += 64) den += exp(z[c] - zmax);
        den = wave_sum_fp(den);
        /* reference: e^{z-1} / (TINY + sum e^{z-1}), here in the max-shifted frame */
        den += exp(fmin((T)LOG_TINY + (T)1 - zmax, (T)(sizeof(T) == 8 ? 700 : 80)));
    }
    T loss = 0, bo = -INFINITY, bt = -INFINITY;
    int io = 1 << 30, it = 1 << 30;
    for (int c = lane; c < n_out; c += 64) {
        T o;
        if (type == 2) o = exp(z[c] - zmax) / den;
        else if (type == 0) o = act_fp<T>(z[c]);
        else o = z[c];
        if (O) O[(size_t)row * ldo + c] = o;
        T d = 0;
        if (valid && Tg) {
            const T t = Tg[(size_t)row * ldt + c];
            if (type == 2) {
                if (o > (T)0) loss += t * log(o + (T)TINY);
                d = t - o;
            } else {
                loss += (t - o) * (t - o);
                d = type == 0 ? (t - o) * dact_fp<T>(o) : t - o;
            }
            if (t > bt) { bt = t; it = c; }
        }
        if (o > bo) { bo = o; io = c; }
        if (D) D[(size_t)row * ldd + c] = d;
    }
    /* first maximum over the row (lowest index on ties) */
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const T ob = __shfl_xor(bo, o, 64), tb = __shfl_xor(bt, o, 64);
        const int oi = __shfl_xor(io, o, 64), ti = __shfl_xor(it, o, 64);
        if (ob > bo || (ob == bo && oi < io)) { bo = ob; io = oi; }
        if (tb > bt || (tb == bt && ti < it)) { bt = tb; it = ti; }
    }
    loss = wave_sum_fp(loss);
    if (lane == 0) {
        if (guess) guess[row] = io;
        if (valid && Tg) {
            const float l = (float)(type == 2 ? -loss / (T)n_out : (T)0.5 * loss);
            if (loss_acc) atomicAdd(loss_acc + HPNN_STAT_SLOT(blockIdx.x), l);
            if (correct && io == it) atomicAdd(correct + HPNN_STAT_SLOT(blockIdx.x), 1u);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void update_fp_kernel(T *__restrict__ W, T *__restrict__ V, const T *__restrict__ G,
                                                        int S, long gstride, long n, T lr, T alpha, T scale,
                                                        int momentum) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        T g = 0;
        for (int s = 0; s < S; s++) g += G[(size_t)s * gstride + i];
        g *= scale;
        if (momentum) {
            T v = V[i] + lr * g;
            W[i] += v;
            V[i] = v * alpha;
        } else {
            W[i] += lr * g;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void reduce_fp_kernel(T *__restrict__ out, const T *__restrict__ G, int S,
                                                        long gstride, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        T g = 0;
        for (int s = 0; s < S; s++) g += G[(size_t)s * gstride + i];
        out[i] = g;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void dact_fp_kernel(T *__restrict__ out, const T *__restrict__ in,
                                                      const T *__restrict__ aux, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        out[i] = in[i] * dact_fp<T>(aux[i]);
}

template <typename T>
int gemm_fp(const void *A, int lda, int ta, const void *B, int ldb, int tb, void *C, int ldc, const void *aux,
            int ldaux, int M, int N, int K, int epi, int splits, long slab_stride, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0 || splits < 1) return -2;
    if (epi == HPNN_EPI_DACT && !aux) return -2;
    const int kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
    const int sp = (K + kchunk - 1) / kchunk;
    /* 128 x 128 tiles once they fill the chip (>= 256 workgroups with the splits); the
     * 64 x 64 kernel below for the small products of narrow layers (HPNN_FP_BIG=0: always) */
    static const bool big_on = [] { const char *e = getenv("HPNN_FP_BIG"); return !(e && e[0] == '0'); }();
    const long tiles_big = (long)((M + BB - 1) / BB) * ((N + BB - 1) / BB);
    if (big_on && tiles_big * sp >= 256) {
        const uintptr_t al = (uintptr_t)A | (uintptr_t)B;
        const int vec = (al % 16 == 0 && lda % FpBig<T>::VW == 0 && ldb % FpBig<T>::VW == 0) ? 1 : 0;
        const int tn = (N + BB - 1) / BB;
        dim3 g2((unsigned)tiles_big, 1, sp);
#define HPNN_GB(E, A_, B_)                                                                                          \
    hipLaunchKernelGGL((gemm_fp_big_kernel<T, E, A_, B_>), g2, dim3(256), 0, s, (const T *)A, lda, (const T *)B, ldb, \
                       (T *)C, ldc, (const T *)aux, ldaux, M, N, K, kchunk, slab_stride, vec, tn)
#define HPNN_GBT(E)                                   \
    if (ta && tb) HPNN_GB(E, true, true);             \
    else if (ta) HPNN_GB(E, true, false);             \
    else if (tb) HPNN_GB(E, false, true);             \
    else HPNN_GB(E, false, false)
        if (epi == HPNN_EPI_ACT) { HPNN_GBT(HPNN_EPI_ACT); }
        else if (epi == HPNN_EPI_DACT) { HPNN_GBT(HPNN_EPI_DACT); }
        else { HPNN_GBT(HPNN_EPI_NONE); }
#undef HPNN_GBT
#undef HPNN_GB
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, sp);
#define HPNN_GF(E, A_, B_)                                                                                        \
    hipLaunchKernelGGL((gemm_fp_kernel<T, E, A_, B_>), grid, dim3(256), 0, s, (const T *)A, lda, (const T *)B, ldb, \
                       (T *)C, ldc, (const T *)aux, ldaux, M, N, K, kchunk, slab_stride)
#define HPNN_GFT(E)                                   \
    if (ta && tb) HPNN_GF(E, true, true);             \
    else if (ta) HPNN_GF(E, true, false);             \
    else if (tb) HPNN_GF(E, false, true);             \
    else HPNN_GF(E, false, false)
    if (epi == HPNN_EPI_ACT) { HPNN_GFT(HPNN_EPI_ACT); }
    else if (epi == HPNN_EPI_DACT) { HPNN_GFT(HPNN_EPI_DACT); }
    else { HPNN_GFT(HPNN_EPI_NONE); }
#undef HPNN_GFT
#undef HPNN_GF
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace

/* slabs a split-K gemm_fp writes for `splits` requested over K (k-chunks are whole BK steps) */
extern "C" int hpnn_gemm_fp_splits(int K, int splits) {
    if (K <= 0 || splits < 1) return 1;
    const int kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
    return (K + kchunk - 1) / kchunk;
}

extern "C" int hpnn_gemm_fp(int f64, const void *A, int lda, int ta, const void *B, int ldb, int tb, void *C, int ldc,
                            const void *aux, int ldaux, int M, int N, int K, int epi, int splits, long slab_stride,
                            hipStream_t stream) {
    return f64 ? gemm_fp<double>(A, lda, ta, B, ldb, tb, C, ldc, aux, ldaux, M, N, K, epi, splits, slab_stride, stream)
               : gemm_fp<float>(A, lda, ta, B, ldb, tb, C, ldc, aux, ldaux, M, N, K, epi, splits, slab_stride, stream);
}

extern "C" int hpnn_output_fp(int f64, const void *Z, int ldz, const void *T, int ldt, void *D, int ldd, void *O,
                              int ldo, int *guess, float *loss_acc, unsigned int *correct, int B, int n_valid,
                              int n_out, int type, hipStream_t stream) {
    if (B <= 0 || n_out < 1) return -2;
    const dim3 grid((B + 3) / 4);
    if (f64)
        hipLaunchKernelGGL(output_fp_kernel<double>, grid, dim3(256), 0, stream, (const double *)Z, ldz,
                           (const double *)T, ldt, (double *)D, ldd, (double *)O, ldo, guess, loss_acc, correct, B,
                           n_valid, n_out, type);
    else
        hipLaunchKernelGGL(output_fp_kernel<float>, grid, dim3(256), 0, stream, (const float *)Z, ldz,
                           (const float *)T, ldt, (float *)D, ldd, (float *)O, ldo, guess, loss_acc, correct, B,
                           n_valid, n_out, type);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_update_fp(int f64, void *W, void *V, const void *G, int S, long gstride, long n, double lr,
                              double alpha, double scale, int momentum, hipStream_t stream) {
    if (n <= 0 || S < 1 || (momentum && !V)) return -2;
    long blocks = (n + 255) / 256;
    const dim3 grid(blocks < 4096 ? blocks : 4096);
    if (f64)
        hipLaunchKernelGGL(update_fp_kernel<double>, grid, dim3(256), 0, stream, (double *)W, (double *)V,
                           (const double *)G, S, gstride, n, lr, alpha, scale, momentum);
    else
        hipLaunchKernelGGL(update_fp_kernel<float>, grid, dim3(256), 0, stream, (float *)W, (float *)V,
                           (const float *)G, S, gstride, n, (float)lr, (float)alpha, (float)scale, momentum);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_dact_fp(int f64, void *out, const void *in, const void *aux, long n, hipStream_t stream) {
    if (n <= 0) return -2;
    long blocks = (n + 255) / 256;
    const dim3 grid(blocks < 4096 ? blocks : 4096);
    if (f64)
        hipLaunchKernelGGL(dact_fp_kernel<double>, grid, dim3(256), 0, stream, (double *)out, (const double *)in,
                           (const double *)aux, n);
    else
        hipLaunchKernelGGL(dact_fp_kernel<float>, grid, dim3(256), 0, stream, (float *)out, (const float *)in,
                           (const float *)aux, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_reduce_fp(int f64, void *out, const void *G, int S, long gstride, long n, hipStream_t stream) {
    if (n <= 0 || S < 1) return -2;
    long blocks = (n + 255) / 256;
    const dim3 grid(blocks < 4096 ? blocks : 4096);
    if (f64)
        hipLaunchKernelGGL(reduce_fp_kernel<double>, grid, dim3(256), 0, stream, (double *)out, (const double *)G, S,
                           gstride, n);
    else
        hipLaunchKernelGGL(reduce_fp_kernel<float>, grid, dim3(256), 0, stream, (float *)out, (const float *)G, S,
                           gstride, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
