/*
 * libhpnn MFMA GEMM kernels for gfx950 (CDNA4), BF16 in / FP32 accumulate.
 *
 * Replaces the reference's per-slice cublasDgemv / cublasDger / fused naive
 * kernels (cuda_ann.cu:77-148, 426-1276, 1310-2093) with
 * batched GEMMs on v_mfma_f32_16x16x32_bf16:
 *
 *   gemm_nt : C[M x N] = epi(A[M x K] . B[N x K]^T)
 *             forward  (A = activations, B = W,  epi = bipolar sigmoid)
 *             backward (A = deltas,      B = Wt, epi = * f'(h))
 *             The MFMA "A" operand is the weight fragment and "B" the
 *             activation fragment, so each lane ends with 4 consecutive
 *             features of one sample: 8-byte (bf16x4) / 16-byte (f32x4)
 *             row-contiguous stores.
 *   gemm_tn : G[N x M] = D^T . H over the batch (weight gradient), split-K
 *             over the batch into FP32 slabs (reduced deterministically by
 *             the optimizer kernel, no atomics).  Both operands are staged
 *             row-major (sample-major) in LDS exactly as they sit in HBM and
 *             read back column-wise with ds_read_b64_tr_b16 (gfx950
 *             transposing LDS read), so neither the input nor the deltas are
 *             ever transposed in memory.
 *
 * Structure: 256 threads (4 wave64), LDS double buffer, register staging
 * with 16-byte global loads, one barrier per K step, XOR-swizzled LDS rows
 * so the 16-lane ds_read_b128 / ds_read_b64_tr_b16 groups hit distinct
 * banks.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace {

__device__ __forceinline__ float bipolar(float x) { return 2.0f / (1.0f + __expf(-x)) - 1.0f; }

/* ---------------------------------------------------------------------- */
/* NT GEMM                                                                 */
/* ---------------------------------------------------------------------- */
/* swizzled byte offset of 16-byte chunk `c` of LDS row `r` (rows of CPR chunks) */
template <int CPR>
__device__ __forceinline__ int nt_off(int r, int c) {
    if constexpr (CPR == 8) return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
    else return r * 64 + ((c ^ ((r >> 2) & 3)) << 4);
}

template <int BM, int BN, int BK, int WM, int WN, int EPI, bool CF32>
__global__ __launch_bounds__(256) void gemm_nt_kernel(const __bf16 *__restrict__ A, int lda,
                                                      const __bf16 *__restrict__ B, int ldb, void *__restrict__ C,
                                                      int ldc, const __bf16 *__restrict__ aux, int ldaux, int K,
                                                      int tiles_n) {
    constexpr int NT = 256;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int CPR = BK / 8;
    constexpr int A_CH = BM * CPR, B_CH = BN * CPR;
    constexpr int A_PER = (A_CH + NT - 1) / NT, B_PER = (B_CH + NT - 1) / NT;
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
    constexpr int STAGE = A_BYTES + B_BYTES;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(FM >= 1 && FN >= 1, "wave tile");
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int tn = blockIdx.x % tiles_n, tm = blockIdx.x / tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int KT = K / BK;

    const char *Ag = (const char *)(A + (size_t)m0 * lda);
    const char *Bg = (const char *)(B + (size_t)n0 * ldb);

    uint4 ra[A_PER], rb[B_PER];
    auto gload = [&](int kt) {
#pragma unroll
        for (int i = 0; i < A_PER; i++) {
            int c = tid + i * NT, r = c / CPR, ch = c % CPR;
            if (A_PER * NT == A_CH || c < A_CH)
                ra[i] = *(const uint4 *)(Ag + ((size_t)r * lda + (size_t)kt * BK + ch * 8) * 2);
        }
#pragma unroll
        for (int i = 0; i < B_PER; i++) {
            int c = tid + i * NT, r = c / CPR, ch = c % CPR;
            if (B_PER * NT == B_CH || c < B_CH)
                rb[i] = *(const uint4 *)(Bg + ((size_t)r * ldb + (size_t)kt * BK + ch * 8) * 2);
        }
    };
    auto lstore = [&](int buf) {
        char *sa = lds + buf * STAGE, *sb = sa + A_BYTES;
#pragma unroll
        for (int i = 0; i < A_PER; i++) {
            int c = tid + i * NT, r = c / CPR, ch = c % CPR;
            if (A_PER * NT == A_CH || c < A_CH) *(uint4 *)(sa + nt_off<CPR>(r, ch)) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < B_PER; i++) {
            int c = tid + i * NT, r = c / CPR, ch = c % CPR;
            if (B_PER * NT == B_CH || c < B_CH) *(uint4 *)(sb + nt_off<CPR>(r, ch)) = rb[i];
        }
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; i++)
#pragma unroll
        for (int j = 0; j < FM; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    gload(0);
    lstore(0);
    __syncthreads();
    const int r16 = lane & 15, q = lane >> 4;
    for (int kt = 0; kt < KT; kt++) {
        const int cur = kt & 1;
        if (kt + 1 < KT) gload(kt + 1);
        const char *sa = lds + cur * STAGE, *sb = sa + A_BYTES;
#pragma unroll
        for (int kk = 0; kk < BK / 32; kk++) {
            const int ch = kk * 4 + q;
            bf16x8 fa[FM], fb[FN];
#pragma unroll
            for (int j = 0; j < FM; j++) fa[j] = *(const bf16x8 *)(sa + nt_off<CPR>(wm * WTM + j * 16 + r16, ch));
#pragma unroll
            for (int i = 0; i < FN; i++) fb[i] = *(const bf16x8 *)(sb + nt_off<CPR>(wn * WTN + i * 16 + r16, ch));
#pragma unroll
            for (int i = 0; i < FN; i++)
#pragma unroll
                for (int j = 0; j < FM; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < KT) lstore(cur ^ 1);
        __syncthreads();
    }

    /* epilogue: lane holds D[f = 4q + r][b = r16] of each 16x16 tile */
#pragma unroll
    for (int i = 0; i < FN; i++) {
#pragma unroll
        for (int j = 0; j < FM; j++) {
            const int b = m0 + wm * WTM + j * 16 + r16;
            const int f = n0 + wn * WTN + i * 16 + 4 * q;
            f32x4 v = acc[i][j];
            if constexpr (EPI == HPNN_EPI_ACT) {
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = bipolar(v[r]);
            } else if constexpr (EPI == HPNN_EPI_DACT) {
                bf16x4 h = *(const bf16x4 *)(aux + (size_t)b * ldaux + f);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    float y = (float)h[r];
                    v[r] *= -0.5f * (y * y - 1.0f);
                }
            }
            if constexpr (CF32) {
                *(f32x4 *)((float *)C + (size_t)b * ldc + f) = v;
            } else {
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)v[r];
                *(bf16x4 *)((__bf16 *)C + (size_t)b * ldc + f) = o;
            }
        }
    }
}

/* ---------------------------------------------------------------------- */
/* TN GEMM (weight gradient)                                               */
/* ---------------------------------------------------------------------- */
/* LDS tile: 64 sample rows x W columns (bf16, W any multiple of 32), stored as W/32
 * sub-tiles of [64 rows][32 cols] (64-byte rows).  Inside a sub-tile the two 32-byte
 * halves of a row are swapped for rows 8..15 mod 16, so the 8 rows that one 32-lane
 * half reads with ds_read_b64_tr_b16 (rows 8g+q, g in {0,1}, q in 0..3) cover all 64
 * banks exactly once. */
template <int W>
__device__ __forceinline__ int tn_off(int r, int col) {
    const int sub = col >> 5, c = col & 31;
    return sub * (64 * 64) + r * 64 + ((((c >> 4) ^ (r >> 3)) & 1) << 5) + (c & 15) * 2;
}

template <int W>
__device__ __forceinline__ bf16x8 tn_frag(const char *tile, int kbase, int c0, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int row = kbase + 8 * g + q;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(tile + tn_off<W>(row, c0 + 4 * p)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(tile + tn_off<W>(row + 4, c0 + 4 * p)));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}

template <int TM, int TN>
__global__ __launch_bounds__(256) void gemm_tn_kernel(const __bf16 *__restrict__ D, int ldd,
                                                      const __bf16 *__restrict__ H, int ldh, float *__restrict__ slab,
                                                      int ldg, int N, int chunk, int tiles_n) {
    constexpr int NT = 256, BK = 64;
    constexpr int WTM = TM / 2, WTN = TN / 2;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int H_CH = BK * TM / 8, D_CH = BK * TN / 8; /* 16-byte chunks per stage */
    constexpr int H_PER = (H_CH + NT - 1) / NT, D_PER = (D_CH + NT - 1) / NT;
    constexpr int H_BYTES = BK * TM * 2, D_BYTES = BK * TN * 2, STAGE = H_BYTES + D_BYTES;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int tn = blockIdx.x % tiles_n, tm = blockIdx.x / tiles_n;
    const int m0 = tm * TM, n0 = tn * TN;
    const int split = blockIdx.y;
    const int b0 = split * chunk;
    const int KT = chunk / BK;

    uint4 rh[H_PER], rd[D_PER];
    auto gload = [&](int kt) {
        const int rbase = b0 + kt * BK;
#pragma unroll
        for (int i = 0; i < H_PER; i++) {
            int c = tid + i * NT;
            if (H_PER * NT == H_CH || c < H_CH) {
                int r = c / (TM / 8), ch = c % (TM / 8);
                rh[i] = *(const uint4 *)(H + (size_t)(rbase + r) * ldh + m0 + ch * 8);
            }
        }
#pragma unroll
        for (int i = 0; i < D_PER; i++) {
            int c = tid + i * NT;
            if (D_PER * NT == D_CH || c < D_CH) {
                int r = c / (TN / 8), ch = c % (TN / 8);
                rd[i] = *(const uint4 *)(D + (size_t)(rbase + r) * ldd + n0 + ch * 8);
            }
        }
    };
    auto lstore = [&](int buf) {
        char *sh = lds + buf * STAGE, *sd = sh + H_BYTES;
#pragma unroll
        for (int i = 0; i < H_PER; i++) {
            int c = tid + i * NT;
            if (H_PER * NT == H_CH || c < H_CH) {
                int r = c / (TM / 8), ch = c % (TM / 8);
                *(uint4 *)(sh + tn_off<TM>(r, ch * 8)) = rh[i];
            }
        }
#pragma unroll
        for (int i = 0; i < D_PER; i++) {
            int c = tid + i * NT;
            if (D_PER * NT == D_CH || c < D_CH) {
                int r = c / (TN / 8), ch = c % (TN / 8);
                *(uint4 *)(sd + tn_off<TN>(r, ch * 8)) = rd[i];
            }
        }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    gload(0);
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < KT; kt++) {
        const int cur = kt & 1;
        if (kt + 1 < KT) gload(kt + 1);
        const char *sh = lds + cur * STAGE, *sd = sh + H_BYTES;
#pragma unroll
        for (int kk = 0; kk < BK / 32; kk++) {
            bf16x8 fh[FM], fd[FN];
#pragma unroll
            for (int i = 0; i < FM; i++) fh[i] = tn_frag<TM>(sh, kk * 32, wm * WTM + i * 16, lane);
#pragma unroll
            for (int j = 0; j < FN; j++) fd[j] = tn_frag<TN>(sd, kk * 32, wn * WTN + j * 16, lane);
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int j = 0; j < FN; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[i], fd[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < KT) lstore(cur ^ 1);
        __syncthreads();
    }
    /* lane holds acc[m = 4*(lane>>4) + r][n = lane & 15] */
    float *out = slab + (size_t)split * N * ldg;
    const int r16 = lane & 15, q = lane >> 4;
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) {
            const int n = n0 + wn * WTN + j * 16 + r16;
            const int m = m0 + wm * WTM + i * 16 + 4 * q;
            *(f32x4 *)(out + (size_t)n * ldg + m) = acc[i][j];
        }
}

template <int BN, int BK, int EPI, bool CF32>
int launch_nt_bn(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux, int ldaux, int M,
                 int N, int K, hipStream_t s) {
    constexpr int BM = 128;
    constexpr int WM = (BN == 128) ? 2 : 4;
    constexpr int WN = 4 / WM;
    const int tiles_n = N / BN, tiles_m = M / BM;
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, BK, WM, WN, EPI, CF32>), dim3(tiles_m * tiles_n), dim3(256), 0, s,
                       (const __bf16 *)A, lda, (const __bf16 *)B, ldb, C, ldc, (const __bf16 *)aux, ldaux, K, tiles_n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

template <int EPI, bool CF32>
int launch_nt_epi(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux, int ldaux, int M,
                  int N, int K, hipStream_t s) {
    const bool k64 = (K % 64) == 0;
#define HPNN_NT(BN_)                                                                                  \
    return k64 ? launch_nt_bn<BN_, 64, EPI, CF32>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, s)      \
               : launch_nt_bn<BN_, 32, EPI, CF32>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, s)
    if (N % 128 == 0 && N >= 128) { HPNN_NT(128); }
    if (N % 64 == 0) { HPNN_NT(64); }
    HPNN_NT(32);
#undef HPNN_NT
}

template <int TM, int TN>
int launch_tn_t(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M, int Bt, int splits,
                hipStream_t s) {
    const int tiles_n = N / TN, tiles_m = M / TM;
    hipLaunchKernelGGL((gemm_tn_kernel<TM, TN>), dim3(tiles_m * tiles_n, splits), dim3(256), 0, s, (const __bf16 *)D,
                       ldd, (const __bf16 *)H, ldh, slab, ldg, N, Bt / splits, tiles_n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

template <int TM>
int launch_tn_m(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M, int Bt, int splits,
                hipStream_t s) {
    if (N % 128 == 0) return launch_tn_t<TM, 128>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, s);
    if (N % 64 == 0) return launch_tn_t<TM, 64>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, s);
    return launch_tn_t<TM, 32>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, s);
}

}  // namespace

extern "C" int hpnn_gemm_nt_bf16(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux,
                                 int ldaux, int M, int N, int K, int epi, int c_f32, hipStream_t stream) {
    if (M <= 0 || N <= 0 || K <= 0) return -1;
    if (M % 128 || N % 32 || K % 32) return -2;
    if (lda % 8 || ldb % 8 || ldc % 8 || ((epi == HPNN_EPI_DACT) && (ldaux % 4 || !aux))) return -3;
    if (c_f32) {
        if (epi == HPNN_EPI_NONE) return launch_nt_epi<HPNN_EPI_NONE, true>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
        if (epi == HPNN_EPI_ACT) return launch_nt_epi<HPNN_EPI_ACT, true>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
        return launch_nt_epi<HPNN_EPI_DACT, true>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
    }
    if (epi == HPNN_EPI_NONE) return launch_nt_epi<HPNN_EPI_NONE, false>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
    if (epi == HPNN_EPI_ACT) return launch_nt_epi<HPNN_EPI_ACT, false>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
    return launch_nt_epi<HPNN_EPI_DACT, false>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
}

extern "C" int hpnn_gemm_tn_bf16(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M,
                                 int Bt, int splits, hipStream_t stream) {
    if (N <= 0 || M <= 0 || Bt <= 0 || splits <= 0) return -1;
    if (N % 32 || M % 32 || Bt % (64 * splits)) return -2;
    if (ldd % 8 || ldh % 8 || ldg % 4 || ldg < M) return -3;
    if (M % 128 == 0) return launch_tn_m<128>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream);
    if (M % 160 == 0) return launch_tn_m<160>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream);
    if (M % 96 == 0) return launch_tn_m<96>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream);
    if (M % 64 == 0) return launch_tn_m<64>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream);
    return launch_tn_m<32>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream);
}
