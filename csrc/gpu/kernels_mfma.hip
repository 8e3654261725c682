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
 * Structure: 256 threads (4 wave64); operands stream HBM -> LDS with
 * global_load_lds_dwordx4 (LDS-DMA, no VGPR staging) through a STAGES-deep
 * ring sized to ~64-72 KiB (2 workgroups per CU); one counted
 * `s_waitcnt vmcnt(N)` + raw s_barrier per K step keeps STAGES-1 stages in
 * flight (a __syncthreads() would drain them); the swizzles of the LDS images
 * are applied on the DMA source address and were checked with a bank
 * simulation (conflict-free ds_read_b128 / ds_read_b64_tr_b16).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.h"

HPNN_CO_PROBE(mfma)
#include "mfma_common.h"

/* kernels_8ph.hip */
int hpnn_gemm_tn8_launch(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M, int Bt,
                         int splits, hipStream_t stream, const hpnn::TnTail &tail);

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace {

using hpnn::bipolar;

/* ---------------------------------------------------------------------- */
/* NT GEMM                                                                 */
/* ---------------------------------------------------------------------- */
/* swizzled byte offset of 16-byte chunk `c` of LDS row `r` (rows of CPR chunks) */
template <int CPR>
__device__ __forceinline__ int nt_off(int r, int c) {
    if constexpr (CPR == 8) return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
    else return r * 64 + ((c ^ ((r >> 1) & 3)) << 4); /* bank-simulated: conflict-free */
}

/* ---------------------------------------------------------------------- */
/* NT GEMM, LDS-DMA pipelined (global_load_lds_dwordx4, STAGES-deep ring)   */
/* ---------------------------------------------------------------------- */
typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
/* wait until at most LPS*rem LDS-DMA loads of this wave are outstanding */
template <int LPS, int STAGES>
__device__ __forceinline__ void wait_stage(int rem) {
    static_assert(LPS * (STAGES - 1) < 64, "vmcnt budget");
    if constexpr (STAGES >= 8) { if (rem >= 7) { wait_vm<LPS * 7>(); return; } }
    if constexpr (STAGES >= 7) { if (rem >= 6) { wait_vm<LPS * 6>(); return; } }
    if constexpr (STAGES >= 6) { if (rem >= 5) { wait_vm<LPS * 5>(); return; } }
    if constexpr (STAGES >= 5) { if (rem >= 4) { wait_vm<LPS * 4>(); return; } }
    if constexpr (STAGES >= 4) { if (rem >= 3) { wait_vm<LPS * 3>(); return; } }
    if constexpr (STAGES >= 3) { if (rem >= 2) { wait_vm<LPS * 2>(); return; } }
    if (rem >= 1) { wait_vm<LPS>(); return; }
    wait_vm<0>();
}

/* One 1-KiB LDS-DMA piece of a [rows][BK] bf16 tile: lane i writes LDS bytes
 * [16i, 16i+16) of the piece, i.e. physical chunk (16i % RB)/16 of row 16i/RB;
 * it fetches the LOGICAL chunk that nt_off<> maps there (source-side swizzle). */
template <int BK>
__device__ __forceinline__ void glds_piece(const char *gbase, size_t ld_bytes, char *lds_piece, int row0, int lane) {
    constexpr int RB = BK * 2;           /* bytes per LDS row */
    constexpr int CPR = BK / 8;
    const int r = row0 + (lane * 16) / RB;
    const int cp = (lane * 16 % RB) >> 4;
    const int cl = (CPR == 8) ? (cp ^ ((r >> 1) & 7)) : (cp ^ ((r >> 1) & 3));
    const char *src = gbase + (size_t)r * ld_bytes + cl * 16;
    hpnn::glds16(src, lds_piece);
}

template <int BM, int BN, int BK, int WM, int WN, int STAGES, int EPI, bool CF32>
__global__ __launch_bounds__(WM * WN * 64) void gemm_nt_pipe_kernel(const __bf16 *__restrict__ A, int lda,
                                                           const __bf16 *__restrict__ B, int ldb,
                                                           void *__restrict__ C, int ldc,
                                                           const __bf16 *__restrict__ aux, int ldaux, int K,
                                                           int tiles_n) {
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int CPR = BK / 8;
    constexpr int RB = BK * 2;
    constexpr int ROWS_PER_PIECE = 1024 / RB;
    constexpr int A_PIECES = BM / ROWS_PER_PIECE, B_PIECES = BN / ROWS_PER_PIECE;
    constexpr int PIECES = A_PIECES + B_PIECES;
    /* every wave issues exactly LPS LDS-DMA loads per stage (a wave short of work
     * re-issues the last piece: same bytes to the same place), so one counted
     * vmcnt is exact for all waves */
    constexpr int NW = WM * WN; /* waves per workgroup (4, or 8 for the 256x256 tile) */
    constexpr int LPS = (PIECES + NW - 1) / NW;
    constexpr int A_BYTES = BM * RB, STAGE = (BM + BN) * RB;
    static_assert((NW == 4 || NW == 8) && FM >= 1 && FN >= 1, "wave tiling");
    __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int tn = blockIdx.x % tiles_n, tm = blockIdx.x / tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int KT = K / BK;
    const char *Ag = (const char *)(A + (size_t)m0 * lda);
    const char *Bg = (const char *)(B + (size_t)n0 * ldb);
    const size_t lda_b = (size_t)lda * 2, ldb_b = (size_t)ldb * 2;

    auto issue = [&](int slot, int kt) {
        char *sa = lds + slot * STAGE, *sb = sa + A_BYTES;
        const char *ga = Ag + (size_t)kt * RB, *gb = Bg + (size_t)kt * RB;
#pragma unroll
        for (int i = 0; i < LPS; i++) {
            int c = wave + NW * i;
            c = c < PIECES ? c : PIECES - 1;
            if (c < A_PIECES) glds_piece<BK>(ga, lda_b, sa + c * 1024, c * ROWS_PER_PIECE, lane);
            else glds_piece<BK>(gb, ldb_b, sb + (c - A_PIECES) * 1024, (c - A_PIECES) * ROWS_PER_PIECE, lane);
        }
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; i++)
#pragma unroll
        for (int j = 0; j < FM; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int st = 0; st < STAGES - 1; st++)
        if (st < KT) issue(st, st);
    const int r16 = lane & 15, q = lane >> 4;
    for (int kt = 0; kt < KT; kt++) {
        const int nxt = kt + STAGES - 1;
        if (nxt < KT) issue(nxt % STAGES, nxt);
        const int last = nxt < KT ? nxt : KT - 1;
        wait_stage<LPS, STAGES>(last - kt);
        __builtin_amdgcn_s_barrier();
        const char *sa = lds + (kt % STAGES) * STAGE, *sb = sa + A_BYTES;
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
        /* every wave's LDS reads of this slot retire before anyone refills it */
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }

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

/* 128 x 128 NT tiles for grids of about one tile per CU (the 8 x 4096 net at its 8-GPU shard,
 * M = 1024: 256 tiles), software-pipelined: gemm_nt_pipe_kernel<128, 128, 64, 2, 4, ...>
 * passes two barriers per 64-wide K-step and reads a step's fragments only after its
 * barrier, so every wave idles through the LDS read latency twice per step.  Here the
 * fragments of each 32-wide half-step go to their own register set, read while the MFMAs of
 * the other set run:
 *     [top of step kt]  issue stage kt + ST - 1 (the slot of kt - 1: every wave is past it)
 *                       read (kt, k32 1) -> R1;  16 MFMAs on R0 = (kt, k32 0)
 *                       counted vmcnt for stage kt + 1; lgkmcnt(0); ONE barrier
 *                       read (kt + 1, k32 0) -> R0;  16 MFMAs on R1
 * Same MFMA order per accumulator as gemm_nt_pipe_kernel: bitwise the same products.
 * BT ("NN"): B given as B^T, i.e. [K][N] row-major (a weight matrix W [N_out][K_in] used as
 * the delta GEMM's right operand without its transposed copy): staged as a T32 image and read
 * with the transposing ds_read_b64_tr_b16, the operands the MFMAs see -- and so the result
 * bits -- are those of the NT form on W^T. */
template <int EPI, bool CF32, int ST, bool BT = false>
__global__ __launch_bounds__(512) void gemm_nt_pp_kernel(const __bf16 *__restrict__ A, int lda,
                                                         const __bf16 *__restrict__ B, int ldb, void *__restrict__ C,
                                                         int ldc, const __bf16 *__restrict__ aux, int ldaux, int K,
                                                         int tiles_n) {
    constexpr int BM = 128, BN = 128, BK = 64, WN = 4, CPR = 8, RB = BK * 2;
    constexpr int A_PIECES = BM / 8, PIECES = A_PIECES + BN / 8, LPS = PIECES / 8; /* 4 per wave */
    constexpr int A_BYTES = BM * RB, STAGE = (BM + BN) * RB;
    static_assert(ST >= 2 && ST * STAGE <= 160 * 1024 && LPS * (ST - 1) < 64, "ring");
    __shared__ __attribute__((aligned(16))) char lds[ST * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN; /* wave tile 64 x 32 */
    const int tn = blockIdx.x % tiles_n, tm = blockIdx.x / tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int KT = K / BK;
    const char *Ag = (const char *)(A + (size_t)m0 * lda);
    const char *Bg = (const char *)(BT ? B + n0 : B + (size_t)n0 * ldb);
    const size_t lda_b = (size_t)lda * 2, ldb_b = (size_t)ldb * 2;
    const int r16 = lane & 15, q = lane >> 4;

    auto issue = [&](int kt) __attribute__((always_inline)) {
        char *sa = lds + (kt % ST) * STAGE, *sb = sa + A_BYTES;
        const char *ga = Ag + (size_t)kt * RB, *gb = BT ? Bg + (size_t)kt * BK * ldb_b : Bg + (size_t)kt * RB;
#pragma unroll
        for (int i = 0; i < LPS; i++) {
            const int c = wave + 8 * i; /* wave-uniform: pieces 0-15 A, 16-31 B */
            if (c < A_PIECES) glds_piece<BK>(ga, lda_b, sa + c * 1024, c * 8, lane);
            else if constexpr (BT) hpnn::glds_t32_piece<BK>(gb, ldb_b, sb, c - A_PIECES, lane);
            else glds_piece<BK>(gb, ldb_b, sb + (c - A_PIECES) * 1024, (c - A_PIECES) * 8, lane);
        }
    };
    bf16x8 fa0[4], fb0[2], fa1[4], fb1[2];
    auto read = [&](int kt, int kk, bf16x8 (&fa)[4], bf16x8 (&fb)[2]) __attribute__((always_inline)) {
        const char *sa = lds + (kt % ST) * STAGE, *sb = sa + A_BYTES;
        const int ch = kk * 4 + q;
#pragma unroll
        for (int j = 0; j < 4; j++) fa[j] = *(const bf16x8 *)(sa + nt_off<CPR>(wm * 64 + j * 16 + r16, ch));
#pragma unroll
        for (int i = 0; i < 2; i++) {
            if constexpr (BT) fb[i] = hpnn::frag_tr<BK>(sb, kk * 32, wn * 32 + i * 16, lane);
            else fb[i] = *(const bf16x8 *)(sb + nt_off<CPR>(wn * 32 + i * 16 + r16, ch));
        }
    };
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    /* EPI_DACT: the epilogue's f'(h) operand loaded now, under the main loop (16 VGPRs): read at
     * the end, its 8 strided loads per lane cost every workgroup ~15 us at M = 1024 */
    bf16x4 hv[2][4];
    if constexpr (EPI == HPNN_EPI_DACT) {
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                hv[i][j] = *(const bf16x4 *)(aux + (size_t)(m0 + wm * 64 + j * 16 + r16) * ldaux + n0 + wn * 32 +
                                             i * 16 + 4 * q);
    }
    auto mma = [&](const bf16x8 (&fa)[4], const bf16x8 (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    };

#pragma unroll
    for (int st = 0; st < ST - 1; st++)
        if (st < KT) issue(st);
    wait_stage<LPS, ST>((ST - 2 < KT - 1 ? ST - 2 : KT - 1));
    __builtin_amdgcn_s_barrier();
    read(0, 0, fa0, fb0);
    for (int kt = 0; kt < KT; kt++) {
        const int nxt = kt + ST - 1;
        if (nxt < KT) issue(nxt);
        read(kt, 1, fa1, fb1);
        mma(fa0, fb0);
        if (kt + 1 < KT) {
            const int last = nxt < KT ? nxt : KT - 1;
            wait_stage<LPS, ST>(last - (kt + 1));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            read(kt + 1, 0, fa0, fb0);
        }
        mma(fa1, fb1);
    }

#pragma unroll
    for (int i = 0; i < 2; i++) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int b = m0 + wm * 64 + j * 16 + r16;
            const int f = n0 + wn * 32 + i * 16 + 4 * q;
            f32x4 v = acc[i][j];
            if constexpr (EPI == HPNN_EPI_ACT) {
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = bipolar(v[r]);
            } else if constexpr (EPI == HPNN_EPI_DACT) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    float y = (float)hv[i][j][r];
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
/* TN GEMM, LDS-DMA pipelined.  Stage = BKR sample rows of the H tile (TM cols) and
 * of the D tile (TN cols), both as T32 images (mfma_common.h) with BKR rows. */
template <int BKR>
__device__ __forceinline__ void glds_tn_piece(const char *gbase, size_t ld_bytes, char *lds_tile, int piece,
                                              int lane) {
    hpnn::glds_t32_piece<BKR>(gbase, ld_bytes, lds_tile, piece, lane);
}
template <int BKR>
__device__ __forceinline__ bf16x8 tnp_frag(const char *tile, int kbase, int c0, int lane) {
    return hpnn::frag_tr<BKR>(tile, kbase, c0, lane);
}

using hpnn::TnTail;
using hpnn::tn_tail_reduce;

template <int TM, int TN, int BKR, int STAGES, int WM = 2, int WN = 2>
__global__ __launch_bounds__(WM * WN * 64) void gemm_tn_pipe_kernel(const __bf16 *__restrict__ D, int ldd,
                                                           const __bf16 *__restrict__ H, int ldh,
                                                           float *__restrict__ slab, int ldg, int N, int units,
                                                           int splits, int tiles_n, int tiles, int xcd_map,
                                                           TnTail tail) {
    if ((int)blockIdx.x >= tiles * splits) { /* appended reduction workgroups: no LDS, no barrier */
        tn_tail_reduce(tail, (int)blockIdx.x - tiles * splits);
        return;
    }
    constexpr int NW = WM * WN; /* 4 waves (2 x 2), or 8 (2 x 4) for the 256x256 tile */
    constexpr int WTM = TM / WM, WTN = TN / WN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int H_PIECES = (TM / 32) * (BKR / 16), D_PIECES = (TN / 32) * (BKR / 16);
    constexpr int PIECES = H_PIECES + D_PIECES;
    constexpr int LPS = (PIECES + NW - 1) / NW;
    constexpr int H_BYTES = BKR * TM * 2, STAGE = BKR * (TM + TN) * 2;
    __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    /* XCD-aware order: workgroups are dealt round-robin to the 8 XCDs in dispatch order;
     * put all output tiles of one batch slice on the same XCD, back to back, so the
     * slice's D (shared by every tile of the slice) is fetched once into that XCD's L2 */
    int tile, split;
    if (xcd_map) {
        const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
        tile = j % tiles;
        split = xcd + 8 * (j / tiles);
    } else {
        tile = blockIdx.x % tiles;
        split = blockIdx.x / tiles;
    }
    const int tn = tile % tiles_n, tm = tile / tiles_n;
    const int m0 = tm * TM, n0 = tn * TN;
    /* uneven splits: split s covers the 64-row units [s*U/S, (s+1)*U/S) of the batch, so
     * any split count gives every workgroup the same share to within one unit and the
     * grid can be sized to fill the CUs evenly (2 workgroups per CU) */
    const int u0 = (int)((long)split * units / splits), u1 = (int)((long)(split + 1) * units / splits);
    const int b0 = u0 * 64;
    const int KT = (u1 - u0) * (64 / BKR);
    const size_t ldh_b = (size_t)ldh * 2, ldd_b = (size_t)ldd * 2;
    const char *Hg = (const char *)(H + (size_t)b0 * ldh + m0);
    const char *Dg = (const char *)(D + (size_t)b0 * ldd + n0);

    auto issue = [&](int slot, int kt) {
        char *sh = lds + slot * STAGE, *sd = sh + H_BYTES;
        const char *gh = Hg + (size_t)kt * BKR * ldh_b, *gd = Dg + (size_t)kt * BKR * ldd_b;
#pragma unroll
        for (int i = 0; i < LPS; i++) {
            int c = wave + NW * i;
            c = c < PIECES ? c : PIECES - 1;
            if (c < H_PIECES) glds_tn_piece<BKR>(gh, ldh_b, sh, c, lane);
            else glds_tn_piece<BKR>(gd, ldd_b, sd, c - H_PIECES, lane);
        }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int st = 0; st < STAGES - 1; st++)
        if (st < KT) issue(st, st);
    for (int kt = 0; kt < KT; kt++) {
        const int nxt = kt + STAGES - 1;
        if (nxt < KT) issue(nxt % STAGES, nxt);
        const int last = nxt < KT ? nxt : KT - 1;
        wait_stage<LPS, STAGES>(last - kt);
        __builtin_amdgcn_s_barrier();
        const char *sh = lds + (kt % STAGES) * STAGE, *sd = sh + H_BYTES;
#pragma unroll
        for (int kk = 0; kk < BKR / 32; kk++) {
            bf16x8 fh[FM], fd[FN];
#pragma unroll
            for (int i = 0; i < FM; i++) fh[i] = tnp_frag<BKR>(sh, kk * 32, wm * WTM + i * 16, lane);
#pragma unroll
            for (int j = 0; j < FN; j++) fd[j] = tnp_frag<BKR>(sd, kk * 32, wn * WTN + j * 16, lane);
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int j = 0; j < FN; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[i], fd[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
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
    /* ring depth: ~64 KiB of staging -> 2 workgroups per CU */
    constexpr int STAGE_BYTES = (BM + BN) * BK * 2;
    constexpr int ST = (65536 / STAGE_BYTES) < 2 ? 2 : ((65536 / STAGE_BYTES) > 5 ? 5 : (65536 / STAGE_BYTES));
    const int tiles_n = N / BN, tiles_m = M / BM;
    hipLaunchKernelGGL((gemm_nt_pipe_kernel<BM, BN, BK, WM, WN, ST, EPI, CF32>), dim3(tiles_m * tiles_n), dim3(256), 0,
                       s, (const __bf16 *)A, lda, (const __bf16 *)B, ldb, C, ldc, (const __bf16 *)aux, ldaux, K,
                       tiles_n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* large GEMMs: 256x256 tiles, 8 waves (2 x 4, each 128x64), 2-stage ring of 64 KiB
 * stages, one workgroup per CU (HPNN_NT_BIG=0 disables).  8192x4096x4096: 974 / 1004
 * TFLOP/s (forward / backward epilogue) vs 870 / 918 with the 128x128 4-wave tile;
 * measured and rejected: BK=32 with 4 stages (913), s_setprio around the MFMA block (910),
 * register-staged operands instead of LDS-DMA, same tiling (916 / 961 vs 926 / 1001 on
 * the same box), 4 waves with 128x128 wave tiles and 256 AGPR accumulators (693 / 570:
 * one wave per SIMD leaves the LDS reads and the MFMAs of a k-step serialized) */
template <int EPI, bool CF32>
int launch_nt_big(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux, int ldaux, int M,
                  int N, int K, hipStream_t s) {
    constexpr int BM = 256, BN = 256;
    const int tiles_n = N / BN, tiles_m = M / BM;
    hipLaunchKernelGGL((gemm_nt_pipe_kernel<BM, BN, 64, 2, 4, 2, EPI, CF32>), dim3(tiles_m * tiles_n), dim3(512), 0, s,
                       (const __bf16 *)A, lda, (const __bf16 *)B, ldb, C, ldc, (const __bf16 *)aux, ldaux, K, tiles_n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* large NT GEMMs on the 8-phase kernel (kernels_8ph.hip); HPNN_NT_8PH=0 keeps the 1-phase
 * 256x256 kernel, hpnn_gemm_nt_set_8ph() switches at run time (A/B benchmarks) */
int g_nt8 = [] { const char *e = getenv("HPNN_NT_8PH"); return !(e && e[0] == '0'); }();
/* large weight gradients on the 8-phase TN kernel (HPNN_TN_8PH=0 keeps the 4-stage kernel) */
int g_tn8 = [] { const char *e = getenv("HPNN_TN_8PH"); return !(e && e[0] == '0'); }();
/* the software-pipelined 128 x 128 NT kernel for grids under two tiles per CU */
int g_ntpp = [] { const char *e = getenv("HPNN_NT_PP"); return !(e && e[0] == '0'); }();

template <int EPI, bool CF32>
int launch_nt_epi(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux, int ldaux, int M,
                  int N, int K, hipStream_t s) {
    const bool k64 = (K % 64) == 0;
    static const int big_off = [] { const char *e = getenv("HPNN_NT_BIG"); return e && e[0] == '0'; }();
    if (!big_off && g_nt8 && K % 128 == 0 && M % 256 == 0 && N % 256 == 0 && (long)(M / 256) * (N / 256) >= 256 &&
        K >= 512)
        return hpnn_gemm_nt8_bf16(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, EPI, CF32 ? 1 : 0, s);
    /* (a split-K form of the 8-phase kernel for grids of fewer 256x256 tiles than CUs,
     * hpnn_gemm_nt8_splitk_bf16, measured slower on the RRUFF-shaped first layer: 168 vs
     * 160 us per step -- the FP32 slabs cost more than the idle CUs; not dispatched here) */
    if (!big_off && k64 && M % 256 == 0 && N % 256 == 0 && (long)(M / 256) * (N / 256) >= 256 && K >= 512)
        return launch_nt_big<EPI, CF32>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, s);
#define HPNN_NT(BN_)                                                                                  \
    return k64 ? launch_nt_bn<BN_, 64, EPI, CF32>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, s)      \
               : launch_nt_bn<BN_, 32, EPI, CF32>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, s)
    /* grids of fewer than two 128 x 128 tiles per CU (the 8 x 4096 net at its 8-GPU shard,
     * M = 1024: 256 tiles): 8 waves (2 x 4, 64 x 32 wave tiles) and a 3-stage ring, one
     * workgroup per CU with two waves per SIMD, instead of the 4-wave tile's one.  Synthetic
     * 8 x 4096 step at batch 1024: 1.60 / 1.60 vs 1.68 / 1.67 ms; 2 stages 1.65, 4 stages
     * 1.59, 5 stages 1.57-1.59, 128 x 64 tiles (two 4-wave workgroups per CU) 1.70
     * (profiles/r5/SUMMARY.md).  HPNN_NT_SMALL=0: the 4-wave tile. */
    static const bool small_off = [] { const char *e = getenv("HPNN_NT_SMALL"); return e && e[0] == '0'; }();
    if (!small_off && k64 && M % 128 == 0 && N % 128 == 0 && (long)(M / 128) * (N / 128) < 512) {
        const int tiles_n = N / 128, tiles_m = M / 128;
        if (g_ntpp) { /* the software-pipelined form (HPNN_NT_PP=0: the kernel below) */
            hipLaunchKernelGGL((gemm_nt_pp_kernel<EPI, CF32, 5>), dim3(tiles_m * tiles_n), dim3(512), 0, s,
                               (const __bf16 *)A, lda, (const __bf16 *)B, ldb, C, ldc, (const __bf16 *)aux, ldaux, K,
                               tiles_n);
            return hipGetLastError() == hipSuccess ? 0 : -5;
        }
        hipLaunchKernelGGL((gemm_nt_pipe_kernel<128, 128, 64, 2, 4, 3, EPI, CF32>), dim3(tiles_m * tiles_n), dim3(512),
                           0, s, (const __bf16 *)A, lda, (const __bf16 *)B, ldb, C, ldc, (const __bf16 *)aux, ldaux,
                           K, tiles_n);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (N % 128 == 0 && N >= 128) { HPNN_NT(128); }
    if (N % 64 == 0) { HPNN_NT(64); }
    HPNN_NT(32);
#undef HPNN_NT
}

template <int TM, int TN, int RING = 73728, int MAXST = 6, int BKR = 32, int WM = 2, int WN = 2>
int launch_tn_t(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M, int Bt, int splits,
                hipStream_t s, const TnTail &tail) {
    const int tiles_n = N / TN, tiles_m = M / TM;
    const int units = Bt / 64;
    /* BKR-row stages (default 32), ring of ~72 KiB (2 workgroups per CU), or the deep ring
     * (~144 KiB, one workgroup per CU: twice the bytes in flight per CU for a grid of <= 1
     * GEMM workgroup per CU, where the stream is latency-bound by the ring depth) */
    constexpr int STAGE = BKR * (TM + TN) * 2;
    constexpr int ST = (RING / STAGE) < 2 ? 2 : ((RING / STAGE) > MAXST ? MAXST : (RING / STAGE));
    const int tiles = tiles_m * tiles_n;
    const int xcd_map = (splits % 8 == 0 && tiles > 1) ? 1 : 0;
    hipLaunchKernelGGL((gemm_tn_pipe_kernel<TM, TN, BKR, ST, WM, WN>), dim3(tiles * splits + tail.blocks),
                       dim3(WM * WN * 64), 0, s, (const __bf16 *)D, ldd, (const __bf16 *)H, ldh, slab, ldg, N, units,
                       splits, tiles_n, tiles, xcd_map, tail);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* (Measured and rejected for MNIST's G0, 800 x 128 over 65536 rows, 48 splits: a deep
 * ~144 KiB ring, one workgroup per CU, 74.3-74.6 vs 73.4-73.5 us per step -- the tail
 * reduction workgroups lose their co-residence; 8-wave / 64-row-stage variants 28.6-33.6
 * vs 29.6-29.8 us for the GEMM alone, none a clear win) */
template <int TM>
int launch_tn_m(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M, int Bt, int splits,
                hipStream_t s, const TnTail &t) {
    if (N % 128 == 0) return launch_tn_t<TM, 128>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, s, t);
    if (N % 64 == 0) return launch_tn_t<TM, 64>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, s, t);
    return launch_tn_t<TM, 32>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, s, t);
}

/* large weight gradients (>= 256 output tiles of 256x256, one split): 8-wave 256x256 tiles,
 * 4-stage ring of 32-row stages (128 KiB), one workgroup per CU (HPNN_TN_BIG=0 disables) */
int launch_tn_big(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M, int Bt,
                  int splits, hipStream_t s, const TnTail &t) {
    constexpr int TM = 256, TN = 256, BKR = 32, ST = 4;
    const int tiles_n = N / TN, tiles_m = M / TM, tiles = tiles_m * tiles_n;
    const int xcd_map = (splits % 8 == 0 && tiles > 1) ? 1 : 0;
    hipLaunchKernelGGL((gemm_tn_pipe_kernel<TM, TN, BKR, ST, 2, 4>), dim3(tiles * splits + t.blocks), dim3(512), 0, s,
                       (const __bf16 *)D, ldd, (const __bf16 *)H, ldh, slab, ldg, N, Bt / 64, splits, tiles_n, tiles,
                       xcd_map, t);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gemm_tn_dispatch(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M, int Bt,
                     int splits, hipStream_t stream, const TnTail &t) {
    if (N <= 0 || M <= 0 || Bt <= 0 || splits <= 0) return -1;
    if (N % 32 || M % 32 || Bt % 64 || splits > Bt / 64) return -2;
    if (ldd % 8 || ldh % 8 || ldg % 4 || ldg < M) return -3;
    static const int big_off = [] { const char *e = getenv("HPNN_TN_BIG"); return e && e[0] == '0'; }();
    if (!big_off && N % 256 == 0 && M % 256 == 0 && (long)(N / 256) * (M / 256) * splits >= 256) {
        if (g_tn8) {
            const int rc = hpnn_gemm_tn8_launch(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
            if (rc != -1) return rc;
        }
        return launch_tn_big(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
    }
    /* 64 x 64 tiles when the 128 x 128 grid leaves CUs idle: RRUFF's G1 (256 x 256 over 16384
     * rows, 32 splits) as 16 x 32 = 512 workgroups instead of 4 x 32 = 128, 145.8 / 146.1 vs
     * 150.6 / 149.4 us per step (profiles/r4/u_rruff_t64.txt; HPNN_TN_T64=0: off) */
    static const int t64 = [] { const char *e = getenv("HPNN_TN_T64"); return e ? atoi(e) : 1; }();
    if (t64 && M % 64 == 0 && N % 64 == 0 && (long)(M / 128) * (N / 128) * splits < 256)
        return launch_tn_t<64, 64>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
    if (M % 128 == 0) return launch_tn_m<128>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
    if (M % 160 == 0) return launch_tn_m<160>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
    if (M % 96 == 0) return launch_tn_m<96>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
    if (M % 64 == 0) return launch_tn_m<64>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
    return launch_tn_m<32>(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
}

}  // namespace

extern "C" void hpnn_gemm_nt_set_8ph(int on) { g_nt8 = on ? 1 : 0; }
extern "C" void hpnn_gemm_tn_set_8ph(int on) { g_tn8 = on ? 1 : 0; }
extern "C" void hpnn_gemm_nt_set_pp(int on) { g_ntpp = on ? 1 : 0; }

/* C[M x N] = epi(A[M x K] . W[K x N]) with W row-major [K][N] (the NT GEMM on W^T without the
 * transposed copy; gemm_nt_pp_kernel<..., BT>): M, N multiples of 128, K of 64 */
extern "C" int hpnn_gemm_nn_ok(int M, int N, int K, int lda, int ldw, int ldc) {
    return M > 0 && N > 0 && K > 0 && M % 128 == 0 && N % 128 == 0 && K % 64 == 0 && lda % 8 == 0 && ldw % 8 == 0 &&
           ldc % 8 == 0 && (size_t)ldw * 2 * 64 < (1u << 31);
}
extern "C" int hpnn_gemm_nn_bf16(const void *A, int lda, const void *W, int ldw, void *C, int ldc, const void *aux,
                                 int ldaux, int M, int N, int K, int epi, int c_f32, hipStream_t stream) {
    if (!hpnn_gemm_nn_ok(M, N, K, lda, ldw, ldc)) return -1;
    if (epi == HPNN_EPI_DACT && (!aux || ldaux % 4)) return -3;
    const int tiles_n = N / 128, grid = (M / 128) * tiles_n;
#define HPNN_NN(E, F)                                                                                              \
    hipLaunchKernelGGL((gemm_nt_pp_kernel<E, F, 5, true>), dim3(grid), dim3(512), 0, stream, (const __bf16 *)A, lda, \
                       (const __bf16 *)W, ldw, C, ldc, (const __bf16 *)aux, ldaux, K, tiles_n)
    if (c_f32) {
        if (epi == HPNN_EPI_NONE) HPNN_NN(HPNN_EPI_NONE, true);
        else if (epi == HPNN_EPI_ACT) HPNN_NN(HPNN_EPI_ACT, true);
        else HPNN_NN(HPNN_EPI_DACT, true);
    } else {
        if (epi == HPNN_EPI_NONE) HPNN_NN(HPNN_EPI_NONE, false);
        else if (epi == HPNN_EPI_ACT) HPNN_NN(HPNN_EPI_ACT, false);
        else HPNN_NN(HPNN_EPI_DACT, false);
    }
#undef HPNN_NN
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_gemm_nt_bf16(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux,
                                 int ldaux, int M, int N, int K, int epi, int c_f32, hipStream_t stream) {
    if (M <= 0 || N <= 0 || K <= 0) return -1;
    /* wide-input layer with a small weight matrix and a large batch: weight-stationary kernel */
    static const int ws_off = [] { const char *e = getenv("HPNN_NO_WS"); return e && atoi(e) ? 1 : 0; }();
    if (!ws_off && M % 32 == 0 && M >= 16384 && N <= 128) {
        int rc = hpnn_gemm_nt_ws_bf16(A, lda, B, ldb, C, ldc, M, N, K, epi, c_f32, stream);
        if (rc <= 0) return rc;
    }
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
    const TnTail none = {nullptr, nullptr, 0, 0, 0, 0, 1, 1, 0};
    return gemm_tn_dispatch(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, none);
}

extern "C" int hpnn_gemm_tn_bf16_reduce(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N,
                                        int M, int Bt, int splits, const float *rslab, int rS, long rstride, long rn,
                                        int rgroups, float *rout, hipStream_t stream) {
    if (rn % 4 || rstride % 4 || rS < 1 || rgroups < 1 || rgroups > rS || !rslab || !rout) return -2;
    const long n4 = rn / 4;
    const int bx = (int)((n4 + 255) / 256);
    const TnTail t = {rslab, rout, rstride, n4, rn, rS, (rS + rgroups - 1) / rgroups, bx, bx * rgroups};
    return gemm_tn_dispatch(D, ldd, H, ldh, slab, ldg, N, M, Bt, splits, stream, t);
}
