/*
 * 256x256-tile GEMMs with an 8-phase software pipeline (gfx950, BF16 in, FP32 acc):
 *   gemm_nt8_kernel  NT (forward / delta GEMMs), also in a split-K form (opt-in);
 *   gemm_tn8_kernel  TN (weight gradient), also with the optimizer step fused into the
 *                    epilogue (hpnn_gemm_tn8_update).
 * Measured on 8192x4096x4096: NT 1.32-1.42, TN 1.42 PFLOP/s (profiles/r2/s5_8ph_gemm.md).
 *
 *   C[M x N] = epi(A[M x K] . B[N x K]^T)   -- the forward (bipolar epilogue) and the
 *   delta (f'(h) epilogue) GEMMs of the large-layer path; same contract and epilogues
 *   as gemm_nt_pipe_kernel (kernels_mfma.hip).  Reference: the per-slice cublasDgemv /
 *   fw_mv_acc / dsigmoid_mul_delta_T of cuda_ann.cu:426-2093, batched.
 *
 * Why a second kernel: the 1-phase 256x256 kernel (one wait + barrier, all of a K-step's
 * LDS reads and MFMAs, barrier) serialises each wave's LDS reads with its MFMAs and keeps
 * only one K-step in flight; it tops out near 1 PFLOP/s on 8192x4096x4096.  Here:
 *
 *  - 8 waves (2 M x 4 N), wave tile 128 x 64 = 2 x 2 quadrants of 64 x 32 (16 MFMAs of
 *    16x16x32 per quadrant per 64-wide K-tile);
 *  - LDS: two K-tile buffers E / O (even / odd K-tiles) of four 16 KiB half-tiles
 *    (A rows 0-127, A rows 128-255, B rows 0-127, B rows 128-255), 128 KiB total, filled by
 *    LDS-DMA (global_load_lds_dwordx4) with the swizzle of nt_off<8> applied on the source
 *    address (conflict-free ds_read_b128);
 *  - one iteration = 2 K-tiles = 8 phases; phase p computes one quadrant:
 *        [ds_reads of the quadrant's new operands; LDS-DMA issue; counted vmcnt]
 *        s_barrier; lgkmcnt(0); setprio 1; 16 MFMAs; setprio 0; s_barrier
 *    quadrant order (0,0) (0,1) (1,1) (1,0): 12, 4, 8 and 0 ds_read_b128 per phase;
 *  - the waves of M-half 1 run one barrier behind those of M-half 0 (one extra barrier at
 *    the start), so on every SIMD one wave issues MFMAs while the other reads LDS;
 *  - prefetch: a half-tile is restaged two phases after its last read (the stagger makes
 *    one phase unsafe) and waited for with a counted vmcnt one phase before its first
 *    read, never vmcnt(0) in the steady state:
 *        P1: A(o) -> O     P4: B(e+2) -> E, vmcnt(4)     P5: A(e+2) -> E
 *        P8: B(o+2) -> O, vmcnt(4)                       (e = 2i, o = 2i + 1)
 *  - XCD-aware block order: each XCD gets a contiguous run of output tiles (bijective for
 *    any grid), so neighbouring tiles that share A / B panels share that XCD's L2.
 * Requires M % 256 == 0, N % 256 == 0, K % 128 == 0.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <mutex>

#include "kernels.h"

HPNN_CO_PROBE(8ph)
#include "mfma_common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int HALF = 16384;   /* bytes of one 128-row x 64-col BF16 half-tile */
constexpr int KBUF = 4 * HALF; /* one K-tile: A0 A1 B0 B1 */

/* swizzled byte offset of 16-byte chunk c of row r in a 128-B-row half-tile image */
__device__ __forceinline__ int off8(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}


template <int EPI, bool CF32>
__global__ __launch_bounds__(512) void gemm_nt8_kernel(const __bf16 *__restrict__ A, int lda,
                                                       const __bf16 *__restrict__ B, int ldb, void *__restrict__ C,
                                                       int ldc, const __bf16 *__restrict__ aux, int ldaux, int K,
                                                       int tiles_n, int ntiles, int splits, long cstride) {
    __shared__ __attribute__((aligned(16))) char lds[2 * KBUF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3; /* wm = stagger group */
    /* XCD-aware, bijective: blocks b, b+8, b+16, ... (one XCD) take consecutive tiles */
    const int total = ntiles * splits;
    const int bid = blockIdx.x, xcd = bid & 7, q8 = total >> 3, r8 = total & 7;
    const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    /* split-K (splits > 1, EPI_NONE into FP32 slabs cstride floats apart): split s takes
     * K-tiles [s KT, (s + 1) KT) */
    const int tile = w % ntiles, split = w / ntiles;
    const int tm = tile / tiles_n, tn = tile % tiles_n;
    const int m0 = tm * 256, n0 = tn * 256;
    const int KT = K / 64 / splits;
    const size_t lda_b = (size_t)lda * 2, ldb_b = (size_t)ldb * 2;
    const char *Ag = (const char *)(A + (size_t)m0 * lda + (size_t)split * KT * 64);
    const char *Bg = (const char *)(B + (size_t)n0 * ldb + (size_t)split * KT * 64);
    if (splits > 1) C = (void *)((float *)C + (size_t)split * cstride);

    /* LDS-DMA of half-tile h (0,1: A rows 128h..; 2,3: B rows 128(h-2)..) of K-tile kt
     * into buffer kt & 1: 16 pieces of 8 rows, two per wave; wave-uniform base in SGPRs,
     * one 32-bit per-lane offset (row, source-swizzled chunk) per piece */
    unsigned int voa[2], vob[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int r = (wave * 2 + i) * 8 + (lane >> 3), cl = (lane & 7) ^ ((r >> 1) & 7);
        voa[i] = (unsigned int)(r * lda_b + cl * 16);
        vob[i] = (unsigned int)(r * ldb_b + cl * 16);
    }
    auto stage = [&](int h, int kt) __attribute__((always_inline)) {
        char *dst = lds + (kt & 1) * KBUF + h * HALF;
        const char *g = h < 2 ? Ag + (size_t)(h * 128) * lda_b : Bg + (size_t)((h - 2) * 128) * ldb_b;
        g += (size_t)kt * 128;
#pragma unroll
        for (int i = 0; i < 2; i++) hpnn::glds16_sv(g, h < 2 ? voa[i] : vob[i], dst + (wave * 2 + i) * 1024);
    };

    /* accumulators: [mi][ni][j: 16-row frag][i: 16-col frag] */
    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int i = 0; i < 2; i++) acc[a][b][j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int r16 = lane & 15, q = lane >> 4;
    /* operand registers, flattened: ra[j * 2 + kk] (4 frags x 2 k32), rb[i * 2 + kk] */
    bf16x8 ra[8], rb0[4], rb1[4];
    auto read_a = [&](const char *buf, int mi) __attribute__((always_inline)) {
        const char *img = buf + wm * HALF;
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int kk = 0; kk < 2; kk++)
                ra[j * 2 + kk] = *(const bf16x8 *)(img + off8(mi * 64 + j * 16 + r16, kk * 4 + q));
    
    };
    auto read_b = [&](const char *buf, int ni, bf16x8 (&rb)[4]) __attribute__((always_inline)) {
        const char *img = buf + (2 + (wn >> 1)) * HALF;
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int kk = 0; kk < 2; kk++)
                rb[i * 2 + kk] = *(const bf16x8 *)(img + off8((wn & 1) * 64 + ni * 32 + i * 16 + r16, kk * 4 + q));
    
    };
    auto mma = [&](int mi, int ni, const bf16x8 (&rb)[4]) __attribute__((always_inline)) {
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; kk++)
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int i = 0; i < 2; i++)
                    acc[mi][ni][j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[i * 2 + kk], ra[j * 2 + kk],
                                                                                acc[mi][ni][j][i], 0, 0, 0);
    
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
    };

    /* prologue: K-tile 0 (A, B) -> E, B of K-tile 1 -> O; K-tile 0 landed everywhere */
    stage(0, 0);
    stage(1, 0);
    stage(2, 0);
    stage(3, 0);
    stage(2, 1);
    stage(3, 1);
    vm_wait<4>();
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier(); /* the stagger */

    for (int e = 0; e < KT; e += 2) {
        const int o = e + 1;
        const bool ne = e + 2 < KT, no = o + 2 < KT;
        const char *bE = lds + (e & 1) * KBUF, *bO = lds + (o & 1) * KBUF;
        /* P1 */
        read_a(bE, 0);
        read_b(bE, 0, rb0);
        stage(0, o);
        stage(1, o);
        __builtin_amdgcn_sched_barrier(0);
        mma(0, 0, rb0);
        /* P2 */
        read_b(bE, 1, rb1);
        __builtin_amdgcn_sched_barrier(0);
        mma(0, 1, rb1);
        /* P3 */
        read_a(bE, 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(1, 1, rb1);
        /* P4: restage E's B for K-tile e+2; K-tile o complete */
        if (ne) {
            stage(2, e + 2);
            stage(3, e + 2);
            vm_wait<4>();
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(1, 0, rb0);
        /* P5 */
        read_a(bO, 0);
        read_b(bO, 0, rb0);
        if (ne) {
            stage(0, e + 2);
            stage(1, e + 2);
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(0, 0, rb0);
        /* P6 */
        read_b(bO, 1, rb1);
        __builtin_amdgcn_sched_barrier(0);
        mma(0, 1, rb1);
        /* P7 */
        read_a(bO, 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(1, 1, rb1);
        /* P8: restage O's B for K-tile o+2; K-tile e+2 complete */
        if (no) {
            stage(2, o + 2);
            stage(3, o + 2);
            vm_wait<4>();
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(1, 0, rb0);
    }
    if (wm == 0) __builtin_amdgcn_s_barrier(); /* pair the stagger barrier */

    /* 4 consecutive features f.. of sample b per store */
    auto emit = [&](int b, int f, f32x4 v) __attribute__((always_inline)) {
        if constexpr (EPI == HPNN_EPI_ACT) {
#pragma unroll
            for (int r = 0; r < 4; r++) v[r] = hpnn::bipolar(v[r]);
        } else if constexpr (EPI == HPNN_EPI_DACT) {
            const bf16x4 h = *(const bf16x4 *)(aux + (size_t)b * ldaux + f);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float y = (float)h[r];
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
    };
#pragma unroll
    for (int mi = 0; mi < 2; mi++)
#pragma unroll
        for (int ni = 0; ni < 2; ni++) {
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int i = 0; i < 2; i++)
                    emit(m0 + wm * 128 + mi * 64 + j * 16 + r16, n0 + wn * 64 + ni * 32 + i * 16 + 4 * q,
                         acc[mi][ni][j][i]);
        
        }
}

/* ---------------------------------------------------------------------- */
/* TN: slab[s][n][m] = sum over the batch rows b of split s of D[b][n] H[b][m] */
/* ---------------------------------------------------------------------- */
/* The weight-gradient GEMM on the same 8-phase schedule.  The operands stay sample-major:
 * a half-tile is 64 batch rows x 128 columns of H (m) or D (n), kept as a T32 image
 * (mfma_common.h: 4 sub-tiles of [64][32], 64-byte rows, chunk permutation) and read
 * column-wise with ds_read_b64_tr_b16 (frag_tr), so nothing is transposed in memory.
 * Wave (wm, wn): m in [128 wm, +128) (H half wm), n in [64 wn, +64) (D half wn / 2);
 * quadrant (mi, ni) = 4 H fragments x 2 D fragments x 2 k-substeps = 16 MFMAs.
 * Split s covers the 64-row units [s U / S, (s + 1) U / S); every split must hold an even
 * number of units (two K-tiles per iteration).  Appended workgroups run the TnTail
 * reduction, as in gemm_tn_pipe_kernel. */
/* optimizer step fused into the TN epilogue (one split: the product is the whole gradient
 * G[n][m]), the math of sgd_tile (kernels_misc.hip) with one slab */
struct Tn8Upd {
    float *W32, *V32;
    __bf16 *Wb, *Wt;
    float lr, alpha, scale;
    int momentum;
    unsigned int *cnt, *err; /* MODE 2: per-tile tickets (32 words apart, zeroed once), error word */
};

constexpr unsigned long long TN8_TIMEOUT = 1000000000ULL; /* wall-clock ticks (~10 s) */

/* MODE 2 side job (hpnn_gemm_tn8_fused_update_side): the NEXT layer's weight gradient
 * G1 = D^T H of a two-layer net (RRUFF: 230 x 230 over the batch) and its step, carried
 * by the layer-0 launch instead of a gradient launch + an update launch of their own.
 * The gradient is cut exactly as gemm_tn_pipe_kernel<64, 64, 32, ...> (kernels_mfma.hip)
 * cuts it for the separate path: 64 x 64 tiles x S splits of units / S 64-row units; each
 * piece runs on one half of a workgroup (waves 0-3 / 4-7, an LDS ring each) with that
 * kernel's staging, fragment reads and MFMA order, so the partial slabs are bitwise the
 * separate launch's.  The pieces run before the layer-0 GEMM and are published
 * write-through; one ticket per workgroup; each workgroup then reduces 1 / grid of G1 over
 * the S slabs in the summation order of sgd_tile (kernels_misc.hip) and applies the step,
 * while it waits for the other splits of its own layer-0 tile. */
struct Tn8Side {
    const __bf16 *D, *H;
    float *slab; /* [S][N][M] */
    float *W32, *V32;
    __bf16 *Wb, *Wt;
    unsigned int *cnt; /* 64-bit arrival counter (one ticket per workgroup per launch) */
    int ldd, ldh, N, M, units, S, tiles_n, tiles, jobs, on;
};

/* 64-row stages (16 KiB per half: 64 H + 64 D columns), a 5-stage ring per half -- all
 * 160 KiB of the CU's LDS for MODE 2 -- and ONE barrier per stage: the pieces are bound by
 * their per-stage overhead (32-row stages with two barriers each: 25.9K ticks for a
 * workgroup's pieces, raw_s6_tr1) */
constexpr int SJ_BKR = 64, SJ_ST = 5, SJ_STAGE = SJ_BKR * 128 * 2, SJ_LPS = 4;
constexpr int TN8_LDS2 = 2 * SJ_ST * SJ_STAGE; /* MODE 2's LDS */
static_assert(TN8_LDS2 >= 2 * KBUF && TN8_LDS2 <= 160 * 1024, "side-job rings fit the CU's LDS");

__device__ __forceinline__ void sj_wait(int rem) { /* SJ_LPS LDS-DMA loads per wave per stage */
    static_assert(SJ_ST <= 5 && SJ_LPS == 4, "counted waits below");
    if (rem >= 4) vm_wait<16>();
    else if (rem == 3) vm_wait<12>();
    else if (rem == 2) vm_wait<8>();
    else if (rem == 1) vm_wait<4>();
    else vm_wait<0>();
}

/* the pieces first, first + step, ... < end of this half (w4: wave within the half); every
 * half of the grid runs the same number of pieces of the same length (host-checked), so the
 * halves meet the workgroup barriers in step.  Staging pieces and fragment reads are those of
 * gemm_tn_pipe_kernel<64, 64, 64, ...> and the MFMAs run in the same k order as its 32-row form:
 * the same partial sums bit for bit. */
__device__ __forceinline__ void side_jobs(const Tn8Side &s, char *ring, int w4, int lane, int first, int step,
                                          int end) {
    const int wm = w4 >> 1, wn = w4 & 1, r16 = lane & 15, q = lane >> 4;
    const int upj = s.units / s.S, KT = upj * (64 / SJ_BKR);
    const size_t ldh_b = (size_t)s.ldh * 2, ldd_b = (size_t)s.ldd * 2;
    for (int j = first; j < end; j += step) {
        const int tile = j % s.tiles, split = j / s.tiles;
        const int m0 = (tile / s.tiles_n) * 64, n0 = (tile % s.tiles_n) * 64;
        const size_t b0 = (size_t)split * upj * 64;
        const char *Hg = (const char *)(s.H + b0 * s.ldh + m0);
        const char *Dg = (const char *)(s.D + b0 * s.ldd + n0);
        auto issue = [&](int kt) __attribute__((always_inline)) {
            char *sh = ring + (kt % SJ_ST) * SJ_STAGE, *sd = sh + SJ_BKR * 64 * 2;
            const char *gh = Hg + (size_t)kt * SJ_BKR * ldh_b, *gd = Dg + (size_t)kt * SJ_BKR * ldd_b;
#pragma unroll
            for (int i = 0; i < SJ_LPS; i++) { /* pieces 0-7 H, 8-15 D */
                const int c = w4 + 4 * i;
                if (c < 8) hpnn::glds_t32_piece<SJ_BKR>(gh, ldh_b, sh, c, lane);
                else hpnn::glds_t32_piece<SJ_BKR>(gd, ldd_b, sd, c - 8, lane);
            }
        };
        f32x4 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int jj = 0; jj < 2; jj++) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < SJ_ST - 1; st++)
            if (st < KT) issue(st);
        for (int kt = 0; kt < KT; kt++) {
            sj_wait((kt + SJ_ST - 2 < KT - 1 ? kt + SJ_ST - 2 : KT - 1) - kt);
            /* stage kt landed everywhere; every wave's reads of stage kt - 1 retired (its MFMAs
             * consumed them), so its slot can be refilled */
            __builtin_amdgcn_s_barrier();
            if (kt + SJ_ST - 1 < KT) issue(kt + SJ_ST - 1);
            const char *sh = ring + (kt % SJ_ST) * SJ_STAGE, *sd = sh + SJ_BKR * 64 * 2;
#pragma unroll
            for (int kk = 0; kk < SJ_BKR / 32; kk++) {
                bf16x8 fh[2], fd[2];
#pragma unroll
                for (int i = 0; i < 2; i++) fh[i] = hpnn::frag_tr<SJ_BKR>(sh, kk * 32, wm * 32 + i * 16, lane);
#pragma unroll
                for (int jj = 0; jj < 2; jj++) fd[jj] = hpnn::frag_tr<SJ_BKR>(sd, kk * 32, wn * 32 + jj * 16, lane);
#pragma unroll
                for (int i = 0; i < 2; i++)
#pragma unroll
                    for (int jj = 0; jj < 2; jj++)
                        acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[i], fd[jj], acc[i][jj], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier(); /* the ring is free for the next piece */
        float *out = s.slab + (size_t)split * s.N * s.M;
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int jj = 0; jj < 2; jj++)
                hpnn::st_sc1(out + (size_t)(n0 + wn * 32 + jj * 16 + r16) * s.M + m0 + wm * 32 + i * 16 + 4 * q,
                             acc[i][jj]);
        /* the stores count in vmcnt: drain them before the next piece's counted waits */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

/* workgroup b's share of G1 (E4 / G float4s): the S partial slabs summed in sgd_tile's order
 * (slab 0; slabs 1.. in four interleaved chains while four remain; the rest into chain 0;
 * chain 0 + ((1 + 2) + 3)), then the step of hpnn_sgd_update */
__device__ __forceinline__ void side_reduce_step(const Tn8Side &s, const Tn8Upd &u, int b, int G) {
    const int E4 = s.N * s.M / 4, per = (E4 + G - 1) / G, m4 = s.M / 4;
    const int e0 = b * per, e1 = min(E4, e0 + per);
    const size_t ss = (size_t)s.N * s.M;
    const int gend = 1 + 4 * ((s.S - 1) / 4);
    for (int e = e0 + (int)threadIdx.x; e < e1; e += (int)blockDim.x) {
        const int n = e / m4, m = 4 * (e % m4);
        const size_t idx = (size_t)n * s.M + m;
        f32x4 ww = *(const f32x4 *)(s.W32 + idx), vv = {0.f, 0.f, 0.f, 0.f}; /* under the slab loads */
        if (u.momentum) vv = *(const f32x4 *)(s.V32 + idx);
        f32x4 g = {0.f, 0.f, 0.f, 0.f}, g1 = g, g2 = g, g3 = g;
        for (int s0 = 0; s0 < s.S; s0 += 16) {
            f32x4 v[16];
            const float *p[16];
#pragma unroll
            for (int j = 0; j < 16; j++) p[j] = s.slab + (size_t)(s0 + j < s.S ? s0 + j : s0) * ss + idx;
            hpnn::ld_sc1_x16(v, p);
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const int k = s0 + j, c = (k - 1) & 3;
                const f32x4 x = v[j];
                if (k < s.S) {
                    if (k == 0) g = x;
                    else if (k >= gend || c == 0) g += x;
                    else if (c == 1) g1 += x;
                    else if (c == 2) g2 += x;
                    else g3 += x;
                }
            }
        }
        g += (g1 + g2) + g3;
        /* the contraction spelled out: sgd_tile's compiled step is fma(lr, g * scale, v) (a
         * free choice of the compiler here measured 1-ulp apart on a few elements) */
        if (u.momentum) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                vv[r] = __builtin_fmaf(u.lr, g[r] * u.scale, vv[r]);
                ww[r] += vv[r];
                vv[r] *= u.alpha;
            }
            *(f32x4 *)(s.V32 + idx) = vv;
        } else {
#pragma unroll
            for (int r = 0; r < 4; r++) ww[r] = __builtin_fmaf(u.lr, g[r] * u.scale, ww[r]);
        }
        *(f32x4 *)(s.W32 + idx) = ww;
        bf16x4 wb;
#pragma unroll
        for (int r = 0; r < 4; r++) wb[r] = (__bf16)ww[r];
        *(bf16x4 *)(s.Wb + idx) = wb;
#pragma unroll
        for (int r = 0; r < 4; r++) s.Wt[(size_t)(m + r) * s.N + n] = wb[r];
    }
}

/* MODE 0: split-K slabs; 3: one split, the product rounded to BF16 into upd.Wb [N][ldg] (the
 * data-parallel exchange's send buffer: no FP32 gradient round trip); 1: one split, the
 * optimizer step in the epilogue; 2: several splits,
 * each publishes its partial tile write-through and takes a ticket, then -- once every split
 * of the tile has arrived -- reduces 1/splits of the tile over the splits in a fixed order
 * and applies the step there (the split-K reduction and the update launch of the RRUFF-shaped
 * first layer move into this launch; the protocol of kernels_g0.hip g0_fused_kernel) */
/* HPNN_TN8_TRACE=1 (profiling only, MODE 2): s_memtime of every workgroup's thread 0 at the
 * phase boundaries, [block][mark]; read back with hpnn_tn8_trace */
constexpr int TN8_TR_BLOCKS = 512, TN8_TR_MARKS = 8;
__device__ unsigned long long g_tn8_trace[TN8_TR_BLOCKS][TN8_TR_MARKS];

/* TM: output-tile width along H (256, or 128 for MODE 2: 256 x 128 tiles -- twice the tiles at
 * half the splits for the same grid, so half the split-K partial bytes; the waves of M-half wm
 * then own H columns 64 wm.. of the one H half-tile, and an iteration has 4 phases) */
template <int MODE, bool TRACE = false, int TM = 256>
__global__ __launch_bounds__(512) void gemm_tn8_kernel(const __bf16 *__restrict__ D, int ldd,
                                                       const __bf16 *__restrict__ H, int ldh,
                                                       float *__restrict__ slab, int ldg, int N, int units,
                                                       int splits, int tiles_n, int ntiles, hpnn::TnTail tail,
                                                       Tn8Upd upd, Tn8Side side) {
    if ((int)blockIdx.x >= ntiles * splits) {
        if (threadIdx.x < 256) hpnn::tn_tail_reduce(tail, (int)blockIdx.x - ntiles * splits);
        return;
    }
    __shared__ __attribute__((aligned(16))) char lds[MODE == 2 ? TN8_LDS2 : 2 * KBUF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    int tile, split;
    if (splits == 1) {
        const int bid = blockIdx.x, xcd = bid & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
        tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
        split = 0;
    } else {
        /* XCD-aware, bijective (as gemm_nt8_kernel): each XCD takes a contiguous run of
         * split-major work items, i.e. whole K slices for every tile, so a slice of D (shared
         * by all tiles) is fetched into one XCD's L2 once instead of into every XCD's */
        const int total = ntiles * splits, bid = blockIdx.x, xcd = bid & 7, q8 = total >> 3, r8 = total & 7;
        const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
        tile = w % ntiles;
        split = w / ntiles;
    }
    static_assert(TM == 256 || (TM == 128 && MODE == 2), "tile width");
    const int tn = tile % tiles_n, tm = tile / tiles_n;
    const int m0 = tm * TM, n0 = tn * 256;
    const int u0 = (int)((long)split * units / splits), u1 = (int)((long)(split + 1) * units / splits);
    const int KT = u1 - u0; /* 64-row K-tiles, even */
    const size_t ldh_b = (size_t)ldh * 2, ldd_b = (size_t)ldd * 2;
    const char *Hg = (const char *)(H + (size_t)u0 * 64 * ldh + m0);
    const char *Dg = (const char *)(D + (size_t)u0 * 64 * ldd + n0);

    auto mark = [&](int i) __attribute__((always_inline)) {
        if constexpr (TRACE) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (tid == 0 && blockIdx.x < TN8_TR_BLOCKS) g_tn8_trace[blockIdx.x][i] = t;
        }
    };
    mark(0);
    unsigned long long want1 = 0; /* the side job's arrival target (thread 0) */
    if constexpr (MODE == 2) {
        if (side.on) {
            const int G = ntiles * splits, bid = blockIdx.x;
            /* the XCD's workgroups take a contiguous, split-major run of pieces (whole K slices
             * of D and H into that XCD's L2 once); host-checked G % 8 == 0 */
            const int per = side.jobs / 8, x0 = (bid & 7) * per;
            side_jobs(side, lds + (wave >> 2) * (SJ_ST * SJ_STAGE), wave & 3, lane, x0 + 2 * (bid >> 3) + (wave >> 2),
                      2 * (G / 8), x0 + per);
            __syncthreads(); /* every piece published; the rings are free for the GEMM */
            if (tid == 0) want1 = hpnn::ticket_arrive(side.cnt, (unsigned)G);
        }
    }
    mark(1);

    unsigned int voh[2], vod[2];
    int dsto[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int pc = wave * 2 + i, sub = pc >> 2, rp = (pc & 3) * 16;
        const int r = rp + (lane >> 2), col = sub * 32 + (((lane & 3) ^ hpnn::t32_g(r)) & 3) * 8;
        voh[i] = (unsigned int)(r * ldh_b + col * 2);
        vod[i] = (unsigned int)(r * ldd_b + col * 2);
        dsto[i] = sub * 4096 + rp * 64;
    }
    auto stage = [&](int h, int kt) __attribute__((always_inline)) {
        char *dst = lds + (kt & 1) * KBUF + h * HALF;
        const char *g = h < 2 ? Hg + (size_t)kt * 64 * ldh_b + h * 256 : Dg + (size_t)kt * 64 * ldd_b + (h - 2) * 256;
#pragma unroll
        for (int i = 0; i < 2; i++) hpnn::glds16_sv(g, h < 2 ? voh[i] : vod[i], dst + dsto[i]);
    };

    f32x4 acc[2][2][4][2]; /* [mi][ni][i: H frag][j: D frag] */
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    /* transposed fragment reads (hpnn::frag_tr on a T32 image with 64 rows), addresses
     * split into a per-lane part -- it depends only on whether the fragment's first column
     * is 0 or 16 mod 32 and on the low / high 4-row group -- and a compile-time constant
     * (sub-tile, k-substep, buffer, half) folded into the ds_read offset */
    int toff[2][2];
    {
        const int g = lane >> 4, qq = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
        for (int cls = 0; cls < 2; cls++)
#pragma unroll
            for (int hl = 0; hl < 2; hl++) {
                const int r = 8 * g + qq + 4 * hl;
                toff[cls][hl] = r * 64 + ((((2 * cls + (p >> 1)) ^ hpnn::t32_g(r)) & 3) << 4) + (p & 1) * 8;
            }
    }
    auto ftr = [&](const char *img, int kbase, int c0) __attribute__((always_inline)) {
        const char *b = img + (c0 >> 5) * 4096 + kbase * 64;
        const int cls = (c0 >> 4) & 1;
        hpnn::s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((hpnn::lds_s16x4 *)(b + toff[cls][0]));
        hpnn::s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((hpnn::lds_s16x4 *)(b + toff[cls][1]));
        hpnn::s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    };
    bf16x8 rh[4][2], rd0[2][2], rd1[2][2];
    auto read_h = [&](const char *buf, int mi) __attribute__((always_inline)) {
        /* TM 128: one H half-tile, M-half wm owns its columns 64 wm.. (mi unused) */
        const char *img = buf + (TM == 256 ? wm * HALF : 0);
        const int c0 = TM == 256 ? mi * 64 : wm * 64;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int kk = 0; kk < 2; kk++) rh[i][kk] = ftr(img, kk * 32, c0 + i * 16);
    };
    auto read_d = [&](const char *buf, int ni, bf16x8 (&rd)[2][2]) __attribute__((always_inline)) {
        const char *img = buf + (2 + (wn >> 1)) * HALF;
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int kk = 0; kk < 2; kk++) rd[j][kk] = ftr(img, kk * 32, (wn & 1) * 64 + ni * 32 + j * 16);
    };
    auto mma = [&](int mi, int ni, const bf16x8 (&rd)[2][2]) __attribute__((always_inline)) {
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; kk++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
                    acc[mi][ni][i][j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(rh[i][kk], rd[j][kk], acc[mi][ni][i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
    };

    /* the schedule of gemm_nt8_kernel with H in the role of A and D in that of B */
    stage(0, 0);
    if constexpr (TM == 256) stage(1, 0);
    stage(2, 0);
    stage(3, 0);
    stage(2, 1);
    stage(3, 1);
    vm_wait<4>();
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();

    if constexpr (TM == 128) {
        /* 4 phases per 2 K-tiles, quadrants (0,0) (0,1) of the one M-quadrant; H(o) is restaged
         * at the top (its O slot was last read two phases before the previous iteration's
         * end), D(e+2) after the even phases, H(e+2) once the odd H is read, D(o+2) last; the
         * counted waits leave only the D pieces just issued in flight */
        for (int e = 0; e < KT; e += 2) {
            const int o = e + 1;
            const bool ne = e + 2 < KT, no = o + 2 < KT;
            const char *bE = lds + (e & 1) * KBUF, *bO = lds + (o & 1) * KBUF;
            read_h(bE, 0);
            read_d(bE, 0, rd0);
            stage(0, o);
            __builtin_amdgcn_sched_barrier(0);
            mma(0, 0, rd0);
            read_d(bE, 1, rd1);
            __builtin_amdgcn_sched_barrier(0);
            mma(0, 1, rd1);
            if (ne) {
                stage(2, e + 2);
                stage(3, e + 2);
                vm_wait<4>();
            } else {
                vm_wait<0>();
            }
            read_h(bO, 0);
            read_d(bO, 0, rd0);
            if (ne) stage(0, e + 2);
            __builtin_amdgcn_sched_barrier(0);
            mma(0, 0, rd0);
            read_d(bO, 1, rd1);
            __builtin_amdgcn_sched_barrier(0);
            mma(0, 1, rd1);
            if (no) {
                stage(2, o + 2);
                stage(3, o + 2);
                vm_wait<4>();
            } else {
                vm_wait<0>();
            }
        }
    } else
    for (int e = 0; e < KT; e += 2) {
        const int o = e + 1;
        const bool ne = e + 2 < KT, no = o + 2 < KT;
        const char *bE = lds + (e & 1) * KBUF, *bO = lds + (o & 1) * KBUF;
        read_h(bE, 0);
        read_d(bE, 0, rd0);
        stage(0, o);
        stage(1, o);
        __builtin_amdgcn_sched_barrier(0);
        mma(0, 0, rd0);
        read_d(bE, 1, rd1);
        __builtin_amdgcn_sched_barrier(0);
        mma(0, 1, rd1);
        read_h(bE, 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(1, 1, rd1);
        if (ne) {
            stage(2, e + 2);
            stage(3, e + 2);
            vm_wait<4>();
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(1, 0, rd0);
        read_h(bO, 0);
        read_d(bO, 0, rd0);
        if (ne) {
            stage(0, e + 2);
            stage(1, e + 2);
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(0, 0, rd0);
        read_d(bO, 1, rd1);
        __builtin_amdgcn_sched_barrier(0);
        mma(0, 1, rd1);
        read_h(bO, 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(1, 1, rd1);
        if (no) {
            stage(2, o + 2);
            stage(3, o + 2);
            vm_wait<4>();
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(1, 0, rd0);
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();
    mark(2);

    float *out = slab + (size_t)split * N * ldg;
    const int r16 = lane & 15, q = lane >> 4;
    if constexpr (MODE == 2) {
#pragma unroll
        for (int mi = 0; mi < TM / 128; mi++)
#pragma unroll
            for (int ni = 0; ni < 2; ni++)
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int n = n0 + wn * 64 + ni * 32 + j * 16 + r16;
                        const int m = m0 + wm * (TM / 2) + mi * 64 + i * 16 + 4 * q;
                        hpnn::st_sc1(out + (size_t)n * ldg + m, acc[mi][ni][i][j]);
                    }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        /* 64-bit tickets (mfma_common.h): no wrap */
        unsigned long long want = 0;
        if (tid == 0) want = hpnn::ticket_arrive(upd.cnt + 32 * tile, (unsigned)splits);
        mark(3);
        if (side.on) { /* G1's share while the tile's other splits finish */
            if (tid == 0) hpnn::ticket_wait(side.cnt, want1, upd.err, TN8_TIMEOUT);
            __syncthreads();
            mark(4);
            side_reduce_step(side, upd, (int)blockIdx.x, ntiles * splits);
        }
        mark(5);
        if (tid == 0) hpnn::ticket_wait(upd.cnt + 32 * tile, want, upd.err, TN8_TIMEOUT);
        __syncthreads();
        mark(6);
        constexpr int NE4 = 256 * TM / 4, R4 = TM / 4;
        const int e0 = (int)((long)split * NE4 / splits), e1 = (int)((long)(split + 1) * NE4 / splits);
        const size_t ss = (size_t)N * ldg;
        for (int e = e0 + tid; e < e1; e += 512) {
            const int n = n0 + e / R4, m = m0 + 4 * (e % R4);
            const float *p = slab + (size_t)n * ldg + m;
            const size_t idx = (size_t)n * ldg + m;
            /* the step's operands first, then every split's partial in ONE batch of 16 loads
             * (one memory round trip per element instead of three) */
            f32x4 ww = *(const f32x4 *)(upd.W32 + idx), vv = {0.f, 0.f, 0.f, 0.f};
            if (upd.momentum) vv = *(const f32x4 *)(upd.V32 + idx);
            f32x4 g = {0.f, 0.f, 0.f, 0.f};
            for (int s0 = 0; s0 < splits; s0 += 16) {
                f32x4 v[16];
                const float *q[16];
#pragma unroll
                for (int j = 0; j < 16; j++) q[j] = p + (size_t)(s0 + j < splits ? s0 + j : s0) * ss;
                hpnn::ld_sc1_x16(v, q);
#pragma unroll
                for (int h = 0; h < 2; h++) /* groups of 8 summed first: the order of sum_sc1_x8 */
                    if (s0 + 8 * h < splits) {
                        f32x4 t = v[8 * h];
#pragma unroll
                        for (int j = 1; j < 8; j++)
                            if (s0 + 8 * h + j < splits) t += v[8 * h + j];
                        g += t;
                    }
            }
            if (upd.momentum) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    vv[r] += upd.lr * (g[r] * upd.scale);
                    ww[r] += vv[r];
                    vv[r] *= upd.alpha;
                }
                *(f32x4 *)(upd.V32 + idx) = vv;
            } else {
#pragma unroll
                for (int r = 0; r < 4; r++) ww[r] += upd.lr * (g[r] * upd.scale);
            }
            *(f32x4 *)(upd.W32 + idx) = ww;
            bf16x4 wb;
#pragma unroll
            for (int r = 0; r < 4; r++) wb[r] = (__bf16)ww[r];
            *(bf16x4 *)(upd.Wb + idx) = wb;
#pragma unroll
            for (int r = 0; r < 4; r++) upd.Wt[(size_t)(m + r) * N + n] = wb[r];
        }
        mark(7);
    } else if constexpr (MODE == 1) {
        /* W [N][ldg]: W32 / V32 / Wb row-major, Wt [ldg][N].  Per quadrant: all loads
         * first (8 fragments in flight), then the step, then the stores -- a load / use /
         * store chain per fragment would leave the epilogue latency-bound */
        float *__restrict__ W32 = upd.W32;
        float *__restrict__ V32 = upd.V32;
        __bf16 *__restrict__ Wb = upd.Wb;
        __bf16 *__restrict__ Wt = upd.Wt;
        __bf16 *tw = (__bf16 *)(lds + wave * 16384);
#pragma unroll
        for (int mi = 0; mi < 2; mi++)
#pragma unroll
            for (int ni = 0; ni < 2; ni++) {
                f32x4 w[4][2], v[4][2];
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const size_t idx = (size_t)(n0 + wn * 64 + ni * 32 + j * 16 + r16) * ldg +
                                           (m0 + wm * 128 + mi * 64 + i * 16 + 4 * q);
                        w[i][j] = *(const f32x4 *)(W32 + idx);
                        if (upd.momentum) v[i][j] = *(const f32x4 *)(V32 + idx);
                    }
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int n = n0 + wn * 64 + ni * 32 + j * 16 + r16;
                        const int m = m0 + wm * 128 + mi * 64 + i * 16 + 4 * q;
                        const size_t idx = (size_t)n * ldg + m;
                        const f32x4 g = acc[mi][ni][i][j];
                        f32x4 ww = w[i][j];
                        if (upd.momentum) {
                            f32x4 vv = v[i][j];
#pragma unroll
                            for (int r = 0; r < 4; r++) {
                                vv[r] += upd.lr * (g[r] * upd.scale);
                                ww[r] += vv[r];
                                vv[r] *= upd.alpha;
                            }
                            *(f32x4 *)(V32 + idx) = vv;
                        } else {
#pragma unroll
                            for (int r = 0; r < 4; r++) ww[r] += upd.lr * (g[r] * upd.scale);
                        }
                        *(f32x4 *)(W32 + idx) = ww;
                        bf16x4 wb;
#pragma unroll
                        for (int r = 0; r < 4; r++) wb[r] = (__bf16)ww[r];
                        *(bf16x4 *)(Wb + idx) = wb;
                        /* W^T through this wave's 16 KiB of the (now idle) LDS: [m][n] image of
                         * its 128 x 64 tile, written out below in 16-byte row pieces */
                        const int ml = mi * 64 + i * 16 + 4 * q, nl = ni * 32 + j * 16 + r16;
#pragma unroll
                        for (int r = 0; r < 4; r++) tw[(ml + r) * 64 + nl] = wb[r];
                    }
            }
        /* every wave is past its last operand read of the main loop (the final barriers),
         * and the region is this wave's own: LDS ops of one wave complete in order; the
         * fence + wave barrier order the cross-lane transpose (stores above by one lane,
         * 16-byte reads below by others) for the compiler as well */
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const int e = t * 64 + lane, ml = e >> 3, nc = (e & 7) * 8;
            *(bf16x8 *)(Wt + (size_t)(m0 + wm * 128 + ml) * N + n0 + wn * 64 + nc) = *(const bf16x8 *)(tw + ml * 64 + nc);
        }
    } else if constexpr (MODE == 3) {
#pragma unroll
        for (int mi = 0; mi < 2; mi++)
#pragma unroll
            for (int ni = 0; ni < 2; ni++)
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int n = n0 + wn * 64 + ni * 32 + j * 16 + r16;
                        const int m = m0 + wm * 128 + mi * 64 + i * 16 + 4 * q;
                        bf16x4 gb;
#pragma unroll
                        for (int r = 0; r < 4; r++) gb[r] = (__bf16)acc[mi][ni][i][j][r];
                        *(bf16x4 *)(upd.Wb + (size_t)n * ldg + m) = gb;
                    }
    } else {
#pragma unroll
        for (int mi = 0; mi < 2; mi++)
#pragma unroll
            for (int ni = 0; ni < 2; ni++)
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int n = n0 + wn * 64 + ni * 32 + j * 16 + r16;
                        const int m = m0 + wm * 128 + mi * 64 + i * 16 + 4 * q;
                        *(f32x4 *)(out + (size_t)n * ldg + m) = acc[mi][ni][i][j];
                    }
    }
}


template <int EPI, bool CF32>
int launch8(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux, int ldaux, int M, int N,
            int K, hipStream_t s, int splits = 1, long cstride = 0) {
    const int tiles_n = N / 256, ntiles = (M / 256) * tiles_n;
    hipLaunchKernelGGL((gemm_nt8_kernel<EPI, CF32>), dim3(ntiles * splits), dim3(512), 0, s, (const __bf16 *)A, lda,
                       (const __bf16 *)B, ldb, C, ldc, (const __bf16 *)aux, ldaux, K, tiles_n, ntiles, splits, cstride);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* C = epi(sum over S FP32 slabs [M][N] of the split-K GEMM), 4 consecutive columns per thread */
template <int EPI, bool CF32>
__global__ __launch_bounds__(256) void nt_splitk_epi_kernel(const float *__restrict__ P, int S, long cstride, int M,
                                                            int N, const __bf16 *__restrict__ aux, int ldaux,
                                                            void *__restrict__ C, int ldc) {
    const long n4 = (long)M * N / 4;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n4; e += (long)gridDim.x * blockDim.x) {
        const int b = (int)(e * 4 / N), f = (int)(e * 4 % N);
        f32x4 v = ((const f32x4 *)P)[e];
        for (int s = 1; s < S; s++) v += ((const f32x4 *)(P + (size_t)s * cstride))[e];
        if constexpr (EPI == HPNN_EPI_ACT) {
#pragma unroll
            for (int r = 0; r < 4; r++) v[r] = hpnn::bipolar(v[r]);
        } else if constexpr (EPI == HPNN_EPI_DACT) {
            const bf16x4 h = *(const bf16x4 *)(aux + (size_t)b * ldaux + f);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float y = (float)h[r];
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

template <int EPI, bool CF32>
int splitk_epi(const float *P, int S, long cstride, int M, int N, const void *aux, int ldaux, void *C, int ldc,
               hipStream_t s) {
    const long n4 = (long)M * N / 4;
    const int blocks = (int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048);
    hipLaunchKernelGGL((nt_splitk_epi_kernel<EPI, CF32>), dim3(blocks), dim3(256), 0, s, P, S, cstride, M, N,
                       (const __bf16 *)aux, ldaux, C, ldc);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* split-K workspace, one per device (train_nn -G drives several GPUs from one process, one
 * host thread each): grown outside stream capture only -- a capture that would need a
 * bigger one gets -1 and the caller takes another kernel.  Split-K GEMMs of one device
 * share it, so they must be stream-ordered (the engines issue GEMMs on one compute stream
 * per device); it lives until the process exits. */
constexpr int WS_DEV = 64;
float *g_ws[WS_DEV] = {};
size_t g_ws_bytes[WS_DEV] = {};
std::mutex g_ws_mu;
float *splitk_ws(size_t bytes, hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= WS_DEV) return nullptr;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    if (bytes <= g_ws_bytes[dev]) return g_ws[dev];
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
    if (hipDeviceSynchronize() != hipSuccess) return nullptr; /* the old buffer may be in use */
    if (g_ws[dev]) hipFree(g_ws[dev]);
    g_ws[dev] = nullptr;
    g_ws_bytes[dev] = 0;
    if (hipMalloc((void **)&g_ws[dev], bytes) != hipSuccess) return nullptr;
    g_ws_bytes[dev] = bytes;
    return g_ws[dev];
}

}  // namespace

extern "C" int hpnn_gemm_nt8_bf16(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux,
                                  int ldaux, int M, int N, int K, int epi, int c_f32, hipStream_t stream) {
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 128) return -1;
    if (lda % 8 || ldb % 8 || ldc % 4 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return -1;
    if ((size_t)lda * 2 * 256 >= (1u << 31) || (size_t)ldb * 2 * 256 >= (1u << 31)) return -1; /* 32-bit offsets */
    if (epi == HPNN_EPI_DACT && (!aux || ldaux % 4)) return -1;
    if (c_f32) {
        if (epi == HPNN_EPI_NONE) return launch8<HPNN_EPI_NONE, true>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
        if (epi == HPNN_EPI_ACT) return launch8<HPNN_EPI_ACT, true>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
        return launch8<HPNN_EPI_DACT, true>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
    }
    if (epi == HPNN_EPI_NONE) return launch8<HPNN_EPI_NONE, false>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
    if (epi == HPNN_EPI_ACT) return launch8<HPNN_EPI_ACT, false>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
    return launch8<HPNN_EPI_DACT, false>(A, lda, B, ldb, C, ldc, aux, ldaux, M, N, K, stream);
}

/* TN entry for gemm_tn_dispatch (kernels_mfma.hip): -1 when the shape does not fit */
int hpnn_gemm_tn8_launch(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M, int Bt,
                         int splits, hipStream_t stream, const hpnn::TnTail &tail) {
    if (N % 256 || M % 256 || Bt % 128 || splits < 1 || ldd % 8 || ldh % 8 || ldg % 4) return -1;
    const int units = Bt / 64;
    if (units % splits || (units / splits) % 2) return -1;
    if ((size_t)ldd * 2 * 64 >= (1u << 31) || (size_t)ldh * 2 * 64 >= (1u << 31)) return -1;
    const int tiles_n = N / 256, ntiles = tiles_n * (M / 256);
    hipLaunchKernelGGL(gemm_tn8_kernel<0>, dim3(ntiles * splits + tail.blocks), dim3(512), 0, stream,
                       (const __bf16 *)D, ldd, (const __bf16 *)H, ldh, slab, ldg, N, units, splits, tiles_n, ntiles,
                       tail, Tn8Upd{}, Tn8Side{});
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* the shape check of hpnn_gemm_tn8_bf16out (without the pointer alignment): 1 when it fits */
extern "C" int hpnn_gemm_tn8_bf16out_ok(int N, int M, int Bt, int ldd, int ldh) {
    if (N % 256 || M % 256 || Bt % 128 || ldd % 8 || ldh % 8 || (Bt / 64) % 2) return 0;
    return (size_t)ldd * 2 * 64 < (1u << 31) && (size_t)ldh * 2 * 64 < (1u << 31);
}

/* G = D^T H over the whole batch (one split), rounded to BF16 into G16 [N][ldg]: -1 when the
 * shape does not fit the 8-phase kernel */
extern "C" int hpnn_gemm_tn8_bf16out(const void *D, int ldd, const void *H, int ldh, void *G16, int ldg, int N, int M,
                                     int Bt, hipStream_t stream) {
    if (N % 256 || M % 256 || Bt % 128 || ldd % 8 || ldh % 8 || ldg % 4 || ((uintptr_t)G16 & 7)) return -1;
    const int units = Bt / 64;
    if (units % 2) return -1;
    if ((size_t)ldd * 2 * 64 >= (1u << 31) || (size_t)ldh * 2 * 64 >= (1u << 31)) return -1;
    const int tiles_n = N / 256, ntiles = tiles_n * (M / 256);
    Tn8Upd u{};
    u.Wb = (__bf16 *)G16;
    hipLaunchKernelGGL(gemm_tn8_kernel<3>, dim3(ntiles), dim3(512), 0, stream, (const __bf16 *)D, ldd,
                       (const __bf16 *)H, ldh, nullptr, ldg, N, units, 1, tiles_n, ntiles, hpnn::TnTail{}, u, Tn8Side{});
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* G = D^T H over the whole batch (one split) with the optimizer step applied in the
 * epilogue: the gradient never goes to memory (saves its write and the update kernel's
 * read of it, and the update launch).  W [N][M] FP32 master (+ V32 momentum), Wbf [N][M],
 * Wt [M][N] BF16 copies, exactly the step of hpnn_sgd_update with one slab.  -1: shape
 * not supported (256x256 tiles, an even number of 64-row units). */
extern "C" int hpnn_gemm_tn8_update(const void *D, int ldd, const void *H, int ldh, int N, int M, int Bt, float *W32,
                                    float *V32, void *Wbf, void *Wt, float lr, float alpha, float scale, int momentum,
                                    hipStream_t stream) {
    if (N % 256 || M % 256 || Bt % 128 || ldd % 8 || ldh % 8 || !W32 || !Wbf || !Wt || (momentum && !V32)) return -1;
    /* the epilogue moves W32 / V32 as float4 and W / W^T as 8- and 16-byte pieces */
    if (((uintptr_t)W32 | (uintptr_t)(momentum ? V32 : W32) | (uintptr_t)Wbf | (uintptr_t)Wt) & 15) return -1;
    if ((size_t)ldd * 2 * 64 >= (1u << 31) || (size_t)ldh * 2 * 64 >= (1u << 31)) return -1;
    const int tiles_n = N / 256, ntiles = tiles_n * (M / 256);
    const Tn8Upd u{W32, V32, (__bf16 *)Wbf, (__bf16 *)Wt, lr, alpha, scale, momentum, nullptr, nullptr};
    hipLaunchKernelGGL(gemm_tn8_kernel<1>, dim3(ntiles), dim3(512), 0, stream, (const __bf16 *)D, ldd,
                       (const __bf16 *)H, ldh, nullptr, M, N, Bt / 64, 1, tiles_n, ntiles, hpnn::TnTail{}, u, Tn8Side{});
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* the same step for a gradient over `splits` splits (>= 2), reduced inside the launch
 * (MODE 2 above): slab is the scratch the partials are published through ([splits][N][M]).
 * -1: shape not covered, or more workgroups than the device holds at once (every split of a
 * tile waits for the others: hpnn_resident_capacity), or HPNN_TN8_FUSED=0. */
extern "C" int hpnn_gemm_tn8_fused_update_side(const void *D, int ldd, const void *H, int ldh, int N, int M, int Bt,
                                               int splits, float *slab, float *W32, float *V32, void *Wbf, void *Wt,
                                               float lr, float alpha, float scale, int momentum, unsigned int *cnt,
                                               unsigned int *err, const hpnn_tn8_side *sd, hipStream_t stream) {
    static const bool on = [] { const char *e = getenv("HPNN_TN8_FUSED"); return !(e && e[0] == '0'); }();
    /* every split of a tile waits for the others: the whole grid must be resident at once */
    static const int cap = hpnn_resident_capacity((const void *)gemm_tn8_kernel<2>, 512, 0);
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev))
            cus = -1;
    }
    if (!on || splits < 2 || !slab || !cnt || !err) return -1;
    if (N % 256 || M % 256 || Bt % 128 || ldd % 8 || ldh % 8 || !W32 || !Wbf || !Wt || (momentum && !V32)) return -1;
    if (((uintptr_t)W32 | (uintptr_t)(momentum ? V32 : W32) | (uintptr_t)Wbf | (uintptr_t)slab) & 15) return -1;
    if ((size_t)ldd * 2 * 64 >= (1u << 31) || (size_t)ldh * 2 * 64 >= (1u << 31)) return -1;
    const int units = Bt / 64;
    if (units % splits || (units / splits) % 2) return -1;
    /* 256 x 128 tiles at half the splits (HPNN_TN8_TM=128; same grid, half the partial bytes) */
    static const int tm_req = [] { const char *e = getenv("HPNN_TN8_TM"); return e ? atoi(e) : 256; }();
    const bool t128 = tm_req == 128 && splits % 2 == 0 && (units / (splits / 2)) % 2 == 0;
    if (t128) splits /= 2;
    const int TMv = t128 ? 128 : 256;
    if (M % TMv) return -1;
    const int tiles_n = N / 256, ntiles = tiles_n * (M / TMv);
    /* 64-bit tickets: 32 words apart in 1024, up to 32 tiles (a block the caller keeps for this GEMM shape: the
     * counters are monotonic, every launch must add `splits` per tile); at least min_wg workgroups (HPNN_TN8_MINWG, default
     * half the CUs: fewer splits leave the chip idle while each reduces a larger share) */
    static const int min_wg = [] { const char *e = getenv("HPNN_TN8_MINWG"); return e ? atoi(e) : 0; }();
    if (ntiles > 32 || ntiles * splits > cap || ntiles * splits < (min_wg > 0 ? min_wg : cus / 2)) return -1;
    const Tn8Upd u{W32, V32, (__bf16 *)Wbf, (__bf16 *)Wt, lr, alpha, scale, momentum, cnt, err};
    Tn8Side side{};
    if (sd) { /* the next layer's gradient + step as the side job: -2 when it does not fit */
        const int G = ntiles * splits, su = Bt / 64;
        if (!sd->D || !sd->H || !sd->slab || !sd->W32 || !sd->Wb || !sd->Wt || !sd->cnt || (momentum && !sd->V32))
            return -2;
        if (sd->N % 64 || sd->M % 64 || sd->S < 1 || su % sd->S || sd->ldd % 8 || sd->ldh % 8) return -2;
        if (((uintptr_t)sd->W32 | (uintptr_t)(momentum ? sd->V32 : sd->W32) | (uintptr_t)sd->slab | (uintptr_t)sd->Wb) &
            15)
            return -2;
        const int tiles = (sd->N / 64) * (sd->M / 64), jobs = tiles * sd->S;
        /* every half-workgroup must run the same number of pieces (they share the barriers) */
        if (G % 8 || jobs % (2 * G)) return -2;
        side = Tn8Side{(const __bf16 *)sd->D, (const __bf16 *)sd->H, sd->slab, sd->W32, sd->V32, (__bf16 *)sd->Wb,
                       (__bf16 *)sd->Wt, sd->cnt, sd->ldd, sd->ldh, sd->N, sd->M, su, sd->S, sd->N / 64, tiles, jobs, 1};
    }
    static const bool trace = [] { const char *e = getenv("HPNN_TN8_TRACE"); return e && e[0] == '1'; }();
    auto kern = t128 ? (trace ? gemm_tn8_kernel<2, true, 128> : gemm_tn8_kernel<2, false, 128>)
                     : (trace ? gemm_tn8_kernel<2, true> : gemm_tn8_kernel<2, false>);
    hipLaunchKernelGGL(kern, dim3(ntiles * splits), dim3(512), 0, stream, (const __bf16 *)D, ldd, (const __bf16 *)H, ldh, slab, M, N, units, splits, tiles_n,
                       ntiles, hpnn::TnTail{}, u, side);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* HPNN_TN8_TRACE=1 stamps: out[512][8] shader-clock ticks (thread 0 of each workgroup) */
extern "C" int hpnn_tn8_trace(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tn8_trace), sizeof(g_tn8_trace)) == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_gemm_tn8_fused_update(const void *D, int ldd, const void *H, int ldh, int N, int M, int Bt,
                                          int splits, float *slab, float *W32, float *V32, void *Wbf, void *Wt,
                                          float lr, float alpha, float scale, int momentum, unsigned int *cnt,
                                          unsigned int *err, hipStream_t stream) {
    return hpnn_gemm_tn8_fused_update_side(D, ldd, H, ldh, N, M, Bt, splits, slab, W32, V32, Wbf, Wt, lr, alpha, scale,
                                           momentum, cnt, err, nullptr, stream);
}

/* split-K form for GEMMs with too few 256x256 tiles to fill the chip (the RRUFF-shaped
 * first layer, 16384 x 256 x 4096: 64 tiles): S splits into FP32 slabs, then one
 * elementwise pass sums them and applies the epilogue.  -1: shape / workspace not
 * available (the caller keeps its other kernels). */
extern "C" int hpnn_gemm_nt8_splitk_bf16(const void *A, int lda, const void *B, int ldb, void *C, int ldc,
                                         const void *aux, int ldaux, int M, int N, int K, int epi, int c_f32,
                                         int splits, hipStream_t stream) {
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || splits < 2 || K % (128 * splits)) return -1;
    if (lda % 8 || ldb % 8 || ldc % 4 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return -1;
    if ((size_t)lda * 2 * 256 >= (1u << 31) || (size_t)ldb * 2 * 256 >= (1u << 31)) return -1;
    if (epi == HPNN_EPI_DACT && (!aux || ldaux % 4)) return -1;
    const long cstride = (long)M * N;
    float *P = splitk_ws((size_t)splits * cstride * 4, stream);
    if (!P) return -1;
    int rc = launch8<HPNN_EPI_NONE, true>(A, lda, B, ldb, P, N, nullptr, 0, M, N, K, stream, splits, cstride);
    if (rc) return rc;
#define HPNN_SKE(E_, F_) return splitk_epi<E_, F_>(P, splits, cstride, M, N, aux, ldaux, C, ldc, stream)
    if (c_f32) {
        if (epi == HPNN_EPI_NONE) HPNN_SKE(HPNN_EPI_NONE, true);
        if (epi == HPNN_EPI_ACT) HPNN_SKE(HPNN_EPI_ACT, true);
        HPNN_SKE(HPNN_EPI_DACT, true);
    }
    if (epi == HPNN_EPI_NONE) HPNN_SKE(HPNN_EPI_NONE, false);
    if (epi == HPNN_EPI_ACT) HPNN_SKE(HPNN_EPI_ACT, false);
    HPNN_SKE(HPNN_EPI_DACT, false);
#undef HPNN_SKE
}


