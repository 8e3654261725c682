/*
 * mlp3_tile: the n_in -> 128 -> 64 -> n_out(<=32) training step up to delta1, one
 * 256-sample tile per workgroup iteration (gfx950).
 *
 * Reference: the per-sample GEMV chain of ann_kernel_train / snn_kernel_train
 * (ann.c:883-888, 1279-1592; snn.c:280-335, 481-794; cuda_ann.cu:426-2093,
 * cuda_snn.cu:156-976 softmax, 2726-3717 train_momentum), batched.
 *
 * Input: the minibatch in FRAGMENT-MAJOR order ([Bp/32][K0/16][64 lanes][8], lane
 * l = 16 g + r of chunk (t, cb) holding X[32 t + 8 g + j][16 cb + r], j < 8; see
 * ops.to_fragment_major), either 8-bit pixels (the exact integers in BF16, the pixel scale
 * xscale applied to the FP32 accumulator: H1 = f(xscale * X W0^T)) or BF16 (xscale 1).
 * It is the SAME buffer the first-layer gradient kernel (kernels_g0.hip,
 * gemm_fm_direct) streams right after this one, so the second read of a step finds it in
 * the 256 MB Infinity Cache.  Where the front's read comes from depends on the data: with
 * bench.py's 4 cycled 52 MB batches part of it is still cached from 4 steps before, with 8
 * (past the cache) the step is 3.5 % slower (profiles/r5/SUMMARY.md; the L2-side counters
 * cannot separate Infinity-Cache hits from HBM reads).
 *
 * One 512-thread workgroup (8 waves) per CU; per 256-sample tile:
 *
 *  A  H1 = f(X W0^T)  [256 x 128]: K0/32 k-steps.  Wave (ng = w&3, sh = w>>2) owns 32
 *     neurons x 128 samples (16 MFMA 16x16x32 per k-step, 64 accumulator registers).
 *     Its two W0 fragments per k-step come straight from the L2-resident fragment-major
 *     copy into registers (1 KiB per wave load); the X slice (256 samples x 32 features,
 *     8 KiB of pixels) is loaded once per workgroup, one 16-byte load per lane,
 *     converted in registers and written as the transposed image X^T [32 feat][256
 *     samples] into one of two LDS stages; MFMA B operands are read from it with
 *     ds_read_b64_tr_b16.  The k-step's MFMAs are interleaved with its conversion VALU and B
 *     reads (sched_group_barrier: MFMA, LDS read, VALU, ...): an MFMA holds the SIMD's vector
 *     issue for 8 of its 16 cycles, so that work issues in the other 8 instead of in series
 *     (phase A 24.0K vs 26.0K ticks).  (Measured and not kept, round 4: every wave loading its X
 *     fragments straight into registers from a row-fragment-major copy -- no X^T stage, no
 *     barrier in phase A: the four neuron-group waves then pull 4x the X bytes through the
 *     vector L1; phase A 31.2K vs 27.0K ticks, the drifted waves meeting at the H1 barrier
 *     16.6K vs 4.7K, 76 vs 61 us per step.  Also measured: three X^T stages with the B
 *     fragments read just before their MFMAs and W0 loads 3 / 4 k-steps ahead, 62.0-62.1 /
 *     61.5-61.6 vs 61.4-61.6 us same box.)  Loads run D k-steps ahead (register ring), one
 *     barrier per k-step.  The K loop is fully unrolled (K0 is a template parameter) so every ring
 *     index is static and the compiler's counted vmcnt waits stay exact.
 *  B  back chain, per wave on ITS OWN 32 samples (no workgroup barrier inside):
 *     H2 = f(H1 W1^T), logits, softmax / sigmoid + loss + delta3 + argmax,
 *     delta2 = (delta3 W2) f'(H2), delta1 = (delta2 W1) f'(H1) -> HBM (fragment-major,
 *     the operand layout of the G0 kernel).
 *  C  one barrier, then G1 += H1^T delta2 and G2 += H2^T delta3 over all 256 samples,
 *     each wave owning output tiles (accumulated in registers over the block's tiles,
 *     written once as the block's [G1 | G2] FP32 slab, the layout of mlp3_mid).
 *
 * Versus mlp3_fused (kernels_mlp3x.hip, 32-sample tiles with a software-pipelined
 * front/back interleave and W0 resident in VGPRs): the tile is 8x larger, so the
 * latency-bound back chain runs once per 256 samples with 8x the independent MFMA work
 * per phase, and needs 2 barriers per tile instead of 4 per 32 samples.
 *
 * LDS (160 KiB, exactly): H1 [256][128] 64 KiB | X^T stages 2 x 16 KiB, aliased by
 * H2 [256][64] in the chain | delta2 [256][64] 32 KiB | delta3 [256][32] 16 KiB |
 * W1 [64][128] 16 KiB.  All images use the T32 layout of mfma_common.h.  (W1 / W1^T operands
 * straight from the L2 into registers instead of the W1 image measured slower: 62.5-62.8 vs
 * 60.2-60.7 us per step -- under phase A's streaming an L2 hit costs ~2-3K shader clocks.)
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"

HPNN_CO_PROBE(mlp3t)
#include "mfma_common.h"
#include "mlp3_common.h"

using namespace hpnn;
using namespace hpnn::mlp3;

namespace {

constexpr int TS = 256;              /* samples per tile */
constexpr int XR = 32;               /* features per k-step (rows of the X^T stage) */
constexpr int IMG_XT = XR * TS * 2;  /* 16 KiB */
constexpr int OFF_H1 = 0;
constexpr int OFF_XT = OFF_H1 + TS * H1 * 2;
constexpr int OFF_H2 = OFF_XT; /* chain only: the X^T stages are dead then */
constexpr int OFF_D2 = OFF_XT + 2 * IMG_XT;
constexpr int OFF_D3 = OFF_D2 + TS * H2 * 2;
constexpr int OFF_W1 = OFF_D3 + TS * NO * 2;
constexpr int LDS_TOTAL = OFF_W1 + IMG_W1;
static_assert(TS * H2 * 2 <= 2 * IMG_XT, "H2 aliases the X^T stages");
static_assert(LDS_TOTAL <= 160 * 1024, "LDS");

/* within-wave ordering of LDS writes before other lanes' reads (one wave's LDS
 * instructions execute in order; this keeps the compiler from moving them) */
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* HPNN_TILE_TRACE=1 (profiling only): s_memtime stamps of every workgroup's wave 0 at the
 * phase boundaries, [block][mark]; read back with hpnn_mlp3_tile_trace */
constexpr int TR_BLOCKS = 1024, TR_MARKS = 12;
__device__ unsigned long long g_tile_trace[TR_BLOCKS][TR_MARKS];

template <int TYPE, bool LABELS, int KS, bool XU8, int D, bool TRACE = false, int ABL = 0, bool EARLY = true,
          bool TRADE = false, bool XORD = false, int IL = 1, bool CB = false>
__global__ __launch_bounds__(512) void mlp3_tile_kernel(const void *__restrict__ Xg, float xscale,
                                                            const __bf16 *__restrict__ W0f,
                                                            const __bf16 *__restrict__ W1,
                                                            const __bf16 *__restrict__ W2,
                                                            const __bf16 *__restrict__ W2t,
                                                            const int *__restrict__ labels,
                                                            const float *__restrict__ T, int ldt, float t_hi,
                                                            float t_lo, __bf16 *__restrict__ D1,
                                                            float *__restrict__ gslab, float *__restrict__ loss_acc,
                                                            unsigned int *__restrict__ correct, int n_tiles,
                                                            int n_valid, int n_out) {
    /* 8 waves (a 16-wave workgroup, 128 VGPRs a wave, measured slower: 65.2 vs 60.2-60.7 us
     * per step, its chain no faster -- the chain is bound by LDS / MFMA throughput, not by
     * per-wave latency).  Phase A on 32 x 128 wave tiles: 64 x 64 (half the B reads, twice
     * the W0 fragments) measured 59.1-59.9 vs 58.1-58.9 us same box. */
    constexpr int NW = 8;
    constexpr int CHUNK = XU8 ? 512 : 1024; /* bytes of one 32 x 16 input chunk */
    constexpr int NCB = 2 * KS;             /* 16-feature blocks per 32-sample row of chunks */
    /* per k-step the workgroup loads 16 chunks (8 sample rows x 2 feature halves): wave w
     * takes row w, lane half h = l >> 5 takes feature half h, XB bytes per lane (2 fm lanes) */
    constexpr int XB = 16 * (XU8 ? 1 : 2); /* bytes per lane per k-step */
    constexpr int XV = XB / 16;            /* 16-byte vectors per lane */
    constexpr int SG = NW / 4;           /* phase A: sample groups (waves per neuron group) */
    constexpr int SPA = TS / SG;         /* phase A: samples per wave */
    constexpr int STA = SPA / 16;        /* phase A: 16-sample tiles per wave */
    constexpr int SPC = TS / NW;         /* chain: samples per wave */
    constexpr int STC = SPC / 16;        /* chain: 16-sample tiles per wave */
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ng = wave & 3, sh = wave >> 2; /* phase A: neurons 32 ng.., samples SPA sh.. */
    const int r16 = lane & 15, q = lane >> 4;
    const LaneOff lo = lane_offsets(lane);
    char *imgH1 = lds + OFF_H1, *imgH2 = lds + OFF_H2, *imgD2 = lds + OFF_D2, *imgD3 = lds + OFF_D3;
    char *imgW1 = lds + OFF_W1;
    auto mark = [&](int i) {
        if constexpr (TRACE) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (tid == 0 && blockIdx.x < TR_BLOCKS) g_tile_trace[blockIdx.x][i] = t;
        }
    };
    mark(0);

    /* ---- once per launch: W1 -> LDS image ---- */
    {
        constexpr int PIECES = (H1 / 32) * (H2 / 16);
        for (int p = wave; p < PIECES; p += NW) glds_t32_piece<H2>((const char *)W1, (size_t)H1 * 2, imgW1, p, lane);
    }
    /* no wait here: the W1 pieces are this wave's oldest vector-memory ops, so phase A's
     * first counted wait (for X(0)) covers them, and its barriers publish them */
    mark(1);

    /* the G1 / G2 partial sums of this block's tiles live in its slab between tiles (not in
     * registers through phase A): stored by the first tile, read-added-stored by later ones;
     * every element belongs to one lane of one wave */
    float *const slab = gslab + (size_t)blockIdx.x * SLAB;
    float my_loss = 0.f;
    unsigned int my_hit = 0;
    const int n_ot = n_out > 16 ? 2 : 1;
    const float inv_nout = 1.0f / (float)n_out;

    /* X^T stage image: row = feature within the k-step, column = sample of the tile.
     * This lane converts fm slots 2i, 2i+1 (i = lane & 31) of chunk (t = wave, cb = 2s + lane/32). */
    int xoff[2];
    const int xi = lane & 31, xcbh = lane >> 5, xg = xi >> 3;
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int row = 16 * xcbh + 2 * (xi & 7) + e;
        xoff[e] = wave * (XR * 64) + row * 64 + (((xg ^ t32_g(row)) & 3) << 4);
    }
    /* write order (XORD, HPNN_TILE_XORD=1; off by default: the selects measured slower than
     * the conflicts): lanes k = xi & 7 with bit 1 set write their odd row first.  Lane k's rows
     * 2k + e sit at bank group 4 e + g(k) (g = t32_g(2k): 0 1 0 1 2 3 2 3), so in-order
     * writes put each 8-lane ds_write_b128 group on 4 bank groups (2-way conflict); the
     * swapped order spreads it over all 8 */
    const int xp = XORD ? (xi >> 1) & 1 : 0;
    const int xa0 = xoff[xp], xa1 = xoff[xp ^ 1];
    const char *xbase = (const char *)Xg + ((size_t)wave * NCB + xcbh) * CHUNK + (size_t)xi * XB;

    /* transposed-read addresses of this wave's STA sample tiles in an X^T stage: sample tile
     * st sits in 32-column sub-tile (STA/2) sh + st/2, with the T32 chunk swap (lo.tr ^ 32)
     * on odd st; two bases + immediate offsets */
    const char *xt_e = lds + OFF_XT + (STA / 2 * sh) * (XR * 64) + lo.tr;
    const char *xt_o = lds + OFF_XT + (STA / 2 * sh) * (XR * 64) + (lo.tr ^ 32);

    for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int T0 = tile * (TS / 32); /* first 32-sample chunk row of the tile */
        const char *xtile = xbase + (size_t)T0 * NCB * CHUNK;
        const __bf16 *wbase = W0f + ((size_t)(2 * ng) * KS * 64 + lane) * 8;

        typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
        u32x4 xr[KS][XV];
        bf16x8 wr[KS][2];
        /* X(sx) and W0(sw) in one batch: an opaque zero pins the loads to this point of the
         * k-loop (the operands are read-only, so the compiler would otherwise hoist every W0
         * load out of the tile loop: spills).  X(k) is consumed two k-steps before W0(k)
         * (converted into the LDS stage the B reads of step k come from), so the batch at
         * step s carries X(s + D + 1) and W0(s + D - 1): step s then waits for exactly one
         * batch, X(s + 2) for its conversion and W0(s) for its MFMAs. */
        auto issue = [&](int sx, int sw) {
            unsigned int z = 0;
            asm volatile("" : "+s"(z));
            /* ABL (profiling only, wrong results): 1 = no W0 loads, 2 = no X loads, 7 = neither (a
             * non-zero register pattern instead: zero operands would raise the clock) */
            const unsigned int pat = z + 0x3c013c01u;
            if (sx < KS) {
#pragma unroll
                for (int n = 0; n < XV; n++)
                    xr[sx][n] = (ABL == 2 || ABL == 7) ? u32x4{pat, pat + 1, pat + 2, pat + 3}
                                                       : *(const u32x4 *)(xtile + z + (size_t)(2 * sx) * CHUNK + 16 * n);
            }
            if (sw >= 0 && sw < KS) {
#pragma unroll
                for (int i = 0; i < 2; i++)
                    wr[sw][i] = (ABL == 1 || ABL == 7)
                                    ? __builtin_bit_cast(bf16x8, u32x4{pat, pat + 4u * i, pat + 2, pat + 3})
                                    : *(const bf16x8 *)(wbase + z + ((size_t)i * KS + sw) * 512);
            }
        };
        /* X^T stage of k-step s: two alternating stages */
        auto soff = [](int s) { return (s & 1) * IMG_XT; };
        auto convert = [&](int s) {
            char *img = lds + OFF_XT + soff(s);
            bf16x8 v[2];
            if constexpr (XU8) {
                v[0] = u8x8_int_bf16(xr[s][0][0], xr[s][0][1]);
                v[1] = u8x8_int_bf16(xr[s][0][2], xr[s][0][3]);
            } else {
                v[0] = __builtin_bit_cast(bf16x8, xr[s][0]);
                v[1] = __builtin_bit_cast(bf16x8, xr[s][1]);
            }
            *(bf16x8 *)(img + xa0) = xp ? v[1] : v[0];
            *(bf16x8 *)(img + xa1) = xp ? v[0] : v[1];
        };

        f32x4 acc[2][STA];
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int st = 0; st < STA; st++) acc[i][st] = f32x4{0.f, 0.f, 0.f, 0.f};

        /* B operand fragments of this wave's STA sample tiles from X^T stage s & 1 */
        auto read_b = [&](int s, bf16x8 (&b)[STA]) {
#pragma unroll
            for (int st = 0; st < STA; st++) {
                const char *pb = ((st & 1) ? xt_o : xt_e) + soff(s) + (st >> 1) * (XR * 64);
                const s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)pb);
                const s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(pb + 256));
                const s16x8 v = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
                b[st] = __builtin_bit_cast(bf16x8, v);
            }
        };
        /* H1 tile -> LDS image [sample][neuron] */
        auto h1_epilogue = [&]() {
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int st = 0; st < STA; st++) {
                    bf16x4 o;
#pragma unroll
                    for (int r = 0; r < 4; r++) o[r] = (__bf16)bipolar(acc[i][st][r] * xscale);
                    st_d4<TS, TRADE>(imgH1, lo, SPA * sh + 16 * st, 32 * ng + 16 * i, o, lane);
                }
        };
        {
            /* the previous tile's chain read H2 (= the X^T stages) and H1 */
            lds_barrier();
#pragma unroll
            for (int s = 0; s <= D && s < KS; s++) issue(s, s - 2);
            convert(0);
            if (KS > 1) convert(1);
            lds_barrier();
            bf16x8 bb[2][STA]; /* B fragments of k-step s in bb[s & 1], read one k-step ahead */
            read_b(0, bb[0]);
            lds_barrier(); /* every wave's stage-0 reads are done before convert(2) refills it */
            mark(2);
            /* ================= phase A: H1 = f(X W0^T) =================
             * k-step s: X(s + 2) is converted into stage s & 1 (its step-s reads finished before
             * the last barrier; EARLY) and the B reads of step s + 1 (stage (s+1) & 1, filled at
             * step s - 1) go out before the MFMAs of step s, so the LDS traffic hides behind
             * them; one barrier publishes stage s & 1 and retires the step-(s+1) reads. */
#pragma unroll
            for (int s = 0; s < KS; s++) {
                issue(s + D + 1, s + D - 1);
                /* EARLY: X(s + 2) goes into stage s & 1 BEFORE the MFMAs of step s -- that stage's
                 * operands already sit in registers (read at step s - 1, retired by its barrier), so
                 * the conversion and its LDS writes overlap the MFMAs and the barrier only waits
                 * for them; otherwise after the MFMAs, in series with them */
                if constexpr (EARLY)
                    if (s + 2 < KS && ABL != 5 && ABL != 8 && ABL != 9) convert(s + 2);
                if (s + 1 < KS && ABL != 4 && ABL != 8 && ABL != 9) read_b(s + 1, bb[(s + 1) & 1]);
                if constexpr (IL == 0) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int st = 0; st < STA; st++) {
                    if constexpr (ABL != 3) {
                        acc[0][st] = mfma(wr[s][0], bb[s & 1][st], acc[0][st]);
                        acc[1][st] = mfma(wr[s][1], bb[s & 1][st], acc[1][st]);
                    } else {
                        acc[0][st] += __builtin_bit_cast(f32x4, wr[s][0]) * 0.f;
                    }
                }
                if constexpr (IL > 0) {
                    /* IL: the k-step's MFMAs interleaved with its conversion VALU and LDS traffic
                     * (one MFMA, one LDS read, IL VALU ops, ...), so the wave issues them in the
                     * shadow of its own MFMA pipe instead of in series with it */
#pragma unroll
                    for (int i = 0; i < 2 * STA; i++) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, IL, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (!EARLY)
                    if (s + 2 < KS && ABL != 5) convert(s + 2);
                if constexpr (ABL == 6 || ABL == 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* no barrier */
                else lds_barrier();
            }
            mark(3);
            h1_epilogue();
        }
        lds_barrier();

        mark(4);
        /* ================= phase B: back chain on this wave's SPC samples ================= */
        const int sw = SPC * wave;
        /* W2 / W2^T operand fragments (L2-resident), not held through phase A */
        bf16x8 w2f[2][2], w2tf[4]; /* P2: A = W2[o][h2] rows; P3: A = W2^T[h2][o] rows */
#pragma unroll
        for (int ot = 0; ot < 2; ot++)
#pragma unroll
            for (int kk = 0; kk < 2; kk++)
                w2f[ot][kk] = *(const bf16x8 *)(W2 + (size_t)(16 * ot + r16) * H2 + 32 * kk + 8 * q);
#pragma unroll
        for (int ht = 0; ht < 4; ht++) w2tf[ht] = *(const bf16x8 *)(W2t + (size_t)(16 * ht + r16) * NO + 8 * q);
        int lab[STC];
#pragma unroll
        for (int st = 0; st < STC; st++) {
            lab[st] = -1;
            if constexpr (LABELS) {
                int s = tile * TS + sw + 16 * st + r16;
                s = s < n_valid ? s : (n_valid > 0 ? n_valid - 1 : 0);
                lab[st] = labels[s];
            }
        }
        /* P1: H2^T [h2][sample] = f(W1 H1^T), this wave's STC sample tiles together: each W1
         * fragment is read from LDS once and feeds STC independent MFMAs */
        {
            f32x4 a[STC][4];
#pragma unroll
            for (int st = 0; st < STC; st++)
#pragma unroll
                for (int ht = 0; ht < 4; ht++) a[st][ht] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H1; k += 32) {
                bf16x8 b[STC];
#pragma unroll
                for (int st = 0; st < STC; st++) b[st] = rd_row<TS>(imgH1, lo, sw + 16 * st, k);
#pragma unroll
                for (int ht = 0; ht < 4; ht++) {
                    const bf16x8 w = rd_row<H2>(imgW1, lo, 16 * ht, k);
#pragma unroll
                    for (int st = 0; st < STC; st++) a[st][ht] = mfma(w, b[st], a[st][ht]);
                }
            }
#pragma unroll
            for (int st = 0; st < STC; st++)
#pragma unroll
                for (int ht = 0; ht < 4; ht++) {
                    bf16x4 o;
#pragma unroll
                    for (int r = 0; r < 4; r++) o[r] = (__bf16)bipolar(a[st][ht][r]);
                    st_d4<TS, TRADE>(imgH2, lo, sw + 16 * st, 16 * ht, o, lane);
                }
        }
        mark(5);
        wave_lds_fence();
        /* P2: logits, output activation, loss, delta3 -> D3 image */
#pragma unroll
        for (int st = 0; st < STC; st++) {
            const int r0 = sw + 16 * st;
            const int s = tile * TS + r0 + r16;
            f32x4 z[2];
            z[0] = z[1] = f32x4{0.f, 0.f, 0.f, 0.f};
            const bf16x8 b0 = rd_row<TS>(imgH2, lo, r0, 0), b1 = rd_row<TS>(imgH2, lo, r0, 32);
            z[0] = mfma(w2f[0][0], b0, z[0]);
            z[0] = mfma(w2f[0][1], b1, z[0]);
            if (n_ot > 1) {
                z[1] = mfma(w2f[1][0], b0, z[1]);
                z[1] = mfma(w2f[1][1], b1, z[1]);
                output_layer<TYPE, LABELS, TS, 2>(z, lab[st], T, ldt, t_hi, t_lo, s, s < n_valid, n_out, imgD3, lo,
                                                  r0, lane, inv_nout, my_loss, my_hit);
            } else {
                output_layer<TYPE, LABELS, TS, 1>(z, lab[st], T, ldt, t_hi, t_lo, s, s < n_valid, n_out, imgD3, lo,
                                                  r0, lane, inv_nout, my_loss, my_hit);
            }
        }
        mark(6);
        wave_lds_fence();
        /* P3: delta2^T [h2][sample] = (W2^T delta3^T) * f'(H2) */
#pragma unroll
        for (int st = 0; st < STC; st++) {
            const int r0 = sw + 16 * st;
            const bf16x8 b = rd_row<TS>(imgD3, lo, r0, 0);
#pragma unroll
            for (int ht = 0; ht < 4; ht++) {
                const f32x4 a = mfma(w2tf[ht], b, f32x4{0.f, 0.f, 0.f, 0.f});
                const bf16x4 h = ld_d4<TS, TRADE>(imgH2, lo, r0, 16 * ht, lane);
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)(a[r] * dbipolar((float)h[r]));
                st_d4<TS, TRADE>(imgD2, lo, r0, 16 * ht, o, lane);
            }
        }
        mark(7);
        /* CB: phase C's barrier (every wave's delta2 in the D2 image) already here, so each wave
         * runs P4 and phase C back to back (neither writes LDS) instead of waiting for the
         * slowest wave's P4 */
        if constexpr (CB) lds_barrier();
        else wave_lds_fence();
        /* P4: delta1 [sample][h1] = (delta2 W1) * f'(H1) -> HBM, fragment-major:
         * chunk (32-sample row, h1 block) = [g][r][j] = delta1[32 t + 8 g + j][16 hb + r] */
        {
            __bf16 *chunk0 = D1 + (size_t)(T0 + (sw >> 5)) * (H1 / 16) * 512;
            const int gb = 2 * ((sw >> 4) & 1);
            bf16x8 d0[STC], d1[STC];
#pragma unroll
            for (int st = 0; st < STC; st++) {
                d0[st] = rd_row<TS>(imgD2, lo, sw + 16 * st, 0);
                d1[st] = rd_row<TS>(imgD2, lo, sw + 16 * st, 32);
            }
            /* each W1^T fragment read once, for all STC sample tiles */
#pragma unroll
            for (int ht = 0; ht < 8; ht++) {
                const bf16x8 w0 = rd_tr<H2>(imgW1, lo, 0, 16 * ht), w1 = rd_tr<H2>(imgW1, lo, 32, 16 * ht);
#pragma unroll
                for (int st = 0; st < STC; st++) {
                    const int r0 = sw + 16 * st;
                    f32x4 a = mfma(d0[st], w0, f32x4{0.f, 0.f, 0.f, 0.f});
                    a = mfma(d1[st], w1, a);
                    /* D[row = sample r0 + 4q + r][col = h1 16 ht + r16]; f'(H1) of those 4 samples */
                    const s16x4 hr = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s16x4 *)(imgH1 + t32<TS>(r0 + 4 * q + (r16 >> 2), 16 * ht + 4 * (r16 & 3))));
                    const bf16x4 hv = __builtin_bit_cast(bf16x4, hr);
                    bf16x4 o;
#pragma unroll
                    for (int r = 0; r < 4; r++) o[r] = (__bf16)(a[r] * dbipolar((float)hv[r]));
                    const int g = gb + 2 * st + (q >> 1);
                    *(bf16x4 *)(chunk0 + (size_t)ht * 512 + (g * 16 + r16) * 8 + 4 * (q & 1)) = o;
                }
            }
        }
        mark(8);
        if constexpr (!CB) lds_barrier();

        /* ================= phase C: G1, G2 over the tile's 256 samples ================= */
        /* [G1 (H2 x H1) | G2 (NO x H2)] slab.  G1: wave w owns the 2 x 2 output tiles h1 tiles
         * ha + i x h2 tiles hb + j, D[h1 = 16 (ha + i) + 4q + r][h2 = 16 (hb + j) + r16]; every
         * operand of the 8 k-steps is read first (64 transposed reads in flight: the chain's
         * registers are free here), then the 32 MFMAs.  G2: wave w < 8 owns h2 tile w&3 x o
         * tile w>>2, D[h2 = 16 (w&3) + 4q + r][o = 16 (w>>2) + r16]. */
        const bool first = tile == (int)blockIdx.x;
        {
            const int ha = 2 * (wave & 3), hb = 2 * (wave >> 2);
            bf16x8 fa[TS / 32][2], fb[TS / 32][2];
#pragma unroll
            for (int k = 0; k < TS / 32; k++)
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    fa[k][i] = rd_tr<TS>(imgH1, lo, 32 * k, 16 * (ha + i)); /* A[h1][sample] */
                    fb[k][i] = rd_tr<TS>(imgD2, lo, 32 * k, 16 * (hb + i)); /* B[sample][h2] */
                }
            f32x4 g[2][2];
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    const float *p = slab + (size_t)((hb + j) * 16 + r16) * H1 + (ha + i) * 16 + 4 * q;
                    g[i][j] = first ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4 *)p;
                }
#pragma unroll
            for (int k = 0; k < TS / 32; k++)
#pragma unroll
                for (int i = 0; i < 2; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) g[i][j] = mfma(fa[k][i], fb[k][j], g[i][j]);
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
                    *(f32x4 *)(slab + (size_t)((hb + j) * 16 + r16) * H1 + (ha + i) * 16 + 4 * q) = g[i][j];
        }
        {
            float *const g2p = slab + H2 * H1 + (size_t)((wave >> 2) * 16 + r16) * H2 + (wave & 3) * 16 + 4 * q;
            f32x4 g2acc = first ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4 *)g2p;
            if ((wave >> 2) < n_ot) {
                bf16x8 fa[TS / 32], fb[TS / 32];
#pragma unroll
                for (int k = 0; k < TS / 32; k++) {
                    fa[k] = rd_tr<TS>(imgH2, lo, 32 * k, 16 * (wave & 3));
                    fb[k] = rd_tr<TS>(imgD3, lo, 32 * k, 16 * (wave >> 2));
                }
#pragma unroll
                for (int k = 0; k < TS / 32; k++) g2acc = mfma(fa[k], fb[k], g2acc);
            }
            *(f32x4 *)g2p = g2acc;
        }
    }

    mark(9);
    lds_barrier();
    float *sl = (float *)(lds + OFF_D3);
    unsigned int *shh = (unsigned int *)(lds + OFF_D3 + 64);
    my_loss = wave_sum(my_loss);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) my_hit += __shfl_xor(my_hit, o, 64);
    if (lane == 0) {
        sl[wave] = my_loss;
        shh[wave] = my_hit;
    }
    __syncthreads();
    if (tid == 0) {
        float a = 0.f;
        unsigned int h = 0;
        for (int w = 0; w < NW; w++) {
            a += sl[w];
            h += shh[w];
        }
        if (loss_acc) atomicAdd(loss_acc + HPNN_STAT_SLOT(blockIdx.x), a);
        if (correct) atomicAdd(correct + HPNN_STAT_SLOT(blockIdx.x), h);
    }
    mark(10);
}

int g_tile_cus = 0;
#ifdef HPNN_ABLATIONS
/* HPNN_TILE_ABL (make ABLATIONS=1 builds only; profiling, wrong results): 1 = no W0 loads,
 * 2 = no X loads, 7 = neither (a register pattern instead), 3 = no phase-A MFMAs, 4 = no
 * phase-A B reads, 5 = no X^T conversion, 6 = no per-k-step barrier, 8 = 4 + 5 + 6, 9 = 4 + 5 */
const int g_tile_abl = [] { const char *e = getenv("HPNN_TILE_ABL"); return e ? atoi(e) : 0; }();
#endif

template <int TYPE, bool LABELS, int KS, bool XU8>
int launch_tile(const void *Xg, float xscale, const void *W0f, const void *W1, const void *W2, const void *W2t,
                const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1, float *gslab,
                float *loss_acc, unsigned int *correct, int n_tiles, int n_valid, int n_out, int grid,
                hipStream_t stream) {
    static const bool trace = [] { const char *e = getenv("HPNN_TILE_TRACE"); return e && e[0] == '1'; }();
    auto go = [&](auto kern, int threads) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL);
            attr = true;
        }
        hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), LDS_TOTAL, stream, Xg, xscale, (const __bf16 *)W0f,
                           (const __bf16 *)W1, (const __bf16 *)W2, (const __bf16 *)W2t, labels, T, ldt, t_hi, t_lo,
                           (__bf16 *)D1, gslab, loss_acc, correct, n_tiles, n_valid, n_out);
        return hipGetLastError() == hipSuccess ? grid : -5;
    };
    /* D = 3 k-steps of loads in flight: 58.7-59.4 us per MNIST step vs 59.6-60.4 at D = 4 and
     * 59.8-60.3 at D = 2 (B reads one k-step ahead; a deeper ring costs the registers the B
     * prefetch needs), profiles/r3/SUMMARY.md; re-measured on the round-4 front (253 VGPRs):
     * D = 2 62.4 / 62.1, D = 4 (spills) 63.0 / 63.3 vs 62.1 us (profiles/r4/dd_tile_d.txt) */
    if constexpr (TYPE == 2 && LABELS && KS == 25 && XU8) {
#ifdef HPNN_ABLATIONS
        /* A/B variants that measured slower (make ABLATIONS=1 builds only):
         * HPNN_TILE_IL=0: the round-4 k-step schedule (conversion, B reads, then the 16 MFMAs as
         *   one block): phase A 26.0K vs 24.0K ticks, 58.9 / 59.0 vs 58.6 / 58.3 us per step
         *   (profiles/r5/SUMMARY.md);
         * HPNN_TILE_EARLY=0: X(s + 2) converted after the MFMAs of step s (equal within noise);
         * HPNN_TILE_TRADE=1: the chain's 8-byte image stores / loads with a lane-pair trade of
         *   halves -- LDS bank conflicts 18.5 % -> 5.6 %, but 60.6 / 61.4 / 62.5 vs 59.9 / 59.8 /
         *   60.0 us per step (profiles/r4/tr_tile_trade_ab.txt);
         * HPNN_TILE_XORD=1: X^T stage writes in a per-lane-pair order (conflicts 60 % -> 18.5 %):
         *   61.5 / 61.5 / 62.0 vs 60.7 / 60.3 / 61.3 us (profiles/r4/xo_tile_xord_ab.txt);
         * HPNN_TILE_ABL=n: phase-A ablations (wrong results), traced with HPNN_TILE_TRACE=1
         *   (profiles/r5/a_tile_phaseA_ablations.txt) */
        static const bool late = [] { const char *e = getenv("HPNN_TILE_EARLY"); return e && e[0] == '0'; }();
        static const bool trade = [] { const char *e = getenv("HPNN_TILE_TRADE"); return e && e[0] == '1'; }();
        static const bool xord = [] { const char *e = getenv("HPNN_TILE_XORD"); return e && e[0] == '1'; }();
        static const bool il0 = [] { const char *e = getenv("HPNN_TILE_IL"); return e && e[0] == '0'; }();
        if (il0) return trace ? go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, true, 0, true, false, false, 0>, 512)
                              : go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, false, 0, true, false, false, 0>, 512);
        if (late) return go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, false, 0, false>, 512);
        if (trade) return go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, false, 0, true, true>, 512);
        if (xord) return go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, false, 0, true, false, true>, 512);
        static const bool cb = [] { const char *e = getenv("HPNN_TILE_CB"); return e && e[0] == '1'; }();
        if (cb) return trace ? go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, true, 0, true, false, false, 1, true>, 512)
                             : go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, false, 0, true, false, false, 1, true>, 512);
#define HPNN_TABL(N_)                                                                                               \
        if (g_tile_abl == N_) return trace ? go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, true, N_>, 512)          \
                                           : go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, false, N_>, 512);
        HPNN_TABL(1) HPNN_TABL(2) HPNN_TABL(3) HPNN_TABL(4) HPNN_TABL(5) HPNN_TABL(6) HPNN_TABL(7) HPNN_TABL(8)
        HPNN_TABL(9)
#undef HPNN_TABL
#endif
        if (trace) return go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3, true>, 512);
    }
    return go(mlp3_tile_kernel<TYPE, LABELS, KS, XU8, 3>, 512);
}

template <int KS>
int launch_tile_k(const void *Xg, int xu8, float xscale, const void *W0f, const void *W1, const void *W2,
                  const void *W2t, const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1,
                  float *gslab, float *loss_acc, unsigned int *correct, int n_tiles, int n_valid, int n_out, int type,
                  int grid, hipStream_t stream) {
#define HPNN_TL(TY, LB, U8)                                                                                     \
    return launch_tile<TY, LB, KS, U8>(Xg, xscale, W0f, W1, W2, W2t, labels, T, ldt, t_hi, t_lo, D1, gslab,     \
                                       loss_acc, correct, n_tiles, n_valid, n_out, grid, stream)
#define HPNN_TL2(TY, LB)       \
    if (xu8) HPNN_TL(TY, LB, true); \
    HPNN_TL(TY, LB, false)
    if (labels) {
        if (type == 2) { HPNN_TL2(2, true); }
        if (type == 0) { HPNN_TL2(0, true); }
        HPNN_TL2(1, true);
    }
    if (type == 2) { HPNN_TL2(2, false); }
    if (type == 0) { HPNN_TL2(0, false); }
    HPNN_TL2(1, false);
#undef HPNN_TL2
#undef HPNN_TL
}

}  // namespace

extern "C" int hpnn_mlp3_tile_grid(int Bp, int grid) {
    if (Bp <= 0 || Bp % TS) return -2;
    if (g_tile_cus <= 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_tile_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            g_tile_cus = 256;
    }
    const int n_tiles = Bp / TS;
    if (grid <= 0) grid = g_tile_cus;
    return grid < n_tiles ? grid : n_tiles;
}

extern "C" int hpnn_mlp3_tile(const void *Xg, int xu8, float xscale, int K0, const void *W0f, const void *W1,
                              const void *W2, const void *W2t, const int *labels, const float *T, int ldt,
                              float t_hi, float t_lo, void *D1, float *gslab, float *loss_acc,
                              unsigned int *correct, int Bp, int n_valid, int n_out, int type, int grid,
                              hipStream_t stream) {
    if (Bp <= 0 || Bp % TS || n_out > NO || n_out < 1) return -2;
    if (!labels && !T) return -1;
    if (((uintptr_t)Xg | (uintptr_t)W0f | (uintptr_t)W1 | (uintptr_t)W2 | (uintptr_t)W2t | (uintptr_t)D1 |
         (uintptr_t)gslab) & 15)
        return -4;
    grid = hpnn_mlp3_tile_grid(Bp, grid);
    if (grid <= 0) return -2;
    const int n_tiles = Bp / TS;
#define HPNN_TK(K_)                                                                                              \
    if (K0 == K_)                                                                                                \
    return launch_tile_k<K_ / 32>(Xg, xu8, xscale, W0f, W1, W2, W2t, labels, T, ldt, t_hi, t_lo, D1, gslab,     \
                                  loss_acc, correct, n_tiles, n_valid, n_out, type, grid, stream)
    HPNN_TK(800);
    HPNN_TK(256);
#undef HPNN_TK
    return -3;
}

/* HPNN_TILE_TRACE=1 stamps: out[TR_BLOCKS][TR_MARKS] shader-clock ticks (wave 0 of each
 * workgroup; s_memtime counts per XCD, so only intervals within a workgroup compare) */
extern "C" int hpnn_mlp3_tile_trace(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tile_trace), sizeof(g_tile_trace)) == hipSuccess ? 0 : -5;
}
