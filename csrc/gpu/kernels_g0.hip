/*
 * Weight-gradient GEMM over fragment-major operands, direct-to-register loads (gfx950).
 *
 *   slab[s][n][m] = sum over the batch rows b of split s of  D[b][n] * H[b][m]
 *
 * (the product of hpnn_gemm_tn_bf16) with both operands stored FRAGMENT-MAJOR:
 * A[b][c] -> [b / 32][c / 16][64 lanes][8], lane l = 16 g + r of fragment (t, cb) holding
 * A[32 t + 8 g + j][16 cb + r], j < 8 -- exactly the per-lane operand of
 * v_mfma_f32_16x16x32_bf16 with k running over the batch (A[row = l&15][k = 8(l>>4)+j]).
 * Every operand fragment is then one contiguous 1 KiB wave load straight into VGPRs; no
 * LDS, no transposes.  Reference: the per-sample weight update of ann_kernel_train /
 * snn_kernel_train (ann.c:1279-1592, cuda_ann.cu ger_acc), batched.
 *
 * Used for MNIST's first-layer gradient G0 = delta1^T X (800 x 128 over 65536 rows): the
 * fused front (kernels_mlp3x.hip, d1fm) writes delta1 in this layout, and an 8-bit pixel
 * batch keeps a fragment-major copy of its bytes, made once when it is prepared
 * (MLP.prepare_input): half the bytes of the BF16 batch, converted in registers to the
 * same bf16(pixel * scale) values the front computes with (8 waves hide the conversion).
 * In the step: 72.5-72.7 us with it vs 74.8-75.6 us for the LDS-DMA TN kernel on the
 * BF16 batch; cold 26.5 us vs 34 standalone (round-2 A/B scripts, since pruned).
 * Measured (48 splits): LDS-staged TN kernel 31.2 us (its LDS-DMA
 * fill, ~27 GB/s per CU, is the bound); this kernel 23.8 us, ~5.1 TB/s of HBM reads --
 * it streams at the memory rate.  Rejected on the way: the same kernel on plain
 * batch-contiguous (transposed row-major) operands, 51 us -- each wave load then hits
 * 16 rows x 64 B, 64 L1 tag lookups per instruction instead of 8, and the vector L1 tag
 * rate (~1 lookup per clock per CU, TCP_TOTAL_CACHE_ACCESSES) is the limit; grouping 2-4
 * k-steps per row visit or padding the row pitch did not change that.
 *
 * Workgroup: 4 x KW waves.  Waves (wm, wn) in 2 x 2 cover a 32 WF x 32 WH output tile
 * (wave tile 16 WF x 16 WH); with KW = 2 a second group of 4 waves takes every other
 * 32-row k-step and the two partial tiles meet in LDS at the end (fixed order).  Each
 * wave keeps PD k-steps of operands in flight in a register ring (PD + 1 slots; the loop
 * is unrolled by PD + 1 so every slot index is static).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"
#include "mfma_common.h"

namespace {

using hpnn::bf16x8;
using hpnn::f32x4;
using hpnn::TnTail;

/* Dg: [Bt/32][N/16][64][8], Hg: [Bt/32][M/16][64][8]; nbd = N / 16, nbh = M / 16.
 * HU8: Hg holds unsigned bytes (8 per lane per fragment), multiplied as exact integers;
 * hscale scales the FP32 result (G = hscale * D^T H) */
template <int WF, int WH, int PD, int KW, bool HU8 = false>
__global__ __launch_bounds__(256 * KW) void gemm_fm_direct_kernel(const __bf16 *__restrict__ Dg, int nbd,
                                                                  const void *__restrict__ Hg, int nbh, float hscale,
                                                                  float *__restrict__ slab, int ldg, int N, int ksteps,
                                                                  int splits, int tiles_n, int tiles, int xcd_map,
                                                                  TnTail tail) {
    if ((int)blockIdx.x >= tiles * splits) {
        if (threadIdx.x < 256) hpnn::tn_tail_reduce(tail, (int)blockIdx.x - tiles * splits);
        return;
    }
    constexpr int R = PD + 1;
    constexpr int TMF = 32 * WF, TNH = 32 * WH; /* workgroup tile: features x delta columns */
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kg = wave >> 2, wm = (wave >> 1) & 1, wn = wave & 1;
    int tile, split;
    if (xcd_map) { /* the tiles of one batch slice on one XCD: its Dt slice is fetched once into that L2 */
        const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
        tile = j % tiles;
        split = xcd + 8 * (j / tiles);
    } else {
        tile = blockIdx.x % tiles;
        split = blockIdx.x / tiles;
    }
    const int m0 = (tile / tiles_n) * TMF + wm * 16 * WF, n0 = (tile % tiles_n) * TNH + wn * 16 * WH;
    const int k0 = (int)((long)split * ksteps / splits), k1 = (int)((long)(split + 1) * ksteps / splits);
    /* this wave group's k-steps: k0 + kg, k0 + kg + KW, ... */
    const int nk = (k1 - k0 - kg + KW - 1) / KW;
    const int r16 = lane & 15;
    constexpr int ES = HU8 ? 1 : 2; /* bytes per H element */
    using HT = typename std::conditional<HU8, uint2, bf16x8>::type;
    const char *pa = (const char *)Hg + (((size_t)(k0 + kg) * nbh + m0 / 16) * 512 + lane * 8) * ES;
    const __bf16 *pb = Dg + ((size_t)(k0 + kg) * nbd + n0 / 16) * 512 + lane * 8;
    const size_t step_a = (size_t)KW * nbh * 512 * ES, step_b = (size_t)KW * nbd * 512; /* this group's next k-step */

    f32x4 acc[WF][WH];
#pragma unroll
    for (int i = 0; i < WF; i++)
#pragma unroll
        for (int j = 0; j < WH; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    HT ra[R][WF];
    bf16x8 rb[R][WH];
    auto load = [&](int slot_, int t) __attribute__((always_inline)) {
        const int tc = t < nk - 1 ? t : nk - 1; /* clamped: the ring tail re-reads the last step */
#pragma unroll
        for (int i = 0; i < WF; i++) ra[slot_][i] = *(const HT *)(pa + i * 512 * ES + (size_t)tc * step_a);
#pragma unroll
        for (int j = 0; j < WH; j++) rb[slot_][j] = *(const bf16x8 *)(pb + j * 512 + (size_t)tc * step_b);
    };
    auto mma = [&](int slot_) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < WF; i++) {
            bf16x8 a;
            if constexpr (HU8) a = hpnn::u8x8_int_bf16(ra[slot_][i].x, ra[slot_][i].y);
            else a = ra[slot_][i];
#pragma unroll
            for (int j = 0; j < WH; j++)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, rb[slot_][j], acc[i][j], 0, 0, 0);
        }
    };
    if (nk > 0) {
#pragma unroll
        for (int p = 0; p < PD; p++) load(p, p);
        int t = 0;
        for (; t + R <= nk; t += R) {
#pragma unroll
            for (int u = 0; u < R; u++) {
                /* program order = issue order: the loads of step t+u+PD go out before the
                 * MFMAs of step t+u, so waiting for step t+u leaves PD steps in flight
                 * (without the barriers the scheduler sinks loads below MFMAs and the
                 * waitcnt pass drains the ring to vmcnt(0) every step) */
                load((u + PD) % R, t + u + PD);
                __builtin_amdgcn_sched_barrier(0);
                mma(u);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        /* remaining nk - t < R steps sit in slots 0.. already (PD = R - 1 loads ahead) */
#pragma unroll
        for (int u = 0; u < R - 1; u++)
            if (t + u < nk) mma(u);
    }

    float *out = slab + (size_t)split * N * ldg;
    const int q = lane >> 4;
    if constexpr (KW > 1) { /* groups 1.. hand their partial tiles to group 0 through LDS, in order */
        __shared__ f32x4 part[4][WF * WH][64];
#pragma unroll
        for (int g = 1; g < KW; g++) {
            if (kg == g) {
#pragma unroll
                for (int i = 0; i < WF; i++)
#pragma unroll
                    for (int j = 0; j < WH; j++) part[wave & 3][i * WH + j][lane] = acc[i][j];
            }
            __syncthreads();
            if (kg == 0) {
#pragma unroll
                for (int i = 0; i < WF; i++)
#pragma unroll
                    for (int j = 0; j < WH; j++) acc[i][j] += part[wave & 3][i * WH + j][lane];
            }
            if (g + 1 < KW) __syncthreads();
        }
        if (kg != 0) return;
    }
#pragma unroll
    for (int i = 0; i < WF; i++)
#pragma unroll
        for (int j = 0; j < WH; j++)
            *(f32x4 *)(out + (size_t)(n0 + j * 16 + r16) * ldg + m0 + i * 16 + 4 * q) =
                HU8 ? acc[i][j] * hscale : acc[i][j];
}

template <int WF, int WH, int PD, int KW, bool HU8 = false>
int launch_fm(const void *Dg, const void *Hg, float hscale, float *slab, int ldg, int N, int M, int Bt, int splits,
              hipStream_t s, const TnTail &tail) {
    constexpr int TMF = 32 * WF, TNH = 32 * WH;
    const int tiles_n = N / TNH, tiles = (M / TMF) * tiles_n;
    const int xcd_map = (splits % 8 == 0 && tiles > 1) ? 1 : 0;
    hipLaunchKernelGGL((gemm_fm_direct_kernel<WF, WH, PD, KW, HU8>), dim3(tiles * splits + tail.blocks),
                       dim3(256 * KW), 0, s, (const __bf16 *)Dg, N / 16, Hg, M / 16, hscale, slab, ldg, N, Bt / 32,
                       splits, tiles_n, tiles, xcd_map, tail);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int fm_dispatch(const void *Dg, const void *Hg, int h_u8, float hscale, float *slab, int ldg, int N, int M, int Bt,
                int splits, hipStream_t s, const TnTail &t) {
    if (N <= 0 || M <= 0 || Bt <= 0 || splits <= 0) return -1;
    if (Bt % 32 || splits > Bt / 32 || M % 32 || N % 32) return -2;
    if (ldg % 4 || ldg < M) return -3;
    /* 160 x 128 tiles: measured alternatives (3 k-steps in flight; 8 waves as two k-interleaved
     * groups with 2 / 1 in flight) were no faster: 23.8 / 25.1 / 24.3 us vs 23.8 us */
#define HPNN_FM(...)                                                                                              \
    return h_u8 ? launch_fm<__VA_ARGS__, true>(Dg, Hg, hscale, slab, ldg, N, M, Bt, splits, s, t)                  \
                : launch_fm<__VA_ARGS__, false>(Dg, Hg, hscale, slab, ldg, N, M, Bt, splits, s, t)
    if (M % 160 == 0 && N % 128 == 0) {
        /* 8-bit H: 8 waves (two k-interleaved groups) hide the byte -> bf16 conversion
         * (23.0 / 26.5 us hot / cold vs 27.0 / 27.2 with 4 waves); bf16 H: 4 waves.
         * Round 3, in the MNIST step (tile front): 59.8-59.9 us per step with this one vs
         * 60.0 with 2 k-steps in flight, 62.3 / 61.4 with 4 waves and 2 / 3 in flight. */
        /* session 7: three k-interleaved groups (12 waves, 3 a SIMD) 24.9 vs 23.4 us in the
         * step, 58.9-59.3 vs 56.2-58.5 us per step (profiles/r3/s7_g0_kw_ab.txt) */
        if (h_u8) { HPNN_FM(5, 4, 1, 2); }
        HPNN_FM(5, 4, 2, 1);
    }
    if (M % 64 == 0 && N % 64 == 0) { HPNN_FM(2, 2, 2, 1); }
    HPNN_FM(1, 1, 3, 1);
#undef HPNN_FM
}

}  // namespace

extern "C" int hpnn_gemm_fm_direct(const void *Dg, const void *Hg, int h_u8, float hscale, float *slab, int ldg, int N,
                                   int M, int Bt, int splits, hipStream_t stream) {
    const TnTail none = {nullptr, nullptr, 0, 0, 0, 0, 1, 1, 0};
    return fm_dispatch(Dg, Hg, h_u8, hscale, slab, ldg, N, M, Bt, splits, stream, none);
}

extern "C" int hpnn_gemm_fm_direct_reduce(const void *Dg, const void *Hg, int h_u8, float hscale, float *slab,
                                          int ldg, int N, int M, int Bt, int splits, const float *rslab, int rS,
                                          long rstride, long rn, int rgroups, float *rout, hipStream_t stream) {
    if (rn % 4 || rstride % 4 || rS < 1 || rgroups < 1 || rgroups > rS || !rslab || !rout) return -2;
    const long n4 = rn / 4;
    const int bx = (int)((n4 + 255) / 256);
    const TnTail t = {rslab, rout, rstride, n4, rn, rS, (rS + rgroups - 1) / rgroups, bx, bx * rgroups};
    return fm_dispatch(Dg, Hg, h_u8, hscale, slab, ldg, N, M, Bt, splits, stream, t);
}
