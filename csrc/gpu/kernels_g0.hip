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
 * BF16 batch (scripts/gpu_ab_input.sh); cold 26.5 us vs 34 in scripts/g0_direct.py.
 * Measured (scripts/g0_direct.py, 48 splits): LDS-staged TN kernel 31.2 us (its LDS-DMA
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

/* 8 unsigned bytes -> bf16x8 of (byte * scale) (exact for pixel values with scale 1) */
__device__ __forceinline__ bf16x8 u8x8_bf16(uint2 v, float scale) {
    bf16x8 r;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        r[e] = (__bf16)((float)((v.x >> (8 * e)) & 0xffu) * scale);
        r[4 + e] = (__bf16)((float)((v.y >> (8 * e)) & 0xffu) * scale);
    }
    return r;
}

/* Dg: [Bt/32][N/16][64][8], Hg: [Bt/32][M/16][64][8]; nbd = N / 16, nbh = M / 16.
 * HU8: Hg holds unsigned bytes (8 per lane per fragment), used as bf16(h * hscale) */
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
            if constexpr (HU8) a = u8x8_bf16(ra[slot_][i], hscale);
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
    if constexpr (KW == 2) { /* group 1 hands its partial tile to group 0 through LDS */
        __shared__ f32x4 part[4][WF * WH][64];
        if (kg == 1) {
#pragma unroll
            for (int i = 0; i < WF; i++)
#pragma unroll
                for (int j = 0; j < WH; j++) part[wave & 3][i * WH + j][lane] = acc[i][j];
        }
        __syncthreads();
        if (kg == 1) return;
#pragma unroll
        for (int i = 0; i < WF; i++)
#pragma unroll
            for (int j = 0; j < WH; j++) acc[i][j] += part[wave & 3][i * WH + j][lane];
    }
#pragma unroll
    for (int i = 0; i < WF; i++)
#pragma unroll
        for (int j = 0; j < WH; j++)
            *(f32x4 *)(out + (size_t)(n0 + j * 16 + r16) * ldg + m0 + i * 16 + 4 * q) = acc[i][j];
}

/* ---------------------------------------------------------------------------------- */
/* Register-staged TN GEMM: row-major operands (D [Bt x ldd], H [Bt x ldh], the layout of */
/* hpnn_gemm_tn_bf16), each 32-row k-step fetched with coalesced 16-byte vector loads      */
/* into VGPRs P steps ahead, written into a T32 LDS image (3 buffers, one barrier per      */
/* step), MFMA operands by transposed LDS reads.  Same math and output as the LDS-DMA      */
/* pipe kernel (kernels_mfma.hip), without its per-CU LDS-DMA fill limit.                  */
/* ---------------------------------------------------------------------------------- */
/* HU8: H holds 8-bit unsigned values (ldh in bytes), converted while staging:
 * bf16(h * hscale) -- exact for pixel data (integers 0..255, hscale 1) */
template <int TM, int TN, int P, bool HU8 = false>
__global__ __launch_bounds__(256) void gemm_tn_rs_kernel(const __bf16 *__restrict__ D, int ldd,
                                                         const void *__restrict__ H, int ldh, float hscale,
                                                         float *__restrict__ slab, int ldg, int N, int units,
                                                         int splits, int tiles_n, int tiles, int xcd_map, TnTail tail) {
    if ((int)blockIdx.x >= tiles * splits) {
        hpnn::tn_tail_reduce(tail, (int)blockIdx.x - tiles * splits);
        return;
    }
    constexpr int WTM = TM / 2, WTN = TN / 2, FM = WTM / 16, FN = WTN / 16;
    constexpr int XE = HU8 ? 16 : 8; /* H elements per 16-byte chunk */
    constexpr int XC = TM / XE, DC = TN / 8, NX = 32 * XC, ND = 32 * DC; /* 16-byte chunks per step */
    constexpr int LX = (NX + 255) / 256, LD = (ND + 255) / 256;
    /* T32 images with sub-tiles padded by 64 bytes: the 16 lanes of one ds_write_b128 cycle
     * (4 chunks of a row in each of 4 consecutive sub-tiles) then hit 16 different
     * 4-bank groups -- unpadded, sub-tiles 2 KiB apart share banks (SQ_LDS_BANK_CONFLICT
     * 1.4M cycles vs 1.8M LDS-active) */
    constexpr int SP = 64;
    constexpr int HB = (TM / 32) * (32 * 64 + SP), STG = HB + (TN / 32) * (32 * 64 + SP);
    __shared__ __attribute__((aligned(16))) char lds[3 * STG];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
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
    const int u0 = (int)((long)split * units / splits), u1 = (int)((long)(split + 1) * units / splits);
    const int KT = (u1 - u0) * 2; /* 32-row steps */
    const size_t ldh_b = (size_t)ldh * (HU8 ? 1 : 2), ldd_b = (size_t)ldd * 2;
    const char *Hg = (const char *)H + (size_t)u0 * 64 * ldh_b + (size_t)m0 * (HU8 ? 1 : 2);
    const char *Dg = (const char *)(D + (size_t)u0 * 64 * ldd + n0);

    /* chunks past the tile (c >= NX / ND) repeat the last one: same bytes to the same LDS
     * slot as its owner -- no predicates, so the waitcnt pass sees straight-line code */
    unsigned int xo[LX], xd[LX], xd2[LX], dO[LD], dd[LD];
#pragma unroll
    for (int i = 0; i < LX; i++) {
        const int c = tid + 256 * i, cc = c < NX ? c : NX - 1;
        const int row = cc / XC, cx = cc % XC;
        xo[i] = (unsigned int)(row * ldh_b + cx * 16);
        xd[i] = (unsigned int)hpnn::t32<32, SP>(row, cx * XE);
        xd2[i] = (unsigned int)hpnn::t32<32, SP>(row, cx * XE + 8); /* HU8: columns + 8 .. 15 */
    }
#pragma unroll
    for (int i = 0; i < LD; i++) {
        const int c = tid + 256 * i, cc = c < ND ? c : ND - 1;
        const int row = cc / DC, c8 = cc % DC;
        dO[i] = (unsigned int)(row * ldd_b + c8 * 16);
        dd[i] = (unsigned int)(HB + hpnn::t32<32, SP>(row, c8 * 8));
    }
    bf16x8 rx[P][LX], rd[P][LD];
    auto load = [&](int slot_, int kt) __attribute__((always_inline)) {
        const int kc = kt < KT ? kt : KT - 1; /* past the end: re-read the last step, never stored */
        const char *hb = Hg + (size_t)kc * 32 * ldh_b, *db = Dg + (size_t)kc * 32 * ldd_b;
#pragma unroll
        for (int i = 0; i < LX; i++)
            rx[slot_][i] = *(const bf16x8 *)(hb + xo[i]);
#pragma unroll
        for (int i = 0; i < LD; i++)
            rd[slot_][i] = *(const bf16x8 *)(db + dO[i]);
    };
    auto store = [&](int slot_, int buf) __attribute__((always_inline)) {
        char *b = lds + buf * STG;
#pragma unroll
        for (int i = 0; i < LX; i++) {
            if constexpr (HU8) {
                const uint4 v = __builtin_bit_cast(uint4, rx[slot_][i]);
                const unsigned int w[4] = {v.x, v.y, v.z, v.w};
                bf16x8 lo8, hi8;
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    lo8[e] = (__bf16)((float)((w[e >> 2] >> (8 * (e & 3))) & 0xffu) * hscale);
                    hi8[e] = (__bf16)((float)((w[2 + (e >> 2)] >> (8 * (e & 3))) & 0xffu) * hscale);
                }
                /* columns cx*16 + 0..7 and + 8..15: two 16-byte slots of the T32 image */
                *(bf16x8 *)(b + xd[i]) = lo8;
                *(bf16x8 *)(b + xd2[i]) = hi8;
            } else {
                *(bf16x8 *)(b + xd[i]) = rx[slot_][i];
            }
        }
#pragma unroll
        for (int i = 0; i < LD; i++)
            *(bf16x8 *)(b + dd[i]) = rd[slot_][i];
    };
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    /* MFMA operands double-buffered in registers: the transposed LDS reads of step t+1
     * are issued right after the barrier and run under the MFMAs of step t */
    bf16x8 fh[2][FM], fd[2][FN];
    auto read = [&](int set, int buf) __attribute__((always_inline)) {
        const char *sh = lds + buf * STG, *sd = sh + HB;
#pragma unroll
        for (int i = 0; i < FM; i++) fh[set][i] = hpnn::frag_tr<32, SP>(sh, 0, wm * WTM + i * 16, lane);
#pragma unroll
        for (int j = 0; j < FN; j++) fd[set][j] = hpnn::frag_tr<32, SP>(sd, 0, wn * WTN + j * 16, lane);
    };
    auto mma = [&](int set) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int j = 0; j < FN; j++)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[set][i], fd[set][j], acc[i][j], 0, 0, 0);
    };
    static_assert(P % 3 == 0, "the loop is unrolled by 6: P register slots, 3 LDS buffers, 2 fragment sets");
    constexpr int UN = (P % 2 == 0) ? P : 2 * P; /* lcm(P, 3, 2) for P in {3, 6, 9} */
    if (KT > 0) {
        /* step s lives in register slot s % P, LDS buffer s % 3, fragment set s % 2 */
#pragma unroll
        for (int sl = 0; sl < P; sl++) load(sl, sl);
        __builtin_amdgcn_sched_barrier(0);
        store(0, 0);
        __builtin_amdgcn_sched_barrier(0);
        load(0, P);
        __builtin_amdgcn_sched_barrier(0);
        store(1 % P, 1);
        __builtin_amdgcn_sched_barrier(0);
        load(1 % P, P + 1);
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
        read(0, 0);
        for (int t = 0; t < KT; t += UN) {
#pragma unroll
            for (int u = 0; u < UN; u++) {
                /* iteration t+u: stage step t+u+2 (slot -> buffer), refill its slot with step
                 * t+u+2+P, one barrier, read step t+u+1, MFMAs of step t+u */
                __builtin_amdgcn_sched_barrier(0);
                store((u + 2) % P, (u + 2) % 3);
                __builtin_amdgcn_sched_barrier(0);
                load((u + 2) % P, t + u + 2 + P);
                __builtin_amdgcn_sched_barrier(0);
                __syncthreads();
                if (t + u + 1 < KT) read((u + 1) % 2, (u + 1) % 3);
                if (t + u < KT) mma(u % 2);
            }
        }
    }
    float *out = slab + (size_t)split * N * ldg;
    const int r16 = lane & 15, q = lane >> 4;
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++)
            *(f32x4 *)(out + (size_t)(n0 + wn * WTN + j * 16 + r16) * ldg + m0 + wm * WTM + i * 16 + 4 * q) = acc[i][j];
}

template <int TM, int TN, int P = 3, bool HU8 = false>
int launch_rs(const void *D, int ldd, const void *H, int ldh, float hscale, float *slab, int ldg, int N, int M, int Bt,
              int splits, hipStream_t s, const TnTail &tail) {
    if (M % TM || N % TN || Bt % 64 || splits > Bt / 64) return -2;
    const int tiles_n = N / TN, tiles = (M / TM) * tiles_n;
    const int xcd_map = (splits % 8 == 0 && tiles > 1) ? 1 : 0;
    hipLaunchKernelGGL((gemm_tn_rs_kernel<TM, TN, P, HU8>), dim3(tiles * splits + tail.blocks), dim3(256), 0, s,
                       (const __bf16 *)D, ldd, H, ldh, hscale, slab, ldg, N, Bt / 64, splits, tiles_n, tiles, xcd_map,
                       tail);
    return hipGetLastError() == hipSuccess ? 0 : -5;
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
    /* HPNN_G0D (experiments) for 160 x 128 tiles: 1 = 3 k-steps in flight, 2 / 3 = 8 waves
     * (two k-interleaved groups) with 2 / 1 in flight; measured 23.8 / 25.1 / 24.3 us vs
     * 23.8 us for the default (2 in flight, 4 waves) */
    static const int var = [] { const char *e = getenv("HPNN_G0D"); return e ? atoi(e) : 0; }();
#define HPNN_FM(...)                                                                                              \
    return h_u8 ? launch_fm<__VA_ARGS__, true>(Dg, Hg, hscale, slab, ldg, N, M, Bt, splits, s, t)                  \
                : launch_fm<__VA_ARGS__, false>(Dg, Hg, hscale, slab, ldg, N, M, Bt, splits, s, t)
    if (M % 160 == 0 && N % 128 == 0) {
        if (var == 1) { HPNN_FM(5, 4, 3, 1); }
        if (var == 2) { HPNN_FM(5, 4, 2, 2); }
        if (var == 3) { HPNN_FM(5, 4, 1, 2); }
        if (var == 4) { HPNN_FM(5, 4, 2, 1); }
        if (var == 5) { HPNN_FM(5, 4, 3, 2); } /* 8-bit H: 23.9 / 27.0 us, no gain */
        if (var == 6) { HPNN_FM(5, 4, 5, 2); } /* 8-bit H: 24.0 / 27.6 us */
        /* 8-bit H: 8 waves (two k-interleaved groups) hide the byte -> bf16 conversion
         * (23.0 / 26.5 us hot / cold vs 27.0 / 27.2 with 4 waves); bf16 H: 4 waves */
        if (h_u8) { HPNN_FM(5, 4, 1, 2); }
        HPNN_FM(5, 4, 2, 1);
    }
    if (M % 64 == 0 && N % 64 == 0) { HPNN_FM(2, 2, 2, 1); }
    HPNN_FM(1, 1, 3, 1);
#undef HPNN_FM
}

}  // namespace

extern "C" int hpnn_gemm_tn_rs(const void *D, int ldd, const void *H, int ldh, int h_u8, float hscale, float *slab,
                               int ldg, int N, int M, int Bt, int splits, const float *rslab, int rS, long rstride,
                               long rn, int rgroups, float *rout, hipStream_t stream) {
    if (N <= 0 || M <= 0 || Bt <= 0 || splits <= 0) return -1;
    if (ldd % 8 || ldh % (h_u8 ? 16 : 8) || ldg % 4 || ldg < M) return -3;
    TnTail t = {nullptr, nullptr, 0, 0, 0, 0, 1, 1, 0};
    if (rslab) {
        if (rn % 4 || rstride % 4 || rS < 1 || rgroups < 1 || rgroups > rS || !rout) return -2;
        const long n4 = rn / 4;
        const int bx = (int)((n4 + 255) / 256);
        t = {rslab, rout, rstride, n4, rn, rS, (rS + rgroups - 1) / rgroups, bx, bx * rgroups};
    }
    static const int pd = [] { const char *e = getenv("HPNN_RS_P"); return e ? atoi(e) : 3; }();
#define HPNN_RS(TM_, P_)                                                                                          \
    return h_u8 ? launch_rs<TM_, 128, P_, true>(D, ldd, H, ldh, hscale, slab, ldg, N, M, Bt, splits, stream, t)    \
                : launch_rs<TM_, 128, P_, false>(D, ldd, H, ldh, hscale, slab, ldg, N, M, Bt, splits, stream, t)
    if (M % 160 == 0 && N % 128 == 0) {
        if (pd == 6) { HPNN_RS(160, 6); }
        HPNN_RS(160, 3);
    }
    if (M % 128 == 0 && N % 128 == 0) { HPNN_RS(128, 3); }
#undef HPNN_RS
    return -2;
}

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
