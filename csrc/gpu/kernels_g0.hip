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
 * it streams at the memory rate.  Round 4, again: the same 160 x 128 tiles with the operands
 * LDS-DMA staged (two k-steps of contiguous fragments per stage, 3-4 stages in flight, no VGPR
 * staging) took 72.9-74.1 vs 61.3-62.0 us per MNIST step (profiles/r4).  Rejected on the way: the same kernel on plain
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

#include <algorithm>
#include <type_traits>

#include "kernels.h"

HPNN_CO_PROBE(g0)
#include "mfma_common.h"

namespace {

/* HPNN_G0_PROTO hand-off diagnostics exist only in make ABLATIONS=1 builds */
#ifdef HPNN_ABLATIONS
#define G0_PROTO(u, bit) ((u).proto & (bit))
#else
#define G0_PROTO(u, bit) 0
#endif

using hpnn::bf16x8;
using hpnn::f32x4;
using hpnn::TnTail;
using hpnn::gu32;
using hpnn::sum_sc1_x8;
using hpnn::st_sc1;

/* Dg: [Bt/32][N/16][64][8], Hg: [Bt/32][M/16][64][8]; nbd = N / 16, nbh = M / 16.
 * HU8: Hg holds unsigned bytes (8 per lane per fragment), multiplied as exact integers;
 * hscale scales the FP32 result (G = hscale * D^T H) */
/* the workgroup's partial product over its split of the batch: on return the waves of group
 * kg == 0 hold the 32 WF x 32 WH tile (wave tile 16 WF x 16 WH) in acc; *tile_, *split_, m0 / n0
 * (this wave's tile origin) are set.  Every wave returns (the caller's barriers need them). */
/* workgroup role: (virtual) block b -> output tile and batch split.  xcd_map: the tiles of
 * one batch slice share b % 8, i.e. one XCD under the observed round-robin placement, so the
 * slice's Dt rows are fetched once into that L2 -- a speed assumption only: every result is
 * the same whichever block takes which role (fixed-order sums; tests permute the order).
 * 8 * (splits / 8) splits map that way; the rest (splits not a multiple of 8) take the last
 * blocks in plain order */
__device__ __forceinline__ void fm_role(int b, int splits, int tiles, int xcd_map, int &tile, int &split) {
    if (xcd_map) {
        const int main = (splits / 8) * 8 * tiles;
        if (b < main) {
            const int xcd = b & 7, j = b >> 3;
            tile = j % tiles;
            split = xcd + 8 * (j / tiles);
        } else {
            tile = (b - main) % tiles;
            split = (splits / 8) * 8 + (b - main) / tiles;
        }
    } else {
        tile = b % tiles;
        split = b / tiles;
    }
}

template <int WF, int WH, int PD, int KW, bool HU8, int WM = 2, int WN = 2, bool X16 = false>
__device__ __forceinline__ void fm_partial(const __bf16 *__restrict__ Dg, int nbd, const void *__restrict__ Hg, int nbh,
                                           int ksteps, int splits, int tiles_n, int tiles, int xcd_map, int vb,
                                           f32x4 (&acc)[WF][WH], int &tile, int &split, int &m0, int &n0) {
    constexpr int R = PD + 1;
    constexpr int GW = WM * WN;                   /* waves per k-group */
    constexpr int TMF = 16 * WF * WM, TNH = 16 * WH * WN; /* workgroup tile: features x delta columns */
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kg = wave / GW, wm = (wave % GW) / WN, wn = wave % WN;
    fm_role(vb, splits, tiles, xcd_map, tile, split);
    m0 = (tile / tiles_n) * TMF + wm * 16 * WF;
    n0 = (tile % tiles_n) * TNH + wn * 16 * WH;
    const int k0 = (int)((long)split * ksteps / splits), k1 = (int)((long)(split + 1) * ksteps / splits);
    /* this wave group's k-steps: k0 + kg, k0 + kg + KW, ... */
    const int nk = (k1 - k0 - kg + KW - 1) / KW;
    const int r16 = lane & 15;
    constexpr int ES = HU8 ? 1 : 2; /* bytes per H element */
    using HT = typename std::conditional<HU8, uint2, bf16x8>::type;
    const char *pa = (const char *)Hg + (((size_t)(k0 + kg) * nbh + m0 / 16) * 512 + lane * 8) * ES;
    const __bf16 *pb = Dg + ((size_t)(k0 + kg) * nbd + n0 / 16) * 512 + lane * 8;
    const size_t step_a = (size_t)KW * nbh * 512 * ES, step_b = (size_t)KW * nbd * 512; /* this group's next k-step */

#pragma unroll
    for (int i = 0; i < WF; i++)
#pragma unroll
        for (int j = 0; j < WH; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    HT ra[R][WF];
    bf16x8 rb[R][WH];
    auto load = [&](int slot_, int t) __attribute__((always_inline)) {
        const int tc = t < nk - 1 ? t : nk - 1; /* clamped: the ring tail re-reads the last step */
        if constexpr (X16 && HU8) {
            /* timing ablation (make ABLATIONS=1, HPNN_G0_X16=1; wrong results): fragment pairs
             * through one 16-byte load per lane instead of two 8-byte loads */
            typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#pragma unroll
            for (int i = 0; i + 1 < WF; i += 2) {
                const u32x4 v = *(const u32x4 *)(pa - lane * 8 + lane * 16 + i * 512 + (size_t)tc * step_a);
                ra[slot_][i] = HT{v.x, v.y};
                ra[slot_][i + 1] = HT{v.z, v.w};
            }
            if constexpr (WF % 2) ra[slot_][WF - 1] = *(const HT *)(pa + (WF - 1) * 512 + (size_t)tc * step_a);
        } else {
#pragma unroll
            for (int i = 0; i < WF; i++) ra[slot_][i] = *(const HT *)(pa + i * 512 * ES + (size_t)tc * step_a);
        }
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

    if constexpr (KW > 1) { /* groups 1.. hand their partial tiles to group 0 through LDS, in order */
        __shared__ f32x4 part[GW][WF * WH][64];
#pragma unroll
        for (int g = 1; g < KW; g++) {
            if (kg == g) {
#pragma unroll
                for (int i = 0; i < WF; i++)
#pragma unroll
                    for (int j = 0; j < WH; j++) part[wave % GW][i * WH + j][lane] = acc[i][j];
            }
            __syncthreads();
            if (kg == 0) {
#pragma unroll
                for (int i = 0; i < WF; i++)
#pragma unroll
                    for (int j = 0; j < WH; j++) acc[i][j] += part[wave % GW][i * WH + j][lane];
            }
            if (g + 1 < KW) __syncthreads();
        }
    }
}

template <int WF, int WH, int PD, int KW, bool HU8 = false, int WM = 2, int WN = 2>
__global__ __launch_bounds__(64 * WM * WN * KW) void gemm_fm_direct_kernel(const __bf16 *__restrict__ Dg, int nbd,
                                                                  const void *__restrict__ Hg, int nbh, float hscale,
                                                                  float *__restrict__ slab, int ldg, int N, int ksteps,
                                                                  int splits, int tiles_n, int tiles, int xcd_map,
                                                                  TnTail tail) {
    if ((int)blockIdx.x >= tiles * splits) {
        if (threadIdx.x < 256) hpnn::tn_tail_reduce(tail, (int)blockIdx.x - tiles * splits);
        return;
    }
    f32x4 acc[WF][WH];
    int tile, split, m0, n0;
    fm_partial<WF, WH, PD, KW, HU8, WM, WN>(Dg, nbd, Hg, nbh, ksteps, splits, tiles_n, tiles, xcd_map,
                                            (int)blockIdx.x, acc, tile, split, m0, n0);
    if ((threadIdx.x >> 6) >= WM * WN) return;
    const int lane = threadIdx.x & 63, r16 = lane & 15, q = lane >> 4;
    float *out = slab + (size_t)split * N * ldg;
#pragma unroll
    for (int i = 0; i < WF; i++)
#pragma unroll
        for (int j = 0; j < WH; j++)
            *(f32x4 *)(out + (size_t)(n0 + j * 16 + r16) * ldg + m0 + i * 16 + 4 * q) =
                HU8 ? acc[i][j] * hscale : acc[i][j];
}

/* ---- G0 with its split-K reduction and the optimizer step in the same launch ----------
 * (the single-GPU MNIST step: front, then this, two launches).  Every GEMM workgroup
 * publishes its FP32 partial tile with write-through (sc1) stores, drains them and adds one
 * ticket to its tile's monotonic counter (agent scope); it then waits (sc1 polls, bounded)
 * until all `splits` partials of the tile have arrived, reduces its 1/splits share of the
 * tile over the splits in a FIXED order (sc1 loads; bitwise repeatable whatever the arrival
 * order) and applies the BP / BPM step to those elements: FP32 master, momentum, BF16 W,
 * W^T and the fragment-major copy the front reads.  The front's [G1 | G2] block slabs are
 * summed completely (fixed order) and layers 1 and 2 stepped by TAIL workgroups appended to
 * the grid, on the CUs the GEMM grid leaves idle (MNIST: 240 GEMM workgroups + 16 tails on 256
 * CUs): the 9 MB of slab reads run beside the GEMM instead of after every workgroup's publish
 * (-2.7 us per step on a slow box, profiles/r6); HPNN_G0_TAIL12 < 100 leaves part of the
 * columns to the GEMM workgroups, between their ticket and their wait.  Tails wait for
 * nothing, so any dispatch order is deadlock-free.  Output tiles are 80 x 128 (10 tiles x 24
 * splits on MNIST: half the split-K partial bytes of 160 x 128 x 48, HPNN_G0_TILE=160 the
 * old form).  Replaces the separate sgd_update_multi launch (6.2 us) and its kernel boundary
 * behind 20 MB of dirty slabs.  All GEMM workgroups are co-resident (grid <= CUs; a wait that
 * times out sets *err instead of hanging).  Reference: the per-layer update of
 * snn_kernel_train_momentum / cuda_snn.cu:2726-3717 (GER into dW, W += dW, dW *= alpha),
 * batched. */
constexpr unsigned long long G0_TIMEOUT = 1000000000ULL; /* wall-clock ticks (~10 s) */

/* the master weight / momentum of the first element a thread steps, loaded right after the
 * GEMM so the load is in flight through the publish, ticket and split-sum waits instead of
 * in series after them (passed by value with a flag: a pointer to it would put it on the
 * stack) */
struct Pre4 {
    f32x4 w, v;
};

__device__ __forceinline__ void bpm_step4(float *__restrict__ W32, float *__restrict__ V32, size_t idx, f32x4 g,
                                          const hpnn_g0_update &u, f32x4 &w, bool use = false, Pre4 pre = {}) {
    w = use ? pre.w : *(const f32x4 *)(W32 + idx);
    if (u.momentum) {
        f32x4 v = use ? pre.v : *(const f32x4 *)(V32 + idx);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            v[r] += u.lr * (g[r] * u.scale);
            w[r] += v[r];
            v[r] *= u.alpha;
        }
        *(f32x4 *)(V32 + idx) = v;
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) w[r] += u.lr * (g[r] * u.scale);
    }
    *(f32x4 *)(W32 + idx) = w;
}

/* element (n, k..k+3) of a [N][K] layer: FP32 master + BF16 W / W^T (+ fragment-major Wf) */
__device__ __forceinline__ void step_elem4(float *W32, float *V32, __bf16 *Wb, __bf16 *Wt, __bf16 *Wf, int N, int K,
                                           int n, int k, f32x4 g, const hpnn_g0_update &u, bool use = false,
                                           Pre4 pre = {}) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    const size_t idx = (size_t)n * K + k;
    f32x4 w;
    bpm_step4(W32, V32, idx, g, u, w, use, pre);
    bf16x4 wb;
#pragma unroll
    for (int r = 0; r < 4; r++) wb[r] = (__bf16)w[r];
    *(bf16x4 *)(Wb + idx) = wb;
    if (Wf) { /* MFMA-fragment-major copy (kernels.h): 4 consecutive k stay contiguous */
        const size_t fo = (((size_t)(n >> 4) * (K / 32) + (k >> 5)) * 64 + (n & 15) + 16 * ((k >> 3) & 3)) * 8 + (k & 7);
        *(bf16x4 *)(Wf + fo) = wb;
    }
    if (!G0_PROTO(u, 2048)) /* 2048: timing ablation, no W^T stores */
#pragma unroll
        for (int r = 0; r < 4; r++) Wt[(size_t)(k + r) * N + n] = wb[r];
}

/* element i of a small array inside the by-value kernel argument, as a chain of selects: a
 * DYNAMIC index into the argument makes the compiler copy the whole 440-byte struct into every
 * thread's scratch at kernel start (seen in the ISA: scratch_store_dwordx4 x 28 per thread) */
template <class T, int N>
__device__ __forceinline__ T pick(const T (&a)[N], int i) {
    T r = a[0];
#pragma unroll
    for (int k = 1; k < N; k++) r = i == k ? a[k] : r;
    return r;
}

/* float4 e4 of [G1 | G2] -> layer l, row n, column k */
__device__ __forceinline__ int g12_elem(const hpnn_g0_update &u, long e4, int &n, int &k) {
    long i = e4 * 4;
    const long n1 = (long)u.Nb[0] * u.Kb[0];
    const int l = i < n1 ? 0 : 1;
    if (l) i -= n1;
    const int kb = pick(u.Kb, l);
    n = (int)(i / kb), k = (int)(i % kb);
    return l;
}
__device__ __forceinline__ Pre4 pre_load(const float *W32, const float *V32, size_t idx, int momentum) {
    Pre4 p;
    p.w = *(const f32x4 *)(W32 + idx);
    p.v = momentum ? *(const f32x4 *)(V32 + idx) : f32x4{0.f, 0.f, 0.f, 0.f};
    return p;
}

/* [G1 | G2]: float4 columns [c0, c1) of the front's block slabs summed over all mrows rows in
 * a fixed order (RG row groups of NT / 16 threads, met in LDS in order), then layers 1 / 2
 * stepped at those elements */
template <int NT>
__device__ __forceinline__ void g12_share(const hpnn_g0_update &u, long c0, long c1, f32x4 *red, float *g12out,
                                          bool use = false, Pre4 pre = {}) {
    constexpr int C4 = 16, RG = NT / C4;
    const int t = threadIdx.x, c = t % C4, rg = t / C4;
    for (long b0 = c0; b0 < c1; b0 += C4) {
        const long e4 = b0 + c;
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        if (e4 < c1) {
            /* 8 rows' loads in flight per batch (a dependent one-at-a-time walk over the rows is
             * latency-bound: ~8 L2 / Infinity-Cache round trips back to back) */
            const float *col = u.mslab + e4 * 4;
            for (int r0 = rg; r0 < u.mrows; r0 += 8 * RG) {
                f32x4 v[8];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const int r = r0 + k * RG;
                    v[k] = r < u.mrows ? *(const f32x4 *)(col + (long)r * u.mstride) : f32x4{0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
                for (int k = 0; k < 8; k++) a += v[k];
            }
        }
        red[t] = a;
        __syncthreads();
        if (rg == 0 && e4 < c1) {
            f32x4 g = red[c];
            for (int r = 1; r < RG; r++) g += red[r * C4 + c];
            long i = e4 * 4;
            if (g12out) {
                *(f32x4 *)(g12out + i) = g;
            } else {
                int n, k;
                const int l = g12_elem(u, e4, n, k);
                step_elem4(pick(u.W32b, l), pick(u.V32b, l), (__bf16 *)pick(u.Wbb, l), (__bf16 *)pick(u.Wtb, l), nullptr,
                           pick(u.Nb, l), pick(u.Kb, l), n,
                           k, g, u, use && b0 == c0 /* this thread's prefetched element */, pre);
            }
        }
        __syncthreads();
    }
}

/* [G1 | G2] on the tail workgroups (blocks past the GEMM grid, on the CUs it leaves idle; they
 * run beside the GEMM instead of after it): float4 columns [c0, c1) summed over all mrows rows,
 * 32 columns (512 contiguous bytes of a row) x NT / 32 row groups per pass and 16 rows of loads
 * in flight per thread (latency-bound otherwise: a pass is one memory round trip); the row
 * groups meet in LDS in a fixed order, then the layer-1/2 step (or the store into g12out) */
template <int NT>
__device__ __forceinline__ void g12_share_wide(const hpnn_g0_update &u, long c0, long c1, f32x4 *red, float *g12out) {
    constexpr int C4 = 32, RG = NT / C4, RB = 16;
    const int t = threadIdx.x, c = t % C4, rg = t / C4;
    for (long b0 = c0; b0 < c1; b0 += C4) {
        const long e4 = b0 + c;
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        if (e4 < c1) {
            const float *col = u.mslab + e4 * 4;
            for (int r0 = rg; r0 < u.mrows; r0 += RB * RG) {
                f32x4 v[RB];
#pragma unroll
                for (int k = 0; k < RB; k++) {
                    const int r = r0 + k * RG;
                    v[k] = r < u.mrows ? *(const f32x4 *)(col + (long)r * u.mstride) : f32x4{0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
                for (int k = 0; k < RB; k++) a += v[k];
            }
        }
        red[t] = a;
        __syncthreads();
        if (rg == 0 && e4 < c1) {
            f32x4 g = red[c];
            for (int r = 1; r < RG; r++) g += red[r * C4 + c];
            if (g12out) {
                *(f32x4 *)(g12out + e4 * 4) = g;
            } else {
                int n, k;
                const int l = g12_elem(u, e4, n, k);
                step_elem4(pick(u.W32b, l), pick(u.V32b, l), (__bf16 *)pick(u.Wbb, l), (__bf16 *)pick(u.Wtb, l), nullptr,
                           pick(u.Nb, l), pick(u.Kb, l), n,
                           k, g, u);
            }
        }
        __syncthreads();
    }
}

/* sum of float4 at offset o over the first `world` ranks' buffers, rank order (identical bits
 * on every rank); all loads in flight at once, system-coherent (sc0 sc1: no cache can serve a
 * stale line, so no acquire fence -- an invalidating acquire per workgroup, while the other
 * workgroups still stream their split sums, cost ~10 us per step) */
static_assert(HPNN_XAR_MAX_RANKS == 8, "one ld_sc1_x8 per element");
__device__ __forceinline__ f32x4 xsum_peers(const hpnn_xar_view &v, long o) {
    const float *q[8];
#pragma unroll
    for (int p = 0; p < 8; p++) q[p] = pick(v.buf, p < v.world ? p : v.rank) + o; /* spare slots: local */
    f32x4 x[8];
    hpnn::ld_sc1_x8<true>(x, q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]);
    f32x4 a = x[0];
#pragma unroll
    for (int p = 1; p < HPNN_XAR_MAX_RANKS; p++)
        if (p < v.world) a += x[p];
    return a;
}

/* data-parallel tail (u.xchg): this workgroup's reduced G0 share (float4 [e0, e1) of its
 * tile) and [G1 | G2] share sit in its half of this rank's exchange buffer (fine-grained,
 * uncached: no cache maintenance between ranks).  One-shot barrier of workgroup b (the
 * protocol of xgmi_ar.hip, release = waiting for the store acknowledgements), then the
 * rank-order sums over the peers' copies of exactly those elements and their steps: the
 * exchange and the update need no launch of their own. */
template <int NT>
__device__ __forceinline__ void g0_exchange_step(const hpnn_g0_update &u, unsigned int e, int N, int ldg, int e0, int e1,
                                              int nt0, int mt0, int TMF, bool pf, Pre4 pg0, Pre4 pg12, int b, long c0,
                                              long c1) {
    const hpnn_xar_view &v = u.xv;
    const int t = threadIdx.x;
    /* the exchanged sums: stepped, or (self-test, u.xres) stored at their flat offsets; the
     * fault hook (u.xfault, tests) corrupts the first G0 element of role 0 on this rank */
    auto out0 = [&](int c, f32x4 g, bool use, Pre4 pre) __attribute__((always_inline)) {
        const int row = c / (TMF / 4), col = mt0 + 4 * (c % (TMF / 4));
        if (u.xfault && b == 0 && c == e0) g[0] += 1.0f;
        if (u.xres) *(f32x4 *)(u.xres + (size_t)(nt0 + row) * ldg + col) = g;
        else step_elem4(u.W32, u.V32, (__bf16 *)u.Wb, (__bf16 *)u.Wt, (__bf16 *)u.Wf, N, ldg, nt0 + row, col, g, u,
                        use, pre);
    };
    auto out12 = [&](long e4, f32x4 g, bool use, Pre4 pre) __attribute__((always_inline)) {
        if (u.xres) {
            *(f32x4 *)(u.xres + (size_t)N * ldg + e4 * 4) = g;
            return;
        }
        int n, k;
        const int l = g12_elem(u, e4, n, k);
        step_elem4(pick(u.W32b, l), pick(u.V32b, l), (__bf16 *)pick(u.Wbb, l), (__bf16 *)pick(u.Wtb, l), nullptr,
                           pick(u.Nb, l), pick(u.Kb, l), n, k, g,
                   u, use, pre);
    };
    const long hoff = (e & 1) ? v.half : 0;
    /* flag barrier `which` of workgroup b with every peer: this workgroup's stores to its buffer
     * acknowledged first (uncached memory: no writeback needed) */
    auto barrier = [&](int which) __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t < v.world && !G0_PROTO(u, 16)) { /* proto & 16: no barrier (one-rank timing ablation only) */
            unsigned int *const sm = pick(v.sig, v.rank), *const sp = pick(v.sig, t);
            unsigned int *const mine = which ? HPNN_XAR_FLAG_B(sm, b, t) : HPNN_XAR_FLAG_A(sm, b, t);
            __hip_atomic_store(which ? HPNN_XAR_FLAG_B(sp, b, v.rank) : HPNN_XAR_FLAG_A(sp, b, v.rank), e,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - t0 > v.timeout) {
                    __hip_atomic_store(pick(v.sig, v.rank) + HPNN_XAR_ERROR_WORD, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
        }
        __syncthreads();
        if (G0_PROTO(u, 8)) /* diagnostics: the invalidating system acquire as well */
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    };
    auto g0_off = [&](int c) __attribute__((always_inline)) {
        return (long)(nt0 + c / (TMF / 4)) * ldg + mt0 + 4 * (c % (TMF / 4));
    };
    const bool two = u.xchg == 2 && v.world > 1;
    barrier(0);
    if (two) {
        /* reduce-scatter: element j of each part belongs to rank j % world, which sums it over
         * all ranks (rank order) into its own buffer; a second barrier; every rank then reads
         * each element from its owner -- each link carries 2 / world of the slice, not all */
        for (int c = e0 + t; c < e1; c += NT)
            if ((c - e0) % v.world == v.rank) {
                const long o = hoff + g0_off(c);
                *(f32x4 *)(pick(v.buf, v.rank) + o) = xsum_peers(v, o);
            }
        for (long e4 = c0 + t; e4 < c1; e4 += NT)
            if ((int)((e4 - c0) % v.world) == v.rank) {
                const long o = hoff + (long)N * ldg + e4 * 4;
                *(f32x4 *)(pick(v.buf, v.rank) + o) = xsum_peers(v, o);
            }
        barrier(1);
    }
    /* at most one G0 and one [G1 | G2] element per thread (the MNIST grid: ~107 and ~11 float4
     * per workgroup): both elements' remote loads go out in ONE block and one wait -- over xGMI
     * each wait is a link round trip, so two in series would cost the step a second one */
    if (e1 - e0 <= NT && c1 - c0 <= NT && (two || v.world <= 4) && !G0_PROTO(u, 32)) { /* 32: ablation */
        const bool h0 = e0 + t < e1, h12 = c0 + t < c1;
        const long oa = h0 ? hoff + g0_off(e0 + t) : hoff, ob = h12 ? hoff + (long)N * ldg + (c0 + t) * 4 : hoff;
        f32x4 ga, gb;
        if (two) { /* the owners' sums (owner of element j = t: rank t % world) */
            const float *qa = pick(v.buf, h0 ? t % v.world : v.rank) + oa;
            const float *qb = pick(v.buf, h12 ? t % v.world : v.rank) + ob;
            asm volatile("global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
                         "global_load_dwordx4 %1, %3, off sc0 sc1\n\t"
                         "s_waitcnt vmcnt(0)"
                         : "=&v"(ga), "=&v"(gb)
                         : "v"(qa), "v"(qb)
                         : "memory");
        } else { /* one-shot, world <= 4: rank-order sums of both, 4 slots each (spares local) */
            f32x4 x[8];
            const float *q[8];
#pragma unroll
            for (int p = 0; p < 4; p++) {
                q[p] = pick(v.buf, p < v.world ? p : v.rank) + oa;
                q[4 + p] = pick(v.buf, p < v.world ? p : v.rank) + ob;
            }
            hpnn::ld_sc1_x8<true>(x, q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]);
            ga = x[0];
            gb = x[4];
#pragma unroll
            for (int p = 1; p < 4; p++)
                if (p < v.world) {
                    ga += x[p];
                    gb += x[4 + p];
                }
        }
        if (h0) out0(e0 + t, ga, pf && t < 128, pg0);
        if (h12) out12(c0 + t, gb, pf && t < 16, pg12);
        return;
    }
    /* one-shot: the rank-order sum over every peer; two-shot: the owner's sum */
    auto fetch = [&](long o, long j) __attribute__((always_inline)) -> f32x4 {
        if (!two) return xsum_peers(v, o);
        const float *q = pick(v.buf, (int)(j % v.world)) + o;
        f32x4 x; /* one system-coherent load and its wait in one asm block (see ld_sc1_x8) */
        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(q) : "memory");
        return x;
    };
    for (int c = e0 + t; c < e1; c += NT) out0(c, fetch(hoff + g0_off(c), c - e0), pf && c == e0 + t && t < 128, pg0);
    for (long e4 = c0 + t; e4 < c1; e4 += NT)
        out12(e4, fetch(hoff + (long)N * ldg + e4 * 4, e4 - c0), pf && e4 == c0 + t && t < 16, pg12);
}

/* self-test pattern of the in-kernel exchange: rank r, flat gradient index i ->
 * (r + 1) (i % 97 + 1) / 16 -- every partial sum over <= 8 ranks exact in FP32 */
__device__ __forceinline__ f32x4 xtest_pattern(int rank, long i) {
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = (float)((rank + 1) * ((i + r) % 97 + 1)) * 0.0625f;
    return v;
}

/* ---- XCD-local first level of the split-K reduction (u.xw, HPNN_G0_XCD=1) -------------
 * The splits of a tile form 8 static groups g = split % 8 of gsz = splits / 8 members (MNIST:
 * 24 splits, 3 a group).  Under the round-robin placement a group's members share one XCD, so
 * they can combine through that XCD's L2 instead of publishing write-through: every member
 * stores its partial tile PLAIN (it stays in the L2), the group's last arriver sums the gsz
 * partials (L1-bypassing loads served by the L2) and publishes ONE write-through partial per
 * (tile, group), and the tile's reducers then read 8 partials instead of `splits`.  The
 * placement is never assumed: at kernel start every member records (launch epoch, hardware
 * XCC_ID) in its group slot, and after its GEMM it stores plain only when every member of the
 * group has recorded this epoch on ITS XCD -- otherwise write-through, which any reader can
 * see.  All sums keep a fixed order (members, then groups): bitwise the same whichever block
 * takes which role and whichever store form ran. */
constexpr int G0X_EP = 0, G0X_SLOTS = 256, G0X_GCNT = 2304, G0X_TCNT = 2816;
static_assert(G0X_TCNT + 32 * HPNN_G0_MAX_TILES <= HPNN_G0X_WORDS, "xw layout");
static_assert(G0X_SLOTS + 64 * HPNN_G0_MAX_TILES <= G0X_GCNT && G0X_GCNT + 16 * HPNN_G0_MAX_TILES <= G0X_TCNT,
              "xw layout");

__device__ __forceinline__ unsigned int xcc_id() {
    return (unsigned int)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u; /* HW_REG_XCC_ID[3:0] */
}

/* the group leader: out[e] = sum over members m (in order) of part[m][e], float4 e of the tile
 * at offsets off(e); NT threads, NE4 float4, G members (static: every index below is
 * compile-time, no scratch); write-through stores */
template <int NT, int NE4, int TMF, int G>
__device__ __forceinline__ void xcd_group_sum_g(const float *slab0, size_t mstride, float *out, int ldg, int nt0,
                                                int mt0) {
    constexpr int KE = (NE4 + NT - 1) / NT, EPB = 16 / G; /* float4 per thread, per 16-load batch */
    const int t = threadIdx.x;
    auto off = [&](int c) __attribute__((always_inline)) {
        return (size_t)(nt0 + c / (TMF / 4)) * ldg + mt0 + 4 * (c % (TMF / 4));
    };
#pragma unroll
    for (int k0 = 0; k0 < KE; k0 += EPB) {
        const float *q[16];
        f32x4 v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int k = k0 + i / G, m = i % G, c = t + k * NT;
            const bool ok = i < EPB * G && k < KE && c < NE4;
            q[i] = slab0 + (ok ? off(c) + (size_t)m * mstride : off(t < NE4 ? t : 0)); /* spares: a valid line */
        }
        hpnn::ld_sc1_x16(v, q);
#pragma unroll
        for (int j = 0; j < EPB; j++) {
            const int k = k0 + j, c = t + k * NT;
            if (k < KE && c < NE4) {
                f32x4 a = v[j * G];
#pragma unroll
                for (int m = 1; m < G; m++) a += v[j * G + m];
                st_sc1(out + off(c), a);
            }
        }
    }
}
template <int NT, int NE4, int TMF>
__device__ __forceinline__ void xcd_group_sum(const float *slab0, size_t mstride, float *out, int gsz, int ldg,
                                              int nt0, int mt0) {
    if (gsz == 2) xcd_group_sum_g<NT, NE4, TMF, 2>(slab0, mstride, out, ldg, nt0, mt0);
    else if (gsz == 3) xcd_group_sum_g<NT, NE4, TMF, 3>(slab0, mstride, out, ldg, nt0, mt0);
    else xcd_group_sum_g<NT, NE4, TMF, 4>(slab0, mstride, out, ldg, nt0, mt0);
}

/* HPNN_G0_TRACE=1 (profiling only): s_memtime stamps of every workgroup's thread 0 at the
 * phase boundaries, [block][mark]; read back with hpnn_g0_trace */
constexpr int G0TR_BLOCKS = 512, G0TR_MARKS = 8;
__device__ unsigned long long g_g0_trace[G0TR_BLOCKS][G0TR_MARKS];

template <int WF, int WH, int PD, int KW, bool HU8, bool TRACE = false, int WM = 2, int WN = 2, bool X16 = false>
__global__ __launch_bounds__(64 * WM * WN * KW) void g0_fused_kernel(const __bf16 *__restrict__ Dg, int nbd,
                                                            const void *__restrict__ Hg, int nbh, float hscale,
                                                            float *__restrict__ slab, int ldg, int N, int ksteps,
                                                            int splits, int tiles_n, int tiles, int xcd_map,
                                                            hpnn_g0_update u) {
    constexpr int GW = WM * WN, NT = 64 * GW * KW, TMF = 16 * WF * WM, TNH = 16 * WH * WN, NE4 = TMF * TNH / 4,
                  PARTS = NT / 128;
    auto mark = [&](int i) __attribute__((always_inline)) {
        if constexpr (TRACE) {
            const unsigned long long tt = __builtin_amdgcn_s_memtime();
            if (threadIdx.x == 0 && blockIdx.x < G0TR_BLOCKS) g_g0_trace[blockIdx.x][i] = tt;
        }
    };
    mark(0);
    __shared__ f32x4 red[NT];
    f32x4 acc[WF][WH];
    int tile, split, m0, n0;
    const long nb = (long)tiles * splits, nf = u.n12 / 4;
    /* [G1 | G2] float4 columns [0, nt4) belong to the tail workgroups (blocks nb..), the rest to
     * the GEMM workgroups after their publish */
    const int ntail = (int)gridDim.x - (int)nb;
    const long nt4 = ntail > 0 ? u.n12t / 4 : 0;
    /* the exchange's parameters, set by whichever path this workgroup takes */
    bool xdo = false, xpf = false;
    int xb = 0, xe0 = 0, xe1 = 0, xnt0 = 0, xmt0 = 0;
    unsigned int xep = 0;
    long xc0 = 0, xc1 = 0;
    Pre4 xpg0 = {}, xpg12 = {};
    if ((long)blockIdx.x >= nb) {
        const int tb = (int)blockIdx.x - (int)nb;
        const long tc0 = (long)tb * nt4 / ntail, tc1 = (long)(tb + 1) * nt4 / ntail;
        __shared__ unsigned int txe_s;
        float *gout = u.gout && u.gsel && !(*u.gsel & 1) ? u.gout + u.galt : u.gout;
        if (u.xchg) {
            if (threadIdx.x == 0) {
                const unsigned int e = u.xv.ep[blockIdx.x] + 1; /* exchange slot: the block itself */
                u.xv.ep[blockIdx.x] = e;
                txe_s = e;
            }
            __syncthreads();
            gout = pick(u.xv.buf, u.xv.rank) + ((txe_s & 1) ? u.xv.half : 0);
        }
        if (u.xtest) {
            if (u.xchg) {
                for (long e4 = tc0 + threadIdx.x; e4 < tc1; e4 += NT) {
                    const long i = (long)N * ldg + e4 * 4;
                    *(f32x4 *)(gout + i) = xtest_pattern(u.xv.rank, i);
                }
            }
        } else {
            g12_share_wide<NT>(u, tc0, tc1, red, gout ? gout + (size_t)N * ldg : nullptr);
        }
        xdo = u.xchg != 0, xb = (int)blockIdx.x, xep = txe_s, xc0 = tc0, xc1 = tc1;
    } else {
        /* the workgroup's role: virtual block vb (u.perm > 0, tests: reversed and rotated order --
         * every result must stay bitwise the same) */
        const int vb = u.perm > 0 ? (int)((nb - 1 - (long)blockIdx.x + u.perm) % nb) : (int)blockIdx.x;
        /* XCD-local first reduction level: this member's (epoch, XCC) in its group slot, before the
         * GEMM (the members check each other's after theirs) */
        const int gsz = splits / 8;
        const bool xg = u.xw && !u.xtest && xcd_map && splits % 8 == 0 && gsz >= 2 && gsz <= 4;
        unsigned int x_me = 0;
        if (xg && threadIdx.x == 0) {
            int tl, sp;
            fm_role(vb, splits, tiles, xcd_map, tl, sp);
            const unsigned int ep =
                __hip_atomic_fetch_add(u.xw + G0X_EP + vb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
            x_me = (ep << 4) | xcc_id();
            __hip_atomic_store(u.xw + G0X_SLOTS + (tl * 8 + (sp & 7)) * 8 + (sp >> 3), x_me, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (u.xtest) /* self-test of the in-kernel exchange: no GEMM (the role only) */
            fm_role(vb, splits, tiles, xcd_map, tile, split);
        else
            fm_partial<WF, WH, PD, KW, HU8, WM, WN, X16>(Dg, nbd, Hg, nbh, ksteps, splits, tiles_n, tiles, xcd_map, vb, acc,
                                                    tile, split, m0, n0);
        mark(1);
        const int t = threadIdx.x, lane = t & 63;
        /* where the reduced gradient goes instead of a step: the plan's buffer, the xGMI
         * all-reduce's next half (gsel), or -- exchanging here -- this workgroup's epoch's half of
         * this rank's exchange buffer */
        __shared__ unsigned int xe_s;
        float *gout = u.gout && u.gsel && !(*u.gsel & 1) ? u.gout + u.galt : u.gout;
        if (u.xchg) {
            if (t == 0) {
                const unsigned int e = u.xv.ep[vb] + 1; /* only this workgroup touches it */
                u.xv.ep[vb] = e;
                xe_s = e;
            }
            __syncthreads();
            gout = pick(u.xv.buf, u.xv.rank) + ((xe_s & 1) ? u.xv.half : 0);
        }
        /* this split's share of the tile (float4 [e0, e1)) and of [G1 | G2] ([c0, c1)); the first
         * element of each that this thread will step: its W / V loads go out now (HPNN_G0_PROTO
         * bit 64 turns the prefetch off) */
        const int e0 = (int)((long)split * NE4 / splits), e1 = (int)((long)(split + 1) * NE4 / splits);
        const int nt0 = (tile % tiles_n) * TNH, mt0 = (tile / tiles_n) * TMF;
        const long c0 = nt4 + vb * (nf - nt4) / nb, c1 = nt4 + (vb + 1) * (nf - nt4) / nb;
        if (u.xtest) {
            /* the known pattern in place of this workgroup's reduced G0 / [G1 | G2] shares, then the
             * exchange with its sums stored (u.xres) for the host to check */
            if (u.xchg) {
                for (int c = e0 + t; c < e1; c += NT) {
                    const long i = (long)(nt0 + c / (TMF / 4)) * ldg + mt0 + 4 * (c % (TMF / 4));
                    *(f32x4 *)(gout + i) = xtest_pattern(u.xv.rank, i);
                }
                for (long e4 = c0 + t; e4 < c1; e4 += NT) {
                    const long i = (long)N * ldg + e4 * 4;
                    *(f32x4 *)(gout + i) = xtest_pattern(u.xv.rank, i);
                }
                xdo = true, xb = vb, xep = xe_s, xe0 = e0, xe1 = e1, xnt0 = nt0, xmt0 = mt0, xc0 = c0, xc1 = c1;
            }
        } else {
            const bool steps = !u.gout || u.xchg, pf = steps && !G0_PROTO(u, 64);
            Pre4 pg0 = {}, pg12 = {};
            if (pf && t < 128 && e0 + t < e1) {
                const int e = e0 + t, row = e / (TMF / 4), col = mt0 + 4 * (e % (TMF / 4));
                pg0 = pre_load(u.W32, u.V32, (size_t)(nt0 + row) * ldg + col, u.momentum);
            }
            if (pf && t < 16 && c0 + t < c1) {
                int n, k;
                const int l = g12_elem(u, c0 + t, n, k);
                pg12 = pre_load(pick(u.W32b, l), pick(u.V32b, l), (size_t)n * pick(u.Kb, l) + k, u.momentum);
            }
            /* publish this split's partial tile (write-through), then one ticket for the workgroup */
            __shared__ int xloc_s, xlead_s;
            const int xgrp = split & 7;
            if (xg) {
                if (t == 0) { /* every member of the group recorded this epoch on this XCD? */
                    bool loc = true;
                    for (int m = 0; m < gsz; m++)
                        loc = loc && __hip_atomic_load(u.xw + G0X_SLOTS + (tile * 8 + xgrp) * 8 + m, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT) == x_me;
                    xloc_s = loc;
                }
                __syncthreads();
            }
            if ((t >> 6) < GW) {
                const int r16 = lane & 15, q = lane >> 4;
                float *out = slab + (size_t)split * N * ldg;
                if (G0_PROTO(u, 256)) {
                    /* timing ablation: no publish at all (wrong results) */
                } else if (xg && xloc_s) { /* the group's leader reads it from this XCD's L2 */
#pragma unroll
                    for (int i = 0; i < WF; i++)
#pragma unroll
                        for (int j = 0; j < WH; j++)
                            *(f32x4 *)(out + (size_t)(n0 + j * 16 + r16) * ldg + m0 + i * 16 + 4 * q) =
                                HU8 ? acc[i][j] * hscale : acc[i][j];
                } else {
#pragma unroll
                    for (int i = 0; i < WF; i++)
#pragma unroll
                        for (int j = 0; j < WH; j++)
                            st_sc1(out + (size_t)(n0 + j * 16 + r16) * ldg + m0 + i * 16 + 4 * q,
                                   HU8 ? acc[i][j] * hscale : acc[i][j]);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            __shared__ unsigned long long want_s;
            unsigned int *const tcnt = xg ? u.xw + G0X_TCNT + 32 * tile : u.cnt + 32 * tile;
            if (t == 0) {
                if (G0_PROTO(u, 1)) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (xg) {
                    /* group ticket: the last arriver of the launch leads; the tile then waits for its 8
                     * group partials (both counters monotonic: gsz and 8 per launch) */
                    unsigned long long *const gc = (unsigned long long *)(u.xw + G0X_GCNT + 2 * (tile * 8 + xgrp));
                    const unsigned long long old = atomicAdd(gc, 1ull);
                    xlead_s = (int)(old % gsz) == gsz - 1;
                    want_s = (old / gsz + 1) * 8ull;
                } else {
                    want_s = hpnn::ticket_arrive(u.cnt + 32 * tile, (unsigned)splits); /* this launch's last ticket */
                }
            }
            if (xg) {
                __syncthreads();
                if (xlead_s) {
                    /* the group's partial: its gsz member slots summed in member order (plain-stored ones
                     * sit in this XCD's L2, write-through ones in memory; both visible to sc1 loads) */
                    xcd_group_sum<NT, NE4, TMF>(slab + (size_t)xgrp * N * ldg, (size_t)8 * N * ldg,
                                                u.xslab + (size_t)xgrp * N * ldg, gsz, ldg, nt0, mt0);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                    if (t == 0) atomicAdd((unsigned long long *)tcnt, 1ull);
                }
            }
            mark(2);
            /* while the other splits finish: this workgroup's share of [G1 | G2] (no dependency on G0) */
            if (!G0_PROTO(u, 512) && c1 > c0) /* 512: timing ablation, no [G1 | G2] share */
                g12_share<NT>(u, c0, c1, red, gout ? gout + (size_t)N * ldg : nullptr, pf && t < 16, pg12);
            mark(3);
            if (t == 0) {
                /* fault hook: this launch reports a timed-out wait (and, like one, reduces what is there) */
                if (u.fault) __hip_atomic_store((gu32 *)u.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else hpnn::ticket_wait(tcnt, want_s, u.err, G0_TIMEOUT);
                if (G0_PROTO(u, 2)) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            __syncthreads();
            mark(4);
            /* this split's share of the tile: float4 e in [e0, e1), 128 at a time; PARTS threads per
             * float4, each summing a fixed run of splits; the runs meet in LDS in order */
            const int f = t % 128, part = t / 128;
            /* the partials to sum: `splits` split slabs, or the 8 XCD-group partials */
            const int rn = xg ? 8 : splits;
            const float *const rbase = xg ? u.xslab : slab;
            const int s0 = part * rn / PARTS, s1 = (part + 1) * rn / PARTS;
            const size_t ss = (size_t)N * ldg;
            for (int cc = e0; cc < e1; cc += 128) {
                const int e = cc + f;
                const int row = e / (TMF / 4), col = mt0 + 4 * (e % (TMF / 4));
                f32x4 sum = {0.f, 0.f, 0.f, 0.f};
                if (e < e1 && !G0_PROTO(u, 1024)) { /* 1024: timing ablation, no split loads */
                    const float *p = rbase + (size_t)(nt0 + row) * ldg + col;
                    if (G0_PROTO(u, 4))
                        for (int s = s0; s < s1; s += 8) sum += sum_sc1_x8<true>(p + (size_t)s * ss, ss, s1 - s);
                    else
                        for (int s = s0; s < s1; s += 8) sum += sum_sc1_x8(p + (size_t)s * ss, ss, s1 - s);
                }
                red[t] = sum;
                __syncthreads();
                if (part == 0 && e < e1) {
                    f32x4 g = red[f];
#pragma unroll
                    for (int pp = 1; pp < PARTS; pp++) g += red[pp * 128 + f];
                    if (gout)
                        *(f32x4 *)(gout + (size_t)(nt0 + row) * ldg + col) = g;
                    else
                        step_elem4(u.W32, u.V32, (__bf16 *)u.Wb, (__bf16 *)u.Wt, (__bf16 *)u.Wf, N, ldg, nt0 + row, col, g, u,
                                   pf && cc == e0, pg0);
                }
                __syncthreads();
            }
            mark(5);
            xdo = u.xchg != 0, xb = vb, xep = xe_s, xe0 = e0, xe1 = e1, xnt0 = nt0, xmt0 = mt0, xc0 = c0, xc1 = c1;
            xpf = pf, xpg0 = pg0, xpg12 = pg12;
        }  /* not the self-test */
    }  /* GEMM workgroups */
    /* ONE inlined copy of the exchange for every path (several copies made the compiler keep the
     * by-value kernel argument in scratch) */
    if (xdo) g0_exchange_step<NT>(u, xep, N, ldg, xe0, xe1, xnt0, xmt0, TMF, xpf, xpg0, xpg12, xb, xc0, xc1);
    if ((long)blockIdx.x >= nb) mark(6);
}

template <int WF, int WH, int PD, int KW, bool HU8 = false, int WM = 2, int WN = 2>
int launch_fm(const void *Dg, const void *Hg, float hscale, float *slab, int ldg, int N, int M, int Bt, int splits,
              hipStream_t s, const TnTail &tail) {
    constexpr int TMF = 16 * WF * WM, TNH = 16 * WH * WN;
    const int tiles_n = N / TNH, tiles = (M / TMF) * tiles_n;
    const int xcd_map = (splits >= 8 && tiles > 1) ? 1 : 0;
    hipLaunchKernelGGL((gemm_fm_direct_kernel<WF, WH, PD, KW, HU8, WM, WN>), dim3(tiles * splits + tail.blocks),
                       dim3(64 * WM * WN * KW), 0, s, (const __bf16 *)Dg, N / 16, Hg, M / 16, hscale, slab, ldg, N,
                       Bt / 32, splits, tiles_n, tiles, xcd_map, tail);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* feature columns per workgroup tile of the 8-bit-input G0 (HPNN_G0_TILE=80 | 160) */
int g0_tile_m(int M) {
    static const int want = [] { const char *e = getenv("HPNN_G0_TILE"); return e ? atoi(e) : 80; }();
    return (want == 80 && M % 80 == 0) ? 80 : 160;
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
    if (N % 128 == 0 && g0_tile_m(M) == 80) { /* 80 x 128: four k-interleaved groups of 1 x 2 waves */
        return h_u8 ? launch_fm<5, 4, 1, 4, true, 1, 2>(Dg, Hg, hscale, slab, ldg, N, M, Bt, splits, s, t)
                    : launch_fm<5, 4, 1, 4, false, 1, 2>(Dg, Hg, hscale, slab, ldg, N, M, Bt, splits, s, t);
    }
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

/* the fused G0 grid (tiles x splits workgroups of 512 threads) fits on the device at once;
 * every instantiation checked (they differ in the operand conversion and the tile) */
static bool g0_fused_resident(int blocks) {
    static const int cap = [] {
        int c = hpnn_resident_capacity((const void *)g0_fused_kernel<5, 4, 1, 2, true>, 512, 0);
        for (const void *k : {(const void *)g0_fused_kernel<5, 4, 1, 2, false>,
                              (const void *)g0_fused_kernel<5, 4, 1, 4, true, false, 1, 2>,
                              (const void *)g0_fused_kernel<5, 4, 1, 4, false, false, 1, 2>}) {
            const int a = hpnn_resident_capacity(k, 512, 0);
            c = a < c ? a : c;
        }
        return c;
    }();
    return blocks <= cap;
}

static bool g0_fused_on() {
    static const bool on = [] { const char *e = getenv("HPNN_G0_FUSED"); return !(e && e[0] == '0'); }();
    return on;
}

/* the fused launch's tile (TMF feature columns x 128) for these operands */
static int g0_fused_tm(int h_u8, int M) {
    (void)h_u8;
    return g0_tile_m(M);
}

extern "C" int hpnn_g0_tile_cols(int M) { return g0_tile_m(M); }

extern "C" int hpnn_g0_tiles(int h_u8, int N, int M) {
    const int tm = g0_fused_tm(h_u8, M);
    return (M % tm || N % 128) ? 0 : (M / tm) * (N / 128);
}

extern "C" int hpnn_gemm_fm_direct_update(const void *Dg, const void *Hg, int h_u8, float hscale, float *slab,
                                          int ldg, int N, int M, int Bt, int splits, const hpnn_g0_update *u,
                                          hipStream_t stream) {
    /* the 8-wave tile configurations of fm_dispatch: 160 x 128, or 80 x 128 for 8-bit H */
    const int tm = g0_fused_tm(h_u8, M);
    if (!g0_fused_on() || !u || M % tm || N % 128 || Bt % 32 || splits < 1 || splits > Bt / 32 || ldg != M) return -1;
    if (!u->cnt || !u->err) return -1;
    const bool steps = !u->gout || u->xchg;
    if (u->n12 % 4 || !u->mslab || u->mrows < 1 || (steps && u->momentum && (!u->V32 || !u->V32b[0] || !u->V32b[1])))
        return -2;
    const int tiles_n = N / 128, tiles = (M / tm) * tiles_n;
    if (tiles > HPNN_G0_MAX_TILES) return -1; /* 64-bit counters 32 words apart, below the error word */
    /* every workgroup waits for the other splits of its tile: all must be resident at once
     * (more splits than that, e.g. forced by HPNN_TN_SPLITS, take the slab form instead of
     * stalling to the timeout) */
    if (!g0_fused_resident(tiles * splits)) return -1;
    /* tail workgroups for the [G1 | G2] share on the CUs the GEMM grid leaves idle (MNIST: 240
     * GEMM workgroups, 16 tails on a 256-CU MI355X); HPNN_G0_TAILS overrides the count (0: off),
     * HPNN_G0_TAIL12 the percentage of the [G1 | G2] columns they take (the GEMM workgroups sum
     * the rest after their publish) */
    static const int cus = [] {
        int dev = 0, n = 0;
        return hipGetDevice(&dev) == hipSuccess &&
                       hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess
                   ? n
                   : 0;
    }();
    static const int tails_env = [] { const char *e = getenv("HPNN_G0_TAILS"); return e ? atoi(e) : -1; }();
    static const int tail_pct = [] { const char *e = getenv("HPNN_G0_TAIL12"); return e ? atoi(e) : 100; }();
    /* one tail per 16 slab rows (each sums ~16 x the [G1 | G2] block, 563 KB on MNIST), at most
     * the CUs the GEMM grid leaves idle: ranks sharing one GPU (tests, rehearsals) keep their
     * grids small enough to co-run */
    int ntail = tails_env >= 0 ? tails_env : std::min(cus - tiles * splits, std::max(1, u->mrows / 16));
    if (ntail < 0 || tail_pct <= 0) ntail = 0;
    if (ntail > 64) ntail = 64;
    while (ntail > 0 && !g0_fused_resident(tiles * splits + ntail)) ntail--;
    if (u->xchg && tiles * splits + ntail > HPNN_XAR_MAX_BLOCKS) ntail = HPNN_XAR_MAX_BLOCKS - tiles * splits;
    if (ntail < 0) ntail = 0;
    if (u->xchg) {
        /* the exchange buffer holds [G0 | G1 | G2]; one epoch / flag slot per workgroup */
        if (tiles * splits + ntail > HPNN_XAR_MAX_BLOCKS || u->xv.world < 1 || u->xv.world > HPNN_XAR_MAX_RANKS ||
            !u->xv.ep || (long)N * ldg + u->n12 > u->xv.half)
            return -1;
        for (int p = 0; p < u->xv.world; p++)
            if (!u->xv.buf[p] || !u->xv.sig[p]) return -1;
    }
    const int xcd_map = (splits >= 8 && tiles > 1) ? 1 : 0;
    hpnn_g0_update uu = *u;
    uu.n12t = ntail ? ((long)(u->n12 / 4) * (tail_pct > 100 ? 100 : tail_pct) / 100) * 4 : 0;
#ifdef HPNN_ABLATIONS
    static const int proto = [] { const char *e = getenv("HPNN_G0_PROTO"); return e ? atoi(e) : 0; }();
    uu.proto |= proto;
#endif
    static const bool trace = [] { const char *e = getenv("HPNN_G0_TRACE"); return e && e[0] == '1'; }();
#define HPNN_G0F(...)                                                                                              \
    hipLaunchKernelGGL((g0_fused_kernel<__VA_ARGS__>), dim3(tiles * splits + ntail), dim3(512), 0, stream,           \
                       (const __bf16 *)Dg,                                                                         \
                       N / 16, Hg, M / 16, hscale, slab, ldg, N, Bt / 32, splits, tiles_n, tiles, xcd_map, uu)
    if (tm == 80) {
        /* HPNN_G0_PD=2 (ABLATIONS builds, tuning): two k-steps of operands in flight */
#ifdef HPNN_ABLATIONS
        static const int pd = [] { const char *e = getenv("HPNN_G0_PD"); return e ? atoi(e) : 1; }();
        static const bool x16 = [] { const char *e = getenv("HPNN_G0_X16"); return e && e[0] == '1'; }();
        if (h_u8 && pd == 2) HPNN_G0F(5, 4, 2, 4, true, false, 1, 2);
        else if (h_u8 && x16) HPNN_G0F(5, 4, 1, 4, true, false, 1, 2, true);
        else
#endif
        if (h_u8 && trace) HPNN_G0F(5, 4, 1, 4, true, true, 1, 2);
        else if (h_u8) HPNN_G0F(5, 4, 1, 4, true, false, 1, 2);
        else HPNN_G0F(5, 4, 1, 4, false, false, 1, 2);
    } else if (h_u8 && trace) HPNN_G0F(5, 4, 1, 2, true, true);
    else if (h_u8) HPNN_G0F(5, 4, 1, 2, true, false);
    else HPNN_G0F(5, 4, 1, 2, false, false);
#undef HPNN_G0F
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_gemm_fm_direct_update_ok(int ldg, int N, int M, int Bt, int splits) {
    const int tiles = hpnn_g0_tiles(1, N, M);
    if (!(g0_fused_on() && tiles > 0 && Bt % 32 == 0 && splits >= 1 && splits <= Bt / 32 && ldg == M &&
          tiles <= HPNN_G0_MAX_TILES))
        return 0;
    return g0_fused_resident(tiles * splits) ? 1 : 0;
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

/* HPNN_G0_TRACE=1 stamps: out[512][8] shader-clock ticks (thread 0 of each workgroup) */
extern "C" int hpnn_g0_trace(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_g0_trace), sizeof(g_g0_trace)) == hipSuccess ? 0 : -5;
}
