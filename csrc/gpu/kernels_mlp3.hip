/*
 * Fused kernels for the 3-weight-layer bias-free MLP (the MNIST-shaped headline
 * network n_in -> 128 -> 64 -> n_out<=32, SNN/ANN/LNN), gfx950.
 *
 * The per-layer path (kernels_mfma.hip) round-trips every activation and delta
 * through HBM and launches ~11 kernels per step.  Here one step is
 *   1. gemm_nt (X . W0^T, bipolar)           -> H1        [B x 128]  (pipelined MFMA)
 *   2. mlp3_mid (this file)                   : H1 -> H2 -> output -> delta3 -> delta2
 *                                              -> delta1 (stored), plus the G1 / G2 weight
 *                                              gradients of the block's samples
 *   3. gemm_tn (delta1^T . X)                -> G0 split-K slabs
 *   4. optimizer (slab reduce + BP/BPM + BF16 W / W^T refresh)
 *
 * mlp3_mid: 256 threads (4 waves), 64-sample tiles, ~72 KiB LDS -> 2 workgroups per
 * CU so one block's barrier / LDS waits overlap the other's MFMA work.  W1 and W2
 * stay in LDS for the whole launch; their transposes are never stored, the
 * delta GEMMs read them column-wise with ds_read_b64_tr_b16.  The next tile's H1
 * lands by LDS-DMA while the current one is processed.  H2 / delta3 / delta2 live
 * only in LDS; G1 / G2 accumulate in registers across the block's tiles (one FP32
 * slab per block).  Every LDS address is a per-lane constant computed once plus a
 * compile-time immediate (the first version spent most of its VALU budget on
 * address arithmetic and was VALU-bound, see profiles/).  HBM traffic per sample:
 * H1 in (256 B) + delta1 out (256 B).
 *
 * Reference math: SURVEY 2.4 (ann.c:883-888, 1279-1592; snn.c:280-335, 481-794).
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include "kernels.h"

HPNN_CO_PROBE(mlp3)
#include "mfma_common.h"
#include "mlp3_common.h"

using namespace hpnn;
using namespace hpnn::mlp3;

namespace {

constexpr int BM = 64;    /* samples per tile */
constexpr int NW = 4;     /* waves per block  */

/* LDS carve (bytes); every image is a T32 image (mfma_common.h) */
constexpr int IMG_H1 = BM * H1 * 2;  /* x2: DMA ring            */
constexpr int IMG_H2 = BM * H2 * 2;
constexpr int IMG_D3 = BM * NO * 2;
constexpr int IMG_D2 = BM * H2 * 2;
constexpr int OFF_H1 = 0;
constexpr int OFF_W1 = OFF_H1 + 2 * IMG_H1;
constexpr int OFF_W2 = OFF_W1 + IMG_W1;
constexpr int OFF_H2 = OFF_W2 + IMG_W2;
constexpr int OFF_D3 = OFF_H2 + IMG_H2;
constexpr int OFF_D2 = OFF_D3 + IMG_D3;
constexpr int OFF_RED = OFF_D2 + IMG_D2;
constexpr int LDS_TOTAL = OFF_RED + 64;
static_assert(LDS_TOTAL <= 80 * 1024, "two workgroups per CU");

template <int R, int C>
__device__ __forceinline__ void load_img(const __bf16 *g, int ld, char *img, int wave, int lane) {
    constexpr int PIECES = (C / 32) * (R / 16);
    static_assert(PIECES % NW == 0, "even DMA split");
#pragma unroll
    for (int p = wave; p < PIECES; p += NW) glds_t32_piece<R>((const char *)g, (size_t)ld * 2, img, p, lane);
}

/* TYPE: 0 ANN, 1 LNN, 2 SNN; LABELS: one-hot targets from int labels */
template <int TYPE, bool LABELS>
__global__ __launch_bounds__(256, 2) void mlp3_mid_kernel(const __bf16 *__restrict__ Hg, const __bf16 *__restrict__ W1,
                                                          const __bf16 *__restrict__ W2, const int *__restrict__ labels,
                                                          const float *__restrict__ T, int ldt, float t_hi,
                                                          float t_lo, __bf16 *__restrict__ D1,
                                                          float *__restrict__ gslab, float *__restrict__ loss_acc,
                                                          unsigned int *__restrict__ correct, int n_tiles,
                                                          int n_valid, int n_out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const LaneOff lo = lane_offsets(lane);
    char *imgW1 = lds + OFF_W1, *imgW2 = lds + OFF_W2;
    char *imgH2 = lds + OFF_H2, *imgD3 = lds + OFF_D3, *imgD2 = lds + OFF_D2;

    load_img<H2, H1>(W1, H1, imgW1, wave, lane);
    load_img<NO, H2>(W2, H2, imgW2, wave, lane);
    int tile = blockIdx.x;
    if (tile < n_tiles) load_img<BM, H1>(Hg + (size_t)tile * BM * H1, H1, lds + OFF_H1, wave, lane);
    int lab_cur = -1;
    if (LABELS && tile < n_tiles) {
        const int s = tile * BM + wave * 16 + r16;
        const int *addr = labels + (s < n_valid ? s : (n_valid > 0 ? n_valid - 1 : 0));
        asm volatile("global_load_dword %0, %1, off" : "=v"(lab_cur) : "v"(addr) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(lab_cur)::"memory");
    lds_barrier();

    /* per-lane output-column mask (c < n_out): c = 16 ot + 4 q + r */
    float cmask[2][4];
#pragma unroll
    for (int ot = 0; ot < 2; ot++)
#pragma unroll
        for (int r = 0; r < 4; r++) cmask[ot][r] = (ot * 16 + 4 * q + r < n_out) ? 1.f : 0.f;
    const int n_ot = n_out > 16 ? 2 : 1;

    f32x4 g1acc[2][4]; /* G1: h1 tiles 2w, 2w+1 ; h2 tiles 0..3 */
    f32x4 g2acc[2];    /* G2: h2 tile w ; o tiles 0, 1          */
#pragma unroll
    for (int i = 0; i < 2; i++) {
        g2acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; j++) g1acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float my_loss = 0.f;
    unsigned int my_hit = 0;

    int buf = 0;
    for (; tile < n_tiles; tile += gridDim.x, buf ^= 1) {
        char *imgH1 = lds + OFF_H1 + buf * IMG_H1;
        const int s0 = tile * BM;
        const int nt = tile + gridDim.x;
        /* next tile: labels (inline asm, so no compiler vmcnt(0) drains the DMA) then H1 */
        int lab_next = -1;
        if (LABELS && nt < n_tiles) {
            int s = nt * BM + wave * 16 + r16;
            s = s < n_valid ? s : (n_valid > 0 ? n_valid - 1 : 0);
            const int *addr = labels + s;
            asm volatile("global_load_dword %0, %1, off" : "=v"(lab_next) : "v"(addr) : "memory");
        }
        if (nt < n_tiles) load_img<BM, H1>(Hg + (size_t)nt * BM * H1, H1, lds + OFF_H1 + (buf ^ 1) * IMG_H1, wave, lane);

        /* ---- P1: H2 = f(H1 . W1^T) [64 x 64]; wave: h2 tile w, sample tiles 0..3 ---- */
        {
            f32x4 acc[4];
#pragma unroll
            for (int j = 0; j < 4; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H1; k += 32) {
                const bf16x8 a = rd_row<H2>(imgW1, lo, wave * 16, k);
#pragma unroll
                for (int j = 0; j < 4; j++) acc[j] = mfma(a, rd_row<BM>(imgH1, lo, j * 16, k), acc[j]);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)bipolar(acc[j][r]);
                *(bf16x4 *)wr_ptr<BM>(imgH2, lo, j * 16, wave * 16) = o;
            }
        }
        lds_barrier();

        /* ---- P2: output layer, samples [16w, 16w+16): logits, loss, delta3 ---- */
        {
            f32x4 z[2];
            z[0] = z[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H2; k += 32) {
                const bf16x8 b = rd_row<BM>(imgH2, lo, wave * 16, k);
                z[0] = mfma(rd_row<NO>(imgW2, lo, 0, k), b, z[0]);
                if (n_ot > 1) z[1] = mfma(rd_row<NO>(imgW2, lo, 16, k), b, z[1]);
            }
            const int s = s0 + wave * 16 + r16;
            const bool valid = s < n_valid;
            const int lab = lab_cur;
            /* masked max of the logits of this sample (4 lanes q share it) */
            float zmax = -INFINITY;
#pragma unroll
            for (int ot = 0; ot < 2; ot++)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (cmask[ot][r] != 0.f) zmax = fmaxf(zmax, z[ot][r]);
            zmax = rows_max(zmax);
            float inv = 0.f;
            float e[2][4];
            if constexpr (TYPE == 2) {
                float den = 0.f;
#pragma unroll
                for (int ot = 0; ot < 2; ot++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        e[ot][r] = __expf(z[ot][r] - zmax) * cmask[ot][r];
                        den += e[ot][r];
                    }
                den = rows_sum(den);
                /* reference e^{z-1}/(TINY + sum e^{z-1}) in the max-shifted form; ln(1e-14) */
                den += __expf(fminf(-32.236191301916641f + 1.0f - zmax, 80.f));
                inv = __builtin_amdgcn_rcpf(den);
            }
            float l = 0.f;
            unsigned int hit = 0;
            float tt[2][4];
            if constexpr (!LABELS) {
#pragma unroll
                for (int ot = 0; ot < 2; ot++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int c = ot * 16 + 4 * q + r;
                        tt[ot][r] = (valid && c < n_out) ? T[(size_t)s * ldt + c] : 0.f;
                    }
            }
            float bt = -INFINITY, zt = -INFINITY; /* dense targets: max target and its logit */
            int ibt = 1 << 30;
#pragma unroll
            for (int ot = 0; ot < 2; ot++) {
                bf16x4 dv;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int c = ot * 16 + 4 * q + r;
                    float t;
                    if constexpr (LABELS) t = (c == lab) ? t_hi : t_lo;
                    else t = tt[ot][r];
                    float o;
                    if constexpr (TYPE == 2) o = e[ot][r] * inv;
                    else if constexpr (TYPE == 0) o = bipolar(z[ot][r]);
                    else o = z[ot][r];
                    float d;
                    if constexpr (TYPE == 0) d = (t - o) * dbipolar(o);
                    else d = t - o;
                    const float m = valid ? cmask[ot][r] : 0.f;
                    d *= m;
                    if constexpr (TYPE == 2) {
                        if (m != 0.f && t != 0.f && o > 0.f) l += t * __logf(o + TINY);
                    } else {
                        l += m * (t - o) * (t - o);
                    }
                    if constexpr (LABELS) {
                        if (c == lab && z[ot][r] >= zmax) hit = 1u;
                    } else {
                        if (m != 0.f && (t > bt || (t == bt && c < ibt))) {
                            bt = t;
                            ibt = c;
                            zt = z[ot][r];
                        }
                    }
                    dv[r] = (__bf16)d;
                }
                *(bf16x4 *)wr_ptr<BM>(imgD3, lo, wave * 16, ot * 16) = dv;
            }
            if constexpr (!LABELS) {
                /* hit iff the logit of the (first) max-target column is the max logit */
#pragma unroll
                for (int off = 16; off <= 32; off <<= 1) {
                    const float ob = __shfl_xor(bt, off, 64), oz = __shfl_xor(zt, off, 64);
                    const int oi = __shfl_xor(ibt, off, 64);
                    if (ob > bt || (ob == bt && oi < ibt)) {
                        bt = ob;
                        ibt = oi;
                        zt = oz;
                    }
                }
                hit = (q == 0 && zt >= zmax) ? 1u : 0u;
            }
            l = rows_sum(l);
            if (valid) {
                if (q == 0) my_loss += (TYPE == 2) ? -l / (float)n_out : 0.5f * l;
                my_hit += hit;
            }
        }
        lds_barrier();

        /* ---- P3: delta2 = (delta3 . W2) * f'(H2) [64 x 64]; wave: h2 tile w ---- */
        {
            f32x4 acc[4];
#pragma unroll
            for (int j = 0; j < 4; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
            const bf16x8 a = rd_tr<NO>(imgW2, lo, 0, wave * 16); /* A[h2][o] = W2[o][h2] */
#pragma unroll
            for (int j = 0; j < 4; j++) acc[j] = mfma(a, rd_row<BM>(imgD3, lo, j * 16, 0), acc[j]);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bf16x4 h = *(const bf16x4 *)wr_ptr<BM>(imgH2, lo, j * 16, wave * 16);
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)(acc[j][r] * dbipolar((float)h[r]));
                *(bf16x4 *)wr_ptr<BM>(imgD2, lo, j * 16, wave * 16) = o;
            }
        }
        lds_barrier();

        /* ---- P4: delta1 = (delta2 . W1) * f'(H1) -> global; wave: h1 tiles 2w, 2w+1 ---- */
        {
            f32x4 acc[2][4];
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H2; k += 32) {
                bf16x8 b[4];
#pragma unroll
                for (int j = 0; j < 4; j++) b[j] = rd_row<BM>(imgD2, lo, j * 16, k);
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const bf16x8 a = rd_tr<H2>(imgW1, lo, k, (2 * wave + i) * 16); /* A[h1][h2] = W1[h2][h1] */
#pragma unroll
                    for (int j = 0; j < 4; j++) acc[i][j] = mfma(a, b[j], acc[i][j]);
                }
            }
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int f = (2 * wave + i) * 16 + 4 * q;
                    const bf16x4 h = *(const bf16x4 *)wr_ptr<BM>(imgH1, lo, j * 16, (2 * wave + i) * 16);
                    bf16x4 o;
#pragma unroll
                    for (int r = 0; r < 4; r++) o[r] = (__bf16)(acc[i][j][r] * dbipolar((float)h[r]));
                    *(bf16x4 *)(D1 + (size_t)(s0 + j * 16 + r16) * H1 + f) = o;
                }
        }
        /* ---- P5: G2 += delta3^T . H2  ([o][h2], k = samples); wave: h2 tile w ---- */
#pragma unroll
        for (int k = 0; k < BM; k += 32) {
            const bf16x8 a = rd_tr<BM>(imgH2, lo, k, wave * 16);
            g2acc[0] = mfma(a, rd_tr<BM>(imgD3, lo, k, 0), g2acc[0]);
            if (n_ot > 1) g2acc[1] = mfma(a, rd_tr<BM>(imgD3, lo, k, 16), g2acc[1]);
        }
        /* ---- P6: G1 += delta2^T . H1  ([h2][h1]); wave: h1 tiles 2w, 2w+1 ---- */
#pragma unroll
        for (int k = 0; k < BM; k += 32) {
            bf16x8 b[4];
#pragma unroll
            for (int t = 0; t < 4; t++) b[t] = rd_tr<BM>(imgD2, lo, k, t * 16);
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const bf16x8 a = rd_tr<BM>(imgH1, lo, k, (2 * wave + i) * 16);
#pragma unroll
                for (int t = 0; t < 4; t++) g1acc[i][t] = mfma(a, b[t], g1acc[i][t]);
            }
        }
        /* next tile's H1 + labels landed; this tile's delta1 stores drained */
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(lab_next)::"memory");
        lab_cur = lab_next;
        lds_barrier();
    }

    /* ---- per-block gradient slab [G1 (H2 x H1) | G2 (NO x H2)] ---- */
    float *slab = gslab + (size_t)blockIdx.x * SLAB;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int t = 0; t < 4; t++) /* D[h1 = 16(2w+i) + 4q + r][h2 = 16t + r16] */
            *(f32x4 *)(slab + (size_t)(t * 16 + r16) * H1 + (2 * wave + i) * 16 + 4 * q) = g1acc[i][t];
#pragma unroll
    for (int ot = 0; ot < 2; ot++) /* D[h2 = 16w + 4q + r][o = 16 ot + r16] */
        *(f32x4 *)(slab + H2 * H1 + (size_t)(ot * 16 + r16) * H2 + wave * 16 + 4 * q) = g2acc[ot];
    /* loss / accuracy: one atomic per block */
    float *sl = (float *)(lds + OFF_RED);
    unsigned int *sh = (unsigned int *)(lds + OFF_RED + 32);
    my_loss = wave_sum(my_loss);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) my_hit += __shfl_xor(my_hit, o, 64);
    if (lane == 0) {
        sl[wave] = my_loss;
        sh[wave] = my_hit;
    }
    __syncthreads();
    if (tid == 0) {
        float a = 0.f;
        unsigned int h = 0;
        for (int w = 0; w < NW; w++) {
            a += sl[w];
            h += sh[w];
        }
        if (loss_acc) atomicAdd(loss_acc + HPNN_STAT_SLOT(blockIdx.x), a);
        if (correct) atomicAdd(correct + HPNN_STAT_SLOT(blockIdx.x), h);
    }
}

/* Slab reduction: out[g*ostride + i] = sum of slabs [g*SG, min(S,(g+1)*SG)) (grid.y =
 * groups).  Two passes (groups -> 1) keep many loads in flight and stay deterministic. */
__global__ __launch_bounds__(256) void reduce_groups_kernel(const float *__restrict__ slab, int S, int SG, long stride,
                                                            long n4, float *__restrict__ out, long ostride) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    const int g = blockIdx.y;
    if (e >= n4) return;
    const int s_end = min(S, (g + 1) * SG);
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    int s = g * SG;
    for (; s + 3 < s_end; s += 4) {
        a0 += ((const f32x4 *)(slab + (long)s * stride))[e];
        a1 += ((const f32x4 *)(slab + (long)(s + 1) * stride))[e];
        a2 += ((const f32x4 *)(slab + (long)(s + 2) * stride))[e];
        a3 += ((const f32x4 *)(slab + (long)(s + 3) * stride))[e];
    }
    for (; s < s_end; s++) a0 += ((const f32x4 *)(slab + (long)s * stride))[e];
    ((f32x4 *)(out + (long)g * ostride))[e] = (a0 + a1) + (a2 + a3);
}


}  // namespace

extern "C" int hpnn_mlp3_mid(const void *H1g, const void *W1, const void *W1t, const void *W2, const void *W2t,
                             const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1,
                             float *gslab, float *loss_acc, unsigned int *correct, int Bp, int n_valid, int n_out,
                             int type, int h1, int h2, int no, int grid, hipStream_t stream) {
    (void)W1t;
    (void)W2t;
    if (h1 != H1 || h2 != H2 || no != NO) return -2;
    if (Bp % BM || n_out > NO || n_out < 1) return -2;
    if (!labels && !T) return -1;
    const int n_tiles = Bp / BM;
    if (grid <= 0 || grid > n_tiles) grid = n_tiles;
#define HPNN_MID(TY, LB)                                                                                          \
    do {                                                                                                          \
        static bool attr = false;                                                                                 \
        if (!attr) {                                                                                              \
            (void)hipFuncSetAttribute((const void *)mlp3_mid_kernel<TY, LB>,                                      \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL);                     \
            attr = true;                                                                                          \
        }                                                                                                         \
        hipLaunchKernelGGL((mlp3_mid_kernel<TY, LB>), dim3(grid), dim3(256), LDS_TOTAL, stream,                   \
                           (const __bf16 *)H1g, (const __bf16 *)W1, (const __bf16 *)W2, labels, T, ldt, t_hi, t_lo, \
                           (__bf16 *)D1, gslab, loss_acc, correct, n_tiles, n_valid, n_out);                     \
    } while (0)
    if (labels) {
        if (type == 2) HPNN_MID(2, true);
        else if (type == 0) HPNN_MID(0, true);
        else HPNN_MID(1, true);
    } else {
        if (type == 2) HPNN_MID(2, false);
        else if (type == 0) HPNN_MID(0, false);
        else HPNN_MID(1, false);
    }
#undef HPNN_MID
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_mlp3_slab_floats(void) { return SLAB; }

/* out[i] = sum_s slab[s*stride + i]: groups of slabs into tmp (>= groups*n floats),
 * then the groups; tmp == NULL or few slabs -> one pass */
extern "C" int hpnn_reduce_slabs2(const float *slab, int S, long stride, long n, float *tmp, float *out,
                                  hipStream_t stream) {
    if (n % 4 || stride % 4 || S < 1) return -2;
    const long n4 = n / 4;
    const int groups = (!tmp || S < 16) ? 1 : (S >= 64 ? 16 : 4);
    const unsigned bx = (unsigned)((n4 + 255) / 256);
    if (groups == 1) {
        hipLaunchKernelGGL(reduce_groups_kernel, dim3(bx, 1), dim3(256), 0, stream, slab, S, S, stride, n4, out, 0L);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    const int SG = (S + groups - 1) / groups;
    hipLaunchKernelGGL(reduce_groups_kernel, dim3(bx, groups), dim3(256), 0, stream, slab, S, SG, stride, n4, tmp, n);
    hipLaunchKernelGGL(reduce_groups_kernel, dim3(bx, 1), dim3(256), 0, stream, (const float *)tmp, groups, groups, n,
                       n4, out, 0L);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* first pass only: out[g*n + i] = sum of slabs [g*ceil(S/groups), ...) -- the optimizer
 * (hpnn_sgd_update_multi with S = groups, gstride = n) sums the groups itself */
extern "C" int hpnn_reduce_groups(const float *slab, int S, long stride, long n, int groups, float *out,
                                  hipStream_t stream) {
    if (n % 4 || stride % 4 || S < 1 || groups < 1 || groups > S) return -2;
    const long n4 = n / 4;
    const unsigned bx = (unsigned)((n4 + 255) / 256);
    const int SG = (S + groups - 1) / groups;
    hipLaunchKernelGGL(reduce_groups_kernel, dim3(bx, groups), dim3(256), 0, stream, slab, S, SG, stride, n4, out, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
