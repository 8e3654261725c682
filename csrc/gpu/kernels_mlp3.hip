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

#include "kernels.h"
#include "mfma_common.h"

using namespace hpnn;

namespace {

constexpr float TINY = 1e-14f;
constexpr int BM = 64;    /* samples per tile */
constexpr int NW = 4;     /* waves per block  */
constexpr int H1 = 128, H2 = 64, NO = 32;

/* LDS carve (bytes); every image is a T32 image (mfma_common.h) */
constexpr int IMG_H1 = BM * H1 * 2;  /* x2: DMA ring            */
constexpr int IMG_W1 = H2 * H1 * 2;  /* [H2 rows][H1 cols]      */
constexpr int IMG_W2 = NO * H2 * 2;  /* [NO rows][H2 cols]      */
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
constexpr int SLAB = H2 * H1 + NO * H2; /* floats per block slab: [G1 | G2] */

/* per-lane constant parts of T32 addresses (see t32<> in mfma_common.h) */
struct LaneOff {
    int row; /* frag_row : + (col0>>5)*R*64 + r0*64                (r0%16==0, col0%32==0) */
    int tr;  /* frag_tr  : + (c0>>5)*R*64 + kbase*64, ^32 if (c0>>4)&1; +256 for rows + 4 */
    int wr;  /* D tile   : + (c0>>5)*R*64 + r0*64, ^32 if (c0>>4)&1                        */
};
__device__ __forceinline__ LaneOff lane_offsets(int lane) {
    const int l15 = lane & 15, q = lane >> 4;
    const int g = t32_g(l15);
    LaneOff o;
    o.row = l15 * 64 + ((q ^ g) << 4);
    const int gg = lane >> 4, qq = (lane & 15) >> 2, p = lane & 3;
    const int G = ((qq >> 1) & 1) | ((gg & 1) << 1);
    o.tr = (8 * gg + qq) * 64 + ((((p >> 1) ^ G) & 3) << 4) + 8 * (p & 1);
    o.wr = l15 * 64 + ((((q >> 1) ^ g) & 3) << 4) + 8 * (q & 1);
    return o;
}

template <int R>
__device__ __forceinline__ bf16x8 rd_row(const char *img, const LaneOff &lo, int r0, int col0) {
    return *(const bf16x8 *)(img + (col0 >> 5) * (R * 64) + r0 * 64 + lo.row);
}
template <int R>
__device__ __forceinline__ bf16x8 rd_tr(const char *img, const LaneOff &lo, int kbase, int c0) {
    const char *b = img + (c0 >> 5) * (R * 64) + kbase * 64 + (lo.tr ^ (((c0 >> 4) & 1) << 5));
    s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)b);
    s16x4 c = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(b + 256));
    s16x8 v = {a[0], a[1], a[2], a[3], c[0], c[1], c[2], c[3]};
    return __builtin_bit_cast(bf16x8, v);
}
/* the 8 bytes (4 bf16) a lane owns in the 16x16 D tile at (r0, c0) */
template <int R>
__device__ __forceinline__ char *wr_ptr(char *img, const LaneOff &lo, int r0, int c0) {
    return img + (c0 >> 5) * (R * 64) + r0 * 64 + (lo.wr ^ (((c0 >> 4) & 1) << 5));
}

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
            zmax = fmaxf(zmax, __shfl_xor(zmax, 16, 64));
            zmax = fmaxf(zmax, __shfl_xor(zmax, 32, 64));
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
                den += __shfl_xor(den, 16, 64);
                den += __shfl_xor(den, 32, 64);
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
            l += __shfl_xor(l, 16, 64);
            l += __shfl_xor(l, 32, 64);
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


/* ====================================================================== */
/* mlp3_fused: X -> delta1 in one persistent kernel                        */
/* ====================================================================== */
/* 512 threads (8 waves, 2 per SIMD), one workgroup per CU, 32-sample tiles.
 *   W0 (128 x K0) lives in VGPRs for the whole launch: wave w holds the A-operand
 *   fragments of neurons [16w, 16w+16) for all K0 (K0/8 registers per lane), read
 *   once from the fragment-major copy W0f (1 KiB contiguous per load).
 *   X tiles stream by LDS-DMA into a 2-slot ring of 128-byte-row images; the slot of
 *   tile i is refilled with tile i+2 as soon as the layer-0 product of tile i is done,
 *   so two tiles (~100 KiB) are in flight during the rest of the tile's work.
 *   H1, H2, delta3, delta2 never leave LDS; delta1 goes to HBM (the G0 GEMM needs it).
 * Memory-counter discipline (one counted s_waitcnt per tile, never vmcnt(0) in the
 * loop): per tile every wave issues, in this order, the label copy of tile i+1 (LDS-DMA
 * into a 2-slot LDS buffer), its 2 delta1 stores, then its LPS X pieces of tile i+2.
 * At the top of tile i+1 the ops younger than label(i+1) are exactly those 2 stores
 * plus tile i+2's pieces. */
constexpr int FR = 32;  /* samples per tile */
constexpr int FNW = 8;  /* waves */
template <int KS>
struct FLay {
    static constexpr int XST = FR * KS * 32 * 2;
    static constexpr int OFF_W1 = 2 * XST;
    static constexpr int OFF_W2 = OFF_W1 + IMG_W1;
    static constexpr int OFF_H1 = OFF_W2 + IMG_W2;
    static constexpr int OFF_H2 = OFF_H1 + FR * H1 * 2;
    static constexpr int OFF_D3 = OFF_H2 + FR * H2 * 2;
    static constexpr int OFF_D2 = OFF_D3 + FR * NO * 2;
    static constexpr int OFF_LAB = OFF_D2 + FR * H2 * 2; /* 2 slots x 64 int labels */
    static constexpr int OFF_RED = OFF_LAB + 2 * 256;
    static constexpr int TOTAL = OFF_RED + 128;
    static_assert(TOTAL <= 160 * 1024, "LDS");
};

template <int R, int C>
__device__ __forceinline__ void load_img_w(const __bf16 *g, int ld, char *img, int wave, int lane) {
    constexpr int PIECES = (C / 32) * (R / 16);
    for (int p = wave; p < PIECES; p += FNW) glds_t32_piece<R>((const char *)g, (size_t)ld * 2, img, p, lane);
}

__device__ __forceinline__ int clamp_sample(int s, int n_valid) { return s < n_valid ? s : (n_valid > 0 ? n_valid - 1 : 0); }

template <int TYPE, bool LABELS, int KS>
__global__ __launch_bounds__(512, 1) void mlp3_fused_kernel(const __bf16 *__restrict__ X, int ldx,
                                                            const __bf16 *__restrict__ W0f,
                                                            const __bf16 *__restrict__ W1,
                                                            const __bf16 *__restrict__ W2,
                                                            const int *__restrict__ labels,
                                                            const float *__restrict__ T, int ldt, float t_hi,
                                                            float t_lo, __bf16 *__restrict__ D1,
                                                            float *__restrict__ gslab, float *__restrict__ loss_acc,
                                                            unsigned int *__restrict__ correct, int n_tiles,
                                                            int n_valid, int n_out) {
    using LY = FLay<KS>;
    constexpr int R = FR;
    constexpr int S64 = KS / 2, TAIL = KS & 1;
    constexpr int XPIECES = S64 * (R / 8) + TAIL * (R / 16);
    constexpr int LPS = (XPIECES + FNW - 1) / FNW;
    static_assert(LPS + 2 < 64, "vmcnt budget");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const LaneOff lo = lane_offsets(lane);
    char *imgW1 = lds + LY::OFF_W1, *imgW2 = lds + LY::OFF_W2, *imgH1 = lds + LY::OFF_H1;
    char *imgH2 = lds + LY::OFF_H2, *imgD3 = lds + LY::OFF_D3, *imgD2 = lds + LY::OFF_D2;
    const int G = gridDim.x;
    const int nloc = (n_tiles - (int)blockIdx.x + G - 1) / G;
    const size_t ldx_b = (size_t)ldx * 2;
    const int ht = wave & 3, hs = wave >> 2; /* (h2 tile | o tile, sample group) for 8-tile phases */

    auto issue_x = [&](int slot, int i) {
        const char *g = (const char *)(X + (size_t)(blockIdx.x + i * G) * R * ldx);
        char *img = lds + slot * LY::XST;
#pragma unroll
        for (int p = 0; p < LPS; p++) {
            int c = wave + FNW * p;
            c = c < XPIECES ? c : XPIECES - 1;
            glds_x_piece<R, S64>(g, ldx_b, img, c, lane);
        }
    };
    /* labels of tile i -> LDS slot i&1 by LDS-DMA (lane l: sample l of the tile, clamped);
     * every wave issues the same copy so the per-wave vm-op counts stay uniform */
    auto load_label = [&](int i) {
        if constexpr (LABELS) {
            const int s = clamp_sample((blockIdx.x + i * G) * R + (lane & 31), n_valid);
            glds4(labels + s, lds + LY::OFF_LAB + (i & 1) * 256);
        }
    };

    /* prologue: X(0), weights, label(0); one full wait the compiler can see (so it adds
     * no drain of its own at the first use of the W0 registers); then X(1) */
    issue_x(0, 0);
    bf16x8 w0[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ks++) w0[ks] = *(const bf16x8 *)(W0f + ((size_t)(wave * KS + ks) * 64 + lane) * 8);
    load_img_w<H2, H1>(W1, H1, imgW1, wave, lane);
    load_img_w<NO, H2>(W2, H2, imgW2, wave, lane);
    load_label(0);
    __builtin_amdgcn_s_waitcnt(0xF70); /* vmcnt(0) */
    if (nloc > 1) issue_x(1, 1);

    float cmask[2][4];
#pragma unroll
    for (int ot = 0; ot < 2; ot++)
#pragma unroll
        for (int r = 0; r < 4; r++) cmask[ot][r] = (ot * 16 + 4 * q + r < n_out) ? 1.f : 0.f;
    const int n_ot = n_out > 16 ? 2 : 1;

    f32x4 g1acc[4], g2acc;
    g2acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; t++) g1acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float my_loss = 0.f;
    unsigned int my_hit = 0;

    for (int i = 0; i < nloc; i++) {
        const int s0 = (blockIdx.x + i * G) * R;
        char *imgX = lds + (i & 1) * LY::XST;
        /* X(i) and label(i) landed; younger ops may stay in flight */
        if (i == 0) {
            if (nloc > 1) wait_vm<LPS>();
            else wait_vm<0>();
        } else {
            if (i + 1 < nloc) wait_vm<LPS + 2>();
            else wait_vm<2>();
        }
        lds_barrier();

        /* ---- P0: H1 = f(X . W0^T) [32 x 128]; wave: neurons [16w, 16w+16), both sample groups ---- */
        {
            f32x4 acc[2];
            acc[0] = acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
            bf16x8 xc[2], xn[2];
            xc[0] = x_frag<R, S64>(imgX, 0, 0, lane);
            xc[1] = x_frag<R, S64>(imgX, 16, 0, lane);
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                if (ks + 1 < KS) {
                    xn[0] = x_frag<R, S64>(imgX, 0, ks + 1, lane);
                    xn[1] = x_frag<R, S64>(imgX, 16, ks + 1, lane);
                }
                acc[0] = mfma(w0[ks], xc[0], acc[0]);
                acc[1] = mfma(w0[ks], xc[1], acc[1]);
                xc[0] = xn[0];
                xc[1] = xn[1];
            }
#pragma unroll
            for (int sg = 0; sg < 2; sg++) {
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)bipolar(acc[sg][r]);
                *(bf16x4 *)wr_ptr<R>(imgH1, lo, sg * 16, wave * 16) = o;
            }
        }
        lds_barrier();

        /* ---- P1: H2 = f(H1 . W1^T) [32 x 64]; wave: h2 tile ht, sample group hs ---- */
        {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H1; k += 32) acc = mfma(rd_row<H2>(imgW1, lo, ht * 16, k), rd_row<R>(imgH1, lo, hs * 16, k), acc);
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; r++) o[r] = (__bf16)bipolar(acc[r]);
            *(bf16x4 *)wr_ptr<R>(imgH2, lo, hs * 16, ht * 16) = o;
        }
        lds_barrier();

        /* ---- P2: output layer; waves 0, 1: samples [16w, 16w+16) ---- */
        if (wave < 2) {
            f32x4 z[2];
            z[0] = z[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H2; k += 32) {
                const bf16x8 b = rd_row<R>(imgH2, lo, wave * 16, k);
                z[0] = mfma(rd_row<NO>(imgW2, lo, 0, k), b, z[0]);
                if (n_ot > 1) z[1] = mfma(rd_row<NO>(imgW2, lo, 16, k), b, z[1]);
            }
            const int s = s0 + wave * 16 + r16;
            const bool valid = s < n_valid;
            const int lab = LABELS ? ((const int *)(lds + LY::OFF_LAB + (i & 1) * 256))[wave * 16 + r16] : -1;
            float zmax = -INFINITY;
#pragma unroll
            for (int ot = 0; ot < 2; ot++)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (cmask[ot][r] != 0.f) zmax = fmaxf(zmax, z[ot][r]);
            zmax = fmaxf(zmax, __shfl_xor(zmax, 16, 64));
            zmax = fmaxf(zmax, __shfl_xor(zmax, 32, 64));
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
                den += __shfl_xor(den, 16, 64);
                den += __shfl_xor(den, 32, 64);
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
            float bt = -INFINITY, zt = -INFINITY;
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
                *(bf16x4 *)wr_ptr<R>(imgD3, lo, wave * 16, ot * 16) = dv;
            }
            if constexpr (!LABELS) {
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
            l += __shfl_xor(l, 16, 64);
            l += __shfl_xor(l, 32, 64);
            if (valid) {
                if (q == 0) my_loss += (TYPE == 2) ? -l / (float)n_out : 0.5f * l;
                my_hit += hit;
            }
        }
        lds_barrier();

        /* ---- P3: delta2 = (delta3 . W2) * f'(H2); wave: h2 tile ht, sample group hs ---- */
        {
            f32x4 acc = mfma(rd_tr<NO>(imgW2, lo, 0, ht * 16), rd_row<R>(imgD3, lo, hs * 16, 0),
                             f32x4{0.f, 0.f, 0.f, 0.f});
            const bf16x4 h = *(const bf16x4 *)wr_ptr<R>(imgH2, lo, hs * 16, ht * 16);
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; r++) o[r] = (__bf16)(acc[r] * dbipolar((float)h[r]));
            *(bf16x4 *)wr_ptr<R>(imgD2, lo, hs * 16, ht * 16) = o;
        }
        lds_barrier();

        /* ---- P4: delta1 = (delta2 . W1) * f'(H1) -> HBM; wave: h1 tile w, both sample groups ---- */
        {
            f32x4 acc[2];
            acc[0] = acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H2; k += 32) {
                const bf16x8 a = rd_tr<H2>(imgW1, lo, k, wave * 16); /* A[h1][h2] = W1[h2][h1] */
                acc[0] = mfma(a, rd_row<R>(imgD2, lo, 0, k), acc[0]);
                acc[1] = mfma(a, rd_row<R>(imgD2, lo, 16, k), acc[1]);
            }
            bf16x4 o[2];
#pragma unroll
            for (int sg = 0; sg < 2; sg++) {
                const bf16x4 h = *(const bf16x4 *)wr_ptr<R>(imgH1, lo, sg * 16, wave * 16);
#pragma unroll
                for (int r = 0; r < 4; r++) o[sg][r] = (__bf16)(acc[sg][r] * dbipolar((float)h[r]));
            }
            /* vm-op order (see header): label(i+1), 2 stores, X(i+2) */
            if (i + 1 < nloc) load_label(i + 1);
#pragma unroll
            for (int sg = 0; sg < 2; sg++)
                *(bf16x4 *)(D1 + (size_t)(s0 + sg * 16 + r16) * H1 + wave * 16 + 4 * q) = o[sg];
            if (i + 2 < nloc) issue_x(i & 1, i + 2);
        }
        /* ---- P5: G2 += delta3^T . H2 ([h2][o] tiles, k = samples); wave: h2 tile ht, o tile hs ---- */
        if (hs < n_ot) g2acc = mfma(rd_tr<R>(imgH2, lo, 0, ht * 16), rd_tr<R>(imgD3, lo, 0, hs * 16), g2acc);
        /* ---- P6: G1 += delta2^T . H1 ([h1][h2] tiles); wave: h1 tile w ---- */
        {
            const bf16x8 a = rd_tr<R>(imgH1, lo, 0, wave * 16);
#pragma unroll
            for (int t = 0; t < 4; t++) g1acc[t] = mfma(a, rd_tr<R>(imgD2, lo, 0, t * 16), g1acc[t]);
        }
        lds_barrier();
    }

    /* ---- per-block gradient slab [G1 (H2 x H1) | G2 (NO x H2)] ---- */
    float *slab = gslab + (size_t)blockIdx.x * SLAB;
#pragma unroll
    for (int t = 0; t < 4; t++) /* D[h1 = 16w + 4q + r][h2 = 16t + r16] */
        *(f32x4 *)(slab + (size_t)(t * 16 + r16) * H1 + wave * 16 + 4 * q) = g1acc[t];
    /* D[h2 = 16 ht + 4q + r][o = 16 hs + r16] */
    *(f32x4 *)(slab + H2 * H1 + (size_t)(hs * 16 + r16) * H2 + ht * 16 + 4 * q) = g2acc;
    float *sl = (float *)(lds + LY::OFF_RED);
    unsigned int *sh = (unsigned int *)(lds + LY::OFF_RED + 64);
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
        for (int w = 0; w < FNW; w++) {
            a += sl[w];
            h += sh[w];
        }
        if (loss_acc) atomicAdd(loss_acc + HPNN_STAT_SLOT(blockIdx.x), a);
        if (correct) atomicAdd(correct + HPNN_STAT_SLOT(blockIdx.x), h);
    }
}

int g_fused_cus = 0;
int fused_grid(int Bp, int grid) {
    if (g_fused_cus <= 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_fused_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            g_fused_cus = 256;
    }
    const int n_tiles = Bp / FR;
    if (grid <= 0) grid = g_fused_cus;
    return grid < n_tiles ? grid : n_tiles;
}

template <int TYPE, bool LABELS, int KS>
int launch_fused(const void *X, int ldx, const void *W0f, const void *W1, const void *W2, const int *labels,
                 const float *T, int ldt, float t_hi, float t_lo, void *D1, float *gslab, float *loss_acc,
                 unsigned int *correct, int Bp, int n_valid, int n_out, int grid, hipStream_t stream) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)mlp3_fused_kernel<TYPE, LABELS, KS>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, FLay<KS>::TOTAL);
        attr = true;
    }
    hipLaunchKernelGGL((mlp3_fused_kernel<TYPE, LABELS, KS>), dim3(grid), dim3(512), FLay<KS>::TOTAL, stream,
                       (const __bf16 *)X, ldx, (const __bf16 *)W0f, (const __bf16 *)W1, (const __bf16 *)W2, labels, T,
                       ldt, t_hi, t_lo, (__bf16 *)D1, gslab, loss_acc, correct, Bp / FR, n_valid, n_out);
    return hipGetLastError() == hipSuccess ? grid : -5;
}

template <int KS>
int launch_fused_k(const void *X, int ldx, const void *W0f, const void *W1, const void *W2, const int *labels,
                   const float *T, int ldt, float t_hi, float t_lo, void *D1, float *gslab, float *loss_acc,
                   unsigned int *correct, int Bp, int n_valid, int n_out, int type, int grid, hipStream_t stream) {
#define HPNN_FZ(TY, LB)                                                                                         \
    return launch_fused<TY, LB, KS>(X, ldx, W0f, W1, W2, labels, T, ldt, t_hi, t_lo, D1, gslab, loss_acc, correct, \
                                    Bp, n_valid, n_out, grid, stream)
    if (labels) {
        if (type == 2) HPNN_FZ(2, true);
        if (type == 0) HPNN_FZ(0, true);
        HPNN_FZ(1, true);
    }
    if (type == 2) HPNN_FZ(2, false);
    if (type == 0) HPNN_FZ(0, false);
    HPNN_FZ(1, false);
#undef HPNN_FZ
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

extern "C" int hpnn_mlp3_fused_grid(int Bp, int grid) { return Bp > 0 && Bp % FR == 0 ? fused_grid(Bp, grid) : -2; }

extern "C" int hpnn_mlp3_fused(const void *X, int ldx, int K0, const void *W0f, const void *W1, const void *W2,
                               const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1,
                               float *gslab, float *loss_acc, unsigned int *correct, int Bp, int n_valid, int n_out,
                               int type, int grid, hipStream_t stream) {
    if (Bp <= 0 || Bp % FR || n_out > NO || n_out < 1 || ldx % 8 || ldx < K0) return -2;
    if (!labels && !T) return -1;
    grid = fused_grid(Bp, grid);
#define HPNN_FK(K_)                                                                                                 if (K0 == K_)                                                                                                   return launch_fused_k<K_ / 32>(X, ldx, W0f, W1, W2, labels, T, ldt, t_hi, t_lo, D1, gslab, loss_acc, correct,                                    Bp, n_valid, n_out, type, grid, stream)
    HPNN_FK(800);
    HPNN_FK(256);
    HPNN_FK(512);
    HPNN_FK(832);
    HPNN_FK(896);
#undef HPNN_FK
    return -3;
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
