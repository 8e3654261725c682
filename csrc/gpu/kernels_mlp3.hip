/*
 * Fused kernels for the 3-weight-layer bias-free MLP (the MNIST-shaped headline
 * network n_in -> H1 -> H2 -> n_out, SNN/ANN/LNN), gfx950.
 *
 * The per-layer path (kernels_mfma.hip) round-trips every activation and delta
 * through HBM and launches ~11 kernels per step.  Here one step is
 *   1. gemm_nt (X . W0^T, bipolar)           -> H1        [B x H1]   (pipelined MFMA)
 *   2. mlp3_mid (this file)                   : H1 -> H2 -> output -> delta3 -> delta2
 *                                              -> delta1 (stored), plus the G1 / G2 weight
 *                                              gradients of the block's samples
 *   3. gemm_tn (delta1^T . X)                -> G0 split-K slabs
 *   4. optimizer (slab reduce + BP/BPM + BF16 W / W^T refresh)
 * mlp3_mid keeps W1, W1^T, W2, W2^T in LDS for the whole launch, streams one
 * 128-sample H1 tile per iteration through a double-buffered LDS-DMA ring (the next
 * tile lands while the current one is processed), holds H2 / delta3 / delta2 in LDS
 * only, and accumulates G1 / G2 in registers across all tiles of the block (one FP32
 * slab per block at the end).  HBM traffic per sample: H1 in + delta1 out.
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
constexpr int BM = 128;   /* samples per tile */
constexpr int NWAVE = 8;  /* 512 threads */

template <int H1, int H2, int NO>
struct Mid {
    /* LDS carve (bytes); every image is a T32 image */
    static constexpr int IMG_H1 = BM * H1 * 2;       /* x2 (ring) */
    static constexpr int IMG_W1 = H2 * H1 * 2;       /* [H2 rows][H1 cols] */
    static constexpr int IMG_W1T = H1 * H2 * 2;      /* [H1 rows][H2 cols] */
    static constexpr int IMG_W2 = NO * H2 * 2;       /* [NO rows][H2 cols] */
    static constexpr int IMG_W2T = H2 * NO * 2;      /* [H2 rows][NO cols] */
    static constexpr int IMG_H2 = BM * H2 * 2;
    static constexpr int IMG_D3 = BM * NO * 2;
    static constexpr int IMG_D2 = BM * H2 * 2;
    static constexpr int OFF_H1 = 0;
    static constexpr int OFF_W1 = OFF_H1 + 2 * IMG_H1;
    static constexpr int OFF_W1T = OFF_W1 + IMG_W1;
    static constexpr int OFF_W2 = OFF_W1T + IMG_W1T;
    static constexpr int OFF_W2T = OFF_W2 + IMG_W2;
    static constexpr int OFF_H2 = OFF_W2T + IMG_W2T;
    static constexpr int OFF_D3 = OFF_H2 + IMG_H2;
    static constexpr int OFF_D2 = OFF_D3 + IMG_D3;
    static constexpr int OFF_RED = OFF_D2 + IMG_D2; /* 8 floats + 8 uints */
    static constexpr int TOTAL = OFF_RED + 64;
    static_assert(TOTAL <= 160 * 1024, "LDS budget");
    static_assert(H1 == 128 && H2 == 64 && NO == 32, "tiling written for 128/64/32");
};

/* copy a row-major [R x C] bf16 global matrix into a T32 image (LDS-DMA pieces,
 * distributed over the 8 waves); returns the number of pieces THIS wave issued */
template <int R, int C>
__device__ __forceinline__ int load_img(const __bf16 *g, int ld, char *img, int wave, int lane) {
    constexpr int PIECES = (C / 32) * (R / 16);
    int n = 0;
    for (int p = wave; p < PIECES; p += NWAVE, n++) glds_t32_piece<R>((const char *)g, (size_t)ld * 2, img, p, lane);
    return n;
}

template <int H1, int H2, int NO>
__global__ __launch_bounds__(512) void mlp3_mid_kernel(const __bf16 *__restrict__ Hg, const __bf16 *__restrict__ W1,
                                                       const __bf16 *__restrict__ W1t,
                                                       const __bf16 *__restrict__ W2,
                                                       const __bf16 *__restrict__ W2t, const int *__restrict__ labels,
                                                       const float *__restrict__ T, int ldt, float t_hi, float t_lo,
                                                       __bf16 *__restrict__ D1, float *__restrict__ gslab,
                                                       float *__restrict__ loss_acc, unsigned int *__restrict__ correct,
                                                       int n_tiles, int n_valid, int n_out, int type) {
    using L = Mid<H1, H2, NO>;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    char *imgW1 = lds + L::OFF_W1, *imgW1t = lds + L::OFF_W1T, *imgW2 = lds + L::OFF_W2, *imgW2t = lds + L::OFF_W2T;
    char *imgH2 = lds + L::OFF_H2, *imgD3 = lds + L::OFF_D3, *imgD2 = lds + L::OFF_D2;

    /* resident weights + first tile */
    load_img<H2, H1>(W1, H1, imgW1, wave, lane);
    load_img<H1, H2>(W1t, H2, imgW1t, wave, lane);
    load_img<NO, H2>(W2, H2, imgW2, wave, lane);
    load_img<H2, NO>(W2t, NO, imgW2t, wave, lane);
    int tile = blockIdx.x;
    if (tile < n_tiles) load_img<BM, H1>(Hg + (size_t)tile * BM * H1, H1, lds + L::OFF_H1, wave, lane);
    wait_vm<0>();
    __syncthreads();

    /* persistent gradient accumulators */
    f32x4 g2acc = {0.f, 0.f, 0.f, 0.f}; /* G2 tile: h-tile = wave>>1, o-tile = wave&1 */
    f32x4 g1acc[4];                     /* G1 tiles: h1-tile = wave, h2-tiles 0..3   */
#pragma unroll
    for (int i = 0; i < 4; i++) g1acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float my_loss = 0.f;
    unsigned int my_hit = 0;
    int lab_cur = -1;
    if (labels && tile < n_tiles) {
        const int s = tile * BM + wave * 16 + r16;
        const int *addr = labels + (s < n_valid ? s : (n_valid > 0 ? n_valid - 1 : 0));
        asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=&v"(lab_cur) : "v"(addr) : "memory");
    }

    int buf = 0;
    for (; tile < n_tiles; tile += gridDim.x, buf ^= 1) {
        char *imgH1 = lds + L::OFF_H1 + buf * L::IMG_H1;
        const int s0 = tile * BM; /* global sample index of row 0 */
        const int nt = tile + gridDim.x;
        /* next tile's labels: inline-asm load issued BEFORE the LDS-DMA prefetch and
         * retired by the end-of-tile wait, so no compiler-inserted vmcnt(0) drains
         * the prefetch in the middle of the tile */
        int lab_next = -1;
        if (labels && nt < n_tiles) {
            int s = nt * BM + wave * 16 + r16;
            s = s < n_valid ? s : (n_valid > 0 ? n_valid - 1 : 0);
            const int *addr = labels + s;
            asm volatile("global_load_dword %0, %1, off" : "=v"(lab_next) : "v"(addr) : "memory");
        }
        if (nt < n_tiles)
            load_img<BM, H1>(Hg + (size_t)nt * BM * H1, H1, lds + L::OFF_H1 + (buf ^ 1) * L::IMG_H1, wave, lane);

        /* ---- phase 1: H2 = f(H1 . W1^T)  [BM x H2]; wave: f-tile wave&3, s-tiles 4*(wave>>2).. */
        {
            const int ft = wave & 3, sb = (wave >> 2) * 4;
            f32x4 acc[4];
#pragma unroll
            for (int j = 0; j < 4; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H1; k += 32) {
                const bf16x8 a = frag_row<H2>(imgW1, ft * 16, k, lane);
#pragma unroll
                for (int j = 0; j < 4; j++) acc[j] = mfma(a, frag_row<BM>(imgH1, (sb + j) * 16, k, lane), acc[j]);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)bipolar(acc[j][r]);
                *(bf16x4 *)(imgH2 + t32<BM>((sb + j) * 16 + r16, ft * 16 + 4 * q)) = o;
            }
        }
        lds_barrier();

        /* ---- phase 2: output layer for samples [16 wave, +16): logits, loss, delta3 ---- */
        {
            f32x4 z[2];
            z[0] = z[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H2; k += 32) {
                const bf16x8 b = frag_row<BM>(imgH2, wave * 16, k, lane);
#pragma unroll
                for (int ot = 0; ot < 2; ot++) z[ot] = mfma(frag_row<NO>(imgW2, ot * 16, k, lane), b, z[ot]);
            }
            /* lane: sample s = 16 wave + r16, outputs 16 ot + 4 q + r */
            const int srow = wave * 16 + r16;
            const int s = s0 + srow;
            const bool valid = s < n_valid;
            const int lab = valid ? lab_cur : -1;
            float o[2][4];
            float zmax = -INFINITY;
            if (type == 2) {
#pragma unroll
                for (int ot = 0; ot < 2; ot++)
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (ot * 16 + 4 * q + r < n_out) zmax = fmaxf(zmax, z[ot][r]);
                zmax = fmaxf(zmax, __shfl_xor(zmax, 16, 64));
                zmax = fmaxf(zmax, __shfl_xor(zmax, 32, 64));
            }
            float den = 0.f;
            if (type == 2) {
#pragma unroll
                for (int ot = 0; ot < 2; ot++)
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (ot * 16 + 4 * q + r < n_out) den += __expf(z[ot][r] - zmax);
                den += __shfl_xor(den, 16, 64);
                den += __shfl_xor(den, 32, 64);
                den += __expf(fminf(logf(TINY) + 1.0f - zmax, 80.f));
            }
            const float inv = type == 2 ? 1.0f / den : 0.f;
            float l = 0.f, bo = -INFINITY, bt = -INFINITY;
            int io = 1 << 30, it = 1 << 30;
#pragma unroll
            for (int ot = 0; ot < 2; ot++) {
                bf16x4 dv;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int c = ot * 16 + 4 * q + r;
                    float d = 0.f;
                    if (c < n_out) {
                        float ov;
                        if (type == 2) ov = __expf(z[ot][r] - zmax) * inv;
                        else if (type == 0) ov = bipolar(z[ot][r]);
                        else ov = z[ot][r];
                        o[ot][r] = ov;
                        if (valid) {
                            const float t = labels ? (c == lab ? t_hi : t_lo) : T[(size_t)s * ldt + c];
                            if (type == 2) {
                                if (t != 0.f && ov > 0.f) l += t * __logf(ov + TINY);
                                d = t - ov;
                            } else if (type == 0) {
                                l += (t - ov) * (t - ov);
                                d = (t - ov) * dbipolar(ov);
                            } else {
                                l += (t - ov) * (t - ov);
                                d = t - ov;
                            }
                            if (ov > bo) { bo = ov; io = c; }
                            if (t > bt) { bt = t; it = c; }
                        }
                    }
                    dv[r] = (__bf16)d;
                }
                *(bf16x4 *)(imgD3 + t32<BM>(srow, ot * 16 + 4 * q)) = dv;
            }
            /* combine the 4 lanes (q) that share a sample */
#pragma unroll
            for (int off = 16; off <= 32; off <<= 1) {
                l += __shfl_xor(l, off, 64);
                const float ob = __shfl_xor(bo, off, 64), tb = __shfl_xor(bt, off, 64);
                const int oi = __shfl_xor(io, off, 64), ti = __shfl_xor(it, off, 64);
                if (ob > bo || (ob == bo && oi < io)) { bo = ob; io = oi; }
                if (tb > bt || (tb == bt && ti < it)) { bt = tb; it = ti; }
            }
            if (valid && q == 0) {
                my_loss += (type == 2) ? -l / (float)n_out : 0.5f * l;
                my_hit += (io == it) ? 1u : 0u;
            }
            (void)o;
        }
        lds_barrier();

        /* ---- phase 3: delta2 = (delta3 . W2) * f'(H2)  [BM x H2] ---- */
        {
            const int ft = wave & 3, sb = (wave >> 2) * 4;
            f32x4 acc[4];
#pragma unroll
            for (int j = 0; j < 4; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < NO; k += 32) {
                const bf16x8 a = frag_row<H2>(imgW2t, ft * 16, k, lane);
#pragma unroll
                for (int j = 0; j < 4; j++) acc[j] = mfma(a, frag_row<BM>(imgD3, (sb + j) * 16, k, lane), acc[j]);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int off = t32<BM>((sb + j) * 16 + r16, ft * 16 + 4 * q);
                const bf16x4 h = *(const bf16x4 *)(imgH2 + off);
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)(acc[j][r] * dbipolar((float)h[r]));
                *(bf16x4 *)(imgD2 + off) = o;
            }
        }
        lds_barrier();

        /* ---- phase 4: delta1 = (delta2 . W1) * f'(H1) -> global  [BM x H1]; wave: f-tile wave ---- */
        {
            f32x4 acc[8];
#pragma unroll
            for (int j = 0; j < 8; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H2; k += 32) {
                const bf16x8 a = frag_row<H1>(imgW1t, wave * 16, k, lane);
#pragma unroll
                for (int j = 0; j < 8; j++) acc[j] = mfma(a, frag_row<BM>(imgD2, j * 16, k, lane), acc[j]);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int srow = j * 16 + r16, f = wave * 16 + 4 * q;
                const bf16x4 h = *(const bf16x4 *)(imgH1 + t32<BM>(srow, f));
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)(acc[j][r] * dbipolar((float)h[r]));
                *(bf16x4 *)(D1 + (size_t)(s0 + srow) * H1 + f) = o;
            }
        }

        /* ---- phase 5: G2 += delta3^T . H2   ([NO x H2], k = samples) ---- */
        {
            const int ht = wave >> 1, ot = wave & 1;
#pragma unroll
            for (int k = 0; k < BM; k += 32)
                g2acc = mfma(frag_tr<BM>(imgH2, k, ht * 16, lane), frag_tr<BM>(imgD3, k, ot * 16, lane), g2acc);
        }
        /* ---- phase 6: G1 += delta2^T . H1   ([H2 x H1]) ---- */
#pragma unroll
        for (int k = 0; k < BM; k += 32) {
            const bf16x8 a = frag_tr<BM>(imgH1, k, wave * 16, lane);
#pragma unroll
            for (int t = 0; t < 4; t++) g1acc[t] = mfma(a, frag_tr<BM>(imgD2, k, t * 16, lane), g1acc[t]);
        }
        /* next tile's H1 + labels landed (and this tile's delta1 stores drained) */
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(lab_next)::"memory");
        lab_cur = lab_next;
        lds_barrier();
    }

    /* ---- per-block gradient slab: [G1 (H2 x H1) | G2 (NO x H2)] ---- */
    float *slab = gslab + (size_t)blockIdx.x * (H2 * H1 + NO * H2);
#pragma unroll
    for (int t = 0; t < 4; t++)  /* D[h1 = 16 wave + 4q + r][h2 = 16 t + r16] */
        *(f32x4 *)(slab + (size_t)(t * 16 + r16) * H1 + wave * 16 + 4 * q) = g1acc[t];
    {
        const int ht = wave >> 1, ot = wave & 1; /* D[h = 16 ht + 4q + r][o = 16 ot + r16] */
        *(f32x4 *)(slab + H2 * H1 + (size_t)(ot * 16 + r16) * H2 + ht * 16 + 4 * q) = g2acc;
    }
    /* loss / accuracy: one atomic per block */
    float *sl = (float *)(lds + L::OFF_RED);
    unsigned int *sh = (unsigned int *)(lds + L::OFF_RED + 32);
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
        for (int w = 0; w < NWAVE; w++) {
            a += sl[w];
            h += sh[w];
        }
        if (loss_acc) atomicAdd(loss_acc, a);
        if (correct) atomicAdd(correct, h);
    }
}

/* Deterministic wide slab reduction: out[i] = sum_s slab[s*stride + i].
 * Block = 256 threads handles 64 float4 columns; the 4 waves split the slabs and
 * combine through LDS, so many loads are in flight per element. */
__global__ __launch_bounds__(256) void reduce_wide_kernel(const float *__restrict__ slab, int S, long stride, long n4,
                                                          float *__restrict__ out) {
    __shared__ f32x4 part[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long e = (long)blockIdx.x * 64 + lane;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    if (e < n4) {
        int s = w;
        for (; s + 12 < S; s += 16) {
            a0 += ((const f32x4 *)(slab + (long)s * stride))[e];
            a1 += ((const f32x4 *)(slab + (long)(s + 4) * stride))[e];
            a2 += ((const f32x4 *)(slab + (long)(s + 8) * stride))[e];
            a3 += ((const f32x4 *)(slab + (long)(s + 12) * stride))[e];
        }
        for (; s < S; s += 4) a0 += ((const f32x4 *)(slab + (long)s * stride))[e];
    }
    part[w][lane] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (w == 0 && e < n4) ((f32x4 *)out)[e] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}

}  // namespace

extern "C" int hpnn_mlp3_mid(const void *H1g, const void *W1, const void *W1t, const void *W2, const void *W2t,
                             const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1,
                             float *gslab, float *loss_acc, unsigned int *correct, int Bp, int n_valid, int n_out,
                             int type, int h1, int h2, int no, int grid, hipStream_t stream) {
    if (h1 != 128 || h2 != 64 || no != 32) return -2;
    if (Bp % BM || n_out > no) return -2;
    if (!labels && !T) return -1;
    using L = Mid<128, 64, 32>;
    const int n_tiles = Bp / BM;
    if (grid <= 0 || grid > n_tiles) grid = n_tiles;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)mlp3_mid_kernel<128, 64, 32>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, L::TOTAL);
        attr = true;
    }
    hipLaunchKernelGGL((mlp3_mid_kernel<128, 64, 32>), dim3(grid), dim3(512), L::TOTAL, stream, (const __bf16 *)H1g,
                       (const __bf16 *)W1, (const __bf16 *)W1t, (const __bf16 *)W2, (const __bf16 *)W2t, labels, T,
                       ldt, t_hi, t_lo, (__bf16 *)D1, gslab, loss_acc, correct, n_tiles, n_valid, n_out, type);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_reduce_slabs_wide(const float *slab, int S, long stride, long n, float *out, hipStream_t stream) {
    if (n % 4 || stride % 4 || S < 1) return -2;
    const long n4 = n / 4;
    hipLaunchKernelGGL(reduce_wide_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, stream, slab, S, stride, n4,
                       out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
