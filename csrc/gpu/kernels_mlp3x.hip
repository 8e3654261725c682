/*
 * mlp3_fused: the whole n_in -> 128 -> 64 -> n_out(<=32) training step up to delta1
 * in ONE persistent kernel (gfx950), software-pipelined across tiles.
 *
 * Reference: the per-sample GEMV chain of ann_kernel_train / snn_kernel_train
 * (ann.c:883-888, 1279-1592; snn.c:280-335, 481-794; cuda_ann.cu:426-2093), batched.
 *
 * One 512-thread workgroup (8 waves, 2 per SIMD) per CU, 32-sample tiles.  In stage t
 * every wave works on TWO tiles at once:
 *   front part (tile t):   H1(t) = f(X(t) . W0^T) for its 16 neurons.  W0 lives in VGPRs
 *                          for the whole launch (16 neurons x K0 per wave, read once from
 *                          the fragment-major copy W0f, 1 KiB contiguous per load).
 *   back part (tile t-1):  H2 = f(H1 W1^T), output layer + loss + delta3, delta2,
 *                          delta1 -> HBM, and the G2 / G1 products (VGPR accumulators
 *                          over all the block's tiles).
 * A stage is 4 intervals separated by workgroup barriers; each interval holds a quarter
 * of the front MFMA work (one X chunk) and one phase of the back chain
 * (P1 | P2 | P3 | P4+P5+P6), so the latency of the dependent back chain hides behind
 * independent MFMA work of the same and of the partner wave instead of serializing
 * with it (the first, phase-serialized version spent >50% of wave time parked at
 * barriers: profiles/).
 *
 * X streams HBM -> LDS by LDS-DMA into a 2-tile ring refilled chunk by chunk as soon as
 * a chunk is consumed (~1.5 tiles, ~77 KiB, in flight).  VM-counter discipline, no
 * vmcnt(0) in the loop: LDS-DMA is inline asm (glds16); waves 4-7 issue the X pieces
 * and the label copies in a fixed periodic order, so every wait is one exact counted
 * s_waitcnt; waves 0-3 issue only the delta1 stores and never wait on them.
 */
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"

HPNN_CO_PROBE(mlp3x)
#include "mfma_common.h"
#include "mlp3_common.h"

using namespace hpnn;
using namespace hpnn::mlp3;

namespace {

constexpr int FR = 32;   /* samples per tile */
constexpr int NCH = 4;   /* X chunks (intervals) per tile */

template <int KS>
struct XPlan {
    static constexpr int S64 = KS / 2, TAIL = KS & 1, NS = S64 + TAIL; /* sub-tiles (64 / 32 cols) */
    static constexpr int PF = FR / 8;                                   /* pieces per full sub-tile */
    /* first sub-tile of chunk c: chunk sizes follow the back-chain phase weights
     * {5, 2, 4, 2}/13 (interval 1 carries the output layer, interval 3 delta1 + G1) */
    static constexpr int sb(int c) {
        constexpr int cw[NCH + 1] = {0, 5, 7, 11, 13};
        return (NS * cw[c] + 6) / 13;
    }
    static constexpr int piece0(int c) { return sb(c) * PF; }
    static constexpr int pieces(int c) {
        const int e = sb(c + 1);
        return ((e < S64 ? e : S64) - sb(c)) * PF + ((TAIL && e > S64) ? FR / 16 : 0);
    }
    static constexpr int L(int c) { return (pieces(c) + 3) / 4; } /* per issuer wave (4 issuers) */

    static constexpr int ks0(int c) { return 2 * sb(c); }
    static constexpr int ks1(int c) { return 2 * sb(c + 1) < KS ? 2 * sb(c + 1) : KS; }
    /* X chunks issued after X(t) chunk j that may stay in flight at its wait */
    static constexpr int newer(int j) {
        int n = 0;
        for (int m = 1; m <= 6; m++) n += L((j + m) % NCH);
        return n;
    }
};

template <int KS>
struct Lay {
    static constexpr int XST = FR * KS * 32 * 2;
    static constexpr int OFF_W1 = 2 * XST;
    static constexpr int OFF_W2 = OFF_W1 + IMG_W1;
    static constexpr int OFF_H1 = OFF_W2 + IMG_W2; /* x2 (front writes t, back reads t-1) */
    static constexpr int IMG_H1 = FR * H1 * 2;
    static constexpr int OFF_H2 = OFF_H1 + 2 * IMG_H1;
    static constexpr int OFF_D3 = OFF_H2 + FR * H2 * 2;
    static constexpr int OFF_D2 = OFF_D3 + FR * NO * 2;
    static constexpr int OFF_LAB = OFF_D2 + FR * H2 * 2; /* 2 slots x 64 ints */
    static constexpr int OFF_RED = OFF_LAB + 2 * 256;
    static constexpr int TOTAL = OFF_RED + 128;
    static_assert(TOTAL <= 160 * 1024, "LDS");
};

template <int R, int C>
__device__ __forceinline__ void load_img8(const __bf16 *g, int ld, char *img, int wave, int lane) {
    constexpr int PIECES = (C / 32) * (R / 16);
    for (int p = wave; p < PIECES; p += 8) glds_t32_piece<R>((const char *)g, (size_t)ld * 2, img, p, lane);
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
                                                            int n_valid, int n_out, int d1fm) {
    using LY = Lay<KS>;
    using XP = XPlan<KS>;
    constexpr int R = FR;
    constexpr int S64 = XP::S64;
    /* exact in-flight counts for waves 4-7 (stream: stage s = label(s), X(s+1).c3 | X(s+2).c0 | .c1 | .c2) */
    constexpr int LABN[4] = {LABELS ? 1 : 0, LABELS ? 2 : 0, LABELS ? 2 : 0, LABELS ? 1 : 0};
    constexpr int W_X0 = XP::newer(0) + LABN[0], W_X2 = XP::newer(2) + LABN[2], W_X3 = XP::newer(3) + LABN[3];
    constexpr int W_LAB = XP::L(3) + XP::L(0) + XP::L(1) + XP::L(2) + 1 + XP::L(3); /* label(t-1) at B1 */
    constexpr int W_B1 = (LABELS && W_LAB < XP::newer(1) + LABN[1]) ? W_LAB : XP::newer(1) + LABN[1];
    static_assert(W_X0 < 64 && W_B1 < 64 && W_X2 < 64 && W_X3 < 64, "vmcnt range");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool issuer = wave >= 4; /* X + label DMA */
    const int iw = wave & 3;
    const int ht = wave & 3, hs = wave >> 2; /* 8-tile phases P1, P3: (h2 tile, sample group) */
    const int r16 = lane & 15, q = lane >> 4;
    const LaneOff lo = lane_offsets(lane);
    char *imgW1 = lds + LY::OFF_W1, *imgW2 = lds + LY::OFF_W2;
    char *imgH2 = lds + LY::OFF_H2, *imgD3 = lds + LY::OFF_D3, *imgD2 = lds + LY::OFF_D2;
    const int G = gridDim.x;
    const int nloc = (n_tiles - (int)blockIdx.x + G - 1) / G;
    const size_t ldx_b = (size_t)ldx * 2;
    auto tile_of = [&](int u) { return (int)blockIdx.x + (u < nloc ? u : nloc - 1) * G; };

    /* chunk c of X tile u by the 4 issuer waves (past the end: tile nloc-1 again, never read) */
    auto issue_chunk = [&](int u, auto cc) {
        constexpr int c = decltype(cc)::value;
        constexpr int P = XP::pieces(c), p0 = XP::piece0(c), LC = XP::L(c);
        if constexpr (LC == 0) return;
        const char *g = (const char *)(X + (size_t)tile_of(u) * R * ldx);
        char *img = lds + (u & 1) * LY::XST;
#pragma unroll
        for (int i = 0; i < LC; i++) {
            int p = iw + 4 * i;
            p = p < P ? p : P - 1;
            glds_x_piece_sv<R, S64>(g, (unsigned int)ldx_b, img, p0 + p, lane);
        }
    };
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
    using C3 = std::integral_constant<int, 3>;
    auto issue_label = [&](int u) {
        if constexpr (LABELS) {
            const int s = clamp_sample(tile_of(u) * R + (lane & 31), n_valid);
            glds4_sv(labels, (unsigned int)s * 4u, lds + LY::OFF_LAB + (u & 1) * 256);
        }
    };

    /* ---- prologue: X(0), W0 -> VGPRs, W1 / W2 -> LDS, one full wait, then X(1) c0..c2 ---- */
    if (issuer) {
        issue_chunk(0, C0{});
        issue_chunk(0, C1{});
        issue_chunk(0, C2{});
        issue_chunk(0, C3{});
    }
    bf16x8 w0[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        w0[ks] = *(const bf16x8 *)(W0f + ((size_t)(wave * KS + ks) * 64 + lane) * 8);
    }
    load_img8<H2, H1>(W1, H1, imgW1, wave, lane);
    load_img8<NO, H2>(W2, H2, imgW2, wave, lane);
    __builtin_amdgcn_s_waitcnt(0xF70); /* vmcnt(0), visible to the compiler: W0 complete */
    if (issuer) {
        issue_chunk(1, C0{});
        issue_chunk(1, C1{});
        issue_chunk(1, C2{});
    }

    f32x4 g1acc[4], g2acc; /* G1: h1 tile w x h2 tiles 0..3; G2: h2 tile ht x o tile hs */
    g2acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; i++) g1acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float my_loss = 0.f;
    unsigned int my_hit = 0;
    const int n_ot = n_out > 16 ? 2 : 1;
    const float inv_nout = 1.0f / (float)n_out;
    f32x4 acc0[2]; /* front: H1 tile (16 neurons x sample group) */

    /* one stage = front part of tile t (FW) + back part of tile t-1 (BW); FW / BW are
     * compile-time so that, inside every interval, the front MFMAs and the back chain of a
     * wave form ONE basic block the scheduler can interleave */
    auto stage = [&](int t, auto FWc, auto BWc) {
        constexpr bool FW = decltype(FWc)::value;
        constexpr bool BW = decltype(BWc)::value;
        const int tb = t - 1;
        const char *imgX = lds + (t & 1) * LY::XST;
        char *H1w = lds + LY::OFF_H1 + (t & 1) * LY::IMG_H1;       /* front writes tile t  */
        char *H1r = lds + LY::OFF_H1 + ((t + 1) & 1) * LY::IMG_H1; /* back reads tile t-1 */
        const int s0b = tile_of(tb < 0 ? 0 : tb) * R;

        auto front_chunk = [&](auto cc) {
            constexpr int c = decltype(cc)::value;
            constexpr int k0 = XP::ks0(c), k1 = XP::ks1(c);
            if constexpr (!FW) return;
            if constexpr (c == 0) acc0[0] = acc0[1] = f32x4{0.f, 0.f, 0.f, 0.f};
            /* the interval is one basic block: the scheduler hoists these reads */
#pragma unroll
            for (int ks = k0; ks < k1; ks++) {
                acc0[0] = mfma(w0[ks], x_frag<R, S64>(imgX, 0, ks, lane), acc0[0]);
                acc0[1] = mfma(w0[ks], x_frag<R, S64>(imgX, 16, ks, lane), acc0[1]);
            }
        };
        auto p1 = [&]() { /* H2 = f(H1 W1^T), tile (ht, hs) */
            f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H1; k += 32) a = mfma(rd_row<H2>(imgW1, lo, ht * 16, k), rd_row<R>(H1r, lo, hs * 16, k), a);
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; r++) o[r] = (__bf16)bipolar(a[r]);
            *(bf16x4 *)wr_ptr<R>(imgH2, lo, hs * 16, ht * 16) = o;
        };
        auto p2 = [&]() { /* output layer, sample group = wave (waves 0, 1) */
            const int sg = wave;
            f32x4 z[2];
            z[0] = z[1] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int s = s0b + sg * 16 + r16;
            const int lab = LABELS ? ((const int *)(lds + LY::OFF_LAB + (tb & 1) * 256))[sg * 16 + r16] : -1;
            if (n_ot > 1) {
#pragma unroll
                for (int k = 0; k < H2; k += 32) {
                    const bf16x8 b = rd_row<R>(imgH2, lo, sg * 16, k);
                    z[0] = mfma(rd_row<NO>(imgW2, lo, 0, k), b, z[0]);
                    z[1] = mfma(rd_row<NO>(imgW2, lo, 16, k), b, z[1]);
                }
                output_layer<TYPE, LABELS, R, 2>(z, lab, T, ldt, t_hi, t_lo, s, s < n_valid, n_out, imgD3, lo,
                                                 sg * 16, lane, inv_nout, my_loss, my_hit);
            } else {
#pragma unroll
                for (int k = 0; k < H2; k += 32)
                    z[0] = mfma(rd_row<NO>(imgW2, lo, 0, k), rd_row<R>(imgH2, lo, sg * 16, k), z[0]);
                output_layer<TYPE, LABELS, R, 1>(z, lab, T, ldt, t_hi, t_lo, s, s < n_valid, n_out, imgD3, lo,
                                                 sg * 16, lane, inv_nout, my_loss, my_hit);
            }
        };
        auto p3 = [&]() { /* delta2 = (delta3 W2) f'(H2), tile (ht, hs) */
            const f32x4 a = mfma(rd_tr<NO>(imgW2, lo, 0, ht * 16), rd_row<R>(imgD3, lo, hs * 16, 0),
                                 f32x4{0.f, 0.f, 0.f, 0.f}); /* A[h2][o] = W2[o][h2] */
            const bf16x4 h = *(const bf16x4 *)wr_ptr<R>(imgH2, lo, hs * 16, ht * 16);
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; r++) o[r] = (__bf16)(a[r] * dbipolar((float)h[r]));
            *(bf16x4 *)wr_ptr<R>(imgD2, lo, hs * 16, ht * 16) = o;
        };
        auto p4 = [&]() { /* delta1 = (delta2 W1) f'(H1) -> HBM; h1 tiles 2w, 2w+1 (waves 0-3) */
            f32x4 a4[2][2];
#pragma unroll
            for (int i = 0; i < 2; i++) a4[i][0] = a4[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (d1fm) {
                /* fragment-major delta1 for the direct-load G0 GEMM (kernels_g0.hip):
                 * chunk (tile, h1 block) = [g][r][j] = delta1[tile*32 + 8g + j][16 block + r].
                 * Operands swapped: D[row = sample 4q + r][col = h1 r16], so every lane owns
                 * 4 consecutive samples of one neuron = 8 contiguous bytes of its chunk;
                 * f'(H1) of the same 4 samples comes from one transposed LDS read. */
#pragma unroll
                for (int k = 0; k < H2; k += 32) {
                    const bf16x8 d0 = rd_row<R>(imgD2, lo, 0, k), d1 = rd_row<R>(imgD2, lo, 16, k);
#pragma unroll
                    for (int i = 0; i < 2; i++) {
                        const bf16x8 a = rd_tr<H2>(imgW1, lo, k, (2 * iw + i) * 16);
                        a4[i][0] = mfma(d0, a, a4[i][0]);
                        a4[i][1] = mfma(d1, a, a4[i][1]);
                    }
                }
                __bf16 *chunk0 = D1 + (size_t)(s0b / R) * (H1 / 16) * 512;
#pragma unroll
                for (int i = 0; i < 2; i++)
#pragma unroll
                    for (int sg = 0; sg < 2; sg++) {
                        const int h = (2 * iw + i) * 16;
                        const s16x4 hr = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_s16x4 *)(H1r + t32<R>(sg * 16 + 4 * q + (r16 >> 2), h + 4 * (r16 & 3))));
                        const bf16x4 hv = __builtin_bit_cast(bf16x4, hr);
                        bf16x4 o;
#pragma unroll
                        for (int r = 0; r < 4; r++) o[r] = (__bf16)(a4[i][sg][r] * dbipolar((float)hv[r]));
                        const int g = 2 * sg + (q >> 1);
                        *(bf16x4 *)(chunk0 + (size_t)(2 * iw + i) * 512 + (g * 16 + r16) * 8 + 4 * (q & 1)) = o;
                    }
                return;
            }
#pragma unroll
            for (int k = 0; k < H2; k += 32) {
                const bf16x8 d0 = rd_row<R>(imgD2, lo, 0, k), d1 = rd_row<R>(imgD2, lo, 16, k);
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const bf16x8 a = rd_tr<H2>(imgW1, lo, k, (2 * iw + i) * 16); /* A[h1][h2] = W1[h2][h1] */
                    a4[i][0] = mfma(a, d0, a4[i][0]);
                    a4[i][1] = mfma(a, d1, a4[i][1]);
                }
            }
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int sg = 0; sg < 2; sg++) {
                    const int h = (2 * iw + i) * 16;
                    const bf16x4 hv = *(const bf16x4 *)wr_ptr<R>(H1r, lo, sg * 16, h);
                    bf16x4 o;
#pragma unroll
                    for (int r = 0; r < 4; r++) o[r] = (__bf16)(a4[i][sg][r] * dbipolar((float)hv[r]));
                    *(bf16x4 *)(D1 + (size_t)(s0b + sg * 16 + r16) * H1 + h + 4 * q) = o;
                }
        };
        auto p5 = [&]() { /* G2 += delta3^T H2 (k = the 32 samples); tile (h2 ht, o hs) */
            if (hs < n_ot) g2acc = mfma(rd_tr<R>(imgH2, lo, 0, ht * 16), rd_tr<R>(imgD3, lo, 0, hs * 16), g2acc);
        };
        auto p6 = [&]() { /* G1 += delta2^T H1; h1 tile w, h2 tiles 0..3 */
            const bf16x8 a = rd_tr<R>(H1r, lo, 0, wave * 16);
#pragma unroll
            for (int t2 = 0; t2 < 4; t2++) g1acc[t2] = mfma(a, rd_tr<R>(imgD2, lo, 0, t2 * 16), g1acc[t2]);
        };

        /* (A variant running the parts in opposite order on the two waves of a SIMD was
         * measured 15% slower than letting the scheduler interleave them.) */
        auto order = [&](auto &&back, auto &&front) {
            /* one basic block per wave role: the scheduler interleaves the two parts */
            front();
            back();
        };

        /* ============ interval 0: X chunk 0 | P1 ============ */
        if (issuer) wait_vm<W_X0>();
        lds_barrier();
        if (issuer) {
            issue_label(t);
            issue_chunk(t + 1, C3{});
        }
        order([&] { if constexpr (BW) p1(); }, [&] { front_chunk(C0{}); });

        /* ============ interval 1: X chunk 1 | P2 (waves 0, 1) ============ */
        if (issuer) wait_vm<W_B1>();
        lds_barrier();
        if (issuer) issue_chunk(t + 2, C0{});
        order([&] { if (BW && wave < 2) p2(); }, [&] { front_chunk(C1{}); });

        /* ============ interval 2: X chunk 2 | P3, P5 ============ */
        if (issuer) wait_vm<W_X2>();
        lds_barrier();
        if (issuer) issue_chunk(t + 2, C1{});
        order(
            [&] {
                if constexpr (BW) p3();
                if constexpr (BW) p5();
            },
            [&] { front_chunk(C2{}); });

        /* ============ interval 3: X chunk 3 + H1(t) | P4 (waves 0-3), P6 ============ */
        if (issuer) wait_vm<W_X3>();
        lds_barrier();
        if (issuer) issue_chunk(t + 2, C2{});
        order(
            [&] {
                if (BW && !issuer) p4();
                if constexpr (BW) p6();
            },
            [&] { front_chunk(C3{}); });
        if constexpr (FW) {
#pragma unroll
            for (int sg = 0; sg < 2; sg++) {
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; r++) o[r] = (__bf16)bipolar(acc0[sg][r]);
                *(bf16x4 *)wr_ptr<R>(H1w, lo, sg * 16, wave * 16) = o;
            }
        }
    };
    using T1 = std::true_type;
    using F0 = std::false_type;
    stage(0, T1{}, F0{});
    for (int t = 1; t < nloc; t++) stage(t, T1{}, T1{});
    stage(nloc, F0{}, T1{});

    /* the dummy X pieces of the last stage land before the workgroup's LDS is released */
    wait_vm<0>();
    /* ---- per-block gradient slab [G1 (H2 x H1) | G2 (NO x H2)] ---- */
    float *slab = gslab + (size_t)blockIdx.x * SLAB;
#pragma unroll
    for (int t2 = 0; t2 < 4; t2++) /* D[h1 = 16w + 4q + r][h2 = 16 t2 + r16] */
        *(f32x4 *)(slab + (size_t)(t2 * 16 + r16) * H1 + wave * 16 + 4 * q) = g1acc[t2];
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
        for (int w = 0; w < 8; w++) {
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
                 unsigned int *correct, int Bp, int n_valid, int n_out, int grid, int d1fm, hipStream_t stream) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)mlp3_fused_kernel<TYPE, LABELS, KS>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, Lay<KS>::TOTAL);
        attr = true;
    }
    hipLaunchKernelGGL((mlp3_fused_kernel<TYPE, LABELS, KS>), dim3(grid), dim3(512), Lay<KS>::TOTAL, stream,
                       (const __bf16 *)X, ldx, (const __bf16 *)W0f, (const __bf16 *)W1, (const __bf16 *)W2, labels, T,
                       ldt, t_hi, t_lo, (__bf16 *)D1, gslab, loss_acc, correct, Bp / FR, n_valid, n_out, d1fm);
    return hipGetLastError() == hipSuccess ? grid : -5;
}

template <int KS>
int launch_fused_k(const void *X, int ldx, const void *W0f, const void *W1, const void *W2, const int *labels,
                   const float *T, int ldt, float t_hi, float t_lo, void *D1, float *gslab, float *loss_acc,
                   unsigned int *correct, int Bp, int n_valid, int n_out, int type, int grid, int d1fm,
                   hipStream_t stream) {
#define HPNN_FZ(TY, LB)                                                                                         \
    return launch_fused<TY, LB, KS>(X, ldx, W0f, W1, W2, labels, T, ldt, t_hi, t_lo, D1, gslab, loss_acc, correct, \
                                    Bp, n_valid, n_out, grid, d1fm, stream)
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

extern "C" int hpnn_mlp3_fused_grid(int Bp, int grid) { return Bp > 0 && Bp % FR == 0 ? fused_grid(Bp, grid) : -2; }

extern "C" int hpnn_mlp3_fused(const void *X, int ldx, int K0, const void *W0f, const void *W1, const void *W2,
                               const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1,
                               float *gslab, float *loss_acc, unsigned int *correct, int Bp, int n_valid, int n_out,
                               int type, int grid, int d1fm, hipStream_t stream) {
    if (Bp <= 0 || Bp % FR || n_out > NO || n_out < 1 || ldx % 8 || ldx < K0) return -2;
    if (!labels && !T) return -1;
    grid = fused_grid(Bp, grid);
#define HPNN_FK(K_)                                                                                             \
    if (K0 == K_)                                                                                               \
    return launch_fused_k<K_ / 32>(X, ldx, W0f, W1, W2, labels, T, ldt, t_hi, t_lo, D1, gslab, loss_acc, correct, \
                                   Bp, n_valid, n_out, type, grid, d1fm, stream)
    HPNN_FK(800);
    HPNN_FK(256);
    HPNN_FK(512);
    HPNN_FK(832);
    HPNN_FK(896);
#undef HPNN_FK
    return -3;
}
