/*
 * Shared pieces of the fused 3-layer MLP kernels (kernels_mlp3.hip: mlp3_mid,
 * kernels_mlp3x.hip: mlp3_fused): padded dims, per-lane T32 offsets, fragment
 * readers/writers and the output layer (softmax / sigmoid / linear + loss + delta).
 * Reference math: SURVEY 2.4 (ann.c:883-888, 1279-1592; snn.c:280-335, 481-794).
 */
#ifndef HPNN_MLP3_COMMON_H
#define HPNN_MLP3_COMMON_H
#include <hip/hip_runtime.h>
#include <math.h>

#include "kernels.h"
#include "mfma_common.h"

namespace hpnn {
namespace mlp3 {

constexpr float TINY = 1e-14f;
constexpr int H1 = 128, H2 = 64, NO = 32;
constexpr int IMG_W1 = H2 * H1 * 2; /* [H2 rows][H1 cols] */
constexpr int IMG_W2 = NO * H2 * 2; /* [NO rows][H2 cols] */
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

/* The same 8 bytes stored / loaded without wr_ptr's 2-way bank conflicts.  A 64-bit LDS
 * access is serviced 16 (store) or 32 (load) lanes at a time, and in wr_ptr's layout those
 * lanes cover 8 / 16 of the 16 / 32 eight-byte bank slots: rows r and r + 4 share a slot
 * (same 16-byte chunk, same half).  Lanes whose row has bit 2 set trade with lane l ^ 16 --
 * same row, other 8-byte half of the same chunk (address ^ 8) -- through v_permlane16_swap,
 * so every group covers all slots.  Both lanes of a pair trade, so each byte is still
 * written / read once.  TRADE = false: the plain wr_ptr access -- what the tile front uses by
 * default, since the shuffles measured slower than the conflicts they remove
 * (profiles/r4/tr_tile_trade_ab.txt). */
template <int R, bool TRADE = true>
__device__ __forceinline__ void st_d4(char *img, const LaneOff &lo, int r0, int c0, bf16x4 v, int lane) {
    if constexpr (!TRADE) { /* plain wr_ptr store (2-way conflicts, no shuffles) */
        *(bf16x4 *)wr_ptr<R>(img, lo, r0, c0) = v;
        return;
    }
    typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
    const u32x2 w = __builtin_bit_cast(u32x2, v);
    const bool trade = (lane >> 2) & 1;
    u32x2 o;
    o[0] = (unsigned int)shfl_xor16((int)w[0], lane);
    o[1] = (unsigned int)shfl_xor16((int)w[1], lane);
    char *p = wr_ptr<R>(img, lo, r0, c0);
    /* the partner's half: bit 3 of the offset is 8 (q & 1) (everything else in wr_ptr's
     * offset is a multiple of 16); pointer arithmetic keeps the access a ds_write */
    const int dh = trade ? (((lane >> 4) & 1) ? -8 : 8) : 0;
    *(u32x2 *)(p + dh) = trade ? o : w;
}
template <int R, bool TRADE = true>
__device__ __forceinline__ bf16x4 ld_d4(const char *img, const LaneOff &lo, int r0, int c0, int lane) {
    if constexpr (!TRADE) return *(const bf16x4 *)wr_ptr<R>((char *)img, lo, r0, c0);
    typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
    const bool trade = (lane >> 2) & 1;
    const char *p = wr_ptr<R>((char *)img, lo, r0, c0);
    const int dh = trade ? (((lane >> 4) & 1) ? -8 : 8) : 0;
    const u32x2 w = *(const u32x2 *)(p + dh);
    u32x2 o;
    o[0] = (unsigned int)shfl_xor16((int)w[0], lane);
    o[1] = (unsigned int)shfl_xor16((int)w[1], lane);
    return __builtin_bit_cast(bf16x4, trade ? o : w);
}

/* Output layer for 16 samples (one wave): logits z (D[row = o 4q+r][col = sample r16],
 * NOT = 1 or 2 o-tiles of 16), targets from the label (LABELS) or dense T, writes delta3
 * (bf16) into the D3 image at rows [r0, r0+16) (zeros in an unused second o-tile),
 * accumulates loss / argmax hits for valid samples.
 * SNN: reference e^{z-1}/(TINY + sum e^{z-1}) evaluated in the max-shifted form. */
/* Hot path of output_layer: SNN, one-hot labels with t_lo == 0: no per-output
 * logarithms or branches -- one log per lane (the label's output), loss -log(o_lab+TINY)/N */
template <int R, int NOT>
__device__ __forceinline__ void output_snn_onehot(const f32x4 (&z)[2], int lab, float t_hi, bool valid, int n_out,
                                                  char *imgD3, const LaneOff &lo, int r0, int lane, float inv_nout,
                                                  float &my_loss, unsigned int &my_hit) {
    const int q = lane >> 4;
    float zmax = -INFINITY;
#pragma unroll
    for (int ot = 0; ot < NOT; ot++)
#pragma unroll
        for (int r = 0; r < 4; r++) zmax = (ot * 16 + 4 * q + r < n_out) ? fmaxf(zmax, z[ot][r]) : zmax;
    zmax = rows_max(zmax);
    float e[NOT][4], den = 0.f;
#pragma unroll
    for (int ot = 0; ot < NOT; ot++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            e[ot][r] = (ot * 16 + 4 * q + r < n_out) ? __expf(z[ot][r] - zmax) : 0.f;
            den += e[ot][r];
        }
    den = rows_sum(den) + __expf(fminf(-32.236191301916641f + 1.0f - zmax, 80.f));
    const float inv = __builtin_amdgcn_rcpf(den);
    const float vm = valid ? 1.f : 0.f;
    float o_lab = 0.f, z_lab = -INFINITY;
#pragma unroll
    for (int ot = 0; ot < 2; ot++) {
        bf16x4 dv = bf16x4{};
        if (ot < NOT) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int c = ot * 16 + 4 * q + r;
                const float o = e[ot][r] * inv;
                const bool is_lab = c == lab;
                o_lab = is_lab ? o : o_lab;
                z_lab = is_lab ? z[ot][r] : z_lab;
                dv[r] = (__bf16)(((is_lab ? t_hi : 0.f) - o) * vm);
            }
        }
        *(bf16x4 *)wr_ptr<R>(imgD3, lo, r0, ot * 16) = dv;
    }
    /* lanes that do not hold the label contribute 0 */
    float l = (z_lab > -INFINITY && valid) ? t_hi * __logf(o_lab + TINY) : 0.f;
    l = rows_sum(l);
    const unsigned int hit = (valid && z_lab > -INFINITY && z_lab >= zmax) ? 1u : 0u;
    if (valid) {
        if (q == 0) my_loss -= l * inv_nout;
        my_hit += hit;
    }
}

template <int TYPE, bool LABELS, int R, int NOT>
__device__ __forceinline__ void output_layer(const f32x4 (&z)[2], int lab, const float *__restrict__ T, int ldt,
                                             float t_hi, float t_lo, int s, bool valid, int n_out, char *imgD3,
                                             const LaneOff &lo, int r0, int lane, float inv_nout,
                                             float &my_loss, unsigned int &my_hit) {
    if constexpr (TYPE == 2 && LABELS) {
        if (t_lo == 0.f) {
            output_snn_onehot<R, NOT>(z, lab, t_hi, valid, n_out, imgD3, lo, r0, lane, inv_nout, my_loss, my_hit);
            return;
        }
    }
    const int q = lane >> 4;
    float cmask[NOT][4];
#pragma unroll
    for (int ot = 0; ot < NOT; ot++)
#pragma unroll
        for (int r = 0; r < 4; r++) cmask[ot][r] = (ot * 16 + 4 * q + r < n_out) ? 1.f : 0.f;
    float zmax = -INFINITY;
#pragma unroll
    for (int ot = 0; ot < NOT; ot++)
#pragma unroll
        for (int r = 0; r < 4; r++)
            if (cmask[ot][r] != 0.f) zmax = fmaxf(zmax, z[ot][r]);
    zmax = rows_max(zmax);
    float inv = 0.f;
    float e[NOT][4];
    if constexpr (TYPE == 2) {
        float den = 0.f;
#pragma unroll
        for (int ot = 0; ot < NOT; ot++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                e[ot][r] = __expf(z[ot][r] - zmax) * cmask[ot][r];
                den += e[ot][r];
            }
        den = rows_sum(den);
        /* TINY in the shifted frame: 1e-14 * e^{1 - zmax}; ln(1e-14) = -32.2361913 */
        den += __expf(fminf(-32.236191301916641f + 1.0f - zmax, 80.f));
        inv = __builtin_amdgcn_rcpf(den);
    }
    float l = 0.f;
    unsigned int hit = 0;
    float tt[NOT][4];
    if constexpr (!LABELS) {
#pragma unroll
        for (int ot = 0; ot < NOT; ot++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int c = ot * 16 + 4 * q + r;
                tt[ot][r] = (valid && c < n_out) ? T[(size_t)s * ldt + c] : 0.f;
            }
    }
    float bt = -INFINITY, zt = -INFINITY;
    int ibt = 1 << 30;
    float o_lab = 0.f;
#pragma unroll
    for (int ot = 0; ot < 2; ot++) {
        bf16x4 dv;
        if (ot >= NOT) {
            dv = bf16x4{};
        } else {
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
                    if constexpr (LABELS) {
                        /* one-hot targets: the t_hi term is the label's; t_lo terms only if t_lo != 0 */
                        if (c == lab) o_lab = o;
                        else if (t_lo != 0.f && m != 0.f && o > 0.f) l += t_lo * __logf(o + TINY);
                    } else {
                        if (m != 0.f && t != 0.f && o > 0.f) l += t * __logf(o + TINY);
                    }
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
        }
        *(bf16x4 *)wr_ptr<R>(imgD3, lo, r0, ot * 16) = dv;
    }
    if constexpr (!LABELS) {
        /* hit iff the logit of the (first) max-target column is the max logit */
        {
            const float ob = shfl_xor16(bt, lane), oz = shfl_xor16(zt, lane);
            const int oi = shfl_xor16(ibt, lane);
            if (ob > bt || (ob == bt && oi < ibt)) {
                bt = ob;
                ibt = oi;
                zt = oz;
            }
        }
        {
            const float ob = shfl_xor32(bt, lane), oz = shfl_xor32(zt, lane);
            const int oi = shfl_xor32(ibt, lane);
            if (ob > bt || (ob == bt && oi < ibt)) {
                bt = ob;
                ibt = oi;
                zt = oz;
            }
        }
        hit = (q == 0 && zt >= zmax) ? 1u : 0u;
    }
    if constexpr (TYPE == 2 && LABELS) {
        /* a single logarithm per lane: only the lane holding the label adds its term */
        if (o_lab > 0.f && valid && t_hi != 0.f) l += t_hi * __logf(o_lab + TINY);
    }
    l = rows_sum(l);
    if (valid) {
        if (q == 0) my_loss += (TYPE == 2) ? -l * inv_nout : 0.5f * l;
        my_hit += hit;
    }
}

}  // namespace mlp3
}  // namespace hpnn
#endif
