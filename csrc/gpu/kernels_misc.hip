/*
 * libhpnn element-wise / reduction kernels for gfx950.
 *
 *   output_delta : output layer activation + loss + output delta + accuracy
 *                  in one pass (replaces the reference's sigmoid/softmax_acc/
 *                  fw_scal/amb/amb_smax/dsigmoid_mul_diff/dsmax_diff kernels
 *                  plus the host-synchronising cublasDasum, cuda_ann.cu:41-113,
 *                  cuda_snn.cu:42-147).  One wave64 per sample, wave-level
 *                  shuffles, one atomic per block; correct for any width
 *                  (the reference reductions read block 0 only: N<=2048).
 *                  SNN uses the reference softmax e^{z-1}/(TINY+sum e^{z-1})
 *                  evaluated in the max-shifted form (identical value, no
 *                  overflow).
 *   reduce_slabs : deterministic sum of split-K partial slabs.
 *   sgd_update   : slab reduce + BP / BPM update on the FP32 master, then
 *                  BF16 W and BF16 W^T (through an LDS transpose so both
 *                  stores are coalesced).  Replaces cublasDger / Daxpy /
 *                  Dscal / ger_acc / ger_dw_acc (cuda_ann.cu:124-148).
 *   pack_bf16    : host-layout FP64/FP32 samples -> padded BF16 tiles.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <tuple>

#include "kernels.h"

HPNN_CO_PROBE(misc)

typedef __attribute__((ext_vector_type(4))) float f32x4;

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
/* first index of the maximum (ties -> lowest index), -1 for empty lanes */
__device__ __forceinline__ void wave_argmax(float &v, int &i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float ov = __shfl_xor(v, o, 64);
        int oi = __shfl_xor(i, o, 64);
        if (oi >= 0 && (i < 0 || ov > v || (ov == v && oi < i))) {
            v = ov;
            i = oi;
        }
    }
}

constexpr float TINY = 1e-14f;

__device__ __forceinline__ void block_reduce_store(float my_loss, unsigned int my_hit, float *loss_acc,
                                                   unsigned int *correct) {
    __shared__ float sloss[4];
    __shared__ unsigned int shit[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    my_loss = wave_sum(my_loss);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) my_hit += __shfl_xor(my_hit, o, 64);
    if (lane == 0) {
        sloss[wave] = my_loss;
        shit[wave] = my_hit;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = sloss[0] + sloss[1] + sloss[2] + sloss[3];
        unsigned int h = shit[0] + shit[1] + shit[2] + shit[3];
        if (loss_acc && s != 0.f) atomicAdd(loss_acc + HPNN_STAT_SLOT(blockIdx.x), s);
        if (correct && h) atomicAdd(correct + HPNN_STAT_SLOT(blockIdx.x), h);
    }
}

/* narrow outputs (n_out <= 64): one LANE per sample row, grid-stride, <= 256 blocks
 * so the loss/accuracy atomics stay few (one per block) */
template <int MAXO>
__global__ __launch_bounds__(256) void output_delta_rows_kernel(const float *__restrict__ Z, int ldz,
                                                                const float *__restrict__ T, int ldt,
                                                                const int *__restrict__ labels, float t_hi, float t_lo,
                                                                __bf16 *__restrict__ D, int ldd, float *__restrict__ O,
                                                                int ldo, float *__restrict__ loss_acc,
                                                                unsigned int *__restrict__ correct, int B, int n_valid,
                                                                int n_out, int type) {
    float my_loss = 0.f;
    unsigned int my_hit = 0;
    for (int row = blockIdx.x * blockDim.x + threadIdx.x; row < B; row += gridDim.x * blockDim.x) {
        const bool valid = row < n_valid;
        float z[MAXO];
        const float *zr = Z + (size_t)row * ldz;
#pragma unroll
        for (int c = 0; c < MAXO; c++) z[c] = c < n_out ? zr[c] : 0.f;
        float zmax = -INFINITY;
        if (type == 2) {
#pragma unroll
            for (int c = 0; c < MAXO; c++)
                if (c < n_out) zmax = fmaxf(zmax, z[c]);
        }
        float denom = 0.f;
        if (type == 2) {
#pragma unroll
            for (int c = 0; c < MAXO; c++)
                if (c < n_out) denom += __expf(z[c] - zmax);
            denom += __expf(fminf(logf(TINY) + 1.0f - zmax, 80.f));
        }
        const float inv = type == 2 ? 1.0f / denom : 0.f;
        const int lab = (labels && valid) ? labels[row] : -1;
        float l = 0.f, bo = -INFINITY, bt = -INFINITY;
        int io = -1, it = -1;
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        __bf16 dv[MAXO];
#pragma unroll
        for (int c = 0; c < MAXO; c++) {
            float d = 0.f;
            if (c < n_out) {
                float o;
                if (type == 2) o = __expf(z[c] - zmax) * inv;
                else if (type == 0) o = 2.0f / (1.0f + __expf(-z[c])) - 1.0f;
                else o = z[c];
                if (valid) {
                    const float t = labels ? (c == lab ? t_hi : t_lo) : T[(size_t)row * ldt + c];
                    if (type == 2) {
                        if (o > 0.f) l += t * logf(o + TINY);
                        d = t - o;
                    } else if (type == 0) {
                        l += (t - o) * (t - o);
                        d = (t - o) * (-0.5f * (o * o - 1.0f));
                    } else {
                        l += (t - o) * (t - o);
                        d = t - o;
                    }
                    if (o > bo) { bo = o; io = c; }
                    if (t > bt) { bt = t; it = c; }
                }
                if (O) O[(size_t)row * ldo + c] = o;
            }
            dv[c] = (__bf16)d;
        }
        /* delta row: ldd bf16 (ldd <= MAXO, multiple of 4) */
        __bf16 *dr = D + (size_t)row * ldd;
#pragma unroll
        for (int c = 0; c < MAXO; c += 4)
            if (c < ldd) *(bf16x4 *)(dr + c) = bf16x4{dv[c], dv[c + 1], dv[c + 2], dv[c + 3]};
        if (valid) {
            my_loss += (type == 2) ? -l / (float)n_out : 0.5f * l;
            my_hit += (io == it) ? 1u : 0u;
        }
    }
    block_reduce_store(my_loss, my_hit, loss_acc, correct);
}

/* wide outputs up to 64*NPL classes (RRUFF: 230): one wave per sample row, the row kept in
 * registers (NPL values per lane) so Z is read once instead of three times, and one row
 * per wave (the grid covers the batch): the three dependent wave reductions of a row no
 * longer serialize over many rows per wave */
template <int NPL>
__global__ __launch_bounds__(256) void output_delta_reg_kernel(const float *__restrict__ Z, int ldz,
                                                               const float *__restrict__ T, int ldt,
                                                               const int *__restrict__ labels, float t_hi, float t_lo,
                                                               __bf16 *__restrict__ D, int ldd, float *__restrict__ O,
                                                               int ldo, float *__restrict__ loss_acc,
                                                               unsigned int *__restrict__ correct, int B, int n_valid,
                                                               int n_out, int type) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float my_loss = 0.f;
    unsigned int my_hit = 0;
    for (int row = blockIdx.x * 4 + wave; row < B; row += gridDim.x * 4) {
        const bool valid = row < n_valid;
        const int lab = (labels && valid) ? labels[row] : -1;
        float z[NPL];
#pragma unroll
        for (int j = 0; j < NPL; j++) {
            const int c = lane + 64 * j;
            z[j] = c < n_out ? Z[(size_t)row * ldz + c] : -INFINITY;
        }
        float inv = 0.f, zmax = 0.f;
        if (type == 2) {
            zmax = z[0];
#pragma unroll
            for (int j = 1; j < NPL; j++) zmax = fmaxf(zmax, z[j]);
            zmax = wave_max(zmax);
            float denom = 0.f;
#pragma unroll
            for (int j = 0; j < NPL; j++)
                if (lane + 64 * j < n_out) denom += __expf(z[j] - zmax);
            denom = wave_sum(denom);
            /* reference: e^{z-1} / (TINY + sum e^{z-1}); shifted by m=zmax */
            denom += __expf(fminf(logf(TINY) + 1.0f - zmax, 80.f));
            inv = 1.0f / denom;
        }
        float bo = -INFINITY, bt = -INFINITY;
        int io = -1, it = -1;
        float l = 0.f;
#pragma unroll
        for (int j = 0; j < NPL; j++) {
            const int c = lane + 64 * j;
            float d = 0.f;
            if (c < n_out) {
                float o;
                if (type == 2) o = __expf(z[j] - zmax) * inv;
                else if (type == 0) o = 2.0f / (1.0f + __expf(-z[j])) - 1.0f;
                else o = z[j];
                if (valid) {
                    const float t = labels ? (c == lab ? t_hi : t_lo) : T[(size_t)row * ldt + c];
                    if (type == 2) {
                        if (o > 0.f) l += t * logf(o + TINY);
                        d = t - o;
                    } else if (type == 0) {
                        l += (t - o) * (t - o);
                        d = (t - o) * (-0.5f * (o * o - 1.0f));
                    } else {
                        l += (t - o) * (t - o);
                        d = t - o;
                    }
                    if (o > bo) { bo = o; io = c; }
                    if (t > bt) { bt = t; it = c; }
                }
                if (O) O[(size_t)row * ldo + c] = o;
            }
            if (c < ldd) D[(size_t)row * ldd + c] = (__bf16)d;
        }
        for (int c = 64 * NPL + lane; c < ldd; c += 64) D[(size_t)row * ldd + c] = (__bf16)0.f;
        l = wave_sum(l);
        wave_argmax(bo, io);
        wave_argmax(bt, it);
        if (valid && lane == 0) {
            my_loss += (type == 2) ? -l / (float)n_out : 0.5f * l;
            my_hit += (io == it) ? 1u : 0u;
        }
    }
    block_reduce_store(my_loss, my_hit, loss_acc, correct);
}

/* wide outputs up to 256 classes (RRUFF: 230), FOUR rows per wave: 16 lanes per row,
 * lane i of a row group owning columns [16 i, 16 i + 16) (four float4 loads, two 16-byte
 * delta stores).  The five row reductions (max, sum, loss, two argmax) run over 16 lanes
 * (4 shuffle steps instead of 6) and for 4 rows at once; the one-row-per-wave kernel above
 * spent ~17 us on 16384 x 230 in these dependent reductions.  Needs ldz, ldd (and ldo)
 * multiples of 16, ldd <= 256. */
__device__ __forceinline__ float g16_max(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 16));
    return v;
}
__device__ __forceinline__ float g16_sum(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
    return v;
}
__device__ __forceinline__ void g16_argmax(float &v, int &i) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 16);
        const int oi = __shfl_xor(i, o, 16);
        if (oi >= 0 && (i < 0 || ov > v || (ov == v && oi < i))) {
            v = ov;
            i = oi;
        }
    }
}

__global__ __launch_bounds__(256) void output_delta_q_kernel(const float *__restrict__ Z, int ldz,
                                                             const float *__restrict__ T, int ldt,
                                                             const int *__restrict__ labels, float t_hi, float t_lo,
                                                             __bf16 *__restrict__ D, int ldd, float *__restrict__ O,
                                                             int ldo, float *__restrict__ loss_acc,
                                                             unsigned int *__restrict__ correct, int B, int n_valid,
                                                             int n_out, int type) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int gi = lane & 15, c0 = 16 * gi;
    float my_loss = 0.f;
    unsigned int my_hit = 0;
    for (int row0 = (blockIdx.x * 4 + wave) * 4; row0 < B; row0 += gridDim.x * 16) {
        const int row = row0 + (lane >> 4);
        const bool in = row < B, valid = row < n_valid;
        const int lab = (labels && valid) ? labels[row] : -1;
        float z[16];
        if (in && c0 < ldz) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float4 v = *(const float4 *)(Z + (size_t)row * ldz + c0 + 4 * j);
                z[4 * j] = v.x;
                z[4 * j + 1] = v.y;
                z[4 * j + 2] = v.z;
                z[4 * j + 3] = v.w;
            }
        }
#pragma unroll
        for (int j = 0; j < 16; j++)
            if (!in || c0 + j >= n_out) z[j] = -INFINITY;
        float inv = 0.f, zmax = 0.f;
        if (type == 2) {
            zmax = z[0];
#pragma unroll
            for (int j = 1; j < 16; j++) zmax = fmaxf(zmax, z[j]);
            zmax = g16_max(zmax);
            float denom = 0.f;
#pragma unroll
            for (int j = 0; j < 16; j++) { /* z[j] <- e^{z - max}: computed once */
                z[j] = c0 + j < n_out ? __expf(z[j] - zmax) : 0.f;
                denom += z[j];
            }
            denom = g16_sum(denom);
            /* reference: e^{z-1} / (TINY + sum e^{z-1}); shifted by m=zmax */
            denom += __expf(fminf(logf(TINY) + 1.0f - zmax, 80.f));
            inv = 1.0f / denom;
        }
        float bo = -INFINITY, bt = -INFINITY, l = 0.f;
        int io = -1, it = -1;
        typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
        bf16x8 dv[2];
        float ov[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int c = c0 + j;
            float d = 0.f, o = 0.f;
            if (in && c < n_out) {
                if (type == 2) o = z[j] * inv;
                else if (type == 0) o = 2.0f / (1.0f + __expf(-z[j])) - 1.0f;
                else o = z[j];
                if (valid) {
                    const float t = labels ? (c == lab ? t_hi : t_lo) : T[(size_t)row * ldt + c];
                    if (type == 2) {
                        if (t != 0.f && o > 0.f) l += t * logf(o + TINY); /* one-hot: one log per row */
                        d = t - o;
                    } else if (type == 0) {
                        l += (t - o) * (t - o);
                        d = (t - o) * (-0.5f * (o * o - 1.0f));
                    } else {
                        l += (t - o) * (t - o);
                        d = t - o;
                    }
                    if (o > bo) { bo = o; io = c; }
                    if (t > bt) { bt = t; it = c; }
                }
            }
            ov[j] = o;
            dv[j >> 3][j & 7] = (__bf16)d;
        }
        if (in && c0 < ldd) {
            *(bf16x8 *)(D + (size_t)row * ldd + c0) = dv[0];
            *(bf16x8 *)(D + (size_t)row * ldd + c0 + 8) = dv[1];
        }
        if (O && in && c0 < ldo) {
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (c0 + j < n_out) O[(size_t)row * ldo + c0 + j] = ov[j];
        }
        l = g16_sum(l);
        g16_argmax(bo, io);
        g16_argmax(bt, it);
        if (valid && gi == 0) {
            my_loss += (type == 2) ? -l / (float)n_out : 0.5f * l;
            my_hit += (io == it) ? 1u : 0u;
        }
    }
    block_reduce_store(my_loss, my_hit, loss_acc, correct);
}

/* very wide outputs (> 256 classes, e.g. the synthetic 4096-wide ANN): one wave per row,
 * every lane handling 4 consecutive columns per step (float4 Z / T loads, 8-byte delta
 * stores); needs ldz and ldd multiples of 4.  The scalar kernel below moved
 * 256 B per wave instruction and ran the 8192 x 4096 output at ~2 TB/s. */
__global__ __launch_bounds__(256) void output_delta_v4_kernel(const float *__restrict__ Z, int ldz,
                                                              const float *__restrict__ T, int ldt,
                                                              const int *__restrict__ labels, float t_hi, float t_lo,
                                                              __bf16 *__restrict__ D, int ldd, float *__restrict__ O,
                                                              int ldo, float *__restrict__ loss_acc,
                                                              unsigned int *__restrict__ correct, int B, int n_valid,
                                                              int n_out, int type) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    float my_loss = 0.f;
    unsigned int my_hit = 0;
    const int cend = ldd > n_out ? ldd : n_out;
    for (int row = blockIdx.x * 4 + wave; row < B; row += gridDim.x * 4) {
        const bool valid = row < n_valid;
        const int lab = (labels && valid) ? labels[row] : -1;
        const float *zr = Z + (size_t)row * ldz;
        float zmax = -INFINITY, denom = 0.f;
        if (type == 2) {
            for (int c = 4 * lane; c < n_out; c += 256) {
                const float4 v = *(const float4 *)(zr + c);
                const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (c + r < n_out) zmax = fmaxf(zmax, e[r]);
            }
            zmax = wave_max(zmax);
            for (int c = 4 * lane; c < n_out; c += 256) {
                const float4 v = *(const float4 *)(zr + c);
                const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (c + r < n_out) denom += __expf(e[r] - zmax);
            }
            denom = wave_sum(denom);
            denom += __expf(fminf(logf(TINY) + 1.0f - zmax, 80.f));
        }
        const float inv = type == 2 ? 1.0f / denom : 0.f;
        float bo = -INFINITY, bt = -INFINITY, l = 0.f;
        int io = -1, it = -1;
        for (int c = 4 * lane; c < cend; c += 256) {
            float e[4] = {0.f, 0.f, 0.f, 0.f}, tv[4] = {t_lo, t_lo, t_lo, t_lo};
            if (c < n_out) {
                const float4 v = *(const float4 *)(zr + c);
                e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
                if (!labels && valid) {
                    const float *tr = T + (size_t)row * ldt + c;
                    if ((ldt & 3) == 0 && ((uintptr_t)T & 15) == 0) {
                        const float4 w = *(const float4 *)tr;
                        tv[0] = w.x; tv[1] = w.y; tv[2] = w.z; tv[3] = w.w;
                    } else { /* unaligned target rows: scalar loads, same values */
#pragma unroll
                        for (int r = 0; r < 4; r++) tv[r] = c + r < n_out ? tr[r] : t_lo;
                    }
                }
            }
            bf16x4 dv;
            float ov[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int cc = c + r;
                float d = 0.f, o = 0.f;
                if (cc < n_out) {
                    if (type == 2) o = __expf(e[r] - zmax) * inv;
                    else if (type == 0) o = 2.0f / (1.0f + __expf(-e[r])) - 1.0f;
                    else o = e[r];
                    if (valid) {
                        const float t = labels ? (cc == lab ? t_hi : t_lo) : tv[r];
                        if (type == 2) {
                            if (t != 0.f && o > 0.f) l += t * logf(o + TINY);
                            d = t - o;
                        } else if (type == 0) {
                            l += (t - o) * (t - o);
                            d = (t - o) * (-0.5f * (o * o - 1.0f));
                        } else {
                            l += (t - o) * (t - o);
                            d = t - o;
                        }
                        if (o > bo) { bo = o; io = cc; }
                        if (t > bt) { bt = t; it = cc; }
                    }
                }
                ov[r] = o;
                dv[r] = (__bf16)d;
            }
            if (c < ldd) *(bf16x4 *)(D + (size_t)row * ldd + c) = dv;
            if (O && c < n_out) {
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (c + r < n_out) O[(size_t)row * ldo + c + r] = ov[r];
            }
        }
        l = wave_sum(l);
        wave_argmax(bo, io);
        wave_argmax(bt, it);
        if (valid && lane == 0) {
            my_loss += (type == 2) ? -l / (float)n_out : 0.5f * l;
            my_hit += (io == it) ? 1u : 0u;
        }
    }
    block_reduce_store(my_loss, my_hit, loss_acc, correct);
}

/* wide outputs: one WAVE per sample row, grid-stride */
__global__ __launch_bounds__(256) void output_delta_kernel(const float *__restrict__ Z, int ldz,
                                                           const float *__restrict__ T, int ldt,
                                                           const int *__restrict__ labels, float t_hi, float t_lo,
                                                           __bf16 *__restrict__ D, int ldd, float *__restrict__ O,
                                                           int ldo, float *__restrict__ loss_acc,
                                                           unsigned int *__restrict__ correct, int B, int n_valid,
                                                           int n_out, int type) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float my_loss = 0.f;
    unsigned int my_hit = 0;
    for (int row = blockIdx.x * 4 + wave; row < B; row += gridDim.x * 4) {
        const bool valid = row < n_valid;
        const int lab = (labels && valid) ? labels[row] : -1;
        float zmax = -INFINITY;
        if (type == 2) {
            for (int c = lane; c < n_out; c += 64) zmax = fmaxf(zmax, Z[(size_t)row * ldz + c]);
            zmax = wave_max(zmax);
        }
        float denom = 0.f;
        if (type == 2) {
            for (int c = lane; c < n_out; c += 64) denom += __expf(Z[(size_t)row * ldz + c] - zmax);
            denom = wave_sum(denom);
            /* reference: e^{z-1} / (TINY + sum e^{z-1}); shifted by m=zmax */
            denom += __expf(fminf(logf(TINY) + 1.0f - zmax, 80.f));
        }
        const float inv = type == 2 ? 1.0f / denom : 0.f;
        float bo = -INFINITY, bt = -INFINITY;
        int io = -1, it = -1;
        float l = 0.f;
        for (int c = lane; c < (ldd > n_out ? ldd : n_out); c += 64) {
            float d = 0.f;
            if (c < n_out) {
                const float z = Z[(size_t)row * ldz + c];
                float o;
                if (type == 2) o = __expf(z - zmax) * inv;
                else if (type == 0) o = 2.0f / (1.0f + __expf(-z)) - 1.0f;
                else o = z;
                if (valid) {
                    const float t = labels ? (c == lab ? t_hi : t_lo) : T[(size_t)row * ldt + c];
                    if (type == 2) {
                        if (o > 0.f) l += t * logf(o + TINY);
                        d = t - o;
                    } else if (type == 0) {
                        l += (t - o) * (t - o);
                        d = (t - o) * (-0.5f * (o * o - 1.0f));
                    } else {
                        l += (t - o) * (t - o);
                        d = t - o;
                    }
                    if (o > bo) { bo = o; io = c; }
                    if (t > bt) { bt = t; it = c; }
                }
                if (O) O[(size_t)row * ldo + c] = o;
            }
            if (c < ldd) D[(size_t)row * ldd + c] = (__bf16)d;
        }
        l = wave_sum(l);
        wave_argmax(bo, io);
        wave_argmax(bt, it);
        if (valid && lane == 0) {
            my_loss += (type == 2) ? -l / (float)n_out : 0.5f * l;
            my_hit += (io == it) ? 1u : 0u;
        }
    }
    block_reduce_store(my_loss, my_hit, loss_acc, correct);
}

/* many slabs: 4 waves per 64 f32x4 of output, wave w adds slabs w, w+4, ... in two
 * independent chains (more loads in flight per lane, 4x the workgroups of the simple
 * kernel); the partials meet in LDS in wave order, so the sum is deterministic */
__global__ __launch_bounds__(256) void reduce_slabs_wide_kernel(const float *__restrict__ slab, int S, long stride,
                                                                long n4, float *__restrict__ out) {
    __shared__ f32x4 part[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long e = (long)blockIdx.x * 64 + lane;
    f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a;
    if (e < n4) {
        int s = w;
        for (; s + 4 < S; s += 8) {
            a += ((const f32x4 *)(slab + (long)s * stride))[e];
            b += ((const f32x4 *)(slab + (long)(s + 4) * stride))[e];
        }
        if (s < S) a += ((const f32x4 *)(slab + (long)s * stride))[e];
    }
    part[w][lane] = a + b;
    __syncthreads();
    if (w == 0 && e < n4) ((f32x4 *)out)[e] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}

__global__ __launch_bounds__(256) void reduce_slabs_kernel(const float *__restrict__ slab, int S, long stride, long n4,
                                                           float *__restrict__ out) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
        f32x4 a = ((const f32x4 *)slab)[i];
        for (int s = 1; s < S; s++) a += ((const f32x4 *)(slab + s * stride))[i];
        ((f32x4 *)out)[i] = a;
    }
}

/* 32x32 tile per block, 256 threads: thread (ty = tid/8, tx = tid%8) owns
 * row ty, columns 4tx..4tx+3 of the tile. */
/* one 32x32 tile of the optimizer step (see hpnn_sgd_update); tile = (tn, tk) */
__device__ __forceinline__ void sgd_tile(float *__restrict__ W32, float *__restrict__ V32, const float *__restrict__ G,
                                         int S, long gstride, __bf16 *__restrict__ Wbf, __bf16 *__restrict__ Wt,
                                         __bf16 *__restrict__ Wf, int N, int K, int tile, float lr, float alpha,
                                         float scale, int momentum, float (*tilebuf)[33]) {
    const int tiles_k = K / 32;
    const int tn = tile / tiles_k, tk = tile % tiles_k;
    const int tx = threadIdx.x & 7, ty = threadIdx.x >> 3;
    const int n = tn * 32 + ty, k = tk * 32 + tx * 4;
    const size_t idx = (size_t)n * K + k;
    f32x4 g = *(const f32x4 *)(G + idx);
    {
        /* four independent partial sums keep several slab loads in flight */
        f32x4 g1 = {0.f, 0.f, 0.f, 0.f}, g2 = g1, g3 = g1;
        int s = 1;
        for (; s + 3 < S; s += 4) {
            g += *(const f32x4 *)(G + (long)s * gstride + idx);
            g1 += *(const f32x4 *)(G + (long)(s + 1) * gstride + idx);
            g2 += *(const f32x4 *)(G + (long)(s + 2) * gstride + idx);
            g3 += *(const f32x4 *)(G + (long)(s + 3) * gstride + idx);
        }
        for (; s < S; s++) g += *(const f32x4 *)(G + (long)s * gstride + idx);
        g += (g1 + g2) + g3;
    }
    f32x4 w = *(const f32x4 *)(W32 + idx);
    if (momentum) {
        f32x4 v = *(const f32x4 *)(V32 + idx);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            v[r] += lr * (g[r] * scale);
            w[r] += v[r];
            v[r] *= alpha;
        }
        *(f32x4 *)(V32 + idx) = v;
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) w[r] += lr * (g[r] * scale);
    }
    *(f32x4 *)(W32 + idx) = w;
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    bf16x4 wb;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        wb[r] = (__bf16)w[r];
        tilebuf[ty][tx * 4 + r] = w[r];
    }
    *(bf16x4 *)(Wbf + idx) = wb;
    if (Wf) {
        /* MFMA-fragment-major copy (kernels.h): 4 consecutive k stay contiguous */
        const size_t fo = (((size_t)(n >> 4) * tiles_k + (k >> 5)) * 64 + (n & 15) + 16 * ((k >> 3) & 3)) * 8 + (k & 7);
        *(bf16x4 *)(Wf + fo) = wb;
    }
    __syncthreads();
    /* transposed: thread writes Wt[k = tk*32 + ty][n = tn*32 + 4tx .. +3] */
    bf16x4 tb;
#pragma unroll
    for (int r = 0; r < 4; r++) tb[r] = (__bf16)tilebuf[tx * 4 + r][ty];
    *(bf16x4 *)(Wt + (size_t)(tk * 32 + ty) * N + tn * 32 + tx * 4) = tb;
}

__global__ __launch_bounds__(256) void sgd_update_kernel(float *__restrict__ W32, float *__restrict__ V32,
                                                         const float *__restrict__ G, int S, long gstride,
                                                         __bf16 *__restrict__ Wbf, __bf16 *__restrict__ Wt, int N,
                                                         int K, float lr, float alpha, float scale, int momentum) {
    __shared__ float tile[32][33];
    sgd_tile(W32, V32, G, S, gstride, Wbf, Wt, nullptr, N, K, blockIdx.x, lr, alpha, scale, momentum, tile);
}

struct UpdArgs {
    hpnn_upd_layer L[HPNN_UPD_MAX];
    int tile0[HPNN_UPD_MAX + 1];
    int n;
    float lr, alpha, scale;
    int momentum;
    int prefetch; /* sub-tile kernel: W / V loads issued with the slab loads (HPNN_UPD_PREFETCH) */
};

__global__ __launch_bounds__(256) void sgd_update_multi_kernel(UpdArgs a) {
    __shared__ float tile[32][33];
    int l = 0;
    while (l + 1 < a.n && (int)blockIdx.x >= a.tile0[l + 1]) l++;
    const hpnn_upd_layer &L = a.L[l];
    sgd_tile(L.W32, L.V32, L.G, L.S, L.gstride, (__bf16 *)L.Wbf, (__bf16 *)L.Wt, (__bf16 *)L.Wf, L.N, L.K,
             blockIdx.x - a.tile0[l], a.lr, a.alpha, a.scale, a.momentum, tile);
}


/* Same step over 8-row sub-tiles (8 x 32 elements, one f32x4 per lane of a wave): four
 * workgroups per 32x32 tile, so MNIST's update (~110 tiles) fills the 256 CUs (~440
 * workgroups) instead of leaving half the chip idle while the slabs stream.  8 waves; wave
 * w sums slabs w, w+8, ..., up to 8 per iteration, added as a fixed pairwise tree (a wave
 * whose layer has fewer than w+1 slabs adds nothing); partials meet in LDS in wave order
 * (deterministic); wave 0 applies the step.  tile0[] counts sub-tiles here.  The slab sum
 * order differs from the HPNN_UPD_MODE=1 kernel, so the two modes agree only to the last
 * FP32 bits. */
__global__ __launch_bounds__(512) void sgd_update_multi_sub_kernel(UpdArgs a) {
    __shared__ f32x4 part[8][64];
    __shared__ float tilebuf[8][33];
    int l = 0;
    while (l + 1 < a.n && (int)blockIdx.x >= a.tile0[l + 1]) l++;
    const hpnn_upd_layer &L = a.L[l];
    const int local = blockIdx.x - a.tile0[l];
    const int tile = local >> 2, sub = local & 3;
    const int tiles_k = L.K / 32;
    const int tn = tile / tiles_k, tk = tile % tiles_k;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ty = lane >> 3, tx = lane & 7;
    const int n = tn * 32 + sub * 8 + ty, k = tk * 32 + tx * 4;
    const size_t idx = (size_t)n * L.K + k;
    /* the updating wave fetches its weights (and momentum) first, so those loads are in
     * flight together with the slab loads instead of a round trip after the barrier */
    f32x4 wv = {0.f, 0.f, 0.f, 0.f}, vv = wv;
    if (w == 0 && a.prefetch) {
        wv = *(const f32x4 *)(L.W32 + idx);
        if (a.momentum) vv = *(const f32x4 *)(L.V32 + idx);
    }
    /* up to 8 slab loads per lane in flight at once (the step is load-latency bound:
     * each wave owns only S/8 slabs), summed in a fixed order */
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s0 = w; s0 < L.S; s0 += 64) {
        f32x4 x[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int s = s0 + 8 * j;
            x[j] = s < L.S ? *(const f32x4 *)(L.G + (long)s * L.gstride + idx) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        acc += ((x[0] + x[1]) + (x[2] + x[3])) + ((x[4] + x[5]) + (x[6] + x[7]));
    }
    part[w][lane] = acc;
    __syncthreads();
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    if (w == 0) {
        f32x4 g = part[0][lane];
#pragma unroll
        for (int ww = 1; ww < 8; ww++) g += part[ww][lane];
        if (!a.prefetch) {
            wv = *(const f32x4 *)(L.W32 + idx);
            if (a.momentum) vv = *(const f32x4 *)(L.V32 + idx);
        }
        if (a.momentum) {
            f32x4 v = vv;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                v[r] += a.lr * (g[r] * a.scale);
                wv[r] += v[r];
                v[r] *= a.alpha;
            }
            *(f32x4 *)(L.V32 + idx) = v;
        } else {
#pragma unroll
            for (int r = 0; r < 4; r++) wv[r] += a.lr * (g[r] * a.scale);
        }
        *(f32x4 *)(L.W32 + idx) = wv;
        bf16x4 wb;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            wb[r] = (__bf16)wv[r];
            tilebuf[ty][tx * 4 + r] = wv[r];
        }
        *(bf16x4 *)((__bf16 *)L.Wbf + idx) = wb;
        if (L.Wf) {
            const size_t fo = (((size_t)(n >> 4) * tiles_k + (k >> 5)) * 64 + (n & 15) + 16 * ((k >> 3) & 3)) * 8 + (k & 7);
            *(bf16x4 *)((__bf16 *)L.Wf + fo) = wb;
        }
    }
    __syncthreads();
    if (w == 0) {
        /* transposed: lane writes Wt[k = tk*32 + lane/2][n = tn*32 + sub*8 + 4(lane&1) .. +3] */
        const int kk = lane >> 1, nh = (lane & 1) * 4;
        bf16x4 tb;
#pragma unroll
        for (int r = 0; r < 4; r++) tb[r] = (__bf16)tilebuf[nh + r][kk];
        *(bf16x4 *)((__bf16 *)L.Wt + (size_t)(tk * 32 + kk) * L.N + tn * 32 + sub * 8 + nh) = tb;
    }
}

/* ---- pieces of the BF16 reduce-scatter data-parallel step (csrc/dist/dp_exchange.cpp) ---- */
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float *__restrict__ src, __bf16 *__restrict__ dst,
                                                            long n4) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const f32x4 v = ((const f32x4 *)src)[i];
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; r++) o[r] = (__bf16)v[r];
        ((bf16x4_t *)dst)[i] = o;
    }
}

/* the optimizer step of this rank's rows from their BF16 gradient sum: W32 / V32 rows (FP32
 * masters, sharded) and the BF16 compute rows Wb (all-gathered afterwards) */
__global__ __launch_bounds__(256) void sgd_rows_bf16g_kernel(float *__restrict__ W32, float *__restrict__ V32,
                                                             const __bf16 *__restrict__ G, long n4, float lr,
                                                             float alpha, float scale, int momentum,
                                                             __bf16 *__restrict__ Wb) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const bf16x4_t g16 = ((const bf16x4_t *)G)[i];
        f32x4 w = ((const f32x4 *)W32)[i];
        if (momentum) {
            f32x4 v = ((const f32x4 *)V32)[i];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                v[r] += lr * ((float)g16[r] * scale);
                w[r] += v[r];
                v[r] *= alpha;
            }
            ((f32x4 *)V32)[i] = v;
        } else {
#pragma unroll
            for (int r = 0; r < 4; r++) w[r] += lr * ((float)g16[r] * scale);
        }
        ((f32x4 *)W32)[i] = w;
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; r++) o[r] = (__bf16)w[r];
        ((bf16x4_t *)Wb)[i] = o;
    }
}

/* Wt [K][N] = Wb^T for a [N][K] BF16 matrix, 32 x 32 tiles through LDS */
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const __bf16 *__restrict__ Wb, __bf16 *__restrict__ Wt,
                                                             int N, int K) {
    __shared__ __bf16 t[32][34];
    const int tk = K / 32, tn = blockIdx.x / tk, tkk = blockIdx.x % tk;
    const int x = threadIdx.x & 31, y = threadIdx.x >> 5; /* y 0..7 */
#pragma unroll
    for (int j = 0; j < 4; j++) t[y + 8 * j][x] = Wb[(size_t)(tn * 32 + y + 8 * j) * K + tkk * 32 + x];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; j++) Wt[(size_t)(tkk * 32 + y + 8 * j) * N + tn * 32 + x] = t[x][y + 8 * j];
}

/* ---- pieces of the BF16 row-sharded tensor-parallel step (tp_engine.cpp TpNetBf16) ---- */
/* dst [rows][P n] <- src [P][rows][n]: the all-gathered per-rank feature blocks of a layer's
 * activations into the batch-major input of the next GEMM (8 bf16 per thread) */
__global__ __launch_bounds__(256) void block_permute_bf16_kernel(const __bf16 *__restrict__ src,
                                                                 __bf16 *__restrict__ dst, int P, long rows, int n) {
    typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
    const int n8 = n / 8;
    const long total = (long)P * rows * n8;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c8 = (int)(i % n8);
        const long pr = i / n8;
        const long r = pr % rows;
        const int p = (int)(pr / rows);
        ((bf16x8_t *)(dst + r * (long)P * n + (long)p * n))[c8] = ((const bf16x8_t *)(src + pr * n))[c8];
    }
}

/* out = bf16(in * f'(H)), f'(y) = -0.5 (y^2 - 1): the f' epilogue on reduce-scattered FP32
 * partial deltas (4 per thread) */
__global__ __launch_bounds__(256) void dact_f32_bf16_kernel(__bf16 *__restrict__ out, const float *__restrict__ in,
                                                            const __bf16 *__restrict__ H, long n4) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const f32x4 v = ((const f32x4 *)in)[i];
        const bf16x4_t h = ((const bf16x4_t *)H)[i];
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const float y = (float)h[r];
            o[r] = (__bf16)(v[r] * (-0.5f * (y * y - 1.0f)));
        }
        ((bf16x4_t *)out)[i] = o;
    }
}

__global__ void pack_bf16_kernel(const void *__restrict__ src, int src_f64, int rows, int cols, int lds,
                                 __bf16 *__restrict__ dst, int prow, int pcol, int ldd) {
    const long total = (long)prow * pcol;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int r = (int)(i / pcol), c = (int)(i % pcol);
        float v = 0.f;
        if (r < rows && c < cols)
            v = src_f64 ? (float)((const double *)src)[(size_t)r * lds + c] : ((const float *)src)[(size_t)r * lds + c];
        dst[(size_t)r * ldd + c] = (__bf16)v;
    }
}

__global__ void fill_kernel(float *p, long n, float v) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v;
}

inline int grid_for(long n, int bs) {
    long g = (n + bs - 1) / bs;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

/* HPNN_OD_WAVE=1: one row per wave for wide outputs (the kernel before output_delta_q) */
static bool od_wave_mode() {
    static const bool v = [] { const char *e = getenv("HPNN_OD_WAVE"); return e && e[0] == '1'; }();
    return v;
}

/* order-independent 64-bit digest of a buffer's 4-byte words: the wrapping sum over i of a
 * murmur3 finalizer of (word << 32 | i).  Equal buffers give equal digests on every device
 * and run (integer adds commute); one changed bit changes it.  Used to check that data-
 * parallel replicas hold bitwise-identical weights (bench.py, train_nn under a launcher). */
__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
__global__ __launch_bounds__(256) void hash_words_kernel(const unsigned int *__restrict__ w, long n, long base,
                                                         unsigned long long *__restrict__ out) {
    unsigned long long h = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        h += mix64(((unsigned long long)w[i] << 32) ^ (unsigned long long)(i + base) ^ 0x9e3779b97f4a7c15ull);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, h);
}

extern "C" int hpnn_hash_words(const void *p, long nbytes, long base, unsigned long long *out, hipStream_t stream) {
    if (!p || !out || nbytes < 0 || nbytes % 4) return -1;
    const long n = nbytes / 4;
    if (n == 0) return 0;
    long blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(hash_words_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const unsigned int *)p, n,
                       base, out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_resident_capacity(const void *kernel, int threads, size_t dyn_lds) {
    static std::mutex mu;
    static std::map<std::tuple<const void *, int, size_t>, int> cache;
    std::lock_guard<std::mutex> g(mu);
    const auto key = std::make_tuple(kernel, threads, dyn_lds);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, dyn_lds) != hipSuccess)
        cus = per = 0; /* unknown: no grid counts as resident (callers take their other forms) */
    return cache[key] = cus * per;
}

extern "C" {
const void *hpnn_co_probe_8ph(void);
const void *hpnn_co_probe_fp(void);
const void *hpnn_co_probe_g0(void);
const void *hpnn_co_probe_mfma(void);
const void *hpnn_co_probe_mlp3(void);
const void *hpnn_co_probe_mlp3t(void);
const void *hpnn_co_probe_mlp3x(void);
const void *hpnn_co_probe_wide(void);
const void *hpnn_co_probe_ws(void);
const void *hpnn_co_probe_online(void);
const void *hpnn_co_probe_xar(void);
}

extern "C" int hpnn_preload_code_objects(void) {
    static std::mutex mu;
    static std::map<int, int> done; /* device -> result */
    std::lock_guard<std::mutex> g(mu);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    auto it = done.find(dev);
    if (it != done.end()) return it->second;
    const void *probes[] = {hpnn_co_probe_8ph(),  hpnn_co_probe_fp(),   hpnn_co_probe_g0(),    hpnn_co_probe_mfma(),
                            hpnn_co_probe_misc(), hpnn_co_probe_mlp3(), hpnn_co_probe_mlp3t(), hpnn_co_probe_mlp3x(),
                            hpnn_co_probe_wide(), hpnn_co_probe_ws(),   hpnn_co_probe_online(), hpnn_co_probe_xar()};
    /* an empty one-thread launch per unit: the launch is what loads its code object */
    hipStream_t s = nullptr;
    int rc = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? 0 : -1;
    for (const void *k : probes)
        if (rc == 0 && hipLaunchKernel(k, dim3(1), dim3(1), nullptr, 0, s) != hipSuccess) rc = -2;
    if (s) {
        if (hipStreamSynchronize(s) != hipSuccess) rc = -3;
        (void)hipStreamDestroy(s);
    }
    return done[dev] = rc;
}

extern "C" int hpnn_output_delta(const float *Z, int ldz, const float *T, int ldt, const int *labels, float t_hi,
                                 float t_lo, void *D, int ldd, float *O, int ldo, float *loss_acc,
                                 unsigned int *correct, int B, int n_valid, int n_out, int type,
                                 hipStream_t stream) {
    if (B <= 0 || n_out <= 0 || ldz < n_out || ldd < n_out) return -1;
    if (!labels && !T) return -1;
    if (ldd <= 32 && ldd % 4 == 0) {
        const int grid = (B + 255) / 256 < 256 ? (B + 255) / 256 : 256;
        hipLaunchKernelGGL(output_delta_rows_kernel<32>, dim3(grid), dim3(256), 0, stream, Z, ldz, T, ldt, labels,
                           t_hi, t_lo, (__bf16 *)D, ldd, O, ldo, loss_acc, correct, B, n_valid, n_out, type);
    } else if (n_out > 64 && ldz % 16 == 0 && ldd % 16 == 0 && ldd <= 256 && ldz >= ldd && (!O || ldo % 16 == 0) &&
               !od_wave_mode()) {
        /* four rows per wave (16 lanes per row): the grid covers the batch */
        const int grid = (B + 15) / 16 < 4096 ? (B + 15) / 16 : 4096;
        hipLaunchKernelGGL(output_delta_q_kernel, dim3(grid), dim3(256), 0, stream, Z, ldz, T, ldt, labels, t_hi, t_lo,
                           (__bf16 *)D, ldd, O, ldo, loss_acc, correct, B, n_valid, n_out, type);
    } else if (n_out <= 256) {
        /* one row per wave: the grid covers the batch (up to 16 waves per CU) */
        const int grid = (B + 3) / 4 < 4096 ? (B + 3) / 4 : 4096;
#define HPNN_OD(NPL_)                                                                                              \
    hipLaunchKernelGGL(output_delta_reg_kernel<NPL_>, dim3(grid), dim3(256), 0, stream, Z, ldz, T, ldt, labels, t_hi, \
                       t_lo, (__bf16 *)D, ldd, O, ldo, loss_acc, correct, B, n_valid, n_out, type)
        if (n_out <= 64) HPNN_OD(1);
        else if (n_out <= 128) HPNN_OD(2);
        else if (n_out <= 192) HPNN_OD(3);
        else HPNN_OD(4);
#undef HPNN_OD
    } else if (ldz % 4 == 0 && ldd % 4 == 0 && ((uintptr_t)Z & 15) == 0 && ((uintptr_t)D & 7) == 0 &&
               !od_wave_mode()) {
        const int grid = (B + 3) / 4 < 4096 ? (B + 3) / 4 : 4096;
        hipLaunchKernelGGL(output_delta_v4_kernel, dim3(grid), dim3(256), 0, stream, Z, ldz, T, ldt, labels, t_hi,
                           t_lo, (__bf16 *)D, ldd, O, ldo, loss_acc, correct, B, n_valid, n_out, type);
    } else {
        const int grid = (B + 3) / 4 < 4096 ? (B + 3) / 4 : 4096;
        hipLaunchKernelGGL(output_delta_kernel, dim3(grid), dim3(256), 0, stream, Z, ldz, T, ldt, labels, t_hi,
                           t_lo, (__bf16 *)D, ldd, O, ldo, loss_acc, correct, B, n_valid, n_out, type);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_reduce_slabs(const float *slab, int S, long stride, long n, float *out, hipStream_t stream) {
    if (n % 4 || stride % 4 || S < 1) return -2;
    if (S >= 8) {
        const long n4 = n / 4;
        hipLaunchKernelGGL(reduce_slabs_wide_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, stream, slab, S,
                           stride, n4, out);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    hipLaunchKernelGGL(reduce_slabs_kernel, dim3(grid_for(n / 4, 256)), dim3(256), 0, stream, slab, S, stride, n / 4,
                       out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_sgd_update(float *W32, float *V32, const float *G, int S, long gstride, void *Wbf, void *Wt,
                               int N, int K, float lr, float alpha, float scale, int momentum, hipStream_t stream) {
    if (N % 32 || K % 32 || S < 1) return -2;
    if (momentum && !V32) return -1;
    hipLaunchKernelGGL(sgd_update_kernel, dim3((N / 32) * (K / 32)), dim3(256), 0, stream, W32, V32, G, S, gstride,
                       (__bf16 *)Wbf, (__bf16 *)Wt, N, K, lr, alpha, scale, momentum);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_sgd_update_multi(const hpnn_upd_layer *layers, int n, float lr, float alpha, float scale,
                                     int momentum, hipStream_t stream) {
    if (n < 1 || n > HPNN_UPD_MAX) return -1;
    UpdArgs a;
    a.n = n;
    a.lr = lr;
    a.alpha = alpha;
    a.scale = scale;
    a.momentum = momentum;
    static const int prefetch = [] { const char *e = getenv("HPNN_UPD_PREFETCH"); return !(e && e[0] == '0'); }();
    a.prefetch = prefetch;
    int t = 0;
    for (int l = 0; l < n; l++) {
        const hpnn_upd_layer &L = layers[l];
        if (L.N % 32 || L.K % 32 || L.S < 1) return -2;
        /* the slab-reduction kernels read 16-byte f32x4 vectors at s * gstride */
        if (L.S > 1 && L.gstride % 4) return -2;
        if (momentum && !L.V32) return -1;
        a.L[l] = L;
        a.tile0[l] = t;
        t += (L.N / 32) * (L.K / 32);
    }
    a.tile0[n] = t;
    int max_s = 0;
    for (int l = 0; l < n; l++) max_s = layers[l].S > max_s ? layers[l].S : max_s;
    static const int wide_off = [] { const char *e = getenv("HPNN_UPD_NARROW"); return e && atoi(e) ? 1 : 0; }();
    if (max_s >= 8 && !wide_off) {
        for (int l = 0; l <= n; l++) a.tile0[l] *= 4;
        hipLaunchKernelGGL(sgd_update_multi_sub_kernel, dim3(4 * t), dim3(512), 0, stream, a);
    } else
        hipLaunchKernelGGL(sgd_update_multi_kernel, dim3(t), dim3(256), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_cast_f32_bf16(const float *src, void *dst, long n, hipStream_t stream) {
    if (n <= 0 || n % 4 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 7)) return -2;
    hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n / 4, 256)), dim3(256), 0, stream, src, (__bf16 *)dst,
                       n / 4);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_sgd_update_rows_bf16g(float *W32, float *V32, const void *G16, long n, float lr, float alpha,
                                          float scale, int momentum, void *Wbf, hipStream_t stream) {
    if (n <= 0 || n % 4 || (momentum && !V32) || (((uintptr_t)W32 | (uintptr_t)(momentum ? V32 : W32)) & 15) ||
        (((uintptr_t)G16 | (uintptr_t)Wbf) & 7))
        return -2;
    hipLaunchKernelGGL(sgd_rows_bf16g_kernel, dim3(grid_for(n / 4, 256)), dim3(256), 0, stream, W32, V32,
                       (const __bf16 *)G16, n / 4, lr, alpha, scale, momentum, (__bf16 *)Wbf);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_block_permute_bf16(const void *src, void *dst, int P, long rows, int n, hipStream_t stream) {
    if (P < 1 || rows < 1 || n < 8 || n % 8 || (((uintptr_t)src | (uintptr_t)dst) & 15)) return -2;
    hipLaunchKernelGGL(block_permute_bf16_kernel, dim3(grid_for((long)P * rows * (n / 8), 256)), dim3(256), 0, stream,
                       (const __bf16 *)src, (__bf16 *)dst, P, rows, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_dact_f32_bf16(void *out, const float *in, const void *H, long n, hipStream_t stream) {
    if (n <= 0 || n % 4 || ((uintptr_t)in & 15) || (((uintptr_t)out | (uintptr_t)H) & 7)) return -2;
    hipLaunchKernelGGL(dact_f32_bf16_kernel, dim3(grid_for(n / 4, 256)), dim3(256), 0, stream, (__bf16 *)out, in,
                       (const __bf16 *)H, n / 4);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_transpose_bf16(const void *Wbf, void *Wt, int N, int K, hipStream_t stream) {
    if (N <= 0 || K <= 0 || N % 32 || K % 32) return -2;
    hipLaunchKernelGGL(transpose_bf16_kernel, dim3((N / 32) * (K / 32)), dim3(256), 0, stream, (const __bf16 *)Wbf,
                       (__bf16 *)Wt, N, K);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_cast_weights(const float *W32, void *Wbf, void *Wt, int N, int K, hipStream_t stream) {
    /* an update with lr = 0 and a zero gradient is exactly a cast: reuse the
     * same kernel with G = W32 and scale 0 */
    return hpnn_sgd_update((float *)W32, NULL, W32, 1, 0, Wbf, Wt, N, K, 0.f, 0.f, 0.f, 0, stream);
}

extern "C" int hpnn_pack_bf16(const void *src, int src_f64, int rows, int cols, int lds, void *dst, int prow,
                              int pcol, int ldd, hipStream_t stream) {
    if (rows > prow || cols > pcol || ldd < pcol) return -1;
    hipLaunchKernelGGL(pack_bf16_kernel, dim3(grid_for((long)prow * pcol, 256)), dim3(256), 0, stream, src, src_f64,
                       rows, cols, lds, (__bf16 *)dst, prow, pcol, ldd);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int hpnn_fill_f32(float *p, long n, float v, hipStream_t stream) {
    hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, p, n, v);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
