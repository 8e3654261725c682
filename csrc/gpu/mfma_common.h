/*
 * Shared gfx950 MFMA / LDS helpers for the libhpnn HIP kernels.
 *
 * LDS activation image ("T32 image"): a [rows][cols] bf16 tile stored as cols/32
 * sub-tiles of [rows][32] (64-byte rows); inside a sub-tile the four 16-byte chunks
 * of row r are permuted by chunk ^ g(r), g(r) = bit1(r) | bit3(r) << 1 (found by
 * an exhaustive bank simulation: conflict-free ds_read_b128 row reads and
 * ds_read_b64_tr_b16 transposed reads, 2-way -- the minimum for this shape --
 * ds_write_b64 of MFMA accumulator rows).  One image serves
 *   - row reads      (ds_read_b128, 8 consecutive columns of one row: MFMA operand
 *                     whose k runs along the features)
 *   - transposed reads (ds_read_b64_tr_b16: MFMA operand whose k runs along the rows,
 *                     i.e. the samples -- weight-gradient products)
 * MFMA: v_mfma_f32_16x16x32_bf16; operand lane maps (cdna guide section 3):
 *   A[row = l&15][k = 8(l>>4)+j], B[k = 8(l>>4)+j][col = l&15],
 *   D[row = 4(l>>4)+r][col = l&15].
 */
#ifndef HPNN_MFMA_COMMON_H
#define HPNN_MFMA_COMMON_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hpnn {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

/* 8 unsigned bytes (pixels 0..255) -> the same 8 integers in BF16, exactly: v_cvt_f32_ubyteN
 * gives the integer as f32, whose low 16 bits are zero (at most 8 significant bits), so
 * v_perm_b32 packs the high halves of two of them into a bf16x2 -- 1.5 VALU per pixel.
 * A pixel scale (e.g. 1/255) is applied to the FP32 MFMA accumulator instead. */
__device__ __forceinline__ unsigned int pk_hi16(float lo, float hi) {
    return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}
__device__ __forceinline__ bf16x8 u8x8_int_bf16(unsigned int a, unsigned int b) {
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    u32x4 r;
    r[0] = pk_hi16((float)((a >> 0) & 0xffu), (float)((a >> 8) & 0xffu));
    r[1] = pk_hi16((float)((a >> 16) & 0xffu), (float)((a >> 24) & 0xffu));
    r[2] = pk_hi16((float)((b >> 0) & 0xffu), (float)((b >> 8) & 0xffu));
    r[3] = pk_hi16((float)((b >> 16) & 0xffu), (float)((b >> 24) & 0xffu));
    return __builtin_bit_cast(bf16x8, r);
}

/* f(x) = 2/(1+e^-x) - 1 with the hardware exp / reciprocal (bf16 outputs) */
__device__ __forceinline__ float bipolar(float x) { return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-x)) - 1.0f; }
__device__ __forceinline__ float dbipolar(float y) { return -0.5f * (y * y - 1.0f); }

__device__ __forceinline__ f32x4 mfma(const bf16x8 &a, const bf16x8 &b, const f32x4 &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

/* byte offset of element (r, col) in a T32 image with R rows */
__device__ __forceinline__ int t32_g(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
/* PAD: bytes between consecutive 32-column sub-tiles beyond R * 64 (a padded image lets
 * 16 lanes writing one row across 4 sub-tiles hit 4 different bank groups) */
template <int R, int PAD = 0>
__device__ __forceinline__ int t32(int r, int col) {
    const int sub = col >> 5, c = col & 31;
    return sub * (R * 64 + PAD) + r * 64 + ((((c >> 3) ^ t32_g(r)) & 3) << 4) + (c & 7) * 2;
}

/* row-read fragment: 8 consecutive columns [col0 + 8(l>>4), +8) of row r0 + (l&15) */
template <int R>
__device__ __forceinline__ bf16x8 frag_row(const char *img, int r0, int col0, int lane) {
    return *(const bf16x8 *)(img + t32<R>(r0 + (lane & 15), col0 + 8 * (lane >> 4)));
}

/* transposed fragment: column c0 + (l&15), rows kbase + 8(l>>4) + 0..7 */
template <int R, int PAD = 0>
__device__ __forceinline__ bf16x8 frag_tr(const char *img, int kbase, int c0, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int row = kbase + 8 * g + q;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(img + t32<R, PAD>(row, c0 + 4 * p)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(img + t32<R, PAD>(row + 4, c0 + 4 * p)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}

/* One LDS-DMA instruction (global_load_lds_dwordx4): lane i copies 16 bytes from
 * gsrc (per lane) to LDS byte lds_dst + 16 i (lds_dst wave-uniform, via M0).
 * Emitted as inline asm on purpose: the compiler's waitcnt pass treats every pending
 * builtin LDS-DMA as a possible alias of any later ds_read and inserts a full
 * s_waitcnt vmcnt(0) before it, which drains the prefetch ring.  The kernels count
 * these loads themselves (wait_vm<N>, barriers); to the compiler they are unknown
 * VMEM ops, which only makes its own vmcnt waits stricter (never unsafe). */
__device__ __forceinline__ void glds16(const void *gsrc, char *lds_dst) {
    const unsigned int m0 =
        __builtin_amdgcn_readfirstlane((unsigned int)(uintptr_t)(__attribute__((address_space(3))) char *)lds_dst);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(m0)
                 : "memory", "m0");
}

/* wave-uniform copy of a 64-bit value (readfirstlane returns int: widen through
 * unsigned int, or a low half with bit 31 set sign-extends into the high half) */
__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long v) {
    const unsigned int lo = (unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)v);
    const unsigned int hi = (unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)(v >> 32));
    return ((unsigned long long)hi << 32) | (unsigned long long)lo;
}

/* Same with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset
 * (global_load_lds_dwordx4 voff, s[base]): one VGPR of addressing per lane instead of
 * two, and the base is not replicated per lane. */
__device__ __forceinline__ void glds16_sv(const void *gbase, unsigned int voff, char *lds_dst) {
    const unsigned int m0 =
        __builtin_amdgcn_readfirstlane((unsigned int)(uintptr_t)(__attribute__((address_space(3))) char *)lds_dst);
    const unsigned long long b = (unsigned long long)(uintptr_t)gbase;
    const unsigned long long bs = uniform_u64(b);
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(bs), "s"(m0)
                 : "memory", "m0");
}
__device__ __forceinline__ void glds4_sv(const void *gbase, unsigned int voff, char *lds_dst) {
    const unsigned int m0 =
        __builtin_amdgcn_readfirstlane((unsigned int)(uintptr_t)(__attribute__((address_space(3))) char *)lds_dst);
    const unsigned long long b = (unsigned long long)(uintptr_t)gbase;
    const unsigned long long bs = uniform_u64(b);
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(bs), "s"(m0)
                 : "memory", "m0");
}

/* 4-byte variant (global_load_lds_dword): lane i -> LDS byte lds_dst + 4 i */
__device__ __forceinline__ void glds4(const void *gsrc, char *lds_dst) {
    const unsigned int m0 =
        __builtin_amdgcn_readfirstlane((unsigned int)(uintptr_t)(__attribute__((address_space(3))) char *)lds_dst);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(gsrc), "s"(m0)
                 : "memory", "m0");
}

/* LDS-DMA: one 1 KiB piece = 16 rows x 32 cols of sub-tile `sub` of a T32 image with
 * R rows, from a row-major global matrix (ld_bytes per row); lane i fills bytes
 * [16i, 16i+16) of the piece, fetching the logical columns the half-swap puts there */
template <int R>
__device__ __forceinline__ void glds_t32_piece(const char *gbase, size_t ld_bytes, char *img, int piece, int lane) {
    constexpr int PPS = R / 16;
    const int sub = piece / PPS, rp = (piece % PPS) * 16;
    const int r = rp + (lane >> 2), cp = lane & 3;
    const int col = sub * 32 + ((cp ^ t32_g(r)) & 3) * 8;
    const char *src = gbase + (size_t)r * ld_bytes + (size_t)col * 2;
    glds16(src, img + sub * (R * 64) + rp * 64);
}

/* X image: K/64 sub-tiles of [R][64] bf16 (128-byte rows, 16-byte chunk c of row r at
 * c ^ ((r >> 1) & 7): conflict-free ds_read_b128 row reads, bank-simulated) and, when
 * K % 64 == 32, one T32 tail sub-tile.  128-byte rows let every LDS-DMA piece fetch
 * 8 rows x 128 B (whole cache lines) instead of 16 rows x 64 B. */
__device__ __forceinline__ int w128_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int R, int S64>
__device__ __forceinline__ void glds_x_piece(const char *g, size_t ld, char *img, int p, int lane) {
    constexpr int PF = R / 8; /* pieces per full sub-tile */
    if (p < S64 * PF) {
        const int sub = p / PF, rp = (p % PF) * 8;
        const int r = rp + (lane >> 3), lc = (lane & 7) ^ ((r >> 1) & 7);
        const char *src = g + (size_t)r * ld + (size_t)(sub * 64 + lc * 8) * 2;
        glds16(src, img + sub * (R * 128) + rp * 128);
    } else {
        glds_t32_piece<R>(g + (size_t)S64 * 128, ld, img + S64 * (R * 128), p - S64 * PF, lane);
    }
}

/* glds_x_piece with a uniform base (SGPRs) and 32-bit lane offsets (ld_bytes * R < 4 GiB) */
template <int R, int S64>
__device__ __forceinline__ void glds_x_piece_sv(const char *g, unsigned int ld, char *img, int p, int lane) {
    constexpr int PF = R / 8;
    if (p < S64 * PF) {
        const int sub = p / PF, rp = (p % PF) * 8;
        const int r = rp + (lane >> 3), lc = (lane & 7) ^ ((r >> 1) & 7);
        glds16_sv(g, (unsigned int)r * ld + (unsigned int)(sub * 64 + lc * 8) * 2u, img + sub * (R * 128) + rp * 128);
    } else {
        constexpr int PPS = R / 16;
        const int pt = p - S64 * PF;
        const int rp = pt * 16; /* one 32-col tail sub-tile: PPS pieces of 16 rows */
        const int r = rp + (lane >> 2), cp = lane & 3;
        const int col = S64 * 64 + ((cp ^ t32_g(r)) & 3) * 8;
        (void)PPS;
        glds16_sv(g, (unsigned int)r * ld + (unsigned int)col * 2u, img + S64 * (R * 128) + rp * 64);
    }
}

template <int R, int S64>
__device__ __forceinline__ bf16x8 x_frag(const char *img, int r0, int ks, int lane) {
    if (ks < 2 * S64) {
        const int r = r0 + (lane & 15), c = (ks & 1) * 4 + (lane >> 4);
        return *(const bf16x8 *)(img + (ks >> 1) * (R * 128) + w128_off(r, c));
    }
    return frag_row<R>(img + S64 * (R * 128), r0, 0, lane);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

/* workgroup barrier that orders LDS traffic but does NOT wait for outstanding
 * vector-memory ops (an in-flight LDS-DMA prefetch survives it; __syncthreads()
 * would emit vmcnt(0) and drain it) */
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

/* value of lane l ^ 16 / l ^ 32: gfx950 v_permlane16_swap / v_permlane32_swap (VALU, no
 * LDS crossbar round trip like the ds_bpermute __shfl_xor compiles to).  With both
 * operands = v, permlane16_swap yields {row-pair even value, odd value} in every lane
 * (rows of 16 lanes), permlane32_swap {lower-half value, upper-half value}. */
__device__ __forceinline__ float shfl_xor16(float v, int lane) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(((lane >> 4) & 1) ? r[0] : r[1]);
}
__device__ __forceinline__ float shfl_xor32(float v, int lane) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float((lane >> 5) ? r[0] : r[1]);
}
__device__ __forceinline__ int shfl_xor16(int v, int lane) {
    return __float_as_int(shfl_xor16(__int_as_float(v), lane));
}
__device__ __forceinline__ int shfl_xor32(int v, int lane) {
    return __float_as_int(shfl_xor32(__int_as_float(v), lane));
}
/* reductions over the 4 rows of 16 lanes (lane>>4): every lane gets the result */
__device__ __forceinline__ float rows_sum(float v) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float rows_max(float v) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return rows_sum(v);
}

typedef __attribute__((address_space(1))) unsigned int gu32;
/* 16-byte write-through store / L1-bypassing load (global_*_dwordx4 ... sc1); the loads
 * are issued in a batch and drained by the caller's s_waitcnt vmcnt(0) */
/* The s_nop: a VALU write of a >8-byte store's data VGPRs right behind the store corrupts the
 * stored bytes (a CDNA VMEM store-data hazard).  The compiler's hazard recognizer pads its own
 * stores, not this one, and it does reuse the data registers at once (seen: the next
 * instruction rewrote v[2:3] of a global_store_dwordx4 v[..], v[2:5]: the first 8 bytes of
 * some lanes' float4 were lost); two wait states inside the asm cover it. */
__device__ __forceinline__ void st_sc1(void *p, const f32x4 &v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ f32x4 ld_sc1(const void *p) {
    f32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}
/* 8 such loads AND their drain in ONE asm block.  With separate asm statements (loads, then
 * "s_waitcnt vmcnt(0)") the compiler may read a destination register -- a select, a copy,
 * an add -- between them, i.e. while the load is still in flight, and get stale data: the
 * outputs of this block only exist once the wait has retired them. */
#define HPNN_LDX8(BITS)                                                                                         \
    asm volatile("global_load_dwordx4 %0, %8, off " BITS "\n\t"                                                   \
                 "global_load_dwordx4 %1, %9, off " BITS "\n\t"                                                   \
                 "global_load_dwordx4 %2, %10, off " BITS "\n\t"                                                  \
                 "global_load_dwordx4 %3, %11, off " BITS "\n\t"                                                  \
                 "global_load_dwordx4 %4, %12, off " BITS "\n\t"                                                  \
                 "global_load_dwordx4 %5, %13, off " BITS "\n\t"                                                  \
                 "global_load_dwordx4 %6, %14, off " BITS "\n\t"                                                  \
                 "global_load_dwordx4 %7, %15, off " BITS "\n\t"                                                  \
                 "s_waitcnt vmcnt(0)"                                                                            \
                 : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),      \
                   "=&v"(v[7])                                                                                   \
                 : "v"(p0), "v"(p1), "v"(p2), "v"(p3), "v"(p4), "v"(p5), "v"(p6), "v"(p7)                       \
                 : "memory")
template <bool SYS = false>
__device__ __forceinline__ void ld_sc1_x8(f32x4 (&v)[8], const float *p0, const float *p1, const float *p2,
                                          const float *p3, const float *p4, const float *p5, const float *p6,
                                          const float *p7) {
    if constexpr (SYS) HPNN_LDX8("sc0 sc1");
    else HPNN_LDX8("sc1");
}
#undef HPNN_LDX8
/* 16 L1-bypassing (sc1) loads and their drain in one asm block (see ld_sc1_x8) */
__device__ __forceinline__ void ld_sc1_x16(f32x4 (&v)[16], const float *const (&p)[16]) {
    asm volatile("global_load_dwordx4 %0, %16, off sc1\n\t"
                 "global_load_dwordx4 %1, %17, off sc1\n\t"
                 "global_load_dwordx4 %2, %18, off sc1\n\t"
                 "global_load_dwordx4 %3, %19, off sc1\n\t"
                 "global_load_dwordx4 %4, %20, off sc1\n\t"
                 "global_load_dwordx4 %5, %21, off sc1\n\t"
                 "global_load_dwordx4 %6, %22, off sc1\n\t"
                 "global_load_dwordx4 %7, %23, off sc1\n\t"
                 "global_load_dwordx4 %8, %24, off sc1\n\t"
                 "global_load_dwordx4 %9, %25, off sc1\n\t"
                 "global_load_dwordx4 %10, %26, off sc1\n\t"
                 "global_load_dwordx4 %11, %27, off sc1\n\t"
                 "global_load_dwordx4 %12, %28, off sc1\n\t"
                 "global_load_dwordx4 %13, %29, off sc1\n\t"
                 "global_load_dwordx4 %14, %30, off sc1\n\t"
                 "global_load_dwordx4 %15, %31, off sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                   "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12]), "=&v"(v[13]),
                   "=&v"(v[14]), "=&v"(v[15])
                 : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7]), "v"(p[8]),
                   "v"(p[9]), "v"(p[10]), "v"(p[11]), "v"(p[12]), "v"(p[13]), "v"(p[14]), "v"(p[15])
                 : "memory");
}
/* sum over n <= 8 consecutive slabs (stride ss floats) of the float4 at p, via ld_sc1_x8:
 * the slots past n load slab 0 again and are dropped after the wait */
template <bool SYS = false>
__device__ __forceinline__ f32x4 sum_sc1_x8(const float *p, size_t ss, int n) {
    f32x4 v[8];
    const float *q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = p + (size_t)(j < n ? j : 0) * ss;
    ld_sc1_x8<SYS>(v, q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]);
    f32x4 g = v[0];
#pragma unroll
    for (int j = 1; j < 8; j++)
        if (j < n) g += v[j];
    return g;
}

/* Split-K arrival tickets: one monotonic 64-bit counter per output tile; every launch adds
 * `splits` tickets to it (one per workgroup of the tile), and a workgroup waits until the last
 * ticket of its own launch has arrived: want = old - old % splits + splits.  The counter is
 * 64-bit because that target is only right while the counter has not wrapped: a 32-bit
 * counter wraps after 2^32 / splits launches (89M at 48 splits, ~1.5 h of MNIST steps), and
 * since 2^32 is not a multiple of 48 every launch after the wrap would compute a wrong target
 * (reducing partial sums, or stalling to the timeout).  At 64 bits the wrap is ~10^10 years of
 * steps away.  Protocol (gfx950 guide, hand-off table row 1): the workgroup's partials are
 * stored sc1 and drained (vmcnt(0) in every storing wave, then the workgroup barrier) before
 * ONE lane takes the ticket (agent-scope atomic add); the waiter polls with relaxed
 * agent-scope (sc1) loads and its workgroup reads the partials with sc1 loads after a
 * barrier.  The wait is bounded: on timeout it sets *err (read back by BPlan::health) and
 * returns false. */
__device__ __forceinline__ unsigned long long ticket_arrive(unsigned int *cnt32, unsigned int splits) {
    unsigned long long *cnt = (unsigned long long *)cnt32;
    const unsigned long long old = atomicAdd(cnt, 1ull);
    return old - old % splits + splits;
}
__device__ __forceinline__ bool ticket_wait(unsigned int *cnt32, unsigned long long want, unsigned int *err,
                                            unsigned long long timeout) {
    typedef __attribute__((address_space(1))) unsigned long long gu64;
    gu64 *cnt = (gu64 *)cnt32;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > timeout) {
            __hip_atomic_store((gu32 *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
    return true;
}

/* Optional tail work of a TN launch: a grouped slab reduction (reduce_groups_kernel of
 * kernels_mlp3.hip: out[g*ostride + i] = sum of slabs [g*SG, min(S, (g+1)*SG)), float4 i)
 * run by extra workgroups appended to the GEMM grid.  The fused MNIST step reduces its
 * [G1 | G2] block slabs this way: the workgroups fill the CUs the 240-tile GEMM leaves
 * idle, and a launch (plus its serialized ~5 us) disappears from the step. */
struct TnTail {
    const float *slab;
    float *out;
    long stride, n4, ostride;
    int S, SG, bx, blocks;
};

__device__ __forceinline__ void tn_tail_reduce(const TnTail &t, int v) {
    const long e = (long)(v % t.bx) * 256 + threadIdx.x;
    const int g = v / t.bx;
    if (e >= t.n4) return;
    const int s_end = min(t.S, (g + 1) * t.SG);
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    int s = g * t.SG;
    for (; s + 3 < s_end; s += 4) {
        a0 += ((const f32x4 *)(t.slab + (long)s * t.stride))[e];
        a1 += ((const f32x4 *)(t.slab + (long)(s + 1) * t.stride))[e];
        a2 += ((const f32x4 *)(t.slab + (long)(s + 2) * t.stride))[e];
        a3 += ((const f32x4 *)(t.slab + (long)(s + 3) * t.stride))[e];
    }
    for (; s < s_end; s++) a0 += ((const f32x4 *)(t.slab + (long)s * t.stride))[e];
    ((f32x4 *)(t.out + (long)g * t.ostride))[e] = (a0 + a1) + (a2 + a3);
}

}  // namespace hpnn
#endif
