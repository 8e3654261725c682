/*
 * Weight-stationary NT GEMM for the wide-input first layer (gfx950).
 *
 *   C[M x N] = epi(X[M x K] . W[N x K]^T),  N <= 128, K <= 1024
 *
 * The reference computes layer 0 as one cublasDgemv per neuron slice per sample
 * (cuda_ann.cu:541-577).  Batched, this is the layer that streams the
 * input matrix (784 bf16 per MNIST sample); with a tiled GEMM every 128-sample
 * tile also re-stages all of W from L2 -- as many bytes as the X tile itself.
 * Here W is loaded ONCE per workgroup into VGPRs as MFMA A-operand fragments
 * (wave w owns neurons [w*N/4, (w+1)*N/4) for all K: N*K/128 registers per lane,
 * 200 for 128 x 800), and only X moves:
 *
 *   persistent grid (one 256-thread workgroup per CU, ~150 KiB LDS ring),
 *   X tiles of R=32 samples arrive by LDS-DMA (global_load_lds_dwordx4) into
 *   T32 images, STAGES-1 tiles in flight, counted vmcnt waits + raw s_barrier,
 *   every wave reads each X fragment (ds_read_b128, conflict-free T32 swizzle)
 *   and issues NT x 2 MFMAs per 32-wide k step.
 *
 * Lane map of the output (A = W rows, B = X rows): D[row = neuron][col = sample],
 * so a lane holds 4 consecutive neurons of one sample -> one 8-byte store.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.h"

HPNN_CO_PROBE(ws)
#include "mfma_common.h"

namespace {

using namespace hpnn;

template <int LPS, int STAGES>
__device__ __forceinline__ void ws_wait(int rem) {
    static_assert(LPS * (STAGES - 1) < 64, "vmcnt budget");
    if constexpr (STAGES >= 4) { if (rem >= 3) { wait_vm<LPS * 3>(); return; } }
    if constexpr (STAGES >= 3) { if (rem >= 2) { wait_vm<LPS * 2>(); return; } }
    if (rem >= 1) { wait_vm<LPS>(); return; }
    wait_vm<0>();
}

/* MODE (profiling experiments only): 0 normal, 1 no MFMA work, 2 no X traffic */
template <int NT, int KS, int STAGES, int EPI, bool CF32, int MODE = 0>
__global__ __launch_bounds__(256, 1) void gemm_nt_ws_kernel(const __bf16 *__restrict__ X, int ldx,
                                                            const __bf16 *__restrict__ W, int ldw,
                                                            void *__restrict__ C, int ldc, int tiles) {
    constexpr int R = 32, SG = R / 16;
    constexpr int K = KS * 32;
    constexpr int S64 = KS / 2, TAIL = KS & 1;
    constexpr int PIECES = S64 * (R / 8) + TAIL * (R / 16);
    constexpr int LPS = (PIECES + 3) / 4;
    constexpr int STAGE = R * K * 2;
    __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int n0 = wave * NT * 16;
    const int nloc = (tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const size_t ldx_b = (size_t)ldx * 2;

    /* W rows of this wave -> registers (A operand: row l&15, k 8(l>>4)..+8) */
    bf16x8 w[NT][KS];
#pragma unroll
    for (int nt = 0; nt < NT; nt++)
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
            w[nt][ks] = *(const bf16x8 *)(W + (size_t)(n0 + nt * 16 + r16) * ldw + ks * 32 + 8 * q);

    auto issue = [&](int slot, int i) {
        const int t = blockIdx.x + i * gridDim.x;
        const char *g = (const char *)(X + (size_t)t * R * ldx);
        char *img = lds + slot * STAGE;
#pragma unroll
        for (int p = 0; p < LPS; p++) {
            int c = wave + 4 * p;
            c = c < PIECES ? c : PIECES - 1;
            glds_x_piece<R, S64>(g, ldx_b, img, c, lane);
        }
    };
#pragma unroll
    for (int st = 0; st < STAGES - 1; st++)
        if (MODE != 2 && st < nloc) issue(st, st);

    for (int i = 0; i < nloc; i++) {
        const int nxt = i + STAGES - 1;
        if (MODE != 2 && nxt < nloc) issue(nxt % STAGES, nxt);
        if (MODE != 2) ws_wait<LPS, STAGES>((nxt < nloc ? nxt : nloc - 1) - i);
        __builtin_amdgcn_s_barrier();
        const char *img = lds + (i % STAGES) * STAGE;
        f32x4 acc[NT][SG];
#pragma unroll
        for (int nt = 0; nt < NT; nt++)
#pragma unroll
            for (int sg = 0; sg < SG; sg++) acc[nt][sg] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE != 1) {
            /* software-pipelined: fragments of step ks+1 are in flight during step ks's MFMAs
             * (one wave per SIMD: nothing else would hide the LDS latency) */
            bf16x8 xc[SG], xn[SG];
#pragma unroll
            for (int sg = 0; sg < SG; sg++) xc[sg] = x_frag<R, S64>(img, sg * 16, 0, lane);
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                if (ks + 1 < KS) {
#pragma unroll
                    for (int sg = 0; sg < SG; sg++) xn[sg] = x_frag<R, S64>(img, sg * 16, ks + 1, lane);
                }
#pragma unroll
                for (int sg = 0; sg < SG; sg++)
#pragma unroll
                    for (int nt = 0; nt < NT; nt++) acc[nt][sg] = mfma(w[nt][ks], xc[sg], acc[nt][sg]);
#pragma unroll
                for (int sg = 0; sg < SG; sg++) xc[sg] = xn[sg];
            }
        }
        /* all LDS reads of this slot retire before any wave refills it */
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const int t = blockIdx.x + i * gridDim.x;
#pragma unroll
        for (int nt = 0; nt < NT; nt++)
#pragma unroll
            for (int sg = 0; sg < SG; sg++) {
                const size_t b = (size_t)t * R + sg * 16 + r16;
                const int f = n0 + nt * 16 + 4 * q;
                f32x4 v = acc[nt][sg];
                if constexpr (EPI == HPNN_EPI_ACT) {
#pragma unroll
                    for (int r = 0; r < 4; r++) v[r] = bipolar(v[r]);
                }
                if constexpr (CF32) {
                    *(f32x4 *)((float *)C + b * ldc + f) = v;
                } else {
                    bf16x4 o;
#pragma unroll
                    for (int r = 0; r < 4; r++) o[r] = (__bf16)v[r];
                    *(bf16x4 *)((__bf16 *)C + b * ldc + f) = o;
                }
            }
    }
}

int g_num_cus = 0;

template <int NT, int KS, int EPI, bool CF32>
int launch_ws(const void *X, int ldx, const void *W, int ldw, void *C, int ldc, int M, hipStream_t s) {
    constexpr int STAGE = 32 * KS * 32 * 2;
    constexpr int ST = (155648 / STAGE) > 4 ? 4 : (155648 / STAGE);
    static_assert(ST >= 2, "ring");
    if (g_num_cus <= 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            g_num_cus = 256;
    }
    const int tiles = M / 32;
    const int grid = tiles < g_num_cus ? tiles : g_num_cus;
    static const int mode = [] { const char *e = getenv("HPNN_WS_MODE"); return e ? atoi(e) : 0; }();
    if (mode == 1)
        hipLaunchKernelGGL((gemm_nt_ws_kernel<NT, KS, ST, EPI, CF32, 1>), dim3(grid), dim3(256), 0, s,
                           (const __bf16 *)X, ldx, (const __bf16 *)W, ldw, C, ldc, tiles);
    else if (mode == 2)
        hipLaunchKernelGGL((gemm_nt_ws_kernel<NT, KS, ST, EPI, CF32, 2>), dim3(grid), dim3(256), 0, s,
                           (const __bf16 *)X, ldx, (const __bf16 *)W, ldw, C, ldc, tiles);
    else
        hipLaunchKernelGGL((gemm_nt_ws_kernel<NT, KS, ST, EPI, CF32>), dim3(grid), dim3(256), 0, s,
                           (const __bf16 *)X, ldx, (const __bf16 *)W, ldw, C, ldc, tiles);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

template <int EPI, bool CF32>
int dispatch_ws(const void *X, int ldx, const void *W, int ldw, void *C, int ldc, int M, int N, int K, hipStream_t s) {
#define HPNN_WS(N_, K_)                                                                     \
    if (N == N_ && K == K_) return launch_ws<N_ / 64, K_ / 32, EPI, CF32>(X, ldx, W, ldw, C, ldc, M, s)
    HPNN_WS(128, 800);
    HPNN_WS(64, 800);
    HPNN_WS(128, 512);
    HPNN_WS(128, 1024);
#undef HPNN_WS
    return 1; /* shape not instantiated */
}

}  // namespace

/* returns 0 when launched, 1 when the shape has no weight-stationary instance */
extern "C" int hpnn_gemm_nt_ws_bf16(const void *X, int ldx, const void *W, int ldw, void *C, int ldc, int M, int N,
                                    int K, int epi, int c_f32, hipStream_t stream) {
    if (M % 32 || ldx % 8 || ldw % 8 || ldc % 8) return 1;
    if (epi == HPNN_EPI_DACT) return 1;
    if (c_f32) {
        if (epi == HPNN_EPI_ACT) return dispatch_ws<HPNN_EPI_ACT, true>(X, ldx, W, ldw, C, ldc, M, N, K, stream);
        return dispatch_ws<HPNN_EPI_NONE, true>(X, ldx, W, ldw, C, ldc, M, N, K, stream);
    }
    if (epi == HPNN_EPI_ACT) return dispatch_ws<HPNN_EPI_ACT, false>(X, ldx, W, ldw, C, ldc, M, N, K, stream);
    return dispatch_ws<HPNN_EPI_NONE, false>(X, ldx, W, ldw, C, ldc, M, N, K, stream);
}
