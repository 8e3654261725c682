/*
 * libhpnn HIP kernel launchers (gfx950).  Plain C ABI: device pointers +
 * hipStream_t, so the native engines and the Python binding share them.
 *
 * Layout conventions (see docs/DESIGN.md):
 *   activations  [rows = samples][cols = features], row-major, BF16
 *   weights      W [N][K] row-major (one row per neuron, as the reference),
 *                plus a transposed BF16 copy Wt [K][N] for the dX GEMM
 *   every feature dimension is padded to a multiple of 32 and every batch
 *   dimension to a multiple of 128 on the device; padded weights/inputs are
 *   zero so they never contribute.
 * Return value of every launcher: 0 = launched, <0 = shape not supported
 * (caller bug: the kernels never guess).
 */
#ifndef HPNN_GPU_KERNELS_H
#define HPNN_GPU_KERNELS_H
#include <hip/hip_runtime_api.h>
#include <libhpnn/xar.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Loss / accuracy statistics are accumulated into HPNN_STAT_SLOTS slots spaced
 * HPNN_STAT_STRIDE floats apart (one 64-byte line each) -- block b adds into slot
 * b % HPNN_STAT_SLOTS -- so thousands of workgroups never serialise on a single
 * atomic address.  `loss_acc` / `correct` arguments point at slot 0; readers sum
 * the slots. */
#define HPNN_STAT_SLOTS 64
#define HPNN_STAT_STRIDE 16
#define HPNN_STAT_SLOT(b) ((size_t)((b) % HPNN_STAT_SLOTS) * HPNN_STAT_STRIDE)

enum {
    HPNN_EPI_NONE = 0,   /* C = acc                                   */
    HPNN_EPI_ACT = 1,    /* C = 2/(1+e^-acc) - 1                      */
    HPNN_EPI_DACT = 2,   /* C = acc * (-0.5)(aux^2 - 1)  (f'(h))      */
};

/* C[M x N] = epi(A[M x K] . B[N x K]^T), A/B BF16, C BF16 (c_f32=0) or
 * FP32 (c_f32=1).  M % 128 == 0, N % 32 == 0, K % 32 == 0. */
int hpnn_gemm_nt_bf16(const void *A, int lda, const void *B, int ldb, void *C, int ldc,
                      const void *aux, int ldaux, int M, int N, int K, int epi, int c_f32,
                      hipStream_t stream);

/* weight-stationary variant for N <= 128, K in {512, 800, 1024}: returns 1 if no instance */
/* the same product on the 8-phase 256x256-tile kernel (kernels_8ph.hip): M % 256 == 0,
 * N % 256 == 0, K % 128 == 0, else -1.  hpnn_gemm_nt_bf16 routes large GEMMs here when
 * HPNN_NT_8PH is not 0. */
/* split-K form of the same (S FP32 slabs in a library workspace, then one epilogue pass):
 * M % 256 == 0, N % 256 == 0, K % (128 S) == 0; -1 when it does not apply */
int hpnn_gemm_nt8_splitk_bf16(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux,
                              int ldaux, int M, int N, int K, int epi, int c_f32, int splits, hipStream_t stream);
/* weight gradient of one layer over the whole batch with the optimizer step fused into the
 * 8-phase TN kernel's epilogue (no gradient in memory): the step of hpnn_sgd_update with one
 * slab.  N % 256 == 0, M % 256 == 0, Bt % 128 == 0, else -1. */
/* G = D^T H (one split) rounded to BF16 into G16 [N][ldg] (8-phase kernel); -1: shape not covered */
int hpnn_gemm_tn8_bf16out_ok(int N, int M, int Bt, int ldd, int ldh);
int hpnn_gemm_tn8_bf16out(const void *D, int ldd, const void *H, int ldh, void *G16, int ldg, int N, int M, int Bt,
                          hipStream_t stream);
int hpnn_gemm_tn8_update(const void *D, int ldd, const void *H, int ldh, int N, int M, int Bt, float *W32, float *V32,
                         void *Wbf, void *Wt, float lr, float alpha, float scale, int momentum, hipStream_t stream);
/* the same with the gradient over `splits` (>= 2) split-K slabs reduced inside the launch (each
 * split publishes its partial write-through; the splits of a tile meet through tickets in
 * cnt, 1024 words zeroed once; err set on a timeout): -1 when not covered */
int hpnn_gemm_tn8_fused_update(const void *D, int ldd, const void *H, int ldh, int N, int M, int Bt, int splits,
                               float *slab, float *W32, float *V32, void *Wbf, void *Wt, float lr, float alpha,
                               float scale, int momentum, unsigned int *cnt, unsigned int *err, hipStream_t stream);
/* the next layer's weight gradient D^T H (N x M over the same Bt rows, S splits of 64 x 64
 * pieces into slab [S][N][M], the pieces of gemm_tn_pipe at 64 x 64) and its step (same lr /
 * alpha / scale / momentum), carried by the fused launch above (kernels_8ph.hip): bitwise the
 * result of hpnn_gemm_tn_bf16 + hpnn_sgd_update.  cnt: a 64-bit counter zeroed once, used by
 * this launch shape only. */
typedef struct {
    const void *D, *H;
    int ldd, ldh;
    float *slab;
    int N, M, S;
    float *W32, *V32;
    void *Wb, *Wt;
    unsigned int *cnt;
} hpnn_tn8_side;
/* hpnn_gemm_tn8_fused_update plus that side job: -1 as above, -2 when the side job does not
 * fit this grid (its pieces must split evenly over the half-workgroups) */
int hpnn_gemm_tn8_fused_update_side(const void *D, int ldd, const void *H, int ldh, int N, int M, int Bt, int splits,
                                    float *slab, float *W32, float *V32, void *Wbf, void *Wt, float lr, float alpha,
                                    float scale, int momentum, unsigned int *cnt, unsigned int *err,
                                    const hpnn_tn8_side *side, hipStream_t stream);
void hpnn_gemm_nt_set_8ph(int on);
void hpnn_gemm_tn_set_8ph(int on); /* same switch for the large weight-gradient GEMMs */
void hpnn_gemm_nt_set_pp(int on);  /* the pipelined 128 x 128 NT kernel for under-filled grids */
/* C[M x N] = epi(A[M x K] . W[K x N]), W row-major [K][N]: the NT product on W^T without the
 * transposed copy (same bits); M, N % 128, K % 64, else -1.  _ok: 1 when the shape fits */
int hpnn_gemm_nn_ok(int M, int N, int K, int lda, int ldw, int ldc);
int hpnn_gemm_nn_bf16(const void *A, int lda, const void *W, int ldw, void *C, int ldc, const void *aux, int ldaux,
                      int M, int N, int K, int epi, int c_f32, hipStream_t stream);
int hpnn_gemm_nt8_bf16(const void *A, int lda, const void *B, int ldb, void *C, int ldc, const void *aux, int ldaux,
                       int M, int N, int K, int epi, int c_f32, hipStream_t stream);
int hpnn_gemm_nt_ws_bf16(const void *X, int ldx, const void *W, int ldw, void *C, int ldc, int M, int N, int K,
                         int epi, int c_f32, hipStream_t stream);

/* slab[s][N x M] = sum_{b in slice s} D[b][n] H[b][m] (FP32 out).
 * D: [Bt x N] BF16, H: [Bt x M] BF16. Bt % 64 == 0, 1 <= splits <= Bt/64, N,M % 32 == 0.
 * Slice s = rows [64*floor(s*U/S), 64*floor((s+1)*U/S)), U = Bt/64 (uneven splits allowed).
 * ldg: row stride of a slab row (>= M); slab stride = N*ldg. */
int hpnn_gemm_tn_bf16(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N,
                      int M, int Bt, int splits, hipStream_t stream);
/* the same GEMM plus, in the same launch, hpnn_reduce_groups(rslab, rS, rstride, rn, rgroups,
 * rout) run by extra workgroups appended to the grid (they fill the CUs the GEMM tiles
 * leave idle; one launch less per fused training step) */
int hpnn_gemm_tn_bf16_reduce(const void *D, int ldd, const void *H, int ldh, float *slab, int ldg, int N, int M,
                             int Bt, int splits, const float *rslab, int rS, long rstride, long rn, int rgroups,
                             float *rout, hipStream_t stream);

/* weight gradient of hpnn_gemm_tn_bf16 over FRAGMENT-MAJOR operands (kernels_g0.hip):
 * Dg [Bt/32][N/16][64][8], Hg [Bt/32][M/16][64][8], lane l = 16 g + r of fragment (t, cb)
 * holding A[32 t + 8 g + j][16 cb + r] (j < 8); slab[s][n][m] as hpnn_gemm_tn_bf16.
 * Bt, M, N multiples of 32.  h_u8: Hg holds unsigned bytes in the same layout, used as
 * bf16(h * hscale) (pixel data).  _reduce: plus hpnn_reduce_groups on appended workgroups. */
int hpnn_gemm_fm_direct(const void *Dg, const void *Hg, int h_u8, float hscale, float *slab, int ldg, int N, int M,
                        int Bt, int splits, hipStream_t stream);
int hpnn_gemm_fm_direct_reduce(const void *Dg, const void *Hg, int h_u8, float hscale, float *slab, int ldg, int N,
                               int M, int Bt, int splits, const float *rslab, int rS, long rstride, long rn,
                               int rgroups, float *rout, hipStream_t stream);

/* the same GEMM with its split-K reduction and the optimizer step of layer 0 in the same
 * launch, plus the [G1 | G2] block-slab reduction and the steps of layers 1, 2 on tail
 * workgroups (the single-GPU fused MNIST step; kernels_g0.hip).  slab: scratch for the
 * published partials.  Returns -1 when the shape is not covered (caller: the 3-launch form),
 * HPNN_G0_FUSED=0 disables it. */
typedef struct {
    float *W32, *V32; /* layer 0 [N][M] FP32 master / momentum (V32 NULL for BP) */
    void *Wb, *Wt, *Wf; /* BF16 W [N][M], W^T [M][N], fragment-major copy (may be NULL) */
    unsigned int *cnt;  /* HPNN_G0CNT_WORDS words, zeroed once: 64-bit tile counters, 32 words apart (monotonic) */
    unsigned int *err;  /* set when a wait for the other splits timed out */
    float lr, alpha, scale;
    int momentum;
    const float *mslab; /* [G1 | G2] block slabs: mrows rows of n12 floats, mstride apart */
    int mrows;
    long mstride, n12;
    float *W32b[2], *V32b[2]; /* layers 1, 2 */
    void *Wbb[2], *Wtb[2];
    int Nb[2], Kb[2];
    /* non-NULL: no step -- the fully reduced gradients are stored instead, G0 [N][M] at gout,
     * [G1 | G2] right after it (the flat layout of the plan's gradient buffer; data parallel) */
    float *gout;
    /* non-NULL (with gout): gout + galt instead of gout when *gsel is even -- gout is then the
     * xGMI all-reduce's own data buffer and *gsel its epoch word, so the gradient lands in the
     * half the next call reads (hpnn_xar_local) and that call needs no copy-in */
    const unsigned int *gsel;
    long galt;
    /* xchg != 0: data parallel with the exchange in this launch -- each workgroup writes its
     * reduced G0 / [G1 | G2] elements into its half of xv's buffer, runs the one-shot flag
     * barrier of workgroup b with every peer (include/libhpnn/xar.h hpnn_xar_view), sums the
     * peers' copies in rank order and steps those elements (scale includes 1 / world) */
    int xchg; /* 1 one-shot, 2 two-shot (each rank reduces 1 / world of every slice, then gathers) */
    hpnn_xar_view xv;
    int proto; /* hand-off diagnostics (HPNN_G0_PROTO, make ABLATIONS=1 builds only): 1 producer agent
                * release, 2 consumer agent acquire, 4 system-scope (sc0 sc1) partial loads, 8 system
                * acquire after the exchange barrier, 16 no exchange barrier, 32 one exchange load
                * block per element (not one for both), 64 no W / V prefetch; timing ablations (wrong
                * results): 256 no partial publish, 512 no [G1 | G2] share, 1024 no split-sum loads */
    /* tests / diagnostics: perm > 0 runs the grid in another block -> role order (reversed,
     * rotated by perm: results must not change); xtest: self-test of the in-kernel exchange
     * (no GEMM: a known pattern is exchanged, the sums land in xres, [G0 | G1 | G2] flat);
     * xfault: corrupt one element of this rank's exchanged sum (HPNN_FAULT=xsum:n) */
    int perm, xtest, xfault;
    float *xres;
    long n12t; /* set by the launcher: [G1 | G2] floats summed by the tail workgroups */
    /* XCD-local first level of the split-K reduction (HPNN_G0_XCD=1): xw = HPNN_G0X_WORDS
     * protocol words (zeroed once), xslab = 8 partial G0 slabs (one per XCD group); NULL: off */
    unsigned int *xw;
    float *xslab;
    int fault; /* test hook (HPNN_FAULT=handoff:n): the split-K wait of that launch reports a
                * timeout (sets *err) as a real one would */
} hpnn_g0_update;
int hpnn_gemm_fm_direct_update(const void *Dg, const void *Hg, int h_u8, float hscale, float *slab, int ldg, int N,
                               int M, int Bt, int splits, const hpnn_g0_update *u, hipStream_t stream);
/* 1 when hpnn_gemm_fm_direct_update covers the shape (launch-free check), including the
 * residency its in-kernel hand-offs need: every workgroup of the grid co-resident */
int hpnn_gemm_fm_direct_update_ok(int ldg, int N, int M, int Bt, int splits);
/* output tiles of the fused G0 launch for these operands (h_u8: 8-bit H), 0 if not covered;
 * the launch's grid is tiles x splits */
int hpnn_g0_tiles(int h_u8, int N, int M);
/* feature columns of that launch's output tile (160, or 80 with HPNN_G0_TILE=80) */
int hpnn_g0_tile_cols(int M);
/* hpnn_g0_update.cnt: HPNN_G0CNT_WORDS words, 64-bit tile counters 32 words apart (tile < 
 * HPNN_G0_MAX_TILES), the error word at HPNN_G0_ERR_WORD */
#define HPNN_G0CNT_WORDS 1024
/* hpnn_g0_update.xw layout: per-role epochs, per-(tile, group) member slots, group and tile
 * counters (64-bit); see kernels_g0.hip */
#define HPNN_G0X_WORDS 4096
#define HPNN_G0_MAX_TILES 31
#define HPNN_G0_ERR_WORD 1000
/* workgroups of `kernel` (threads per workgroup, dynamic LDS bytes) the device can hold at once:
 * the occupancy API's blocks per CU x CUs (cached per kernel).  Kernels whose workgroups wait
 * for each other inside one launch (split-K tickets, tile-pair hand-offs, the in-kernel DP
 * exchange) refuse grids above it: the first wave of workgroups would spin on partners that
 * cannot be scheduled until the wait times out. */
int hpnn_resident_capacity(const void *kernel, int threads, size_t dyn_lds);
/* (Best effort: the count assumes the launch has the device to itself.  Kernels of another
 * stream or process on the same GPU -- a side-stream collective, ranks sharing one GPU in
 * tests / rehearsals -- can hold CUs meanwhile; a waiting grid then stretches until they
 * finish, and a wait that outlives its bound sets the error word read by BPlan::health.) */
/* *out += order-independent 64-bit digest of the nbytes / 4 words at p (word index offset by
 * base, so several buffers can be folded into one digest); *out must be initialised */
int hpnn_hash_words(const void *p, long nbytes, long base, unsigned long long *out, hipStream_t stream);
/* load every kernel translation unit's code object onto the current device now (HIP loads a
 * code object at its first launch): training loops call it before their clock starts, so a
 * first eager step does not pay for it.  Once per device; 0 on success. */
int hpnn_preload_code_objects(void);

/* output layer: logits Z [B x ldz] FP32 (n_out valid columns) ->
 *   delta  D [B x ldd] BF16  (zero in padded rows/cols)
 *   loss_acc[slot] += sum of per-sample loss over valid rows (slot array, above)
 *   correct[slot]  += argmax hits
 *   optional O [B x ldo] FP32 network output (NULL to skip)
 * targets: dense T [B x ldt] FP32 (labels == NULL) or int32 labels with
 * one-hot values (t_hi at the label, t_lo elsewhere).
 * type: 0 ANN, 1 LNN, 2 SNN (nn_type). */
int hpnn_output_delta(const float *Z, int ldz, const float *T, int ldt, const int *labels, float t_hi,
                      float t_lo, void *D, int ldd, float *O, int ldo, float *loss_acc,
                      unsigned int *correct, int B, int n_valid, int n_out, int type,
                      hipStream_t stream);

/* sum S slabs of n floats: out[i] = sum_s slab[s*stride + i] */
int hpnn_reduce_slabs(const float *slab, int S, long stride, long n, float *out, hipStream_t stream);

/* optimizer step for one layer, W32/V32 FP32 master [N x K]:
 *   g = scale * sum_s G[s*gstride + i]
 *   BP : w += lr g              (momentum == 0)
 *   BPM: v += lr g; w += v; v *= alpha
 * then writes BF16 W [N x K] and BF16 Wt [K x N] (ldwt = N). */
int hpnn_sgd_update(float *W32, float *V32, const float *G, int S, long gstride, void *Wbf, void *Wt,
                    int N, int K, float lr, float alpha, float scale, int momentum,
                    hipStream_t stream);

/* all layers' optimizer steps in ONE launch (same math as hpnn_sgd_update per layer).
 * Wf (optional, may be NULL): BF16 copy of W in MFMA-fragment-major order, the operand
 * layout of the register-resident first-layer weights (hpnn_mlp3_fused):
 *   element (n, k) at (((n/16)*(K/32) + k/32)*64 + n%16 + 16*((k/8)%4))*8 + k%8 */
#define HPNN_UPD_MAX 8
typedef struct {
    float *W32;
    float *V32;
    const float *G;
    long gstride;
    void *Wbf;
    void *Wt;
    void *Wf;
    int S, N, K;
} hpnn_upd_layer;
int hpnn_sgd_update_multi(const hpnn_upd_layer *layers, int n, float lr, float alpha, float scale, int momentum,
                          hipStream_t stream);

/* dense FP64/FP32 host-layout matrix -> padded BF16 device matrix:
 * dst[r][c] = src[r][c] for r<rows,c<cols, 0 in the padding.
 * src_f64 selects double vs float input. */
int hpnn_pack_bf16(const void *src, int src_f64, int rows, int cols, int lds, void *dst, int prow,
                   int pcol, int ldd, hipStream_t stream);

/* FP32 master <-> BF16 copies without an update (after load/broadcast) */
int hpnn_cast_weights(const float *W32, void *Wbf, void *Wt, int N, int K, hipStream_t stream);

/* BF16 reduce-scatter data parallelism (csrc/dist/dp_exchange.cpp): dst = bf16(src), n % 4 == 0;
 * the step of n consecutive master elements from a BF16 gradient sum (W32, V32, Wbf rows);
 * Wt [K][N] = Wbf^T */
int hpnn_cast_f32_bf16(const float *src, void *dst, long n, hipStream_t stream);
int hpnn_sgd_update_rows_bf16g(float *W32, float *V32, const void *G16, long n, float lr, float alpha, float scale,
                               int momentum, void *Wbf, hipStream_t stream);
int hpnn_transpose_bf16(const void *Wbf, void *Wt, int N, int K, hipStream_t stream);

/* BF16 row-sharded tensor parallelism (tp_engine.cpp): dst [rows][P n] <- src [P][rows][n]
 * (n % 8 == 0); out = bf16(in * f'(H)) elementwise (n % 4 == 0) */
int hpnn_block_permute_bf16(const void *src, void *dst, int P, long rows, int n, hipStream_t stream);
int hpnn_dact_f32_bf16(void *out, const float *in, const void *H, long n, hipStream_t stream);

/* zero-fill helper usable inside graphs */
int hpnn_fill_f32(float *p, long n, float v, hipStream_t stream);

/* fused middle of a 3-layer MLP (kernels_mlp3.hip): H1 [Bp x 128] -> delta1
 * [Bp x 128] + per-block [G1 (64 x 128) | G2 (32 x 64)] FP32 slabs (grid of them),
 * loss / accuracy.  Dims must be h1=128, h2=64, no=32 (padded), n_out <= 32,
 * Bp % 64 == 0.  W1t / W2t are unused (transposed LDS reads of W1 / W2). */
int hpnn_mlp3_mid(const void *H1g, const void *W1, const void *W1t, const void *W2, const void *W2t,
                  const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1, float *gslab,
                  float *loss_acc, unsigned int *correct, int Bp, int n_valid, int n_out, int type, int h1, int h2,
                  int no, int grid, hipStream_t stream);
/* the whole 3-layer step up to delta1 in one persistent kernel (kernels_mlp3.hip):
 *   X [Bp x K0] -> H1 = f(X W0^T) -> H2 -> output/loss -> delta3 -> delta2 -> delta1 (D1)
 * plus per-block [G1 | G2] slabs (grid of them, same layout as hpnn_mlp3_mid).  W0 is
 * read once per workgroup into registers from its fragment-major copy W0f (see
 * hpnn_sgd_update_multi); K0 in {256, 512, 800, 832, 896}, Bp % 32 == 0.  grid <= 0:
 * one workgroup per CU.  d1fm: delta1 written fragment-major ([Bp/32][8][64][8], the
 * operand layout of hpnn_gemm_fm_direct) instead of row-major [Bp x 128].  Returns the
 * grid used (> 0) or an error (< 0). */
int hpnn_mlp3_fused(const void *X, int ldx, int K0, const void *W0f, const void *W1, const void *W2,
                    const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1, float *gslab,
                    float *loss_acc, unsigned int *correct, int Bp, int n_valid, int n_out, int type, int grid,
                    int d1fm, hipStream_t stream);
/* grid hpnn_mlp3_fused will use for Bp samples (slab rows to allocate) */
int hpnn_mlp3_fused_grid(int Bp, int grid);
/* the same step up to delta1 with 256-sample tiles (kernels_mlp3t.hip): X given
 * FRAGMENT-MAJOR ([Bp/32][K0/16][64][8], ops.to_fragment_major), 8-bit (xu8: used as
 * bf16(byte * xscale)) or BF16; W0f fragment-major BF16 W0, W1 [64][128], W2 [32][64] and
 * W2t [64][32] BF16; delta1 written fragment-major ([Bp/32][8][64][8]); per-block
 * [G1 | G2] slabs as hpnn_mlp3_mid.  Bp % 256 == 0, K0 in {256, 800}.  grid <= 0: one
 * workgroup per CU (capped at Bp / 256).  Returns the grid used (> 0) or an error (< 0). */
int hpnn_mlp3_tile(const void *Xg, int xu8, float xscale, int K0, const void *W0f, const void *W1, const void *W2,
                   const void *W2t, const int *labels, const float *T, int ldt, float t_hi, float t_lo, void *D1,
                   float *gslab, float *loss_acc, unsigned int *correct, int Bp, int n_valid, int n_out, int type,
                   int grid, hipStream_t stream);
int hpnn_mlp3_tile_grid(int Bp, int grid);
/* profiling (HPNN_TILE_TRACE=1): per-workgroup s_memtime stamps [1024][12] */
int hpnn_mlp3_tile_trace(unsigned long long *out);
/* HPNN_G0_TRACE=1 phase stamps of the fused G0 launch: out[512][8] */
int hpnn_g0_trace(unsigned long long *out);
/* ---- wide-input one-hidden-layer front (kernels_wide.hip): K0 (4096) -> 256 -> 256 ----
 * X [Bp][ldx] bf16 row-major, W0 [256][K0], W1 / W1t [256][256] bf16; outputs H0, D2 (delta
 * of the output layer), D1 (delta of the hidden layer), all [Bp][256] bf16 row-major; labels
 * or T [Bp][ldt]; with 2 workgroups per 128-sample tile (hpnn_wide2_ksplit) pbuf
 * (hpnn_wide2_pbuf_bytes), cnt / flag (Bp / 128 words each, zero once, self-resetting) and
 * err (one word, set on a hand-over timeout) are required. */
typedef struct {
    const void *X, *W0, *W1, *W1t;
    int ldx, K0;
    const int *labels;
    const float *T;
    int ldt;
    float t_hi, t_lo;
    void *H0, *D2, *D1, *pbuf;
    unsigned int *cnt, *flag, *err;
    float *loss_acc;
    unsigned int *correct;
    int Bp, n_valid, n_out, type;
    int ksplit; /* workgroups per tile: 1, 2, or 0 = hpnn_wide2_ksplit */
} hpnn_wide2_args;
int hpnn_wide2_front(const hpnn_wide2_args *a, hipStream_t stream);
int hpnn_wide2_ksplit(int Bp, int K0);
long hpnn_wide2_pbuf_bytes(int Bp);
/* profiling (HPNN_WIDE_TRACE=1): per-workgroup s_memtime stamps [512][12] */
int hpnn_wide2_trace(unsigned long long *out);
int hpnn_tn8_trace(unsigned long long *out); /* HPNN_TN8_TRACE=1: [512][8] MODE-2 phase stamps */
/* ---- FP64 / FP32 batched engine (kernels_fp.hip): f64 selects double, else float ----
 * gemm_fp: C[M x N] (ldc) = sum_k A(m, k) B(n, k) with A(m, k) = A[m*lda + k] (ta = 0) or
 * A[k*lda + m] (ta = 1), B(n, k) = B[n*ldb + k] (tb = 0) or B[k*ldb + n] (tb = 1), on the FP64 /
 * FP32 MFMA; epi as hpnn_gemm_nt_bf16 (aux [M x N], ldaux); splits > 1: split-K into
 * hpnn_gemm_fp_splits(K, splits) slabs slab_stride elements apart.  Any sizes. */
int hpnn_gemm_fp(int f64, const void *A, int lda, int ta, const void *B, int ldb, int tb, void *C, int ldc,
                 const void *aux, int ldaux, int M, int N, int K, int epi, int splits, long slab_stride,
                 hipStream_t stream);
int hpnn_gemm_fp_splits(int K, int splits);
/* output layer in FP64 / FP32: O (optional) = output, D (optional) = delta, guess (optional)
 * = argmax per row (first maximum), loss / hits into the stat slots for rows < n_valid
 * (T required for D, loss, hits) */
int hpnn_output_fp(int f64, const void *Z, int ldz, const void *T, int ldt, void *D, int ldd, void *O, int ldo,
                   int *guess, float *loss_acc, unsigned int *correct, int B, int n_valid, int n_out, int type,
                   hipStream_t stream);
/* W += step(scale * sum_s G[s]) (BP / BPM), n elements */
int hpnn_update_fp(int f64, void *W, void *V, const void *G, int S, long gstride, long n, double lr, double alpha,
                   double scale, int momentum, hipStream_t stream);
/* out = sum_s G[s] */
int hpnn_reduce_fp(int f64, void *out, const void *G, int S, long gstride, long n, hipStream_t stream);
/* out[i] = in[i] * f'(aux[i]) (in place allowed): f' applied to reduced partial deltas */
int hpnn_dact_fp(int f64, void *out, const void *in, const void *aux, long n, hipStream_t stream);

/* floats per block slab written by hpnn_mlp3_mid */
int hpnn_mlp3_slab_floats(void);
/* deterministic 2-pass slab reduction: groups of slabs into tmp (>= 16*n floats,
 * NULL = single pass), then the groups into out */
int hpnn_reduce_slabs2(const float *slab, int S, long stride, long n, float *tmp, float *out,
                       hipStream_t stream);

/* first pass of hpnn_reduce_slabs2 only: out[g*n + i], g < groups (groups <= S) */
int hpnn_reduce_groups(const float *slab, int S, long stride, long n, int groups, float *out, hipStream_t stream);

/* online (batch-1) FP64 persistent engine, see online.hip */
typedef struct {
    int L;
    int n_in;
    int N[16];
    int M[16];
    double *W[16];
    double *dW[16];
    int type;     /* 0 ANN 1 LNN 2 SNN */
    int momentum;
    double lr;
    double alpha;
    double delta;
    int min_iter;
    int max_iter;
    const double *x;
    const double *t;
    double *out;       /* n_out, final network output */
    double *scratch;   /* vectors when they do not fit in LDS */
    double *result;    /* [0]=dEp [1]=init_err [2]=iter [3]=ok [4]=first_ok */
    int use_lds;
    int forward_only;
    /* multi-workgroup (cooperative) variant, online.hip: exchange vectors + partials
     * (hpnn_online_coop_xch_bytes) and the control words (HPNN_ONLINE_CTL_BYTES) */
    double *xch;
    unsigned int *ctl;
    /* device-spanning cooperative grid (online training over several GPUs, the reference's
     * row sharding of cuda_ann.cu:533-1275 over n_gpu x n_streams): this launch is slot
     * `dev_slot` of `n_slots` launches of `grid` workgroups each (one per GPU, or several
     * virtual slots on one GPU); workgroup g = dev_slot * grid + blockIdx.x of
     * n_slots * grid owns rows j == g (mod n_slots * grid) of every layer, and only those
     * rows of its slot's W / dW are read or written.  xch / ctl are ONE allocation that
     * every slot's device maps (fine-grained), accessed at system scope.  n_slots <= 1:
     * the single-device kernel. */
    int dev_slot, n_slots;
} hpnn_online_args;

#define HPNN_ONLINE_CTL_BYTES 1024
/* grid of the cooperative online kernel (0: not applicable -> single-workgroup kernel) */
int hpnn_online_coop_grid(const hpnn_online_args *a);
long hpnn_online_coop_xch_bytes(const hpnn_online_args *a, int grid);
/* one sample on `grid` workgroups (all resident): every layer's rows are spread over the
 * workgroups, vectors and delta partials are exchanged through write-through stores and
 * a counter barrier; returns 0, or < 0 (launch error) */
int hpnn_online_coop_launch(const hpnn_online_args *a, int grid, hipStream_t stream);
/* device-spanning form: workgroups per slot for n_slots slots (0: not applicable);
 * per_device_cap bounds one device's share of resident workgroups */
int hpnn_online_coop_grid_slots(const hpnn_online_args *a, int n_slots, int per_device_cap);
/* 0, or -1 when a barrier of the last cooperative launch timed out (ctl read back) */
int hpnn_online_coop_status(const hpnn_online_args *a);

int hpnn_online_launch(const hpnn_online_args *a, hipStream_t stream);
/* bytes of vector storage the online kernel needs */
long hpnn_online_vec_bytes(const hpnn_online_args *a);

#ifdef __cplusplus
}
#endif

/* one probe kernel per translation unit: hpnn_preload_code_objects() queries its attributes,
 * which loads that unit's code object onto the device */
#define HPNN_CO_PROBE(tu)                                                                  \
    __global__ void hpnn_co_probe_kernel_##tu() {}                                         \
    extern "C" const void *hpnn_co_probe_##tu(void) { return (const void *)hpnn_co_probe_kernel_##tu; }
#endif
