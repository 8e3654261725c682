/*
 * The batched BF16 training plan: ONE orchestrator of the gfx950 kernels, used by the C
 * library's batched engine (train_nn -m batched: gpu_engine.cpp train_single / train_dp /
 * train_dp_mp, batched run_nn) and, through the pybind11 module, by hpnn_amd.models.MLP
 * (bench.py, the data-parallel driver, the tests).  Reference being replaced: the per-layer
 * GEMV / GER sequence of nn_train_kernel -> {ann,snn}_train_BP[M] (libhpnn.c:1149-1302,
 * cuda_snn.cu:2726-3717), here over a minibatch.
 *
 * A plan is
 *   - a configuration (host only, no device needed): padded dims, the step structure
 *     ("mode"), split-K factors, grids, and the table of device buffers it needs;
 *   - memory: either allocated by the plan (C engine) or bound to buffers the host
 *     framework allocated from that table (Python: torch tensors, so they are views);
 *   - launches on a caller-given HIP stream, all capturable in a HIP graph.
 *
 * Modes (the step's kernel sequence):
 *   't'  MNIST-shaped n_in(800|256)-128-64-(<=32): mlp3_tile front (X -> delta1 + [G1|G2]
 *        block slabs) -> G0 with its split-K reduction and every layer's optimizer step in
 *        the same launch (kernels_g0.hip g0_fused_kernel): two launches per step.  Input
 *        fragment-major (8-bit pixels or BF16).
 *   'x'  same shape, 32-sample pipelined front (mlp3_fused), row-major BF16 input (plus an
 *        optional fragment-major 8-bit copy for G0).
 *   'm'  same shape, gemm_nt layer 0 + mlp3_mid.
 *   'w'  K0 = 4096 -> 256 -> 256 (padded): wide2_front, then per-layer weight gradients
 *        (8-phase TN with the update in its epilogue where it applies) and updates.
 *   0    any net: per-layer gemm_nt forward / output_delta / gemm_nt deltas / gemm_tn
 *        gradients / one multi-layer update.
 */
#ifndef HPNN_GPU_BPLAN_H
#define HPNN_GPU_BPLAN_H
#include <hip/hip_runtime_api.h>
#include <stdlib.h>

#include <functional>
#include <string>
#include <vector>

#include "kernels.h"

namespace hpnn {

enum BDtype { BD_F32 = 0, BD_BF16 = 1, BD_U8 = 2, BD_I32 = 3 };

/* one device buffer of the plan */
struct BufSpec {
    std::string name; /* "W32", "V32", "Wb", "Wt", "slab", "gflat", "H", "D", "Z", "stats", ... */
    int layer;        /* -1: not per layer */
    int dtype;        /* BDtype */
    int ndim;
    long shape[4];
    bool zero; /* must start zeroed */
    size_t bytes() const;
};

/* one prepared minibatch: x = the front's input (row-major [Bp][Kp0] BF16, or fragment-major
 * [Bp/32][Kp0/16][64][8] for mode 't', 8-bit when u8), xg = fragment-major 8-bit copy for the
 * first-layer gradient (mode 'x' only, may be null); the network sees bf16(byte * scale) */
struct XIn {
    const void *x = nullptr;
    const void *xg = nullptr;
    int u8 = 0;
    float scale = 1.f;
};

/* gradient ready for exchange: layers lo..hi (contiguous in gflat) are final */
typedef std::function<bool(int lo, int hi)> ReadyFn;

/* the gradient of a step left in its unreduced form (the xGMI all-reduce sums the slabs in its
 * copy-in): segment i = sum over cnt[i] slabs of n[i] floats, stride[i] apart, at base[i] */
struct SlabSegs {
    int count = 0;
    const float *base[2];
    int cnt[2];
    long n[2], stride[2];
};

class BPlan {
  public:
    /* ---- configuration ---- */
    int L = 0, type = 2, batch = 0, Bp = 0, n_out = 0;
    bool momentum = false, on_device = true;
    int M[16], N[16], Kp[16], Np[16], S[16];
    char mode = 0;
    int mid_grid = 0, mid_groups = 1, wide_ksplit = 1, slab_f = 0;
    bool g0_fused = true; /* modes t / x: G0 + reduction + every step in one launch when it applies */
    int g0_perm = 0;      /* tests: > 0 runs the fused G0 grid in a permuted block -> role order */
    /* the fused G0's XCD-local first reduction level (kernels_g0.hip; HPNN_G0_XCD=1) */
    bool g0_xcd = [] { const char *e = getenv("HPNN_G0_XCD"); return e && e[0] == '1'; }();
    bool tn_update = true; /* the step in the 8-phase TN gradient's epilogue where it applies */
    /* two-layer nets: layer 1's gradient + step as the side job of layer 0's fused TN launch */
    bool tn8_side = [] { const char *e = getenv("HPNN_TN8_SIDE"); return !(e && e[0] == '0'); }();
    long side_launches = 0; /* launches issued with that side job (tests) */
    /* per-layer: the delta GEMM reads W (NN form, hpnn_gemm_nn_bf16) instead of W^T, which is
     * then not kept current (the sharded data-parallel step sets it: no transpose per update) */
    bool nn_bwd[16] = {false};
    size_t goff[17] = {0};
    std::vector<BufSpec> specs;

    /* fused: -1 auto (the fastest eligible mode), 0 per-layer only, or 't' / 'x' / 'm' / 'w'
     * (an error when not eligible); splits: per-layer split-K override (null / 0 = pick);
     * mid_grid_req: block slabs of mode 'm'; on_device = false: a host-only configuration
     * (CPU emulation: grids of 1).  Returns 0 or a negative error (message in err). */
    int configure(const int *sizes, int n_layers, int net_type, int batch_size, bool momentum_, int fused,
                  const int *splits, int mid_grid_req, bool device, std::string *err = nullptr);
    /* the layout prepare_input must produce: 1 = fragment-major main input (mode 't'),
     * 2 = row-major BF16 plus a fragment-major 8-bit copy when the data are 8-bit (mode 'x'),
     * 0 = row-major BF16 */
    int input_layout() const { return mode == 't' ? 1 : (mode == 'x' ? 2 : 0); }
    /* split-K factor of a weight gradient (N x K over Bp rows) for this plan's kernels */
    static int pick_splits(int Np, int Kp, int Bp);

    /* ---- memory ---- */
    int allocate(hipStream_t s); /* every spec via hpnn_dev_malloc, zeroed where required */
    int bind(void *const *ptrs); /* one pointer per spec, in spec order (caller owns them) */
    ~BPlan();
    void *buf(const char *name, int layer = -1) const;

    /* ---- launches (stream s) ---- */
    int cast_weights(hipStream_t s); /* BF16 copies (and W0f) from the FP32 masters */
    int zero_stats(hipStream_t s);
    /* per-layer building blocks */
    int forward(const void *X, hipStream_t s); /* row-major BF16 input -> H[], Z */
    int output(const int *labels, const float *T, int ldt, int n_valid, float *O, int ldo, bool stats,
               hipStream_t s);
    int backward_layer(int l, hipStream_t s);                                 /* D[l-1] from D[l] */
    int grad_layer(int l, const XIn &x, bool reduce, hipStream_t s);         /* slab[l] / G[l] */
    int update_layer(int l, float lr, float alpha, float scale, bool from_g, hipStream_t s);
    /* fused front of modes t / x / m / w (X -> deltas, [G1|G2] block slabs) */
    int front(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, hipStream_t s);
    /* whole training step: fwd + bwd + update (no host sync) */
    int step(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, float lr, float alpha,
             hipStream_t s);
    /* data parallel: gradients summed over this replica's samples into gflat, ready(lo, hi) as
     * each bucket becomes final (last layers first) */
    int grads(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, const ReadyFn &ready,
              hipStream_t s);
    std::vector<std::pair<int, int>> buckets() const;
    /* fused modes: front + G0 with the gradient left in slabs (the xGMI all-reduce's copy-in
     * sums them); segs[0] = G0 slabs, segs[1] = [G1|G2] groups -- or, when the G0 launch
     * reduces in-kernel, ONE segment: gflat itself, fully reduced.  dst (with sel / alt, see
     * hpnn_g0_update.gsel): the in-kernel reduced gradient goes there instead (the xGMI
     * all-reduce's own buffer half) and segs->count = 0 */
    int grads_slabs(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, SlabSegs *segs,
                    hipStream_t s, float *dst = nullptr, const unsigned int *sel = nullptr, long alt = 0);
    /* fused modes: front + every layer's gradient summed over this replica's samples into
     * gflat, with G0's split-K and [G1|G2] reductions inside the G0 launch when it applies
     * (two launches; the exchange then moves one copy) */
    int grads_local(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, hipStream_t s);
    /* fused modes, data parallel: front, then G0 with its split-K reduction, the exchange over
     * xv (one-shot xGMI protocol inside the launch, kernels_g0.hip) and every layer's step --
     * the single-GPU step's two launches; scale includes 1 / world.  -1 (nothing launched)
     * when the fused G0 does not cover the shape or the input. */
    int xchg_step(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, float lr, float alpha,
                  float scale, const hpnn_xar_view &xv, hipStream_t s);
    /* collective self-test of that in-kernel exchange on xv (known pattern, exact sums checked
     * on the host): 0 when every float arrived right, > 0 wrong floats, -1 not covered */
    int xchg_self_test(const hpnn_xar_view &xv, hipStream_t s);
    int update_flat(const float *G, float lr, float alpha, float scale, hipStream_t s);
    /* layer l's weight gradient and step run as ONE 8-phase TN launch */
    bool tn_update_ok(int l) const;
    /* network outputs O [Bp][ldo] FP32 of a row-major BF16 batch */
    int predict(const void *X, int n_valid, float *O, int ldo, hipStream_t s);
    /* 0, or -9 when an in-kernel hand-over (wide front partials, fused G0 splits) timed out
     * since the plan was created (synchronises s) */
    int health(hipStream_t s);
    /* the same words copied into dst[0..2] (pinned host memory, zeroed by the caller) on s
     * without waiting: a training loop checks them one replay later, so the check never
     * leaves the GPU idle; any non-zero word = a timed-out hand-off */
    int health_enqueue(hipStream_t s, unsigned int *dst);
    /* 64-bit digest of the weights (bit 1: BF16 copies W / W^T of every layer, bit 2: the FP32
     * masters); data-parallel replicas must agree on it bit for bit (synchronises s) */
    int weights_digest(int which, unsigned long long *out, hipStream_t s);
    /* (loss sum, hits) summed over the stat slots (synchronises s) */
    int read_stats(double *loss, unsigned int *hits, hipStream_t s);

    /* named pointers (valid after allocate / bind) */
    float *W32[16] = {0}, *V32[16] = {0}, *slab[16] = {0};
    void *Wb[16] = {0}, *Wt[16] = {0}, *H[16] = {0}, *D[16] = {0};
    float *Z = nullptr, *stats = nullptr, *gflat = nullptr, *midslab = nullptr, *midtmp = nullptr;
    void *W0f = nullptr;
    float *wpbuf = nullptr;
    unsigned int *wwords = nullptr, *g0cnt = nullptr, *tncnt = nullptr, *g0xw = nullptr;
    float *g0xs = nullptr;
    int *lab0 = nullptr;
    /* data-parallel BF16 exchange (csrc/dist/dp_exchange.cpp): where grad_layer(reduce) may
     * write layer l's gradient as BF16 instead of FP32 into gflat (NULL: FP32), and whether the
     * last call did (shapes the 8-phase kernel does not cover stay FP32) */
    void *g16[16] = {0};
    bool g16_used[16] = {0};

  private:
    std::vector<void *> ptr_;
    bool owns_ = false;
    unsigned long long *digest_ = nullptr; /* device word of weights_digest */
    int grad_and_update_layers(const XIn &x, float lr, float alpha, float scale, hipStream_t s);
    int g0_reduce(const XIn &x, hipStream_t s);
    int g0_fused_step(const XIn &x, float lr, float alpha, float scale, hipStream_t s, float *gout = nullptr,
                      const unsigned int *gsel = nullptr, long galt = 0, const hpnn_xar_view *xv = nullptr);
    const void *fm_input(const XIn &x) const;
    void name_pointers();
};

}  // namespace hpnn

#endif
