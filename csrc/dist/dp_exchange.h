/*
 * Native data-parallel step over RCCL (one process per GPU): the library's batched plan
 * (csrc/gpu/bplan.h) computes each layer's gradient sum into the flat buffer and reports it
 * ready (last layers first); the exchange runs on the communicator's side stream while the
 * backward of the layers below continues on the compute stream.  Replaces the reference's
 * MPI tier, which replicated the same sample on every rank and all-gathered every weight
 * matrix after each update (ann.c:1638).
 *
 *   FP32    every layer bucket all-reduced (FP32 sum), then every rank steps the whole net
 *           from the identical sums (the update launch joins the buckets).
 *   BF16RS  for layers whose padded rows split evenly over the ranks: the gradient is cast to
 *           BF16 and reduce-scattered (rank r receives the sum of its rows), rank r steps its
 *           rows of the FP32 masters / momentum (a sharded optimizer: the masters live
 *           sharded), the BF16 compute rows are all-gathered in place and W^T rebuilt --
 *           (W-1)/W x P x (2 + 2) bytes per rank and step instead of the ring all-reduce's
 *           2 (W-1)/W x P x 4: half.  All of it on the side stream, per layer, as soon as the
 *           gradient is final; other layers take the FP32 path.
 * No per-step allocation: the BF16 staging buffers are sized once for the widest layer.
 */
#ifndef HPNN_DIST_DP_EXCHANGE_H
#define HPNN_DIST_DP_EXCHANGE_H
#include <libhpnn/comm.h>

#include <vector>

#include "../gpu/bplan.h"

namespace hpnn {

class DpExchange {
  public:
    enum Mode { FP32 = 0, BF16RS = 1 };
    /* plan: this rank's replica (modes t / x / m / w / per-layer); BF16RS needs the per-layer
     * plan (mode 0).  Returns 0 or < 0 (and the exchange must not be used). */
    int init(BPlan *plan, hpnn_comm *comm, int mode);
    ~DpExchange();
    /* one data-parallel step: n_total = samples of the global minibatch (the gradient scale) */
    int step(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, int n_total, float lr, float alpha,
             hipStream_t s);
    /* BF16RS: every rank's rows of the FP32 masters / momentum onto every rank (checkpoints) */
    int gather_masters(hipStream_t s);
    bool sharded(int l) const { return l < (int)sharded_.size() && sharded_[l]; }

  private:
    BPlan *p_ = nullptr;
    hpnn_comm *c_ = nullptr;
    int rank_ = 0, world_ = 1;
    /* shard count: world_, or HPNN_DPX_EMULATE_WORLD on one rank (emu_): that rank runs the
     * sharded step at that world's per-rank sizes -- 1/W of the rows reduce-scattered and
     * stepped, the all-gather's receive bytes copied locally -- for timing the per-rank
     * compute of a W-GPU run on one GPU (timing only: the other rows are never updated) */
    int vw_ = 1;
    bool emu_ = false;
    void *emu16_ = nullptr;
    Mode mode_ = FP32;
    std::vector<bool> sharded_;
    std::vector<bool> nn_; /* sharded layers whose delta GEMM reads W (no W^T rebuild per step) */
    void *send16_ = nullptr, *recv16_ = nullptr;
    void *grad16_ = nullptr; /* per-layer BF16 gradients written by the plan's TN GEMM (sharded layers) */
};

}  // namespace hpnn

#endif
