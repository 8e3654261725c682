/*
 * Native data-parallel step over RCCL: FP32 bucket all-reduce or BF16 reduce-scatter +
 * sharded optimizer step + BF16 all-gather, overlapped with the backward (dp_exchange.h).
 */
#include "dp_exchange.h"

#include <stdlib.h>

#include <algorithm>

#include <libhpnn.h>
#include <libhpnn/devmem.h>

namespace hpnn {

DpExchange::~DpExchange() {
    if (p_)
        for (int l = 0; l < p_->L; l++) {
            p_->g16[l] = nullptr;
            if (l < (int)nn_.size() && nn_[l]) { /* the plan goes back to W^T: make it current */
                p_->nn_bwd[l] = false;
                (void)hpnn_transpose_bf16(p_->Wb[l], p_->Wt[l], p_->Np[l], p_->Kp[l], nullptr);
            }
        }
    if (p_ && std::find(nn_.begin(), nn_.end(), true) != nn_.end()) (void)hipDeviceSynchronize();
    hpnn_dev_free(grad16_);
    hpnn_dev_free(send16_);
    hpnn_dev_free(recv16_);
    hpnn_dev_free(emu16_);
}

int DpExchange::init(BPlan *plan, hpnn_comm *comm, int mode) {
    if (!plan || !comm) return -1;
    p_ = plan;
    c_ = comm;
    rank_ = hpnn_comm_rank(comm);
    world_ = hpnn_comm_size(comm);
    mode_ = mode == BF16RS ? BF16RS : FP32;
    sharded_.assign(p_->L, false);
    vw_ = world_;
    if (const char *e = getenv("HPNN_DPX_EMULATE_WORLD")) {
        const int w = atoi(e);
        if (w > 1 && world_ == 1 && mode_ == BF16RS) {
            vw_ = w;
            emu_ = true;
            NN_WARN(stderr, "HPNN_DPX_EMULATE_WORLD=%d: one rank runs the sharded step at %d-rank sizes "
                            "(timing only, not a training run)\n", w, w);
        }
    }
    if (mode_ == FP32) return 0;
    if (p_->mode) {
        NN_ERROR(stderr, "BF16 reduce-scatter exchange needs the per-layer plan (mode %c)\n", p_->mode);
        return -2;
    }
    size_t mx = 0;
    /* HPNN_DPX_SHARD1=1 (tests): the sharded path even on one rank (the collectives are then
     * copies), so its kernels and ordering run on a one-GPU box */
    const char *s1 = getenv("HPNN_DPX_SHARD1");
    const bool one = s1 && s1[0] == '1';
    for (int l = 0; l < p_->L; l++) {
        /* rows split evenly over the ranks (any block height: the transpose runs on the whole
         * all-gathered matrix) */
        sharded_[l] = (vw_ > 1 || one) && p_->Np[l] % vw_ == 0;
        if (sharded_[l]) mx = mx > (size_t)p_->Np[l] * p_->Kp[l] ? mx : (size_t)p_->Np[l] * p_->Kp[l];
    }
    /* the BF16 send staging buffer is only for sharded layers whose gradient the 8-phase TN GEMM
     * cannot write in BF16 itself (split-K, or a shape it does not take): cast from FP32 */
    size_t mx_cast = 0;
    for (int l = 0; l < p_->L; l++)
        if (sharded_[l] && !(p_->S[l] == 1 && hpnn_gemm_tn8_bf16out_ok(p_->Np[l], p_->Kp[l], p_->Bp, p_->Np[l], p_->Kp[l])))
            mx_cast = mx_cast > (size_t)p_->Np[l] * p_->Kp[l] ? mx_cast : (size_t)p_->Np[l] * p_->Kp[l];
    if (mx_cast && hpnn_dev_malloc(&send16_, mx_cast * 2) != hipSuccess) return -7;
    if (mx && hpnn_dev_malloc(&recv16_, mx * 2 / vw_ + 64) != hipSuccess) return -7;
    if (emu_ && mx && hpnn_dev_malloc(&emu16_, mx * 2) != hipSuccess) return -7;
    /* one BF16 gradient buffer per sharded layer: the plan's TN GEMM writes it directly (no
     * FP32 round trip and cast), the side stream reduce-scatters it while the next layer's
     * gradient goes into its own buffer */
    size_t tot = 0;
    for (int l = 0; l < p_->L; l++)
        if (sharded_[l]) tot += (size_t)p_->Np[l] * p_->Kp[l];
    if (tot && hpnn_dev_malloc(&grad16_, tot * 2) != hipSuccess) return -7;
    for (size_t l = 0, o = 0; l < (size_t)p_->L; l++)
        if (sharded_[l]) {
            p_->g16[l] = (char *)grad16_ + o * 2;
            o += (size_t)p_->Np[l] * p_->Kp[l];
        }
    /* the delta GEMM of a sharded layer reads the all-gathered W directly (NN form, same bits),
     * so the step needs no W^T rebuild (a 2 x P-byte transpose per layer; HPNN_DPX_NN=0: keep
     * it); W^T is made current again by gather_masters and when the exchange goes away */
    const char *nn = getenv("HPNN_DPX_NN");
    nn_.assign(p_->L, false);
    for (int l = 1; l < p_->L; l++)
        if (sharded_[l] && !(nn && nn[0] == '0') &&
            hpnn_gemm_nn_ok(p_->Bp, p_->Np[l - 1], p_->Np[l], p_->Np[l], p_->Kp[l], p_->Np[l - 1]) &&
            p_->Kp[l] == p_->Np[l - 1])
            nn_[l] = p_->nn_bwd[l] = true;
    return 0;
}

int DpExchange::step(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, int n_total, float lr,
                     float alpha, hipStream_t s) {
    const float scale = 1.0f / (float)(n_total > 0 ? n_total : 1);
    const int mom = p_->momentum ? 1 : 0;
    int err = 0;
    auto layer_rs = [&](int l) -> int {
        /* on the side stream, after the compute stream's work so far (this gradient) */
        hipStream_t side = hpnn_comm_fork(c_, s);
        if (!side) return -2;
        const int N = p_->Np[l], K = p_->Kp[l], rp = N / vw_;
        const long cnt = (long)rp * K, off = (long)rank_ * cnt;
        const void *src = send16_;
        int r = 0;
        if (p_->g16[l] && p_->g16_used[l]) src = p_->g16[l]; /* the GEMM wrote BF16 already */
        else if (!send16_) r = -9; /* init judged this layer's gradient to come in BF16 */
        else r = hpnn_cast_f32_bf16(p_->gflat + p_->goff[l], send16_, (long)N * K, side);
        if (!r) r = hpnn_comm_reduce_scatter(c_, src, recv16_, cnt, HPNN_DT_BF16, HPNN_OP_SUM, side);
        if (!r)
            r = hpnn_sgd_update_rows_bf16g(p_->W32[l] + off, p_->V32[l] ? p_->V32[l] + off : nullptr, recv16_, cnt, lr,
                                           alpha, scale, mom, (char *)p_->Wb[l] + off * 2, side);
        if (!r && emu_) /* the (W-1) / W of the rows a rank receives, as a local copy */
            r = hipMemcpyAsync(emu16_, (const char *)p_->Wb[l] + cnt * 2, (size_t)(vw_ - 1) * cnt * 2,
                               hipMemcpyDeviceToDevice, side) == hipSuccess ? 0 : -5;
        else if (!r)
            r = hpnn_comm_all_gather(c_, (char *)p_->Wb[l] + off * 2, p_->Wb[l], cnt, HPNN_DT_BF16, side);
        if (!r && !nn_[l]) r = hpnn_transpose_bf16(p_->Wb[l], p_->Wt[l], N, K, side);
        const int rd = hpnn_comm_fork_done(c_);
        return r ? r : rd;
    };
    auto ready = [&](int lo, int hi) -> bool {
        if (err) return true; /* keep issuing nothing more; the step reports the error */
        if (mode_ == BF16RS) {
            for (int l = hi; l >= lo && !err; l--) {
                if (sharded_[l]) err = layer_rs(l);
                else err = hpnn_comm_all_reduce_async(c_, p_->gflat + p_->goff[l], (long)(p_->goff[l + 1] - p_->goff[l]),
                                                      HPNN_DT_F32, s);
            }
            return err == 0;
        }
        err = hpnn_comm_all_reduce_async(c_, p_->gflat + p_->goff[lo], (long)(p_->goff[hi + 1] - p_->goff[lo]),
                                         HPNN_DT_F32, s);
        return err == 0;
    };
    int r = p_->grads(x, labels, T, ldt, n_valid, ready, s);
    const int j = hpnn_comm_join(c_, s);
    if (r || err || j) {
        NN_ERROR(stderr, "data-parallel step failed (grads %d, exchange %d, join %d)\n", r, err, j);
        return r ? r : (err ? err : j);
    }
    if (mode_ == FP32) return p_->update_flat(p_->gflat, lr, alpha, scale, s);
    for (int l = 0; l < p_->L; l++)
        if (!sharded_[l] && (r = p_->update_layer(l, lr, alpha, scale, true, s))) return r;
    return 0;
}

int DpExchange::gather_masters(hipStream_t s) {
    if (mode_ != BF16RS) return 0;
    for (int l = 0; l < p_->L; l++) {
        if (!sharded_[l]) continue;
        /* W^T current for the readers outside the step (checkpoints, tests, digests) */
        if (nn_[l] && hpnn_transpose_bf16(p_->Wb[l], p_->Wt[l], p_->Np[l], p_->Kp[l], s)) return -3;
        if (emu_) continue; /* an emulated run has no other ranks' rows to gather */
        const long cnt = (long)(p_->Np[l] / world_) * p_->Kp[l], off = (long)rank_ * cnt;
        float *bufs[2] = {p_->W32[l], p_->V32[l]};
        for (float *b : bufs) {
            if (!b) continue;
            /* in place: this rank's rows sit at rank * cnt already */
            if (hpnn_comm_all_gather(c_, b + off, b, cnt, HPNN_DT_F32, s)) return -3;
        }
    }
    return 0;
}

}  // namespace hpnn
