/*
 * Row-sharded tensor parallelism for the batched GPU engine ([parallel] tp; [dtype] f64 | f32
 * below, [dtype] bf16 in TpNetBf16 further down): the reference's model-parallel scheme (every layer's neuron rows
 * split over MPI ranks / GPUs, ann.c:912-1236 with MPI_Allgather at ann.c:925, 957, 990;
 * cuda_ann.cu:533-1275 over n_gpu x n_streams), with the whole minibatch on every rank.
 *
 * Activations are kept FEATURE-MAJOR (H^T [features][batch]): rank r owns the feature rows
 * [r n_l, (r+1) n_l) of every hidden layer, so an all-gather of the local rows IS the full
 * H^T, with no re-ordering.  Per step, rank r:
 *
 *   forward   H_l^T[R_r] = f(W_l[R_r] H_{l-1}^T)            FP64/FP32 MFMA GEMM, local
 *             H_l^T      = all_gather(H_l^T[R_r])            n_l x B elements per rank
 *   output    the output layer is replicated (it is narrow: n_out <= a few hundred):
 *             Z = H_{L-1} W_L^T, softmax / loss / delta_L on every rank, bit-identical
 *   backward  delta_{L-1}^T[R_r] = (W_L[:, R_r])^T delta_L^T * f'(H)   local, no comm
 *             G_l[R_r] = delta_l^T[R_r] H_{l-1}                          local
 *             P^T = W_l[R_r]^T delta_l^T[R_r]  (this rank's share of every input's delta)
 *             delta_{l-1}^T[R_r] = reduce_scatter(P^T) * f'(H_{l-1}^T[R_r])
 *                                  (the f' epilogue runs on the reduced rows: hpnn_dact_fp)
 *   update    local rows only (the replicated output layer: the same update everywhere)
 *
 * so the weights are never moved (the reference all-gathered every N_l x M_l weight
 * matrix after each update); a step moves B x (sum of hidden widths) activations and
 * partial deltas.  Rows are padded to P x ceil(N_l / P) with zero weights, which keep
 * their activations, deltas and gradients at zero.
 *
 * Collectives: RCCL (one process per GPU under a launcher, or one host thread per GPU of
 * this process with train_nn -G N) or, with HPNN_LOOPBACK_RANKS = P, P host threads on ONE
 * GPU exchanging through a device staging buffer (tests and CI without a multi-GPU node).
 */
#include <hip/hip_runtime.h>
#include <hip/hip_runtime_api.h>
#include <libhpnn/ann.h>
#include <libhpnn/bootstrap.h>
#include <libhpnn/comm.h>
#include <libhpnn/devmem.h>
#include <libhpnn/observe.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../core/runtime_internal.h"
#include "bplan.h"
#include "engine.h"
#include "kernels.h"

#define TPCHK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            NN_ERROR(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return FALSE;                                                                         \
        }                                                                                         \
    } while (0)

namespace {

layer_ann *layer_at(kernel_ann *k, int l) { return l < (int)k->n_hiddens ? &k->hiddens[l] : &k->output; }
constexpr size_t ACC_BYTES = (size_t)HPNN_STAT_SLOTS * HPNN_STAT_STRIDE * 4;

/* ---------------------------------------------------------------- collectives */
template <typename T>
struct TpColl {
    virtual ~TpColl() {}
    /* recv [P][count] <- every rank's send [count] */
    virtual bool all_gather(const T *send, T *recv, long count, hipStream_t s) = 0;
    /* recv [count] <- sum over ranks of their send[r * count ...] (send: [P][count]) */
    virtual bool reduce_scatter(const T *send, T *recv, long count, hipStream_t s) = 0;
    /* full weights for the host copy: same as all_gather, off the hot path */
    virtual bool gather_rows(const T *send, T *recv, long count, hipStream_t s) { return all_gather(send, recv, count, s); }
    virtual void abort() {}
    /* the collectives only enqueue on the stream (no host waits): an epoch can be captured */
    virtual bool capturable() const { return false; }
};

template <typename T>
struct RcclColl : TpColl<T> {
    hpnn_comm *c;
    static constexpr hpnn_comm_dtype DT = sizeof(T) == 8 ? HPNN_DT_F64 : HPNN_DT_F32;
    explicit RcclColl(hpnn_comm *cc) : c(cc) {}
    bool all_gather(const T *send, T *recv, long count, hipStream_t s) override {
        return hpnn_comm_all_gather(c, send, recv, count, DT, s) == 0;
    }
    bool reduce_scatter(const T *send, T *recv, long count, hipStream_t s) override {
        return hpnn_comm_reduce_scatter(c, send, recv, count, DT, HPNN_OP_SUM, s) == 0;
    }
    bool capturable() const override { return true; }
};

/* host-thread ranks on one device: a generation barrier (abortable, so one failing rank
 * cannot leave the others waiting) and a device staging buffer */
struct HostBarrier {
    std::mutex m;
    std::condition_variable cv;
    int P = 1, count = 0;
    unsigned gen = 0;
    bool aborted = false;
    bool wait() {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) return false;
        const unsigned g = gen;
        if (++count == P) {
            count = 0;
            gen++;
            cv.notify_all();
            return true;
        }
        cv.wait(lk, [&] { return gen != g || aborted; });
        return !aborted;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m);
        aborted = true;
        cv.notify_all();
    }
};

template <typename T>
struct HostShared {
    int P = 1;
    T *stage = nullptr;
    HostBarrier bar;
    ~HostShared() { hpnn_dev_free(stage); }
};

template <typename T>
struct HostColl : TpColl<T> {
    HostShared<T> *sh;
    int r;
    HostColl(HostShared<T> *s_, int rank) : sh(s_), r(rank) {}
    bool all_gather(const T *send, T *recv, long count, hipStream_t s) override {
        const size_t b = (size_t)count * sizeof(T);
        if (hipMemcpyAsync(sh->stage + (size_t)r * count, send, b, hipMemcpyDeviceToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess || !sh->bar.wait())
            return false;
        if (hipMemcpyAsync(recv, sh->stage, b * sh->P, hipMemcpyDeviceToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return false;
        return sh->bar.wait();
    }
    bool reduce_scatter(const T *send, T *recv, long count, hipStream_t s) override {
        const long blk = (long)sh->P * count; /* rank q's whole send at stage + q * blk */
        if (hipMemcpyAsync(sh->stage + (size_t)r * blk, send, (size_t)blk * sizeof(T), hipMemcpyDeviceToDevice, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess || !sh->bar.wait())
            return false;
        /* sum in rank order: deterministic */
        if (hpnn_reduce_fp(sizeof(T) == 8, recv, sh->stage + (size_t)r * count, sh->P, blk, count, s) != 0 ||
            hipStreamSynchronize(s) != hipSuccess)
            return false;
        return sh->bar.wait();
    }
    void abort() override { sh->bar.abort(); }
};

/* ---------------------------------------------------------------- one rank's shard */
template <typename T>
struct TpNet {
    typedef T coll_t; /* element type of the collectives */
    static constexpr int F64 = sizeof(T) == 8 ? 1 : 0;
    static const char *name() { return sizeof(T) == 8 ? "f64" : "f32"; }
    int L = 0, P = 1, r = 0, Bp = 0, n_out = 0, type = 2;
    int Ntrue[16], Mtrue[16], n[16], Mp[16], S[16];
    T *W[16] = {0}, *V[16] = {0}, *slab[16] = {0}, *Hloc[16] = {0}, *Hfull[16] = {0}, *Dloc[16] = {0};
    T *DL = nullptr, *Z = nullptr, *part = nullptr;
    T *Xt = nullptr, *Td = nullptr; /* the sample set: X^T [n_in][cols], targets [cols][n_out] */
    int cols = 0;
    float *acc = nullptr;
    hipStream_t s = nullptr;
    TpColl<T> *coll = nullptr;

    ~TpNet() {
        if (s) hipStreamSynchronize(s);
        hpnn_dev_free(Xt);
        hpnn_dev_free(Td);
        for (int l = 0; l < 16; l++) {
            hpnn_dev_free(W[l]);
            hpnn_dev_free(V[l]);
            hpnn_dev_free(slab[l]);
            hpnn_dev_free(Hloc[l]);
            hpnn_dev_free(Hfull[l]);
            hpnn_dev_free(Dloc[l]);
        }
        hpnn_dev_free(DL);
        hpnn_dev_free(Z);
        hpnn_dev_free(part);
        hpnn_dev_free(acc);
    }

    static int pick(int Nn, int Mm, int B) {
        const int tiles = ((Nn + 63) / 64) * ((Mm + 63) / 64);
        int sp = (256 + tiles - 1) / tiles;
        const int maxs = B / 256 > 0 ? B / 256 : 1;
        sp = sp < maxs ? sp : maxs;
        return hpnn_gemm_fp_splits(B, sp < 1 ? 1 : sp);
    }

    /* rows of layer l this rank holds in the host weights: global row of local row j */
    int grow(int l, int j) const { return l < L - 1 ? r * n[l] + j : j; }

    BOOL init(kernel_ann *k, int P_, int r_, int B, nn_type t, bool momentum, hipStream_t st, TpColl<T> *c) {
        P = P_, r = r_, s = st, coll = c, Bp = B;
        L = (int)k->n_hiddens + 1;
        n_out = (int)k->n_outputs;
        type = t == NN_TYPE_ANN ? 0 : (t == NN_TYPE_LNN ? 1 : 2);
        size_t part_elems = 0;
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_at(k, l);
            Ntrue[l] = (int)ly->n_neurons;
            Mtrue[l] = (int)ly->n_inputs;
            n[l] = l < L - 1 ? (Ntrue[l] + P - 1) / P : Ntrue[l];
            Mp[l] = l == 0 ? Mtrue[0] : (l - 1 < L - 1 ? P * n[l - 1] : Mtrue[l]);
            S[l] = pick(n[l], Mp[l], Bp);
            const size_t nw = (size_t)n[l] * Mp[l];
            TPCHK(hpnn_dev_malloc(&W[l], nw * sizeof(T)));
            TPCHK(hpnn_dev_malloc(&slab[l], nw * sizeof(T) * S[l]));
            if (momentum) {
                TPCHK(hpnn_dev_malloc(&V[l], nw * sizeof(T)));
                TPCHK(hipMemsetAsync(V[l], 0, nw * sizeof(T), s));
            }
            if (l < L - 1) {
                TPCHK(hpnn_dev_malloc(&Hloc[l], (size_t)n[l] * Bp * sizeof(T)));
                TPCHK(hpnn_dev_malloc(&Hfull[l], (size_t)P * n[l] * Bp * sizeof(T)));
                TPCHK(hpnn_dev_malloc(&Dloc[l], (size_t)n[l] * Bp * sizeof(T)));
            }
            if (l >= 1 && l < L - 1) part_elems = std::max(part_elems, (size_t)Mp[l] * Bp);
            std::vector<T> tmp(nw, (T)0);
            for (int j = 0; j < n[l]; j++) {
                const int g = grow(l, j);
                if (g >= Ntrue[l]) continue;
                for (int m = 0; m < Mtrue[l]; m++) tmp[(size_t)j * Mp[l] + m] = (T)ly->weights[(size_t)g * Mtrue[l] + m];
            }
            TPCHK(hipMemcpyAsync(W[l], tmp.data(), nw * sizeof(T), hipMemcpyHostToDevice, s));
            TPCHK(hipStreamSynchronize(s));
        }
        TPCHK(hpnn_dev_malloc(&Z, (size_t)Bp * n_out * sizeof(T)));
        TPCHK(hpnn_dev_malloc(&DL, (size_t)Bp * n_out * sizeof(T)));
        if (part_elems) TPCHK(hpnn_dev_malloc(&part, part_elems * sizeof(T)));
        TPCHK(hpnn_dev_malloc(&acc, ACC_BYTES));
        TPCHK(hipMemsetAsync(acc, 0, ACC_BYTES, s));
        return TRUE;
    }

    BOOL upload_momentum(const kernel_ann *k) {
        if (!k->dw) return TRUE;
        for (int l = 0; l < L; l++) {
            if (!V[l]) continue;
            std::vector<T> tmp((size_t)n[l] * Mp[l], (T)0);
            for (int j = 0; j < n[l]; j++) {
                const int g = grow(l, j);
                if (g >= Ntrue[l]) continue;
                for (int m = 0; m < Mtrue[l]; m++) tmp[(size_t)j * Mp[l] + m] = (T)k->dw[l][(size_t)g * Mtrue[l] + m];
            }
            TPCHK(hipMemcpyAsync(V[l], tmp.data(), tmp.size() * sizeof(T), hipMemcpyHostToDevice, s));
            TPCHK(hipStreamSynchronize(s));
        }
        return TRUE;
    }

#define TPK(call, what)                                                 \
    do {                                                                \
        const int rc_ = (call);                                         \
        if (rc_) {                                                      \
            NN_ERROR(stderr, "tensor-parallel %s failed (%d)\n", what, rc_); \
            return FALSE;                                               \
        }                                                               \
    } while (0)

    /* one minibatch: Xt = X^T columns of this batch (ldx = row pitch of the uploaded X^T),
     * Tt [Bp][n_out] targets, nv valid samples */
    BOOL step(const T *Xt, int ldx, const T *Tt, int nv, double lr, double alpha, bool mom) {
        auto hin = [&](int l, int *ld) -> const T * {
            if (l == 0) {
                *ld = ldx;
                return Xt;
            }
            *ld = Bp;
            return Hfull[l - 1];
        };
        /* forward of the sharded hidden layers */
        for (int l = 0; l < L - 1; l++) {
            int ld;
            const T *A = hin(l, &ld);
            TPK(hpnn_gemm_fp(F64, W[l], Mp[l], 0, A, ld, 1, Hloc[l], Bp, nullptr, 0, n[l], Bp, Mp[l], HPNN_EPI_ACT, 1,
                             0, s),
                "forward GEMM");
            if (!coll->all_gather(Hloc[l], Hfull[l], (long)n[l] * Bp, s)) return FALSE;
        }
        /* replicated output layer */
        const int o = L - 1;
        int ldo;
        const T *Ho = hin(o, &ldo);
        TPK(hpnn_gemm_fp(F64, Ho, ldo, 1, W[o], Mp[o], 0, Z, n_out, nullptr, 0, Bp, n_out, Mp[o], HPNN_EPI_NONE, 1, 0,
                         s),
            "output GEMM");
        TPK(hpnn_output_fp(F64, Z, n_out, Tt, n_out, DL, n_out, nullptr, 0, nullptr, acc, (unsigned int *)(acc + 1),
                           Bp, nv, n_out, type, s),
            "output layer");
        /* output layer gradient (replicated) and the local rows of the last hidden delta */
        TPK(hpnn_gemm_fp(F64, DL, n_out, 1, Ho, ldo, 0, slab[o], Mp[o], nullptr, 0, n_out, Mp[o], Bp, HPNN_EPI_NONE,
                         S[o], (long)n_out * Mp[o], s),
            "output gradient");
        if (L >= 2) {
            const int h = L - 2;
            TPK(hpnn_gemm_fp(F64, W[o] + (size_t)r * n[h], Mp[o], 1, DL, n_out, 0, Dloc[h], Bp, Hloc[h], Bp, n[h], Bp,
                             n_out, HPNN_EPI_DACT, 1, 0, s),
                "delta GEMM");
        }
        for (int l = L - 2; l >= 0; l--) {
            int ld;
            const T *A = hin(l, &ld);
            TPK(hpnn_gemm_fp(F64, Dloc[l], Bp, 0, A, ld, 0, slab[l], Mp[l], nullptr, 0, n[l], Mp[l], Bp, HPNN_EPI_NONE,
                             S[l], (long)n[l] * Mp[l], s),
                "weight gradient");
            if (l > 0) {
                /* this rank's share of every input's delta, summed over ranks for the local rows */
                TPK(hpnn_gemm_fp(F64, W[l], Mp[l], 1, Dloc[l], Bp, 1, part, Bp, nullptr, 0, Mp[l], Bp, n[l],
                                 HPNN_EPI_NONE, 1, 0, s),
                    "partial delta GEMM");
                if (!coll->reduce_scatter(part, Dloc[l - 1], (long)n[l - 1] * Bp, s)) return FALSE;
                TPK(hpnn_dact_fp(F64, Dloc[l - 1], Dloc[l - 1], Hloc[l - 1], (long)n[l - 1] * Bp, s), "f' epilogue");
            }
        }
        const double scale = 1.0 / (double)(nv > 0 ? nv : 1);
        for (int l = 0; l < L; l++)
            TPK(hpnn_update_fp(F64, W[l], V[l], slab[l], S[l], (long)n[l] * Mp[l], (long)n[l] * Mp[l], lr, alpha, scale,
                               mom ? 1 : 0, s),
                "update");
        return hpnn_debug_check("tensor-parallel step") == 0;
    }

    /* the whole sample set as X^T [n_in][cols] (batch b at columns b B) and targets */
    BOOL upload_data(const DOUBLE *X, const DOUBLE *Tg, UINT ns, int n_in, int cols_) {
        cols = cols_;
        std::vector<T> h((size_t)n_in * cols, (T)0);
        for (UINT i = 0; i < ns; i++)
            for (int c = 0; c < n_in; c++) h[(size_t)c * cols + i] = (T)X[(size_t)i * n_in + c];
        TPCHK(hpnn_dev_malloc(&Xt, h.size() * sizeof(T)));
        TPCHK(hipMemcpyAsync(Xt, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
        std::vector<T> t((size_t)cols * n_out, (T)0);
        for (size_t i = 0; i < (size_t)ns * n_out; i++) t[i] = (T)Tg[i];
        TPCHK(hpnn_dev_malloc(&Td, t.size() * sizeof(T)));
        TPCHK(hipMemcpyAsync(Td, t.data(), t.size() * sizeof(T), hipMemcpyHostToDevice, s));
        TPCHK(hipStreamSynchronize(s));
        return TRUE;
    }
    BOOL batch_step(int b, int B, int nv, double lr, double alpha, bool mom) {
        return step(Xt + (size_t)b * B, cols, Td + (size_t)b * B * n_out, nv, lr, alpha, mom);
    }
    /* elements of the loopback staging buffer the collectives of P ranks need */
    size_t stage_elems() const {
        size_t st = 0;
        for (int l = 0; l < L - 1; l++) {
            st = std::max(st, (size_t)P * n[l] * Bp);
            if (l + 1 < L - 1) st = std::max(st, (size_t)P * Mp[l + 1] * Bp);
        }
        for (int l = 0; l < L; l++) st = std::max(st, (size_t)P * n[l] * Mp[l]);
        return st;
    }
    BOOL host_rows(kernel_ann *k, bool mom) { return download_rows(k, r, W, mom ? V : nullptr); }

    BOOL read_stats(double *loss, unsigned int *hits) {
        std::vector<float> h(ACC_BYTES / 4);
        TPCHK(hipMemcpyAsync(h.data(), acc, ACC_BYTES, hipMemcpyDeviceToHost, s));
        TPCHK(hipStreamSynchronize(s));
        double l = 0.0;
        unsigned int c = 0;
        for (int i = 0; i < HPNN_STAT_SLOTS; i++) {
            l += h[(size_t)i * HPNN_STAT_STRIDE];
            unsigned int u;
            memcpy(&u, &h[(size_t)i * HPNN_STAT_STRIDE + 1], 4);
            c += u;
        }
        *loss = l;
        *hits = c;
        return TRUE;
    }

    /* every rank's rows of every layer -> the host kernel of this rank (all-gather) */
    BOOL gather_to_host(kernel_ann *k, TpColl<T> &cl, int W_, bool mom) {
        BOOL ok = TRUE;
        for (int l = 0; l < L && ok; l++) {
            const long cnt = (long)n[l] * Mp[l];
            T *full = nullptr;
            const int sh = l < L - 1 ? W_ : 1;
            for (int pass = 0; pass < (mom ? 2 : 1) && ok; pass++) {
                const T *src = pass ? V[l] : W[l];
                ok = hpnn_dev_malloc(&full, (size_t)cnt * sh * sizeof(T)) == hipSuccess;
                if (ok && sh > 1) ok = cl.gather_rows(src, full, cnt, s);
                else if (ok) ok = hipMemcpyAsync(full, src, cnt * sizeof(T), hipMemcpyDeviceToDevice, s) == hipSuccess;
                std::vector<T> h((size_t)cnt * sh);
                if (ok) ok = hipMemcpyAsync(h.data(), full, h.size() * sizeof(T), hipMemcpyDeviceToHost, s) ==
                             hipSuccess && hipStreamSynchronize(s) == hipSuccess;
                hpnn_dev_free(full);
                full = nullptr;
                if (!ok) break;
                layer_ann *ly = layer_at(k, l);
                DOUBLE *dst = pass ? k->dw[l] : ly->weights;
                const int rows = sh * n[l];
                for (int g = 0; g < rows && g < Ntrue[l]; g++)
                    for (int m = 0; m < Mtrue[l]; m++) dst[(size_t)g * Mtrue[l] + m] = (DOUBLE)h[(size_t)g * Mp[l] + m];
            }
        }
        return ok;
    }

    /* this rank's rows -> the host kernel (rows of other ranks untouched) */
    BOOL download_rows(kernel_ann *k, int rank_rows_of, const T *const *Wsrc, const T *const *Vsrc) {
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_at(k, l);
            const int rr = rank_rows_of;
            const size_t nw = (size_t)n[l] * Mp[l];
            std::vector<T> tmp(nw);
            for (int pass = 0; pass < 2; pass++) {
                const T *src = pass ? (Vsrc ? Vsrc[l] : nullptr) : Wsrc[l];
                if (!src) continue;
                DOUBLE *dst = pass ? k->dw[l] : ly->weights;
                TPCHK(hipMemcpyAsync(tmp.data(), src, nw * sizeof(T), hipMemcpyDeviceToHost, s));
                TPCHK(hipStreamSynchronize(s));
                for (int j = 0; j < n[l]; j++) {
                    const int g = l < L - 1 ? rr * n[l] + j : j;
                    if (g >= Ntrue[l]) continue;
                    for (int m = 0; m < Mtrue[l]; m++) dst[(size_t)g * Mtrue[l] + m] = (DOUBLE)tmp[(size_t)j * Mp[l] + m];
                }
            }
        }
        return TRUE;
    }
};

/* ---------------------------------------------------------------- the BF16 shard
 * [parallel] tp with [dtype] bf16: the same row sharding on the BF16 MFMA kernels of the
 * batched engine, activations BATCH-major (the BF16 GEMMs' layout: H [Bp][features]):
 *
 *   forward   Hloc_l [Bp][n_l] = f(A [Bp][Mp_l] . Wb_l[R_r]^T)            gemm_nt, ACT epilogue
 *             stage [P][Bp][n_l] = all_gather(Hloc_l)   (BF16, half the FP32 bytes)
 *             Hfull_l [Bp][P n_l] = block_permute(stage)                  one pass
 *   output    replicated: Z = Hfull_{L-2} Wb_o^T (FP32), output_delta -> DL (BF16)
 *   backward  Dloc_{L-2} = f'(Hloc) * (DL . Wt_o[R_r]^T)                 gemm_nt, DACT epilogue
 *             slab_l = Dloc_l^T A                                          gemm_tn, split-K
 *             part[p] [Bp][n_{l-1}] = Dloc_l . Wt_l[rows of rank p]^T      P gemm_nt, FP32 out
 *             Dloc_{l-1} = bf16(f'(Hloc_{l-1}) * reduce_scatter(part))    FP32 sum, one pass
 *   update    hpnn_sgd_update_multi over this rank's rows (FP32 masters, BF16 W and W^T)
 *
 * The weights never move; per step a rank sends (P-1)/P x Bp x (2 B per gathered activation +
 * 4 B per reduced delta) x (sum of hidden widths).  Rows padded to P x 32 ceil(N / 32 P) with
 * zero weights; the batch padded to a multiple of 128 with zero samples (no gradient). */
static inline unsigned short bf16_rne(float f) {
    unsigned int u;
    memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (unsigned short)(u >> 16); /* inf / nan */
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}

struct TpNetBf16 {
    typedef float coll_t;
    static const char *name() { return "bf16"; }
    int L = 0, P = 1, r = 0, B = 0, Bp = 0, n_out = 0, No = 0, type = 2, nb = 0;
    int Ntrue[16], Mtrue[16], n[16], Mp[16], S[16];
    float *W32[16] = {0}, *V32[16] = {0}, *slab[16] = {0};
    void *Wb[16] = {0}, *Wt[16] = {0}, *Hloc[16] = {0}, *Hfull[16] = {0}, *Dloc[16] = {0};
    void *DL = nullptr, *hstage = nullptr, *X16 = nullptr;
    float *Z = nullptr, *part = nullptr, *dred = nullptr, *T32 = nullptr;
    float *acc = nullptr;
    hipStream_t s = nullptr;
    TpColl<float> *coll = nullptr;

    ~TpNetBf16() {
        if (s) hipStreamSynchronize(s);
        for (int l = 0; l < 16; l++) {
            void *bufs[] = {W32[l], V32[l], slab[l], Wb[l], Wt[l], Hloc[l], Hfull[l], Dloc[l]};
            for (void *b : bufs) hpnn_dev_free(b);
        }
        void *bufs[] = {DL, hstage, X16, Z, part, dred, T32, acc};
        for (void *b : bufs) hpnn_dev_free(b);
    }
    static int pad32(int v) { return (v + 31) / 32 * 32; }
    int grow(int l, int j) const { return l < L - 1 ? r * n[l] + j : j; }

    BOOL put_rows(float *dst, const DOUBLE *src, int l) {
        std::vector<float> tmp((size_t)n[l] * Mp[l], 0.f);
        for (int j = 0; j < n[l]; j++) {
            const int g = grow(l, j);
            if (g >= Ntrue[l]) continue;
            for (int m = 0; m < Mtrue[l]; m++) tmp[(size_t)j * Mp[l] + m] = (float)src[(size_t)g * Mtrue[l] + m];
        }
        TPCHK(hipMemcpyAsync(dst, tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice, s));
        TPCHK(hipStreamSynchronize(s));
        return TRUE;
    }

    BOOL init(kernel_ann *k, int P_, int r_, int B_, nn_type t, bool momentum, hipStream_t st, TpColl<float> *c) {
        P = P_, r = r_, s = st, coll = c, B = B_;
        Bp = (B + 127) / 128 * 128;
        L = (int)k->n_hiddens + 1;
        n_out = (int)k->n_outputs;
        No = pad32(n_out);
        type = t == NN_TYPE_ANN ? 0 : (t == NN_TYPE_LNN ? 1 : 2);
        if (L > 1 + HPNN_UPD_MAX * 2) return FALSE;
        size_t part_elems = 0, stage_b = 0, red = 0;
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_at(k, l);
            Ntrue[l] = (int)ly->n_neurons;
            Mtrue[l] = (int)ly->n_inputs;
            n[l] = l < L - 1 ? pad32((Ntrue[l] + P - 1) / P) : No;
            Mp[l] = l == 0 ? pad32(Mtrue[0]) : P * n[l - 1];
            S[l] = hpnn::BPlan::pick_splits(n[l], Mp[l], Bp);
            const size_t nw = (size_t)n[l] * Mp[l];
            TPCHK(hpnn_dev_malloc(&W32[l], nw * 4));
            TPCHK(hpnn_dev_malloc(&Wb[l], nw * 2));
            TPCHK(hpnn_dev_malloc(&Wt[l], nw * 2));
            TPCHK(hpnn_dev_malloc(&slab[l], nw * 4 * S[l]));
            if (momentum) {
                TPCHK(hpnn_dev_malloc(&V32[l], nw * 4));
                TPCHK(hipMemsetAsync(V32[l], 0, nw * 4, s));
            }
            if (l < L - 1) {
                TPCHK(hpnn_dev_malloc(&Hloc[l], (size_t)Bp * n[l] * 2));
                TPCHK(hpnn_dev_malloc(&Dloc[l], (size_t)Bp * n[l] * 2));
                if (P > 1) {
                    TPCHK(hpnn_dev_malloc(&Hfull[l], (size_t)Bp * P * n[l] * 2));
                    stage_b = std::max(stage_b, (size_t)Bp * P * n[l] * 2);
                } else {
                    Hfull[l] = nullptr; /* the local rows are the whole layer */
                }
            }
            if (l >= 1 && l < L - 1) {
                part_elems = std::max(part_elems, (size_t)P * Bp * n[l - 1]);
                red = std::max(red, (size_t)Bp * n[l - 1]);
            }
            if (!put_rows(W32[l], ly->weights, l)) return FALSE;
            TPK(hpnn_cast_weights(W32[l], Wb[l], Wt[l], n[l], Mp[l], s), "weight cast");
        }
        TPCHK(hpnn_dev_malloc(&Z, (size_t)Bp * No * 4));
        TPCHK(hpnn_dev_malloc(&DL, (size_t)Bp * No * 2));
        TPCHK(hipMemsetAsync(DL, 0, (size_t)Bp * No * 2, s));
        if (stage_b) TPCHK(hpnn_dev_malloc(&hstage, stage_b));
        if (part_elems) TPCHK(hpnn_dev_malloc(&part, part_elems * 4));
        if (red) TPCHK(hpnn_dev_malloc(&dred, red * 4));
        TPCHK(hpnn_dev_malloc(&acc, ACC_BYTES));
        TPCHK(hipMemsetAsync(acc, 0, ACC_BYTES, s));
        TPCHK(hipStreamSynchronize(s));
        return TRUE;
    }

    BOOL upload_momentum(const kernel_ann *k) {
        if (!k->dw) return TRUE;
        for (int l = 0; l < L; l++)
            if (V32[l] && !put_rows(V32[l], k->dw[l], l)) return FALSE;
        return TRUE;
    }

    /* the sample set per batch, zero-padded: X [nb][Bp][Mp0] BF16, targets [nb][Bp][n_out] FP32 */
    BOOL upload_data(const DOUBLE *X, const DOUBLE *Tg, UINT ns, int n_in, int) {
        nb = (int)((ns + B - 1) / B);
        const int K0 = Mp[0];
        std::vector<unsigned short> h((size_t)nb * Bp * K0, 0);
        std::vector<float> t((size_t)nb * Bp * n_out, 0.f);
        for (UINT i = 0; i < ns; i++) {
            const size_t row = (size_t)(i / B) * Bp + i % B;
            for (int c = 0; c < n_in; c++) h[row * K0 + c] = bf16_rne((float)X[(size_t)i * n_in + c]);
            for (int c = 0; c < n_out; c++) t[row * n_out + c] = (float)Tg[(size_t)i * n_out + c];
        }
        TPCHK(hpnn_dev_malloc(&X16, h.size() * 2));
        TPCHK(hipMemcpyAsync(X16, h.data(), h.size() * 2, hipMemcpyHostToDevice, s));
        TPCHK(hpnn_dev_malloc(&T32, t.size() * 4));
        TPCHK(hipMemcpyAsync(T32, t.data(), t.size() * 4, hipMemcpyHostToDevice, s));
        TPCHK(hipStreamSynchronize(s));
        return TRUE;
    }

    const void *hin(int l, const void *X) const {
        if (l == 0) return X;
        return P > 1 ? Hfull[l - 1] : Hloc[l - 1];
    }

    BOOL step(const void *X, const float *Tt, int nv, double lr, double alpha, bool mom) {
        /* forward of the sharded hidden layers */
        for (int l = 0; l < L - 1; l++) {
            TPK(hpnn_gemm_nt_bf16(hin(l, X), Mp[l], Wb[l], Mp[l], Hloc[l], n[l], nullptr, 0, Bp, n[l], Mp[l],
                                  HPNN_EPI_ACT, 0, s),
                "forward GEMM");
            if (P > 1) {
                if (!coll->all_gather((const float *)Hloc[l], (float *)hstage, (long)Bp * n[l] / 2, s)) {
                    NN_ERROR(stderr, "tensor-parallel activation all-gather failed (layer %d)\n", l);
                    return FALSE;
                }
                TPK(hpnn_block_permute_bf16(hstage, Hfull[l], P, Bp, n[l], s), "activation permute");
            }
        }
        /* replicated output layer */
        const int o = L - 1;
        const void *Ho = hin(o, X);
        TPK(hpnn_gemm_nt_bf16(Ho, Mp[o], Wb[o], Mp[o], Z, No, nullptr, 0, Bp, No, Mp[o], HPNN_EPI_NONE, 1, s),
            "output GEMM");
        TPK(hpnn_output_delta(Z, No, Tt, n_out, nullptr, 1.f, -1.f, DL, No, nullptr, 0, acc, (unsigned int *)(acc + 1),
                              Bp, nv, n_out, type, s),
            "output layer");
        TPK(hpnn_gemm_tn_bf16(DL, No, Ho, Mp[o], slab[o], Mp[o], No, Mp[o], Bp, S[o], s), "output gradient");
        if (L >= 2) {
            const int h = L - 2;
            TPK(hpnn_gemm_nt_bf16(DL, No, (const char *)Wt[o] + (size_t)r * n[h] * No * 2, No, Dloc[h], n[h], Hloc[h],
                                  n[h], Bp, n[h], No, HPNN_EPI_DACT, 0, s),
                "delta GEMM");
        }
        for (int l = L - 2; l >= 0; l--) {
            TPK(hpnn_gemm_tn_bf16(Dloc[l], n[l], hin(l, X), Mp[l], slab[l], Mp[l], n[l], Mp[l], Bp, S[l], s),
                "weight gradient");
            if (l > 0) {
                const int m = n[l - 1];
                for (int q = 0; q < P; q++)
                    TPK(hpnn_gemm_nt_bf16(Dloc[l], n[l], (const char *)Wt[l] + (size_t)q * m * n[l] * 2, n[l],
                                          part + (size_t)q * Bp * m, m, nullptr, 0, Bp, m, n[l], HPNN_EPI_NONE, 1, s),
                        "partial delta GEMM");
                const float *sum = part;
                if (P > 1) {
                    if (!coll->reduce_scatter(part, dred, (long)Bp * m, s)) {
                        NN_ERROR(stderr, "tensor-parallel delta reduce-scatter failed (layer %d)\n", l);
                        return FALSE;
                    }
                    sum = dred;
                }
                TPK(hpnn_dact_f32_bf16(Dloc[l - 1], sum, Hloc[l - 1], (long)Bp * m, s), "f' epilogue");
            }
        }
        const float scale = 1.0f / (float)(nv > 0 ? nv : 1);
        hpnn_upd_layer u[HPNN_UPD_MAX];
        for (int l0 = 0; l0 < L; l0 += HPNN_UPD_MAX) {
            const int cnt = std::min(HPNN_UPD_MAX, L - l0);
            for (int i = 0; i < cnt; i++) {
                const int l = l0 + i;
                u[i] = hpnn_upd_layer{W32[l], V32[l], slab[l], (long)n[l] * Mp[l], Wb[l], Wt[l], nullptr, S[l], n[l],
                                      Mp[l]};
            }
            TPK(hpnn_sgd_update_multi(u, cnt, (float)lr, (float)alpha, scale, mom ? 1 : 0, s), "update");
        }
        return hpnn_debug_check("tensor-parallel bf16 step") == 0;
    }
    BOOL batch_step(int b, int, int nv, double lr, double alpha, bool mom) {
        return step((const char *)X16 + (size_t)b * Bp * Mp[0] * 2, T32 + (size_t)b * Bp * n_out, nv, lr, alpha, mom);
    }
    size_t stage_elems() const { /* in floats: every rank's whole send buffer */
        size_t st = 0;
        for (int l = 0; l < L - 1; l++) {
            st = std::max(st, (size_t)P * Bp * n[l] / 2);                     /* all-gather (BF16) */
            if (l + 1 < L - 1) st = std::max(st, (size_t)P * P * Bp * n[l]); /* reduce-scatter */
        }
        for (int l = 0; l < L; l++) st = std::max(st, (size_t)P * n[l] * Mp[l]);
        return st;
    }
    BOOL read_stats(double *loss, unsigned int *hits) {
        std::vector<float> h(ACC_BYTES / 4);
        TPCHK(hipMemcpyAsync(h.data(), acc, ACC_BYTES, hipMemcpyDeviceToHost, s));
        TPCHK(hipStreamSynchronize(s));
        double l = 0.0;
        unsigned int c = 0;
        for (int i = 0; i < HPNN_STAT_SLOTS; i++) {
            l += h[(size_t)i * HPNN_STAT_STRIDE];
            unsigned int u;
            memcpy(&u, &h[(size_t)i * HPNN_STAT_STRIDE + 1], 4);
            c += u;
        }
        *loss = l;
        *hits = c;
        return TRUE;
    }
    /* rows [rank_rows_of ...] of h ([sh n_l][Mp_l] FP32) -> host weights / momentum of layer l */
    void to_host(kernel_ann *k, int l, bool momentum, const std::vector<float> &h, int rows, int row0) {
        layer_ann *ly = layer_at(k, l);
        DOUBLE *dst = momentum ? k->dw[l] : ly->weights;
        for (int j = 0; j < rows; j++) {
            const int g = row0 + j;
            if (g >= Ntrue[l]) continue;
            for (int m = 0; m < Mtrue[l]; m++) dst[(size_t)g * Mtrue[l] + m] = (DOUBLE)h[(size_t)j * Mp[l] + m];
        }
    }
    BOOL host_rows(kernel_ann *k, bool mom) {
        for (int l = 0; l < L; l++)
            for (int pass = 0; pass < (mom ? 2 : 1); pass++) {
                const float *src = pass ? V32[l] : W32[l];
                if (!src) continue;
                std::vector<float> h((size_t)n[l] * Mp[l]);
                TPCHK(hipMemcpyAsync(h.data(), src, h.size() * 4, hipMemcpyDeviceToHost, s));
                TPCHK(hipStreamSynchronize(s));
                to_host(k, l, pass == 1, h, n[l], l < L - 1 ? r * n[l] : 0);
            }
        return TRUE;
    }
    BOOL gather_to_host(kernel_ann *k, TpColl<float> &cl, int W_, bool mom) {
        for (int l = 0; l < L; l++) {
            const long cnt = (long)n[l] * Mp[l];
            const int sh = l < L - 1 ? W_ : 1;
            for (int pass = 0; pass < (mom ? 2 : 1); pass++) {
                const float *src = pass ? V32[l] : W32[l];
                if (!src) continue;
                float *full = nullptr;
                TPCHK(hpnn_dev_malloc(&full, (size_t)cnt * sh * 4));
                bool ok = sh > 1 ? cl.gather_rows(src, full, cnt, s)
                                 : hipMemcpyAsync(full, src, cnt * 4, hipMemcpyDeviceToDevice, s) == hipSuccess;
                std::vector<float> h((size_t)cnt * sh);
                ok = ok && hipMemcpyAsync(h.data(), full, h.size() * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
                     hipStreamSynchronize(s) == hipSuccess;
                hpnn_dev_free(full);
                if (!ok) return FALSE;
                to_host(k, l, pass == 1, h, sh * n[l], 0);
            }
        }
        return TRUE;
    }
};
#undef TPK

/* the epoch loop of one rank; over RCCL each epoch's launches (collectives included) are
 * captured once in a HIP graph and replayed (HPNN_GRAPH=0 or HPNN_DEBUG: eager) */
template <class Net>
BOOL run_rank(Net &net, UINT n, const hpnn_batched_opts *o, int B, double *ep_loss, unsigned int *ep_hits) {
    const bool mom = o->train == NN_TRAIN_BPM;
    const int n_batches = (int)((n + B - 1) / B);
    auto epoch = [&]() -> bool {
        for (int b = 0; b < n_batches; b++) {
            const int nv = (b == n_batches - 1) ? (int)n - b * B : B;
            if (!net.batch_step(b, B, nv, o->lr, o->alpha, mom)) return false;
        }
        return true;
    };
    const char *ge = getenv("HPNN_GRAPH");
    hipGraphExec_t gx = nullptr;
    if (net.coll->capturable() && !(ge && ge[0] == '0') && !hpnn_debug_enabled() && n_batches <= 4096) {
        hipGraph_t g = nullptr;
        bool ok = hipStreamBeginCapture(net.s, hipStreamCaptureModeRelaxed) == hipSuccess;
        const bool okb = ok && epoch();
        ok = ok && hipStreamEndCapture(net.s, &g) == hipSuccess && g && okb &&
             hipGraphInstantiate(&gx, g, nullptr, nullptr, 0) == hipSuccess;
        if (g) hipGraphDestroy(g);
        if (!ok) {
            gx = nullptr;
            hipGetLastError();
            NN_DBG(stdout, "tensor-parallel rank %d: epoch not capturable, eager launches\n", net.r);
        }
    }
    for (UINT e = 0; e < o->epochs; e++) {
        TPCHK(hipMemsetAsync(net.acc, 0, ACC_BYTES, net.s));
        if (gx) {
            if (hipGraphLaunch(gx, net.s) != hipSuccess) {
                hipGraphExecDestroy(gx);
                return FALSE;
            }
        } else if (!epoch()) {
            return FALSE;
        }
        if (!net.read_stats(ep_loss, ep_hits)) {
            if (gx) hipGraphExecDestroy(gx);
            return FALSE;
        }
        if (net.r == 0 && hpnn_metrics_active())
            hpnn_metrics_epoch("gpu-tp", o->epoch0 + e + 1, *ep_loss / (double)n, *ep_hits, n, 0.0,
                               (UINT64)n * (e + 1));
    }
    if (gx) hipGraphExecDestroy(gx);
    TPCHK(hipStreamSynchronize(net.s));
    return TRUE;
}

/* P ranks as host threads of this process: loopback (all on device 0, staging-buffer
 * collectives) or one per GPU (RCCL) */
template <class Net>
BOOL train_tp_threads(kernel_ann *k, const DOUBLE *X, const DOUBLE *Tg, UINT n, const hpnn_batched_opts *o,
                      hpnn_batched_stats *st, int P, bool loopback) {
    typedef typename Net::coll_t T;
    const int B = (int)(o->batch ? o->batch : 256);
    const int n_batches = (int)((n + B - 1) / B);
    const int cols = n_batches * B;
    const bool mom = o->train == NN_TRAIN_BPM;
    std::vector<int> dev(P);
    std::vector<hipStream_t> str(P);
    for (int g = 0; g < P; g++) {
        dev[g] = loopback ? hpnn_rt_device(0) : hpnn_rt_device((UINT)g);
        str[g] = loopback ? nullptr : hpnn_rt_stream((UINT)g, 0);
    }
    HostShared<T> shared;
    shared.P = P;
    shared.bar.P = P;
    std::vector<hpnn_comm *> comms(P, nullptr);
    std::vector<std::unique_ptr<TpColl<T>>> colls(P);
    if (!loopback) {
        if (!hpnn_comm_available() || hpnn_comm_init_all(comms.data(), P, dev.data()) != 0) {
            NN_ERROR(stderr, "tensor parallelism over %d GPUs needs RCCL\n", P);
            return FALSE;
        }
        for (int g = 0; g < P; g++) colls[g].reset(new RcclColl<T>(comms[g]));
    } else {
        for (int g = 0; g < P; g++) colls[g].reset(new HostColl<T>(&shared, g));
    }
    std::vector<std::unique_ptr<Net>> nets(P);
    std::vector<int> tok(P, 1);
    std::vector<double> losses(P, 0.0);
    std::vector<unsigned int> hits(P, 0);
    if (mom) ann_momentum_init(k);
    BOOL ok = TRUE;
    /* setup (serial: allocation sizes of the staging buffer depend on every shard) */
    for (int g = 0; g < P && ok; g++) {
        if (hipSetDevice(dev[g]) != hipSuccess) ok = FALSE;
        if (ok && loopback && hipStreamCreateWithFlags(&str[g], hipStreamNonBlocking) != hipSuccess) ok = FALSE;
        if (!ok) break;
        nets[g].reset(new Net());
        ok = nets[g]->init(k, P, g, B, o->type, mom, str[g], colls[g].get());
        if (ok && mom && o->resume) ok = nets[g]->upload_momentum(k);
        if (ok) ok = nets[g]->upload_data(X, Tg, n, (int)k->n_inputs, cols + B);
    }
    if (ok && loopback) {
        const size_t stage = nets[0]->stage_elems();
        hipSetDevice(dev[0]);
        if (hpnn_dev_malloc(&shared.stage, (stage ? stage : 1) * sizeof(T)) != hipSuccess) ok = FALSE;
    }
    NN_OUT(stdout, "tensor-parallel batched training: %d ranks (%s, %s), rows of every hidden layer sharded, "
                   "%d samples per step\n",
           P, loopback ? "loopback on one GPU" : "RCCL", Net::name(), B);
    for (int g = 0; g < P; g++) {
        hipSetDevice(dev[g]);
        hpnn_preload_code_objects();
    }
    hipSetDevice(dev[0]);
    auto t0 = std::chrono::steady_clock::now();
    if (ok) {
        std::vector<std::thread> th;
        for (int g = 0; g < P; g++)
            th.emplace_back([&, g]() {
                if (hipSetDevice(dev[g]) != hipSuccess || !run_rank<Net>(*nets[g], n, o, B, &losses[g], &hits[g])) {
                    tok[g] = 0;
                    colls[g]->abort();
                }
            });
        for (auto &t : th) t.join();
        for (int g = 0; g < P; g++) ok = ok && tok[g];
    }
    auto t1 = std::chrono::steady_clock::now();
    if (ok && !loopback)
        for (int g = 0; g < P; g++) ok = ok && hpnn_comm_check(comms[g]) == 0;
    /* every rank's rows -> the host kernel */
    for (int g = 0; g < P && ok; g++) {
        hipSetDevice(dev[g]);
        ok = nets[g]->host_rows(k, mom);
    }
    if (ok && st) {
        st->seconds = std::chrono::duration<double>(t1 - t0).count();
        st->samples = (UINT64)n * o->epochs;
        st->epoch_loss = losses[0] / (double)n;
        st->correct = hits[0];
        st->last_loss = st->epoch_loss;
    }
    for (int g = 0; g < P; g++) {
        hipSetDevice(dev[g]);
        nets[g].reset();
        if (loopback && str[g]) hipStreamDestroy(str[g]);
        if (comms[g]) hpnn_comm_destroy(comms[g]);
    }
    hipSetDevice(hpnn_rt_device(0));
    return ok;
}

/* one process per GPU under a launcher (RANK / WORLD_SIZE / LOCAL_RANK): RCCL collectives;
 * every rank ends with the full weights in its host kernel (all-gather of the rows) */
template <class Net>
BOOL train_tp_mp(kernel_ann *k, const DOUBLE *X, const DOUBLE *Tg, UINT n, const hpnn_batched_opts *o,
                 hpnn_batched_stats *st) {
    typedef typename Net::coll_t T;
    const int W = hpnn_boot_world(), R = hpnn_boot_rank();
    const int dev = hpnn_rt_device(0);
    TPCHK(hipSetDevice(dev));
    hipStream_t s = hpnn_rt_stream(0, 0);
    if (!hpnn_comm_available()) {
        NN_ERROR(stderr, "tensor parallelism across processes needs RCCL\n");
        return FALSE;
    }
    unsigned char id[HPNN_COMM_ID_BYTES] = {0};
    std::vector<unsigned char> all((size_t)W * HPNN_COMM_ID_BYTES);
    if (R == 0 && hpnn_comm_unique_id(id) != 0) return FALSE;
    if (hpnn_boot_allgather(id, sizeof id, all.data()) != 0) return FALSE;
    hpnn_comm *comm = hpnn_comm_init_rank(all.data(), W, R, dev);
    if (!comm) return FALSE;
    RcclColl<T> coll(comm);
    const int B = (int)(o->batch ? o->batch : 256);
    const int n_batches = (int)((n + B - 1) / B);
    const int cols = n_batches * B + B;
    const bool mom = o->train == NN_TRAIN_BPM;
    if (mom) ann_momentum_init(k);
    Net net;
    BOOL ok = net.init(k, W, R, B, o->type, mom, s, &coll);
    if (ok && mom && o->resume) ok = net.upload_momentum(k);
    if (ok) ok = net.upload_data(X, Tg, n, (int)k->n_inputs, cols);
    NN_OUT(stdout, "tensor-parallel batched training: %d processes (RCCL, %s), %d samples per step\n", W,
           Net::name(), B);
    double loss = 0.0;
    unsigned int hits = 0;
    hpnn_preload_code_objects();
    auto t0 = std::chrono::steady_clock::now();
    if (ok) ok = run_rank<Net>(net, n, o, B, &loss, &hits);
    auto t1 = std::chrono::steady_clock::now();
    if (ok) ok = hpnn_comm_check(comm) == 0;
    /* all ranks agree before the weights are gathered (a failed rank issues no collective) */
    int okv = ok ? 1 : 0;
    std::vector<int> oks(W);
    if (hpnn_boot_allgather(&okv, sizeof okv, oks.data()) != 0) ok = FALSE;
    for (int v : oks) ok = ok && v;
    if (ok) ok = net.gather_to_host(k, coll, W, mom);
    if (ok && st) {
        st->seconds = std::chrono::duration<double>(t1 - t0).count();
        st->samples = (UINT64)n * o->epochs;
        st->epoch_loss = loss / (double)n;
        st->correct = hits;
        st->last_loss = st->epoch_loss;
    }
    hipStreamSynchronize(s);
    hpnn_boot_finish();
    hpnn_comm_destroy(comm);
    return ok;
}

template <class Net>
BOOL train_tp(kernel_ann *k, const DOUBLE *X, const DOUBLE *Tg, UINT n, const hpnn_batched_opts *o,
              hpnn_batched_stats *st) {
    if (k->n_hiddens + 1 > 16) return FALSE;
    hpnn_gpu_sync_host(k);
    const char *lb = getenv("HPNN_LOOPBACK_RANKS");
    const int lbr = lb ? atoi(lb) : 0;
    BOOL ok;
    /* HPNN_FORCE_RCCL=1: RCCL collectives (and the epoch graphs) even for one GPU */
    const char *fr = getenv("HPNN_FORCE_RCCL");
    const bool rccl1 = fr && fr[0] == '1';
    if (lbr >= 2) ok = train_tp_threads<Net>(k, X, Tg, n, o, st, lbr, true);
    else if (hpnn_boot_world() > 1) ok = train_tp_mp<Net>(k, X, Tg, n, o, st);
    else if (o->n_gpu > 1 || rccl1)
        ok = train_tp_threads<Net>(k, X, Tg, n, o, st, o->n_gpu > 1 ? (int)o->n_gpu : 1, false);
    else ok = train_tp_threads<Net>(k, X, Tg, n, o, st, 1, true);
    if (ok) hpnn_gpu_mark_host_dirty(k);
    return ok;
}

}  // namespace

extern "C" BOOL hpnn_gpu_train_tp(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n, const hpnn_batched_opts *o,
                                  hpnn_batched_stats *st) {
    if (o->dtype == NN_DTYPE_F64) return train_tp<TpNet<double>>(k, X, T, n, o, st);
    if (o->dtype == NN_DTYPE_F32) return train_tp<TpNet<float>>(k, X, T, n, o, st);
    return train_tp<TpNetBf16>(k, X, T, n, o, st);
}
